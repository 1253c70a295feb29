"""The C-ABI boundary on CPU: the library loads, exports every symbol
include/ec_method.h declares, keeps the 120-byte ec_matrix_list_t layout, and
its host-side math (GF(2^8), encode matrix, inverse) matches the oracle.
Without a GPU, ec_method_init selects the CPU engine (tests/test_cpu_engine.py
checks its output against the oracle)."""
import ctypes
import itertools
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "include", "ec_method.h")
LIB = os.path.join(ROOT, "glusterfs_amd", "lib", "libec_mi355x.so")


def declared():
    text = open(HDR).read()
    return sorted(set(re.findall(r"\b(ec_method_\w+)\s*\(", text)))


def test_header_matches_python_mirror():
    import glusterfs_amd.ec_method as m
    assert sorted(m.EXPORTS) == declared()


def test_library_exports_every_declared_symbol():
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True,
                         text=True, check=True).stdout
    syms = set(l.split()[-1] for l in out.splitlines() if " T " in l)
    missing = [s for s in declared() if s not in syms]
    assert not missing, missing
    lib = ctypes.CDLL(LIB)
    for s in declared():
        assert getattr(lib, s)


def test_library_is_not_unloadable():
    """The library owns registered host memory, a registration thread and
    the free hook the integration patch installs in libglusterfs's iobuf
    layer (iobuf_set_data_allocator keeps it for buffers still out), so it
    is linked -z nodelete: dlclose of the ec xlator must not unmap it."""
    out = subprocess.run(["readelf", "-d", LIB], capture_output=True, text=True,
                         check=True).stdout
    assert "NODELETE" in out, out


def test_reference_prototypes_unchanged():
    """The five drop-in prototypes are those of ec-method.h:31-46."""
    text = " ".join(open(HDR).read().split())
    for proto in (
        "int32_t ec_method_init(xlator_t *xl, ec_matrix_list_t *list, uint32_t columns, "
        "uint32_t rows, uint32_t max, const char *gen);",
        "void ec_method_fini(ec_matrix_list_t *list);",
        "int32_t ec_method_update(xlator_t *xl, ec_matrix_list_t *list, const char *gen);",
        "void ec_method_encode(ec_matrix_list_t *list, uint64_t size, void *in, void **out);",
        "int32_t ec_method_decode(ec_matrix_list_t *list, uint64_t size, uintptr_t mask, "
        "uint32_t *rows, void **in, void *out);",
    ):
        assert proto in text, proto


def _build_c_check(tmp_path):
    exe = str(tmp_path / "abi_check")
    subprocess.run(["gcc", "-std=c11", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "c", "abi_check.c"), "-o", exe,
                    "-L", os.path.dirname(LIB), "-lec_mi355x",
                    "-Wl,-rpath," + os.path.dirname(LIB)], check=True)
    return exe


def test_c_caller_layout_and_cpu_engine(tmp_path):
    """A plain C caller: layout, -EINVAL on a bad geometry, fini after a
    failed init, and an encode/decode round trip on the CPU engine
    (cpu-extensions=none), GPU or not."""
    exe = _build_c_check(tmp_path)
    r = subprocess.run([exe, "cpu"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "roundtrip ok" in r.stdout, r.stdout + r.stderr
    assert "engine cpu/" in r.stdout


@pytest.mark.gpu
def test_c_caller_roundtrip_on_gpu(tmp_path):
    exe = _build_c_check(tmp_path)
    r = subprocess.run([exe, "gpu"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "roundtrip ok" in r.stdout, r.stdout + r.stderr


def test_python_init_without_gpu_selects_cpu_engine():
    """The reference's coder always starts (ec-method.c:300-353): on a node
    without gfx950 the library codes on the CPU instead of failing."""
    import glusterfs_amd as g
    if g.device_count() > 0:
        pytest.skip("GPU visible")
    with g.ECMatrixList(4, 6) as L:
        assert L.engine.startswith("cpu/")
    with g.ECMatrixList(4, 6, gen="hip") as L:
        assert L.engine.startswith("cpu/")


def test_pool_and_deferred_registration_without_gpu():
    """Without a device the pinned pool hands out nothing (the integration
    patch's iobuf allocator then falls back to GF_MALLOC / GF_CALLOC), puts
    of foreign pointers are refused (the caller frees them), and deferred
    registration reports -ENODEV."""
    import errno
    import glusterfs_amd as g
    if g.device_count() > 0:
        pytest.skip("GPU visible")
    L = g.ec_method.lib
    assert not L.ec_method_buffer_get(1 << 20)
    buf = (ctypes.c_uint8 * 4096)()
    assert L.ec_method_buffer_put(ctypes.addressof(buf)) == 0
    assert L.ec_method_buffer_put(None) == 0
    assert L.ec_method_host_register_async(ctypes.addressof(buf), 4096) == -errno.ENODEV
    L.ec_method_host_register_flush()
    st = g.pool_stats()
    assert st["pool_bytes"] == 0 and st["gets"] == 0 and st["deferred_registers"] == 0
    b = g.PoolBuffer(8192)
    assert not b.pooled and b.array.nbytes == 8192


def test_encode_rows_device_argument_errors_without_gpu():
    """ec_method_encode_rows_device: bits beyond the volume's bricks and NULL
    output slots of selected bricks are -EINVAL before any device work; an
    empty mask or zero stripes are no-ops; a real request without a device is
    -ENODEV (device-resident entry points have no CPU path to fall back to)."""
    import errno
    import glusterfs_amd as g
    if g.device_count() > 0:
        pytest.skip("GPU visible")
    with g.ECMatrixList(4, 6) as L:
        lib = g.ec_method.lib
        src = (ctypes.c_uint8 * (512 * 4))()
        dst = [(ctypes.c_uint8 * 512)() for _ in range(6)]
        outs = (ctypes.c_void_p * 6)(*[ctypes.addressof(d) for d in dst])
        call = lambda nst, m, o: lib.ec_method_encode_rows_device(  # noqa: E731
            ctypes.byref(L._list), 0, None, nst, ctypes.addressof(src), m, o)
        assert call(1, 1 << 6, outs) == -errno.EINVAL
        holes = (ctypes.c_void_p * 6)(None, *[ctypes.addressof(d) for d in dst[1:]])
        assert call(1, 0x1, holes) == -errno.EINVAL
        assert call(1, 0, outs) == 0 and call(0, 0x3, outs) == 0
        assert call(1, 0x3, outs) == -errno.ENODEV


def test_host_matrices_match_oracle(oracle):
    import glusterfs_amd as g
    for k, n in ((2, 3), (4, 6), (8, 12), (16, 20), (16, 31), (5, 7)):
        assert np.array_equal(np.array(g.encode_matrix(k, n)), oracle.encode_matrix(k, n))
    rng = np.random.default_rng(3)
    for k, n in ((2, 3), (3, 5), (4, 6), (8, 12), (16, 20), (16, 31)):
        if n <= 12:
            picks = list(itertools.combinations(range(1, n + 1), k))
        else:
            picks = [sorted(rng.choice(n, k, replace=False) + 1) for _ in range(60)]
        for rows in picks:
            rows = [int(r) for r in rows]
            assert g.inverse_matrix(list(rows)) == oracle.inverse_matrix(list(rows)).tolist()


def test_host_gf_semantics():
    import glusterfs_amd as g
    from test_oracle import py_gf_mul, py_gf_inv
    for a in range(256):
        for b in (0, 1, 7, 0x80, 0xFF):
            assert g.gf_mul(a, b) == py_gf_mul(a, b)
    for a in range(1, 256):
        assert g.gf_div(1, a) == py_gf_inv(a)
    assert g.gf_mul(300, 1) == 256 and g.gf_div(5, 0) == 256


def test_inverse_rejects_bad_rows():
    import glusterfs_amd as g
    with pytest.raises(OSError):
        g.inverse_matrix([1, 1, 2, 3])       # repeated evaluation point
    with pytest.raises(OSError):
        g.inverse_matrix([0, 1, 2, 3])       # rows are brick index + 1 >= 1
