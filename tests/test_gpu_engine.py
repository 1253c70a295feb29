"""Engine selection on a GPU node: the CPU fallback after a device error
(fault injection), the CPU/GPU crossover at its default thresholds, and the
cpu-extensions values that pin the CPU engine.  Outputs are compared with the
oracle bit for bit."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

CHUNK = 512
HERE = os.path.dirname(os.path.abspath(__file__))


def rnd(n, seed):
    return np.random.default_rng(seed).integers(0, 256, size=n, dtype=np.uint8)


@pytest.fixture(scope="module")
def ec():
    import glusterfs_amd as g
    if g.device_count() < 1:
        pytest.fail("no MI355X visible")
    return g


def test_auto_engine_is_gfx950(ec):
    with ec.ECMatrixList(4, 6) as L:
        assert L.engine.startswith("gfx950")
    with ec.ECMatrixList(4, 6, gen="none") as L:
        assert L.engine.startswith("cpu/")


def test_device_fault_falls_back_to_cpu(ec, oracle):
    """A failed device submission is redone on the CPU engine: every host
    entry point still returns oracle-exact data (ec-method.c:393-408 cannot
    fail), and the fallback is counted."""
    import ctypes
    k, n, nst = 8, 12, 300
    data = rnd(CHUNK * k * nst, 1)
    want = oracle.encode(k, n, data)
    with ec.ECMatrixList(k, n) as L:
        f0 = ec.stats()["cpu_fallbacks"]
        # ec_method_encode (void): the drop-in call
        bufs = [np.zeros(CHUNK * nst, np.uint8) for _ in range(n)]
        ptrs = (ctypes.c_void_p * n)(*[b.ctypes.data for b in bufs])
        ec.inject_device_faults(1)
        ec.ec_method.lib.ec_method_encode(ctypes.byref(L._list), data.size, data.ctypes.data,
                                          ptrs)
        assert all(np.array_equal(a, b) for a, b in zip(bufs, want))
        # decode
        rows = [2, 3, 5, 6, 7, 9, 10, 12]
        mask = sum(1 << (r - 1) for r in rows)
        out = np.zeros(data.size, np.uint8)
        ec.inject_device_faults(1)
        L.decode(CHUNK * nst, mask, rows, [want[r - 1] for r in rows], out)
        assert np.array_equal(out, data)
        # mixed-pattern decode
        out[:] = 0
        ec.inject_device_faults(1)
        L.decode_mixed(nst, 16, [mask, 0xFF0] * 10, want, out)
        assert np.array_equal(out, data)
        # heal
        tgt = [0, 3, 7, 10]
        outs = [np.zeros(CHUNK * nst, np.uint8) for _ in tgt]
        ec.inject_device_faults(1)
        L.heal(nst, mask, [want[r - 1] for r in rows], sum(1 << t for t in tgt), outs)
        assert all(np.array_equal(o, want[t]) for o, t in zip(outs, tgt))
        # partial-stripe write
        S = CHUNK * k
        user = rnd(5 * S + 77, 2)
        oh, ot = rnd(S, 3), rnd(S, 4)
        v = oracle.writev_merge(k, 100, user, oh, ot)
        wv = oracle.encode(k, n, v)
        outs = [np.zeros(v.size // k, np.uint8) for _ in range(n)]
        ec.inject_device_faults(1)
        L.writev_encode(100, user, oh, ot, outs)
        assert all(np.array_equal(a, b) for a, b in zip(outs, wv))
        assert ec.stats()["cpu_fallbacks"] == f0 + 5


def test_cpu_engine_pinned_by_gen_on_gpu_node(ec, oracle):
    k, n, nst = 16, 20, 64
    data = rnd(CHUNK * k * nst, 5)
    want = oracle.encode(k, n, data)
    for gen in ("none", "x64", "sse", "avx"):
        g0 = ec.stats()
        with ec.ECMatrixList(k, n, gen=gen) as L:
            assert L.engine.startswith("cpu/")
            outs = [np.zeros(CHUNK * nst, np.uint8) for _ in range(n)]
            L.encode_batch(nst, data, outs)
        assert all(np.array_equal(a, b) for a, b in zip(outs, want)), gen
        g1 = ec.stats()
        assert g1["gpu_calls"] == g0["gpu_calls"] and g1["cpu_calls"] == g0["cpu_calls"] + 1


CHILD = r'''
import json, sys
import numpy as np
sys.path[:0] = [sys.argv[1], sys.argv[1] + "/oracle"]
import glusterfs_amd as g, oracle as O
res = {}
def run(name, k, n, op, user, pinned=False):
    nst = user // (512 * k)
    data = np.random.default_rng(nst).integers(0, 256, 512 * k * nst, dtype=np.uint8)
    with g.ECMatrixList(k, n) as L:
        frags = O.encode(k, n, data)
        s0 = g.stats()
        if op == "enc":
            pins = [g.PinnedArray(512 * nst) for _ in range(n)] if pinned else []
            outs = [p.array for p in pins] or [np.zeros(512 * nst, np.uint8) for _ in range(n)]
            src = g.PinnedArray(data.size) if pinned else None
            if src is not None:
                src.array[:] = data
            L.encode_batch(nst, src.array if src is not None else data, outs)
            ok = all(np.array_equal(a, b) for a, b in zip(outs, frags))
            for p in pins + ([src] if src is not None else []):
                p.free()
        else:
            rows = list(range(n - k + 1, n + 1))
            out = np.zeros(data.size, np.uint8)
            L.decode(512 * nst, sum(1 << (r - 1) for r in rows), rows,
                     [frags[r - 1] for r in rows], out)
            ok = bool(np.array_equal(out, data))
        s1 = g.stats()
    res[name] = dict(gpu=s1["gpu_calls"] - s0["gpu_calls"],
                     cpu=s1["cpu_calls"] - s0["cpu_calls"], ok=ok)
run("enc4+2_128K", 4, 6, "enc", 128 << 10)
run("enc4+2_8M", 4, 6, "enc", 8 << 20)
run("dec16+4_16M", 16, 20, "dec", 16 << 20)
run("enc4+2_64M_pinned", 4, 6, "enc", 64 << 20, pinned=True)
print("XOVER " + json.dumps(res))
'''


def _crossover_child(hybrid):
    env = {k: v for k, v in os.environ.items()
           if not (k.startswith("EC_GPU_") or k.startswith("EC_CPU_") or k.startswith("EC_HYBRID"))}
    env["EC_MI355X_QUIET"] = "1"
    env["EC_HYBRID"] = "1" if hybrid else "0"
    r = subprocess.run([sys.executable, "-c", CHILD, os.path.dirname(HERE)], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("XOVER ")][0]
    return json.loads(line[6:])


def test_crossover_defaults():
    """Default cost model with split calls off (no other overrides, DESIGN.md
    1.1): FUSE-sized and cache-sized encodes on the calling thread, a 16 MiB
    16+4 decode (pageable) and a 64 MiB encode from pinned buffers on the GPU."""
    res = _crossover_child(hybrid=False)
    assert res["enc4+2_128K"] == dict(gpu=0, cpu=1, ok=True), res
    assert res["enc4+2_8M"] == dict(gpu=0, cpu=1, ok=True), res
    assert res["dec16+4_16M"] == dict(gpu=1, cpu=0, ok=True), res
    assert res["enc4+2_64M_pinned"] == dict(gpu=1, cpu=0, ok=True), res


def test_crossover_defaults_with_split_calls():
    """The same calls with split calls on (the default since r05): below
    1 MiB a call stays whole on its engine; the larger ones run whole on the
    engine the crossover picks or split across both (gpu and cpu each
    counted once), and every output is exact."""
    res = _crossover_child(hybrid=True)
    assert res["enc4+2_128K"] == dict(gpu=0, cpu=1, ok=True), res
    for name, whole in (("enc4+2_8M", dict(gpu=0, cpu=1)), ("dec16+4_16M", dict(gpu=1, cpu=0)),
                        ("enc4+2_64M_pinned", dict(gpu=1, cpu=0))):
        got = dict(res[name])
        assert got.pop("ok") is True, (name, res)
        assert got in (whole, dict(gpu=1, cpu=1)), (name, res)
