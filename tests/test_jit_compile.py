"""The run-time compiled whole-matrix kernels (glusterfs_amd/csrc/ec_jit.hip)
without a device: the library generates the kernel source of a decode
matrix and hiprtc compiles it for gfx950 here, as it does on a GPU node
(cross-compilation needs no GPU).  Checks that real inverses of 16+4 and
12+4 volumes compile and that their programs need fewer XOR instructions
per dword column than the row-by-row searched programs the shipped kernel
runs (tools/gen/gf8_prog.txt lengths).  The GPU results are checked in
tests/test_gpu_jit.py."""
import ctypes
import os

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _inverse(g, k, mask):
    rows = [i + 1 for i in range(32) if (mask >> i) & 1]
    assert len(rows) == k
    r = (ctypes.c_uint32 * k)(*rows)
    m = (ctypes.c_uint32 * (k * k))()
    assert g.ec_method.lib.ec_method_inverse_matrix(k, r, m) == 0
    return np.array(list(m), np.uint8)


def _rowwise_ops(coef):
    lens = {}
    for line in open(os.path.join(ROOT, "tools", "gen", "gf8_prog.txt")):
        f = line.split()
        lens[int(f[0])] = int(f[1])
    return sum(lens[int(c)] for c in coef if c)


@pytest.mark.parametrize("k,mask", [(16, 0xFFFF0), (16, 0x5FFF5), (12, 0xFFF0)])
def test_jit_kernel_compiles_without_gpu(k, mask):
    import glusterfs_amd as g
    coef = _inverse(g, k, mask)
    size, ops = g.jit_compile_check(k, k, coef)
    if size == -38:                                   # -ENOSYS: no hiprtc in this image
        pytest.skip("libhiprtc not available")
    assert size > 0, size
    assert 0 < ops < _rowwise_ops(coef), (ops, _rowwise_ops(coef))


def test_jit_compile_check_rejects_bad_geometry():
    import glusterfs_amd as g
    assert g.jit_compile_check(17, 16, np.ones(17 * 16, np.uint8))[0] == -22
    assert g.jit_compile_check(16, 1, np.ones(16, np.uint8))[0] == -22


EXIT_SCRIPT = r"""
import sys, numpy as np
sys.path.insert(0, %r)
import glusterfs_amd as g
rng = np.random.default_rng(int(sys.argv[1]))
coef = rng.integers(1, 256, 256, dtype=np.uint8)       # a fresh matrix: no compiler cache hit
assert g.jit_prepare(16, 16, coef) in (0, -38), "prepare"
print("queued", flush=True)
"""


def test_exit_while_a_matrix_compiles():
    """A client that exits while a matrix is still being compiled exits
    cleanly (the compile runs in the ec_jitc process; round 6's first
    version compiled on a library thread and crashed such exits in 3 of 3
    runs).  Five processes, each exiting right after queueing."""
    import subprocess
    import sys
    env = dict(os.environ, EC_MI355X_QUIET="1")
    env.pop("EC_MI355X_JIT_SYNC", None)
    for seed in range(5):
        r = subprocess.run([sys.executable, "-c", EXIT_SCRIPT % ROOT, str(seed)], env=env,
                           capture_output=True, text=True, timeout=120)
        assert r.returncode == 0 and "queued" in r.stdout, (r.returncode, r.stderr[-2000:])
