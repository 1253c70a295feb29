"""GPU parity of the run-time compiled whole-matrix kernels (r06,
glusterfs_amd/csrc/ec_jit.hip): a single-pattern device combine of a wide
code (k >= 12, >= 12 output rows) runs a kernel compiled for its coefficient
matrix once the code exists.  Every result is compared with the oracle:

  * 16+4 decodes of device fragments for the contiguous masks and scattered
    ones, tile-aligned and ragged stripe counts, fragments at an odd byte
    address (LDS-DMA reads them in place), with EC_MI355X_JIT_SYNC=1 so the
    first call compiles and every call runs the compiled kernel;
  * 12+4 decodes (12 rows: programs of 6 rows per wave) and a 16+12
    row-masked encode of 12 rows (fragment-major outputs, 512-byte runs);
  * 1 GiB calls (non-temporal staging), five per mask, as round trips;
  * the default asynchronous mode: the first call of a matrix runs the
    shipped kernel while a library thread compiles, later calls the
    compiled one -- exact both ways;
  * a process exiting while its matrix compiles exits cleanly;
  * EC_MI355X_JIT=0: never compiled, never launched.
Each case runs in its own process through the C ABI (the settings are read
once per process)."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

COMMON = r"""
import itertools, sys, time
sys.path.insert(0, "oracle")
import numpy as np, torch
import glusterfs_amd as g
import oracle as O           # the checker

rng = np.random.default_rng(11)
def rb(n):
    return rng.integers(0, 256, n, dtype=np.uint8)
def dev(a, off=0):
    if off == 0:
        return torch.from_numpy(a).cuda()
    t = torch.empty(a.size + off, dtype=torch.uint8, device="cuda")
    t[off:] = torch.from_numpy(a).cuda()
    return t[off:]

def decode_check(L, k, n, nst, mask, off=0):
    frags = [rb(512 * nst) for _ in range(n)]
    rows = O.mask_rows(mask)
    out = torch.empty(512 * k * nst, dtype=torch.uint8, device="cuda")
    out.fill_(0xA5)
    L.decode_batch(nst, mask, rows, [dev(frags[r - 1], off) for r in rows], out)
    exp = O.decode(k, rows, [frags[r - 1] for r in rows])
    assert np.array_equal(out.cpu().numpy(), exp), ("dec", k, n, nst, hex(mask), off)
"""

SYNC = COMMON + r"""
s0 = g.jit_stats()
with g.ECMatrixList(16, 20) as L:
    allm = [sum(1 << b for b in c) for c in itertools.combinations(range(20), 16)]
    masks = [0xFFFF0, 0x0FFFF, 0xF0FFF] + [allm[i] for i in rng.choice(len(allm), 3, replace=False)]
    for m in masks:
        for nst in (1024, 4099):
            decode_check(L, 16, 20, nst, m)
    decode_check(L, 16, 20, 2051, masks[3], off=3)
    decode_check(L, 16, 20, 1000, masks[0])          # below the threshold: shipped kernel
with g.ECMatrixList(12, 16) as L:
    decode_check(L, 12, 16, 1030, 0xFFF0)
    decode_check(L, 12, 16, 1030, 0x7BDE)
# a row-masked encode of 12 rows of a 16+12 volume: fragment-major outputs
with g.ECMatrixList(16, 28) as L:
    nst = 1027
    data = rb(512 * 16 * nst)
    want = O.encode(16, 28, data)
    rm = sum(1 << i for i in range(16, 28))
    outs = [torch.empty(512 * nst, dtype=torch.uint8, device="cuda") if (rm >> i) & 1 else None
            for i in range(28)]
    L.encode_rows_device(0, None, nst, dev(data), rm, outs)
    g.sync_device(0)
    for i in range(16, 28):
        assert np.array_equal(outs[i].cpu().numpy(), want[i]), ("rows", i)
s1 = g.jit_stats()
d = {k: s1[k] - s0[k] for k in s1}
print("JIT", d)
assert d["failed"] == 0, d
assert d["compiled"] >= len(masks) + 3, d
# every eligible call ran a compiled kernel (sync mode): 6 masks x 2 sizes,
# the odd-offset call, two 12+4 decodes and the 12-row encode
assert d["launches"] >= 2 * len(masks) + 1 + 2 + 1, d
print("ok")
"""

ASYNC = COMMON + r"""
with g.ECMatrixList(16, 20) as L:
    decode_check(L, 16, 20, 2048, 0xFFFF0)          # first sight: queued, shipped kernel
    s = g.jit_stats()
    assert s["launches"] == 0, s
    t0 = time.time()
    while g.jit_stats()["compiled"] + g.jit_stats()["failed"] < 1 and time.time() - t0 < 60:
        time.sleep(0.05)
    s = g.jit_stats()
    assert s["compiled"] == 1 and s["failed"] == 0, s
    for _ in range(3):
        decode_check(L, 16, 20, 2048, 0xFFFF0)
    s = g.jit_stats()
    assert s["launches"] == 3, s
print("ok", s)
"""

# 1 GiB of user data per call (the size the bench decodes, non-temporal
# staging): the round trip data -> shipped encode -> compiled decode == data,
# five calls per mask (a tile read before every wave's staging landed shows
# as a mismatch somewhere in 131,072 stripes)
FULL = COMMON + r"""
k, n = 16, 20
nst = (1 << 30) // (512 * k)
data = torch.randint(0, 256, (512 * k * nst,), dtype=torch.uint8, device="cuda")
frags = [torch.empty(512 * nst, dtype=torch.uint8, device="cuda") for _ in range(n)]
out = torch.empty_like(data)
with g.ECMatrixList(k, n) as L:
    L.encode_batch(nst, data, frags)
    for m in (0xFFFF0, 0xF0FFF, 0x5FFF5):
        rows = O.mask_rows(m)
        for _ in range(5):
            out.fill_(0)
            L.decode_batch(nst, m, rows, [frags[r - 1] for r in rows], out)
            assert torch.equal(out, data), hex(m)
s = g.jit_stats()
assert s["launches"] >= 15 and s["failed"] == 0, s
print("ok", s)
"""

# a process that exits while its matrix is still being compiled: the compile
# thread is joined at exit (a compile running through the compiler's static
# destructors would crash the exit)
EXIT = COMMON + r"""
with g.ECMatrixList(16, 20) as L:
    decode_check(L, 16, 20, 2048, 0xFFFF0)
print("ok", g.jit_stats())
"""

OFF = COMMON + r"""
with g.ECMatrixList(16, 20) as L:
    for _ in range(2):
        decode_check(L, 16, 20, 2048, 0xFFFF0)
s = g.jit_stats()
assert s["compiled"] == 0 and s["launches"] == 0 and s["lookups"] == 0, s
print("ok")
"""


def _run(script, **env):
    e = dict(os.environ, EC_MI355X_QUIET="1", EC_GPU_ALWAYS="1")
    e.update(env)
    r = subprocess.run([sys.executable, "-c", script], cwd=ROOT, env=e, capture_output=True,
                       text=True, timeout=280)
    assert r.returncode == 0 and "ok" in r.stdout, r.stdout[-2000:] + r.stderr[-3000:]
    return r.stdout


def test_jit_kernels_match_oracle():
    print(_run(SYNC, EC_MI355X_JIT_SYNC="1"))


def test_jit_full_size_round_trip():
    print(_run(FULL, EC_MI355X_JIT_SYNC="1"))


def test_jit_async_first_call_shipped_then_compiled():
    print(_run(ASYNC))


def test_jit_exit_while_compiling():
    print(_run(EXIT))


def test_jit_off():
    _run(OFF, EC_MI355X_JIT="0")
