"""Split host calls (r05, ec_method.c hybrid_share / encode_split /
decode_split): a host call both engines would code in comparable times runs
on both -- the first share of its stripes on a GPU (from a helper thread),
the rest on the calling thread's CPU engine -- and must be bit-exact with the
oracle for every host entry point, pattern-group alignment and buffer kind;
a failed GPU share is redone on the CPU with the helper's error text handed
to the caller.

Runs in a child process with the crossover on (conftest.py sets
EC_GPU_ALWAYS=1, which never splits), the CPU model slowed so every call is
near a tie, and the GPU share fixed (EC_HYBRID_SHARE) so the split is
deterministic."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = r"""
import ctypes, json, sys
sys.path[:0] = [%(root)r, %(oracle)r]
import numpy as np
import torch  # noqa: F401  (one HIP runtime)
import glusterfs_amd as g
import oracle as O
CH = 512
res = {}

def rnd(n, seed):
    return np.random.default_rng(seed).integers(0, 256, n, dtype=np.uint8)

def host(n, kind, seed=None):
    if kind == "pinned":
        p = g.PinnedArray(n)
        keep.append(p)
        a = p.array[:n]
    else:
        a = np.empty(n, np.uint8)
    if seed is not None:
        a[:] = rnd(n, seed)
    return a

def split_count(fn):
    s0 = g.stats()
    fn()
    s1 = g.stats()
    return s1["gpu_calls"] - s0["gpu_calls"], s1["cpu_calls"] - s0["cpu_calls"]

keep = []
for kind in ("pageable", "pinned"):
    for (k, r) in ((4, 2), (8, 4), (16, 4), (5, 2)):
        n = k + r
        nst = (4 << 20) // (CH * k) + 3                 # > 1 MiB, odd stripe count
        with g.ECMatrixList(k, n) as L:
            data = host(CH * k * nst, kind, seed=k)
            want = O.encode(k, n, np.array(data), nthreads=8)
            outs = [host(CH * nst, kind) for _ in range(n)]
            gc, cc = split_count(lambda: L.encode_batch(nst, data, outs))
            assert (gc, cc) == (1, 1), ("encode not split", kind, k, gc, cc)
            assert all(np.array_equal(o, w) for o, w in zip(outs, want)), ("encode", kind, k)
            # decode
            rows = list(range(r + 1, n + 1))
            mask = sum(1 << (x - 1) for x in rows)
            fr = [host(CH * nst, kind) for _ in rows]
            for f, x in zip(fr, rows):
                f[:] = want[x - 1]
            out = host(CH * k * nst, kind)
            gc, cc = split_count(lambda: L.decode_batch(nst, mask, rows, fr, out))
            assert (gc, cc) == (1, 1), ("decode not split", kind, k, gc, cc)
            assert np.array_equal(out, data), ("decode", kind, k)
            # mixed decode, groups of 64 stripes (the share is cut at a group)
            pool = [mask, sum(1 << (x - 1) for x in range(1, k + 1))]
            ng = (nst + 63) // 64
            gm = [pool[i %% 2] for i in range(ng)]
            allf = [host(CH * nst, kind) for _ in range(n)]
            for i in range(n):
                allf[i][:] = want[i]
            out2 = host(CH * k * nst, kind)
            L.decode_mixed(nst, 64, gm, allf, out2)
            assert np.array_equal(out2, data), ("mixed", kind, k)
            # heal: regenerate the first r fragments from the others
            tmask = (1 << r) - 1
            hout = [host(CH * nst, kind) for _ in range(r)]
            L.heal(nst, mask, fr, tmask, hout)
            assert all(np.array_equal(h, want[i]) for i, h in enumerate(hout)), ("heal", kind, k)
            # row-masked encode of bricks 1 and n
            rm = 1 | (1 << (n - 1))
            ro = [host(CH * nst, kind) if (rm >> i) & 1 else None for i in range(n)]
            L.encode_rows(data.size, data, rm, ro)
            assert np.array_equal(ro[0], want[0]) and np.array_equal(ro[n - 1], want[n - 1]), \
                ("encode_rows", kind, k)
        res["%%s_%%d+%%d" %% (kind, k, r)] = "ok"

# a failed GPU share: redone on the CPU, counted, its reason handed over
with g.ECMatrixList(8, 12) as L:
    nst = 2048
    data = rnd(CH * 8 * nst, 5)
    want = O.encode(8, 12, data)
    outs = [np.zeros(CH * nst, np.uint8) for _ in range(12)]
    f0 = g.stats()["cpu_fallbacks"]
    g.inject_device_faults(1)
    L.encode_batch(nst, data, outs)
    assert all(np.array_equal(o, w) for o, w in zip(outs, want))
    assert g.stats()["cpu_fallbacks"] == f0 + 1
    assert "injected" in (g.ec_method.lib.ec_method_last_error() or b"").decode()
res["fallback"] = "ok"
print(json.dumps(res))
print("OK")
"""


def test_split_calls_match_oracle():
    env = dict(os.environ)
    env.pop("EC_GPU_ALWAYS", None)
    env.update(EC_HYBRID_SHARE="450", EC_CPU_ENC_GBPS_K2="6", EC_CPU_DEC_GBPS_K="4",
               EC_XOVER_ADAPT="0", EC_MI355X_QUIET="1")
    code = SCRIPT % dict(root=ROOT, oracle=os.path.join(ROOT, "oracle"))
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True,
                       text=True, timeout=280)
    assert r.returncode == 0 and "OK" in r.stdout, r.stdout[-3000:] + r.stderr[-3000:]
    print(json.loads(r.stdout.strip().splitlines()[-2]))


def test_split_off_keeps_calls_whole():
    """EC_HYBRID=0: the same near-tie calls run whole on one engine."""
    env = dict(os.environ)
    env.pop("EC_GPU_ALWAYS", None)
    env.update(EC_HYBRID="0", EC_HYBRID_SHARE="450", EC_CPU_ENC_GBPS_K2="6",
               EC_CPU_DEC_GBPS_K="4", EC_XOVER_ADAPT="0", EC_MI355X_QUIET="1")
    code = r"""
import sys
sys.path[:0] = [%(root)r]
import numpy as np
import torch  # noqa: F401
import glusterfs_amd as g
with g.ECMatrixList(8, 12) as L:
    nst = 2048
    data = np.arange(512 * 8 * nst, dtype=np.uint32).astype(np.uint8)
    outs = [np.zeros(512 * nst, np.uint8) for _ in range(12)]
    s0 = g.stats()
    L.encode_batch(nst, data, outs)
    s1 = g.stats()
    d = (s1["gpu_calls"] - s0["gpu_calls"], s1["cpu_calls"] - s0["cpu_calls"])
    assert d in ((1, 0), (0, 1)), d
print("OK")
""" % dict(root=ROOT)
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True,
                       text=True, timeout=200)
    assert r.returncode == 0 and "OK" in r.stdout, r.stdout[-3000:] + r.stderr[-3000:]


def test_learned_shares_stay_exact():
    """Split calls without a fixed share: the library learns each class's
    share from the two shares' times (ec_method.c share_learn), so the split
    point moves from call to call; every result must stay bit-exact, and the
    learned share must be a real split."""
    env = dict(os.environ)
    env.pop("EC_GPU_ALWAYS", None)
    env.update(EC_CPU_ENC_GBPS_K2="60", EC_CPU_DEC_GBPS_K="60", EC_MI355X_QUIET="1")
    env.pop("EC_HYBRID_SHARE", None)
    code = r"""
import ctypes, sys
sys.path[:0] = [%(root)r, %(oracle)r]
import numpy as np
import torch  # noqa: F401
import glusterfs_amd as g
import oracle as O
k, n = 8, 12
nst = (4 << 20) // (512 * k)
rng = np.random.default_rng(11)
splits = 0
with g.ECMatrixList(k, n) as L:
    keep = []
    def pinned(nb):
        p = g.PinnedArray(nb)
        keep.append(p)
        return p.array[:nb]
    data = pinned(512 * k * nst)
    frags = [pinned(512 * nst) for _ in range(n)]
    out = pinned(512 * k * nst)
    rows = list(range(5, 13))
    mask = sum(1 << (r - 1) for r in rows)
    for it in range(24):
        data[:] = rng.integers(0, 256, data.size, dtype=np.uint8)
        s0 = g.stats()
        L.encode_batch(nst, data, frags)
        want = O.encode(k, n, np.array(data), nthreads=8)
        assert all(np.array_equal(f, w) for f, w in zip(frags, want)), ("encode", it)
        L.decode_batch(nst, mask, rows, [frags[r - 1] for r in rows], out)
        assert np.array_equal(out, data), ("decode", it)
        s1 = g.stats()
        splits += (s1["gpu_calls"] - s0["gpu_calls"]) > 0 and (s1["cpu_calls"] - s0["cpu_calls"]) > 0
    sh = ctypes.c_int32(-2)
    g.ec_method.lib.ec_method_xover_plan(k, 1, data.size, 2 * data.size, 0, 0, 0, ctypes.byref(sh))
print("splits", splits, "share", sh.value)
assert splits >= 4, splits
print("OK")
""" % dict(root=ROOT, oracle=os.path.join(ROOT, "oracle"))
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True,
                       text=True, timeout=280)
    assert r.returncode == 0 and "OK" in r.stdout, r.stdout[-3000:] + r.stderr[-3000:]
    print(r.stdout.strip().splitlines()[-2])
