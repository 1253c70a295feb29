#!/usr/bin/env python3
"""Host-buffer decode time per call by size (development probe, GPU box):
8+4 and 4+2 decodes and encodes from pinned buffers (ec_method_host_alloc,
i.e. the zero-copy kernels) at ZC_SIZES MiB of user data (default 4 16 64
256), median of repeated calls.  Run once per knob setting (EC_MI355X_ZCDB,
EC_ZC_TPB, EC_ZC_INFLIGHT_KB: read at library load); EC_GPU_ALWAYS=1 keeps every
call on the GPU.  Usage: python tools/zc_sizes.py"""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401  (torch first: one HIP runtime)
import glusterfs_amd as g  # noqa: E402


def pinned(lib, nb):
    p = lib.ec_method_host_alloc(nb)
    if not p:
        raise MemoryError
    return p, np.ctypeslib.as_array((ctypes.c_uint8 * nb).from_address(p))


def main():
    lib = g.ec_method.lib
    knobs = " ".join("%s=%s" % (v, os.environ.get(v, "unset"))
                     for v in ("EC_MI355X_ZCDB", "EC_ZC_TPB", "EC_ZC_INFLIGHT_KB", "EC_MI355X_ZCENC16"))
    print(knobs)
    sizes = [float(x) for x in os.environ.get("ZC_SIZES", "4 16 64 256").split()]
    geos = [tuple(int(x) for x in gk.split("+")) for gk in
            os.environ.get("ZC_GEOS", "8+4 4+2").split()]
    for k, r in geos:
        n = k + r
        for mib in sizes:
            S = int(mib * (1 << 20)) // (512 * k) * (512 * k)
            nst = S // (512 * k)
            bufs = []
            try:
                din_p, din = pinned(lib, S)
                bufs.append(din_p)
                din[:] = np.random.default_rng(int(mib * 16)).integers(0, 256, S, dtype=np.uint8)
                fr = [pinned(lib, nst * 512) for _ in range(n)]
                bufs += [p for p, _ in fr]
                dout_p, dout = pinned(lib, S)
                bufs.append(dout_p)
                with g.ECMatrixList(k, n) as L:
                    L.encode_batch(nst, din_p, [p for p, _ in fr])
                    rows = list(range(n - k + 1, n + 1))
                    mask = sum(1 << (r - 1) for r in rows)
                    ins = [fr[r - 1][0] for r in rows]
                    L.decode_batch(nst, mask, rows, ins, dout_p)
                    reps = max(5, min(60, (512 << 20) // S))
                    ts = []
                    for _ in range(reps):
                        t0 = time.perf_counter()
                        L.decode_batch(nst, mask, rows, ins, dout_p)
                        ts.append(time.perf_counter() - t0)
                    ok = bool(np.array_equal(dout, din))
                    te = []
                    frs = [p for p, _ in fr]
                    want = [a.copy() for _, a in fr]
                    for _ in range(reps):
                        t0 = time.perf_counter()
                        L.encode_batch(nst, din_p, frs)
                        te.append(time.perf_counter() - t0)
                    ok = ok and all(np.array_equal(a, w) for (_, a), w in zip(fr, want))
                    # heal of the n - k bricks outside `rows` (fragments in,
                    # their fragments out) and the row-masked re-encode of a
                    # heal write to them (user data in, their fragments out)
                    lost = [b for b in range(n) if not (mask >> b) & 1]
                    hp = [pinned(lib, nst * 512) for _ in lost]
                    bufs += [p for p, _ in hp]
                    th, tr = [], []
                    for _ in range(reps):
                        t0 = time.perf_counter()
                        L.heal(nst, mask, ins, sum(1 << b for b in lost), [p for p, _ in hp])
                        th.append(time.perf_counter() - t0)
                    ok = ok and all(np.array_equal(a, want[b]) for (_, a), b in zip(hp, lost))
                    sel = sum(1 << b for b in lost)
                    arg = [None] * n
                    for (p, _), b in zip(hp, lost):
                        arg[b] = p
                    for (_, a) in hp:
                        a[:] = 0
                    for _ in range(reps):
                        t0 = time.perf_counter()
                        L.encode_rows(S, din_p, sel, list(arg))
                        tr.append(time.perf_counter() - t0)
                    ok = ok and all(np.array_equal(a, want[b]) for (_, a), b in zip(hp, lost))
                ts.sort()
                te.sort()
                th.sort()
                tr.sort()
                med, mede = ts[len(ts) // 2], te[len(te) // 2]
                medh, medr = th[len(th) // 2], tr[len(tr) // 2]
                print("%d+%d %7.2f MiB: decode %8.1f us %6.2f GB/s, encode %8.1f us %6.2f GB/s,"
                      " heal %8.1f us, encode_rows %8.1f us, ok %s [%s]"
                      % (k, n - k, mib, med * 1e6, S / med / 1e9, mede * 1e6, S / mede / 1e9,
                         medh * 1e6, medr * 1e6, ok, knobs))
            finally:
                for p in bufs:
                    lib.ec_method_host_free(p)


if __name__ == "__main__":
    main()
