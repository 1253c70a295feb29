#!/usr/bin/env python3
"""Default-stream mixed decodes through the device pattern-table cache from
1 and 8 threads (development tool, GPU box).

Each call is a 16+4 self-heal window on device buffers: 512 stripes (4 MiB
of data), 64 pattern groups of 8 stripes, 64 masks (past the kernel-argument
space: the decode matrices come from the device table).  Every thread passes
stream NULL (its per-thread default stream) and the same hot mask set -- a
heal sweep -- and syncs every call.  r04's release() created an event per
NULL-stream call and, past 16 readers, waited for the oldest under the
cache mutex; r05's re-records one event per (stream, thread).

Usage: EC_MI355X_LIB=<lib> python tools/patcache_threads.py [secs]
prints one JSON line per thread count."""
import itertools
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402  (torch first: one HIP runtime)
import glusterfs_amd as g  # noqa: E402

CHUNK = 512
K, N, NST, GRP = 16, 20, 512, 8
NMASK = int(os.environ.get("PC_MASKS", "64"))   # 1..7: kernel-argument patterns, no table


def run(L, nth, secs, dfr, gp, masks):
    outs = [torch.empty(CHUNK * K * NST, dtype=torch.uint8, device="cuda") for _ in range(nth)]
    calls = [0] * nth
    go = threading.Barrier(nth + 1)
    t_end = [0.0]

    def worker(t):
        go.wait()
        while time.time() < t_end[0]:
            L.decode_mixed_device(0, None, NST, GRP, gp, masks, dfr, outs[t])
            g.sync_device(0)
            calls[t] += 1

    th = [threading.Thread(target=worker, args=(t,)) for t in range(nth)]
    for t in th:
        t.start()
    t_end[0] = time.time() + secs
    t0 = time.time()
    go.wait()
    for t in th:
        t.join()
    dt = time.time() - t0
    c = sum(calls)
    return dict(threads=nth, calls=c, secs=round(dt, 3), us_per_call=round(dt / c * 1e6, 2),
                data_GBps=round(c * CHUNK * K * NST / dt / 1e9, 2))


def main():
    secs = float(sys.argv[1]) if len(sys.argv) > 1 else 3.0
    allm = [sum(1 << b for b in c) for c in itertools.combinations(range(N), K)]
    rng = np.random.default_rng(3)
    masks = sorted(int(x) for x in rng.choice(allm, NMASK, replace=False))
    dfr = [torch.randint(0, 256, (CHUNK * NST,), dtype=torch.uint8, device="cuda") for _ in range(N)]
    gp = torch.arange(NST // GRP, device="cuda").remainder(NMASK).to(torch.uint8)
    torch.cuda.synchronize()
    lib = os.environ.get("EC_MI355X_LIB") or "in-tree"
    with g.ECMatrixList(K, N) as L:
        run(L, 1, 0.5, dfr, gp, masks)                 # warm up: table, kernels
        for nth in (1, 8, 1, 8):
            r = run(L, nth, secs, dfr, gp, masks)
            r["lib"] = os.path.basename(lib)
            r["masks"] = NMASK
            print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
