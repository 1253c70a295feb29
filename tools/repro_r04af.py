#!/usr/bin/env python3
"""Cause of r04af's wrong device partial write (development tool, GPU box).

profiles/r04/r04af_fuzz.log:14305 recorded a 4+2 writev on device buffers
(head 1517, 6040 user bytes) whose two interior stripes -- the ones the
fused encoder reads in place from the user buffer -- were wrong, while the
two edge stripes (gathered first, into library scratch) were right.

tools/fuzz_api.py passed that user buffer as a temporary,
`L.writev_encode_device(..., A.buf(user), ...)`: the tensor was freed when the
call returned, BEFORE g.sync_device(); the call is asynchronous on the
calling thread's per-thread stream, which torch's caching allocator knows
nothing of, so the block went back to torch's stream for reuse while the
library's kernels had not yet read it.

This tool tests that hypothesis directly:
  order    one thread: queue work on the per-thread stream, free a user
           tensor right after the writev call, reallocate the same size on
           torch's stream and overwrite it.  Reports whether torch's stream
           waited for the library's per-thread stream (HIP's null-stream
           semantics) -- if not, the overwrite can land before the read.
  cross    two threads: X's writev frees its user tensor on return, Y
           takes a block from torch's allocator and a library call on Y's
           own per-thread stream writes it (another fuzz call's output);
           whether Y got X's block, and whether X's result was then wrong;
           also with Y on a torch side stream (non-blocking, after
           wait_stream on torch's current stream), as the fuzzer's
           stream_chain op wrote its outputs
  fuzz     FUZZ-like threads, the writev of r04af's shape, with the user
           tensor freed before the sync (as the fuzzer did) and kept until
           after it (fixed), mismatches counted for each.
Prints one JSON line.  Usage: python tools/repro_r04af.py [secs per mode]
"""
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import numpy as np  # noqa: E402
import torch  # noqa: E402  (torch first: one HIP runtime)
import glusterfs_amd as g  # noqa: E402
import oracle as O  # noqa: E402  (the checker)

CHUNK = 512
K, N, HEAD, US = 4, 6, 1517, 6040


def want_of(user, oh, ot):
    return O.encode(K, N, O.writev_merge(K, HEAD, user, oh, ot))


def one(L, rng, keep, overwrite):
    S = CHUNK * K
    user = rng.integers(0, 256, US, dtype=np.uint8)
    oh = rng.integers(0, 256, S, dtype=np.uint8)
    ot = rng.integers(0, 256, S, dtype=np.uint8)
    nst = (HEAD + US + S - 1) // S
    outs = [torch.empty(CHUNK * nst, dtype=torch.uint8, device="cuda") for _ in range(N)]
    dh = torch.from_numpy(oh).cuda()
    dt = torch.from_numpy(ot).cuda()
    du = torch.from_numpy(user).cuda()
    L.writev_encode_device(0, None, HEAD, US, du, dh, dt, outs)
    if not keep:
        del du                           # back to torch's allocator, unsynced
        if overwrite:                    # what another fuzz thread did next
            junk = torch.empty(US, dtype=torch.uint8, device="cuda")
            junk.fill_(0x5A)
    g.sync_device(0)
    want = want_of(user, oh, ot)
    return all(np.array_equal(o.cpu().numpy(), w) for o, w in zip(outs, want))


def order_probe(L, secs):
    """Single thread: keep the per-thread stream busy first (a 256 MiB 4+2
    encode, ~0.1 ms each, 20 of them), so the writev's kernels are still
    queued when torch reuses and overwrites the freed block."""
    big = torch.randint(0, 256, (256 << 20,), dtype=torch.uint8, device="cuda")
    bouts = [torch.empty((256 << 20) // K, dtype=torch.uint8, device="cuda") for _ in range(N)]
    nst_big = (256 << 20) // (CHUNK * K)
    rng = np.random.default_rng(1)
    bad = calls = 0
    t_end = time.time() + secs
    while time.time() < t_end:
        for _ in range(20):
            L.encode_device(0, None, nst_big, big, bouts)
        ok = one(L, rng, keep=False, overwrite=True)
        bad += not ok
        calls += 1
    return dict(calls=calls, wrong=bad, torch_stream=int(torch.cuda.current_stream().cuda_stream))


def cross_probe(L, secs, keep, side=False):
    """Two threads.  X queues a backlog on its per-thread stream, then the
    r04af writev with the user tensor freed on return (keep=False) or held
    until after its sync (keep=True); Y then takes a block of the same size
    from torch's allocator -- as another fuzz thread's output buffer -- and a
    library call on Y's own (idle) per-thread stream writes it.  Nothing
    orders two per-thread streams, so if Y got X's freed block, Y's kernel can
    write it before X's encoder reads it."""
    S = CHUNK * K
    big = torch.randint(0, 256, (256 << 20,), dtype=torch.uint8, device="cuda")
    bouts = [torch.empty((256 << 20) // K, dtype=torch.uint8, device="cuda") for _ in range(N)]
    nst_big = (256 << 20) // (CHUNK * K)
    nst_y = 12                                   # 6144-byte fragments: du's size class
    ysrc = torch.randint(0, 256, (CHUNK * K * nst_y,), dtype=torch.uint8, device="cuda")
    youts = [torch.empty(CHUNK * nst_y, dtype=torch.uint8, device="cuda") for _ in range(N - 1)]
    rng = np.random.default_rng(7)
    handoff, done = threading.Event(), threading.Event()
    box = {}
    stats = dict(calls=0, wrong=0, reused=0, wrong_when_reused=0)
    t_end = time.time() + secs

    def y_thread():
        while True:
            handoff.wait()
            handoff.clear()
            if box.get("stop"):
                return
            junk = torch.empty(CHUNK * nst_y, dtype=torch.uint8, device="cuda")
            box["reused"] = junk.data_ptr() == box["p"]
            if side:      # as the fuzzer's stream_chain: a torch side stream (non-blocking)
                st = ys
                st.wait_stream(torch.cuda.current_stream())
                L.encode_device(0, st.cuda_stream, nst_y, ysrc, [junk] + youts)
                st.synchronize()
            else:
                L.encode_device(0, None, nst_y, ysrc, [junk] + youts)   # Y's per-thread stream
                g.sync_device(0)
            box["junk"] = junk
            done.set()

    ys = torch.cuda.Stream()
    ty = threading.Thread(target=y_thread)
    ty.start()
    try:
        while time.time() < t_end:
            user = rng.integers(0, 256, US, dtype=np.uint8)
            oh = rng.integers(0, 256, S, dtype=np.uint8)
            ot = rng.integers(0, 256, S, dtype=np.uint8)
            nst = (HEAD + US + S - 1) // S
            outs = [torch.empty(CHUNK * nst, dtype=torch.uint8, device="cuda") for _ in range(N)]
            dh = torch.from_numpy(oh).cuda()
            dt = torch.from_numpy(ot).cuda()
            du = torch.from_numpy(user).cuda()
            # the backlog AFTER the inputs exist: a copy on torch's (null)
            # stream waits for every blocking stream, so made later the
            # inputs would drain it first (r05c/d's probe did, and saw 0)
            torch.cuda.synchronize()
            for _ in range(20):
                L.encode_device(0, None, nst_big, big, bouts)
            L.writev_encode_device(0, None, HEAD, US, du, dh, dt, outs)
            box["p"] = du.data_ptr()
            held = du if keep else None
            del du
            handoff.set()
            done.wait()
            done.clear()
            g.sync_device(0)
            del held
            box.pop("junk", None)
            want = want_of(user, oh, ot)
            ok = all(np.array_equal(o.cpu().numpy(), w) for o, w in zip(outs, want))
            stats["calls"] += 1
            stats["wrong"] += not ok
            stats["reused"] += box["reused"]
            stats["wrong_when_reused"] += box["reused"] and not ok
    finally:
        box["stop"] = True
        handoff.set()
        ty.join()
    return stats


def fuzz_mode(L, secs, keep, nth=8):
    bad, calls = [0], [0]
    lock = threading.Lock()
    t_end = time.time() + secs

    def worker(t):
        rng = np.random.default_rng(1000 + t)
        while time.time() < t_end:
            ok = one(L, rng, keep=keep, overwrite=True)
            with lock:
                calls[0] += 1
                bad[0] += not ok

    th = [threading.Thread(target=worker, args=(t,)) for t in range(nth)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    return dict(calls=calls[0], wrong=bad[0])


def main():
    secs = float(sys.argv[1]) if len(sys.argv) > 1 else 10.0
    res = {}
    with g.ECMatrixList(K, N) as L:
        res["order_freed_before_sync"] = order_probe(L, secs)
        print("order probe done", flush=True)
        res["cross_freed_before_sync"] = cross_probe(L, secs, keep=False)
        print("cross probe (freed) done", flush=True)
        res["cross_kept_until_sync"] = cross_probe(L, secs, keep=True)
        print("cross probe (kept) done", flush=True)
        res["cross_side_freed_before_sync"] = cross_probe(L, secs, keep=False, side=True)
        print("cross probe, side stream (freed) done", flush=True)
        res["cross_side_kept_until_sync"] = cross_probe(L, secs, keep=True, side=True)
        print("cross probe, side stream (kept) done", flush=True)
        res["threads_freed_before_sync"] = fuzz_mode(L, secs, keep=False)
        print("freed mode done", flush=True)
        res["threads_kept_until_sync"] = fuzz_mode(L, secs, keep=True)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
