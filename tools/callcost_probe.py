#!/usr/bin/env python3
"""Host cost of one device-resident call (development probe).

Times back-to-back ec_method_decode_device / encode_device calls on tiny and
on 64K-stripe batches: the Python wrapper, the bare ctypes call with the
arguments built once, and the GPU time per launch (events), to tell host
submission cost from kernel time in bench.py's event-timed figures."""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import glusterfs_amd as g  # noqa: E402
from glusterfs_amd import ec_method as em  # noqa: E402


def run(k, n, nst, reps=200):
    dev = torch.device("cuda", 0)
    sp = torch.cuda.current_stream(dev).cuda_stream
    data = torch.randint(0, 255, (nst * 512 * k,), dtype=torch.uint8, device=dev)
    frags = [torch.empty(nst * 512, dtype=torch.uint8, device=dev) for _ in range(n)]
    L = g.ECMatrixList(k, n)
    L.encode_device(0, sp, nst, data, frags)
    rows = list(range(n - k + 1, n + 1))
    mask = sum(1 << (r - 1) for r in rows)
    ins = [frags[r - 1] for r in rows]
    out = torch.empty_like(data)
    res = {}
    for name, fn in (
            ("wrapper", lambda: L.decode_device(0, sp, nst, mask, ins, out)),
            ("ctypes", None)):
        if fn is None:
            arr = em._ptr_array(ins)
            o = em.addr(out)
            lst = ctypes.byref(L._list)
            f = em.lib.ec_method_decode_device

            def fn():
                f(lst, 0, sp, nst, mask, arr, o)
        for _ in range(10):
            fn()
        torch.cuda.synchronize()
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        host = (time.perf_counter() - t0) / reps
        e1.record()
        torch.cuda.synchronize()
        res[name] = dict(host_us=round(host * 1e6, 1),
                         gpu_us_per_call=round(e0.elapsed_time(e1) * 1e3 / reps, 1))
    print("k=%d n=%d nst=%d" % (k, n, nst), res, flush=True)


if __name__ == "__main__":
    for k, n, nst in ((4, 6, 8), (8, 12, 8), (8, 12, 65536), (4, 6, 524288)):
        run(k, n, nst)
