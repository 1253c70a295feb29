#!/usr/bin/env python3
"""Host-side cost of one device-resident call (development probe, GPU box).

For the headline call (4+2 decode of 1 GiB, mask 0x3C, device buffers) it
reports:
  * host time per ec_method_decode_device call through the ctypes wrapper
    (GPU busy, queue ahead), and through a direct ctypes call with the
    argument arrays built once;
  * the event-timed gap an idle GPU waits for the first launch;
  * event time per launch for 20 and 100 back-to-back launches, as the
    bench times them.
Usage: python tools/host_latency.py
"""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402  (torch first: one HIP runtime)
import glusterfs_amd as g  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    k, n, S = 4, 6, 1 << 30
    nst = S // (512 * k)
    data = torch.randint(0, 256, (S,), dtype=torch.uint8, device=dev)
    frags = [torch.empty(nst * 512, dtype=torch.uint8, device=dev) for _ in range(n)]
    out = torch.empty_like(data)
    sp = torch.cuda.current_stream().cuda_stream
    with g.ECMatrixList(k, n) as L:
        L.encode_device(0, sp, nst, data, frags)
        mask = 0x3C
        rows = g.mask_rows(mask)
        ins = [frags[r - 1] for r in rows]
        fn = lambda: L.decode_device(0, sp, nst, mask, ins, out)  # noqa: E731
        lib = g.ec_method.lib
        arr = (ctypes.c_void_p * k)(*[t.data_ptr() for t in ins])
        lst = ctypes.byref(L._list)
        optr = ctypes.c_void_p(out.data_ptr())
        spv = ctypes.c_void_p(sp)
        raw = lambda: lib.ec_method_decode_device(lst, 0, spv, nst, mask, arr, optr)  # noqa: E731
        for f in (fn, raw):
            for _ in range(5):
                f()
        torch.cuda.synchronize()
        for name, f in (("wrapper", fn), ("direct ctypes", raw)):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(20):
                f()
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            print("host time per call, %-14s %.1f us" % (name, (t1 - t0) / 20 * 1e6))
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e2 = torch.cuda.Event(enable_timing=True)
        for name, f in (("wrapper", fn), ("direct ctypes", raw)):
            gaps = []
            for _ in range(5):
                torch.cuda.synchronize()
                e0.record()
                f()
                e1.record()
                f()
                e2.record()
                torch.cuda.synchronize()
                gaps.append((e0.elapsed_time(e1) - e1.elapsed_time(e2)) * 1e3)
            print("first launch after idle (%s): event span exceeds a queued launch by %s us"
                  % (name, " ".join("%.0f" % x for x in gaps)))
        for steps in (20, 100):
            for f, name in ((fn, "wrapper"), (raw, "direct ctypes")):
                torch.cuda.synchronize()
                e0.record()
                for _ in range(steps):
                    f()
                e1.record()
                torch.cuda.synchronize()
                print("%3d launches (%s): %.4f ms per launch" % (steps, name,
                                                                 e0.elapsed_time(e1) / steps))
        ok = torch.equal(out, data)
        print("decode ok", ok)


if __name__ == "__main__":
    main()
