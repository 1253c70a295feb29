#!/usr/bin/env python3
"""PCIe ceiling of the host-buffer path (development probe, GPU box): DMA
copies between pinned host memory and HBM, one direction at a time and both
at once (two streams), so the zero-copy kernels' rates (DESIGN.md 5,
extra.e2e_pcie_*) can be read against what the link itself carries.
Usage: python tools/pcie_probe.py [MiB]   (default 256)"""
import sys
import time

import torch


def rate(fn, nbytes, reps=10):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    return nbytes / ts[len(ts) // 2] / 1e9


def main():
    mib = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    n = mib << 20
    h_in = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    h_out = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    d_in = torch.empty(n, dtype=torch.uint8, device="cuda")
    d_out = torch.randint(0, 255, (n,), dtype=torch.uint8, device="cuda")
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def h2d():
        d_in.copy_(h_in, non_blocking=True)

    def d2h():
        h_out.copy_(d_out, non_blocking=True)

    def both():
        with torch.cuda.stream(s1):
            d_in.copy_(h_in, non_blocking=True)
        with torch.cuda.stream(s2):
            h_out.copy_(d_out, non_blocking=True)

    up = rate(h2d, n)
    down = rate(d2h, n)
    duplex = rate(both, n)   # per direction: n bytes each way in the time
    print('{"pcie_probe_MiB": %d, "h2d_GBps": %.2f, "d2h_GBps": %.2f, '
          '"duplex_per_direction_GBps": %.2f}' % (mib, up, down, duplex))


if __name__ == "__main__":
    main()
