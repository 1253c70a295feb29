#!/usr/bin/env python3
"""Reproducer for the one mismatch tools/fuzz_api.py found with registered
host ranges (r04x: 3+2 encode + decode, ~4 MiB, every buffer its own
hipHostRegister'd numpy array, registered / unregistered per call while
other threads do the same).  Runs the call pattern under variants and
reports which stage (encode fragments, decode output) differs from the
oracle, and where:
  fresh   new numpy arrays every iteration, registered, unregistered after
          (virtual addresses are reused by later arrays)
  keep    the same registered arrays for every iteration
  nounreg new arrays, registered, never unregistered (no address reuse)
each single-threaded and with REPRO_THREADS threads (default 4).
Usage: python tools/reg_repro.py [iterations]"""
import ctypes
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401
import glusterfs_amd as g  # noqa: E402
import oracle as O  # noqa: E402

CHUNK = 512
lib = g.ec_method.lib


def reg_array(n, regs):
    raw = np.empty(n + 8192, np.uint8)
    a = raw[(-raw.ctypes.data) % 4096:][:n + 4096]
    rc = lib.ec_method_host_register(a.ctypes.data, a.nbytes)
    if rc == 0:
        regs.append(a.ctypes.data)
    return raw, a[:n], rc


def first_diff(x, y):
    d = np.nonzero(x != y)[0]
    return (int(d[0]), int(d.size)) if d.size else None


def run(variant, iters, tid, out, k=3, r=2, nst=2730):
    n = k + r
    rng = np.random.default_rng(1000 + tid)
    L = g.ECMatrixList(k, n)
    kept = None
    bad = []
    held, held_regs = [], []          # nounreg: alive (and registered) to the end
    if variant == "nounreg":
        iters = min(iters, 40)
    for it in range(iters):
        regs = []
        if variant == "keep" and kept is not None:
            raws, src, frs, dout, rcs = kept
        else:
            raws, rcs = [], []
            raw, src, rc = reg_array(CHUNK * k * nst, regs)
            raws.append(raw)
            rcs.append(rc)
            frs = []
            for _ in range(n):
                raw, f, rc = reg_array(CHUNK * nst, regs)
                raws.append(raw)
                rcs.append(rc)
                frs.append(f)
            raw, dout, rc = reg_array(CHUNK * k * nst, regs)
            raws.append(raw)
            rcs.append(rc)
            if variant == "keep":
                kept = (raws, src, frs, dout, rcs)
        data = rng.integers(0, 256, CHUNK * k * nst, dtype=np.uint8)
        src[:] = data
        L.encode(data.size, src, frs)
        want = O.encode(k, n, data)
        enc_bad = [(i, first_diff(f, w)) for i, (f, w) in enumerate(zip(frs, want))
                   if first_diff(f, w)]
        rows = sorted(rng.choice(n, k, replace=False) + 1)
        m = sum(1 << (x - 1) for x in rows)
        dout[:] = 0
        L.decode(CHUNK * nst, m, [int(x) for x in rows], [frs[x - 1] for x in rows], dout)
        dec_bad = first_diff(dout, data)
        if enc_bad or dec_bad:
            bad.append(dict(it=it, enc=enc_bad[:3], dec=dec_bad, mask=m, rcs=rcs,
                            src=hex(src.ctypes.data)))
        if variant == "fresh":
            for p in regs:
                lib.ec_method_host_unregister(p)
            del raws
        elif variant == "nounreg":
            held.append(raws)
            held_regs += regs
        elif it == 0:
            held_regs += regs                 # keep: registered once
    for p in held_regs:
        lib.ec_method_host_unregister(p)
    L.fini()
    out[tid] = bad


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 100
    nth = int(os.environ.get("REPRO_THREADS", "4"))
    for variant in ("keep", "nounreg", "fresh"):
        for threads in (1, nth):
            out = {}
            t0 = time.time()
            th = [threading.Thread(target=run, args=(variant, iters, t, out))
                  for t in range(threads)]
            for t in th:
                t.start()
            for t in th:
                t.join()
            bad = [b for t in sorted(out) for b in out[t]]
            st = g.ec_method.stats()
            print("%-8s threads %d: %d iterations each, %d bad, %.1f s, engine calls so far "
                  "gpu %d cpu %d %s" % (variant, threads, iters, len(bad), time.time() - t0,
                                         st["gpu_calls"], st["cpu_calls"], bad[:3] if bad else ""),
                  flush=True)


if __name__ == "__main__":
    main()
