#!/usr/bin/env python3
"""Add the strong-scaled configs[3] fixtures to tests/golden/fullsize_sha256.json:
one fixed 16+4 job of 1,048,576 stripes (8 GiB of user data, SURVEY 8(d)
config 4) split by glusterfs_amd.dist.stripe_range over N = 2, 4, 8 ranks.
Case "16+4_8GiBjob_N<N>_r<r>" holds SHA-256 of rank r's input slice and of
each of its 20 fragment slices.

The stream is filled sequentially by the oracle (oracle/ec_oracle.c
or_fill_xorshift returns the generator state, so 1 GiB slices chain) and each
1 GiB slice is oracle-encoded once; every N's hashers are fed the slices they
cover (N = 8: one slice, N = 4: two, N = 2: four), so the 8 GiB job is never
held in memory.

    python3 tests/golden/gen_strong_sha.py       # ~1-2 min, 8 threads, ~3 GiB RAM
"""
import ctypes
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]

import oracle as O  # noqa: E402  (test infrastructure)

K, N_FRAG = 16, 20
STRIPES = 1 << 20
SLICE = (1 << 30)                       # bytes per 1/8 of the job
WAYS = (1, 2, 4, 8)


def main():
    path = os.path.join(HERE, "fullsize_sha256.json")
    with open(path) as f:
        fx = json.load(f)
    lib = O.lib()
    h = {}                              # (N, rank) -> [data hasher, frag hashers]
    for w in WAYS:
        for r in range(w):
            h[(w, r)] = [hashlib.sha256(), [hashlib.sha256() for _ in range(N_FRAG)]]
    state = int(fx["seed"], 16)
    buf = np.empty(SLICE, dtype=np.uint8)
    for s in range(8):
        state = lib.or_fill_xorshift(buf.ctypes.data_as(ctypes.c_void_p), SLICE, state)
        frags = O.encode(K, N_FRAG, buf, nthreads=8)
        for w in WAYS:
            hd, hf = h[(w, s * w // 8)]
            hd.update(memoryview(buf))
            for i in range(N_FRAG):
                hf[i].update(memoryview(frags[i]))
        del frags
        print("slice", s, flush=True)
    nb_job = STRIPES * 512 * K
    for w in WAYS:
        for r in range(w):
            hd, hf = h[(w, r)]
            fx["cases"]["16+4_8GiBjob_N%d_r%d" % (w, r)] = {
                "k": K, "n": N_FRAG, "bytes": nb_job // w, "rank": r,
                "word0": r * (nb_job // w) // 8, "job_stripes": STRIPES, "ranks": w,
                "data": hd.hexdigest(), "frags": [x.hexdigest() for x in hf]}
    with open(path, "w") as f:
        json.dump(fx, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
