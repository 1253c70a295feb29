#!/usr/bin/env python3
"""Generate tests/golden/fullsize_sha256.json: SHA-256 of the synthetic input
and of every oracle-encoded fragment at BASELINE.json's full sizes
(SURVEY.md 8(c)(2)), so the GPU box -- where neither the reference nor a
1 GiB oracle run is at hand inside the timed bench -- can check full-size
runs by hash.

Input: the xorshift64 stream of SURVEY.md 8(d) (seed 0x9E3779B97F4A7C15),
filled here by the oracle (oracle/ec_oracle.c or_fill_xorshift); rank r of
an N-GPU job owns the r-th slice of one global stream (glusterfs_amd/synth.py
enters the stream at word r * bytes / 8 on the device).  Fragments: oracle
encode (the CPU restatement of ec-method.c:394-408).  Decode outputs of valid
fragments are the data itself, so a decode is checked against "data".

    python3 tests/golden/gen_fullsize_sha.py      # ~2-4 min, 8 threads, ~5 GiB RAM
"""
import hashlib
import json
import os
import sys
from concurrent.futures import ThreadPoolExecutor

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]

import oracle as O  # noqa: E402  (test infrastructure)

GiB = 1 << 30
# name: (k, n, bytes per rank, ranks, with fragments)
CASES = {
    "4+2_1GiB": (4, 6, GiB, 8, True),          # configs[0]/[1], headline per rank
    "8+4_64Kstripes": (8, 12, 65536 * 4096, 1, True),   # configs[2]
    "8+4_1GiB": (8, 12, GiB, 8, False),        # configs[4] self-heal, 8+4 1 GiB decode
    "16+4_1GiB": (16, 20, GiB, 1, True),       # 16+4 decode / mixed
    "16+4_2GiB": (16, 20, 2 * GiB, 8, True),   # configs[3] per rank
}


def sha(a):
    return hashlib.sha256(memoryview(a)).hexdigest()


def stream(nbytes, word0):
    """Words [word0, word0 + nbytes/8) of the stream (oracle fill of the
    prefix, then sliced: cheap next to the encode)."""
    full = O.fill_xorshift(word0 * 8 + nbytes)
    return full[word0 * 8:].copy()


def main():
    out = {"seed": "0x9E3779B97F4A7C15",
           "stream": "xorshift64 (13,7,17), u64 word i = state after i+1 steps, little-endian",
           "rank_slice": "rank r owns words [r*bytes/8, (r+1)*bytes/8) of one stream",
           "cases": {}}
    pool = ThreadPoolExecutor(8)
    for name, (k, n, nb, ranks, frags) in CASES.items():
        for r in range(ranks):
            word0 = r * nb // 8
            full = O.fill_xorshift(word0 * 8 + nb)
            data = full[word0 * 8:]
            ent = {"k": k, "n": n, "bytes": nb, "rank": r, "word0": word0,
                   "data": sha(data)}
            if frags:
                fr = O.encode(k, n, data, nthreads=8)
                ent["frags"] = list(pool.map(sha, fr))
                del fr
            del full, data
            out["cases"]["%s_r%d" % (name, r)] = ent
            print(name, r, ent["data"][:16], flush=True)
    with open(os.path.join(HERE, "fullsize_sha256.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
