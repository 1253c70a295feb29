#!/usr/bin/env python3
"""Generate tests/golden/gf8_muladd_ref.npz from the reference's own kernels.

The reference's portable coding kernels are 256 straight-line functions
``gf8_muladd_XX(out, in)`` in xlators/cluster/ec/src/ec-code-c.c:20-11571
(each computes ``out = out * 0xXX ^ in`` over one 512-byte bit-sliced chunk).
Those sources cannot be compiled in this image (their headers need liburcu,
libuuid and a generated config.h), so this script *reads the source text* and
evaluates every function body statement by statement with numpy.  The
statement forms are the few the generated file uses::

    uint64_t inN = out_ptr[WIDTH * N];        load plane N of `out`
    X = A ^ B [^ C ...];                      XOR of loaded/temporary words
    out_ptr[WIDTH * N] = X ^ in_ptr[WIDTH * N];
    out_ptr[WIDTH * N] ^= in_ptr[WIDTH * N];  (gf8_muladd_01)
    memcpy(out, in, ...)                      (gf8_muladd_00)

Each loop iteration ``i`` touches only word ``i`` of every plane, so the loop
is evaluated for all 8 words at once.  The output file holds only data: the
random input chunks and, for every constant, the reference's result.  Run it
in the development container (the reference is not present on the GPU box):

    python tests/golden/gen_gf8_muladd.py
"""
import os
import re
import sys

import numpy as np

REF = "/root/reference/xlators/cluster/ec/src/ec-code-c.c"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "gf8_muladd_ref.npz")
SAMPLES = 3
SEED = 0x5EED_EC


def _index(expr):
    expr = expr.strip()
    if expr == "0":
        return 0
    if expr == "WIDTH":
        return 1
    m = re.fullmatch(r"WIDTH\s*\*\s*(\d+)", expr)
    if not m:
        raise ValueError("unexpected index " + expr)
    return int(m.group(1))


def _functions(text):
    for m in re.finditer(r"\ngf8_muladd_([0-9A-F]{2})\(void \*out, void \*in\)\n\{(.*?)\n\}\n",
                         text, re.S):
        yield int(m.group(1), 16), m.group(2)


def evaluate(body, out, inp):
    """Run one gf8_muladd body on chunks out/inp of shape [S, 8 planes, 8 words]."""
    out = out.copy()
    if "memcpy(out, in" in body:
        return inp.copy()
    loop = re.search(r"for \(i = 0; i < WIDTH; i\+\+\) \{(.*)\}", body, re.S)
    if not loop:
        raise ValueError("no loop")
    env = {}

    def term(t):
        t = t.strip()
        m = re.fullmatch(r"in_ptr\[(.+)\]", t)
        if m:
            return inp[:, _index(m.group(1))]
        m = re.fullmatch(r"out_ptr\[(.+)\]", t)
        if m:
            return out[:, _index(m.group(1))]
        return env[t]

    for stmt in loop.group(1).split(";"):
        s = " ".join(stmt.split())
        if not s or s.startswith("uint64_t out0") or s.startswith("uint64_t tmp") \
                or s in ("in_ptr++", "out_ptr++"):
            continue
        m = re.fullmatch(r"uint64_t (in\d+) = out_ptr\[(.+)\]", s)
        if m:
            env[m.group(1)] = out[:, _index(m.group(2))].copy()
            continue
        m = re.fullmatch(r"out_ptr\[(.+)\] \^= (.+)", s)
        if m:
            out[:, _index(m.group(1))] ^= term(m.group(2))
            continue
        m = re.fullmatch(r"(out_ptr\[.+\]|\w+) = (.+)", s)
        if m:
            val = None
            for t in m.group(2).split("^"):
                v = term(t)
                val = v.copy() if val is None else val ^ v
            dst = m.group(1)
            dm = re.fullmatch(r"out_ptr\[(.+)\]", dst)
            if dm:
                out[:, _index(dm.group(1))] = val
            else:
                env[dst] = val
            continue
        raise ValueError("unhandled statement: " + s)
    return out


def main():
    if not os.path.exists(REF):
        sys.exit("reference source not present; fixtures are already committed")
    text = open(REF).read()
    funcs = dict(_functions(text))
    if sorted(funcs) != list(range(256)):
        sys.exit("expected 256 gf8_muladd functions, found %d" % len(funcs))
    rng = np.random.default_rng(SEED)
    shape = (SAMPLES, 8, 8)  # samples x planes x u64 words  (one 512-B chunk)
    out0 = rng.integers(0, 2**64, size=shape, dtype=np.uint64)
    inp = rng.integers(0, 2**64, size=shape, dtype=np.uint64)
    # sample 0: a chunk whose planes are single-bit impulses, to touch every
    # (plane, bit) position deterministically
    out0[0] = np.uint64(1) << np.arange(64, dtype=np.uint64).reshape(8, 8)
    expected = np.empty((256,) + shape, dtype=np.uint64)
    for c in range(256):
        expected[c] = evaluate(funcs[c], out0, inp)
    np.savez_compressed(OUT, out0=out0, inp=inp, expected=expected,
                        source=np.array("ec-code-c.c:20-11571 gf8_muladd_00..FF"))
    print("wrote", OUT, expected.nbytes, "bytes of expected chunks")


if __name__ == "__main__":
    main()
