#!/usr/bin/env python3
"""Whole-matrix XOR programs for ONE fixed 16 x 16 GF(2^8) decode matrix
(VERDICT r05 "do this" #2: the k = 16 lever never measured).

The shipped k = 16 combine evaluates each output row as 16 multiply-
accumulates, each a searched program over one input's 8 bit-planes
(tools/gen/gf8_search.c: 12.85 v_bitop3 / v_xor per multiply on average),
so it shares nothing across coefficients: ~3,300 instructions per dword
column for a dense 16 x 16 matrix.  Over the whole 128 x 128 GF(2) matrix
(output plane (r, b) x input plane (p, j); entry = bit b of c_rp * x^j) a
four-Russians program shares sub-sums: every input's 8 planes are split
into two groups of 4, each group's 15 nonzero XOR combinations are built
once (11 instructions with a 3-input XOR: 6 pairs, 4 triples, 1 quad), and
each output plane takes one table entry per group -- both groups of an
input in one v_bitop3 (acc ^ T0[m0] ^ T1[m1]).

Emits tools/kbench/kb_wm16.h: device functions that run this program on
one lane's dword column of a plane-major LDS tile (kb3's layout: input p,
plane b at (p * 8 + b) * T * 64), for all 16 output rows or for 8 of them,
plus the instruction counts of both programs and of the row-by-row
programs for the same matrix (from tools/gen/gf8_prog.txt).

The matrix is kb3's dense decode matrix: c(r, p) = 1 + ((r*16 + p) * 173
+ 11) % 255 (tools/kbench/kb3.hip ct_coef), so the probe's output is
checked against the shipped run-time kernel on the same coefficients.

    python3 tools/gen/gen_wm16.py > tools/kbench/kb_wm16.h
"""
import os

HERE = os.path.dirname(os.path.abspath(__file__))
K = 16


def gf_mul(a, b):
    r = 0
    while b:
        if b & 1:
            r ^= a
        a <<= 1
        if a & 0x100:
            a ^= 0x11D
        b >>= 1
    return r


def coef(r, p):
    return 1 + ((r * K + p) * 173 + 11) % 255


def row_mask(r, b, p):
    """bits j of input p's planes that feed output plane (r, b)"""
    c = coef(r, p)
    return sum(((gf_mul(c, 1 << j) >> b) & 1) << j for j in range(8))


def rowwise_ops():
    lens = {}
    for line in open(os.path.join(HERE, "gf8_prog.txt")):
        f = line.split()
        lens[int(f[0])] = int(f[1])
    return sum(lens[coef(r, p)] for r in range(K) for p in range(K))


TABLE = {}      # 4-bit mask -> (op, operands as masks)


def table_program(need):
    """instructions building the needed nonzero combinations of 4 planes;
    singletons are the planes themselves"""
    have = {1, 2, 4, 8}
    ops = []

    def build(m):
        if m in have:
            return
        bits = [1 << i for i in range(4) if m >> i & 1]
        if len(bits) == 2:
            ops.append((m, bits))
        elif len(bits) == 3:
            ops.append((m, bits))
        else:                                   # 4 planes: (ab) ^ c ^ d
            ab = bits[0] | bits[1]
            build(ab)
            ops.append((m, [ab, bits[2], bits[3]]))
        have.add(m)

    for m in sorted(need, key=lambda x: bin(x).count("1")):
        build(m)
    return ops


def emit_prog(name, rows, T):
    outs = [(r, b) for r in rows for b in range(8)]
    lines = []
    nops = 0
    ntab = 0
    lines.append("template <int T>")
    lines.append("__device__ __forceinline__ void %s(const uint8_t *col, u32 (&acc)[%d])"
                 % (name, len(outs)))
    lines.append("{")
    lines.append("    u32 x[8], nx[8];")
    lines.append("#pragma unroll")
    lines.append("    for (int b = 0; b < 8; ++b)")
    lines.append("        nx[b] = *reinterpret_cast<const u32 *>(col + (u32)b * (T * 64u));")
    started = [False] * len(outs)
    for p in range(K):
        lines.append("    /* input %d */" % p)
        lines.append("#pragma unroll")
        lines.append("    for (int b = 0; b < 8; ++b)")
        lines.append("        x[b] = nx[b];")
        if p + 1 < K:
            lines.append("#pragma unroll")
            lines.append("    for (int b = 0; b < 8; ++b)")
            lines.append("        nx[b] = *reinterpret_cast<const u32 *>(col + (u32)(%d * 8 + b) * (T * 64u));"
                         % (p + 1))
        lines.append("    __builtin_amdgcn_sched_barrier(0);")
        lines.append("    {")
        masks = [row_mask(r, b, p) for (r, b) in outs]
        for h in range(2):
            need = {(m >> (4 * h)) & 15 for m in masks} - {0}
            prog = table_program(need)
            for j in range(4):
                lines.append("        const u32 t%d_%d = x[%d];" % (h, 1 << j, 4 * h + j))
            for m, srcs in prog:
                args = ", ".join("t%d_%d" % (h, s) for s in srcs)
                if len(srcs) == 2:
                    lines.append("        const u32 t%d_%d = %s ^ %s;" % (h, m, "t%d_%d" % (h, srcs[0]),
                                                                      "t%d_%d" % (h, srcs[1])))
                else:
                    lines.append("        const u32 t%d_%d = ecgf::xor3(%s);" % (h, m, args))
                nops += 1
                ntab += 1
        for o, m in enumerate(masks):
            m0, m1 = m & 15, m >> 4
            terms = ["t0_%d" % m0] if m0 else []
            terms += ["t1_%d" % m1] if m1 else []
            if not terms:
                continue
            if not started[o]:
                if len(terms) == 2:
                    lines.append("        acc[%d] = %s ^ %s;" % (o, terms[0], terms[1]))
                    nops += 1
                else:
                    lines.append("        acc[%d] = %s;" % (o, terms[0]))
                started[o] = True
            elif len(terms) == 2:
                lines.append("        acc[%d] = ecgf::xor3(acc[%d], %s, %s);" % (o, o, terms[0], terms[1]))
                nops += 1
            else:
                lines.append("        acc[%d] ^= %s;" % (o, terms[0]))
                nops += 1
        lines.append("    }")
        lines.append("    __builtin_amdgcn_sched_barrier(0);")
    for o in range(len(outs)):
        if not started[o]:
            lines.append("    acc[%d] = 0;" % o)
    lines.append("}")
    return lines, nops, ntab


def main():
    T = 4
    full, n_full, t_full = emit_prog("wm16_rows16", list(range(16)), T)
    h0, n_h0, t_h0 = emit_prog("wm16_rows_lo", list(range(8)), T)
    h1, n_h1, t_h1 = emit_prog("wm16_rows_hi", list(range(8, 16)), T)
    rw = rowwise_ops()
    out = ["/* Generated by tools/gen/gen_wm16.py -- do not edit.  Development probe",
           " * (tools/kbench/kb3.hip group dec16wm), not product code.",
           " * Whole-matrix four-Russians programs (two 4-plane groups per input) of",
           " * kb3's dense 16 x 16 decode matrix c(r, p) = 1 + ((r*16+p)*173 + 11) % 255.",
           " * Instructions per dword column (v_xor / v_bitop3):",
           " *   row by row, searched programs (shipped kernel): %d" % rw,
           " *   whole matrix, all 16 rows in one program:       %d (%d of them table builds)" % (n_full, t_full),
           " *   two programs of 8 rows (tables built twice):     %d + %d = %d" % (n_h0, n_h1, n_h0 + n_h1),
           " */",
           "#pragma once",
           "#define WM16_OPS_ROWWISE %d" % rw,
           "#define WM16_OPS_FULL %d" % n_full,
           "#define WM16_OPS_HALVES %d" % (n_h0 + n_h1),
           ""]
    out += full + [""] + h0 + [""] + h1
    print("\n".join(out))


if __name__ == "__main__":
    main()
