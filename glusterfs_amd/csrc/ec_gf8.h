/*
 * ec_gf8.h -- GF(2^8) multiply-by-constant on bit-sliced 512-byte chunks,
 * evaluated by gfx950 VALU XOR trees.
 *
 * Layout (ec-method.h:27-29): a chunk is 8 bit-planes of
 * 64 bytes; bit b of GF symbol s (s = 0..511) is bit s%8 of byte b*64 + s/8.
 * A lane owns W consecutive dwords (32*W symbols) of every plane, so a GF
 * multiply by a constant C is a fixed 8x8 GF(2) matrix applied plane-wise:
 * out plane p = XOR of the input planes b whose bit p is set in C*2^b.  That
 * is the operation each reference gf8_muladd_XX routine (ec-code-c.c:20-11571)
 * and each JIT program (ec-gf8.c:13-5882) evaluates.  Here C is a template
 * parameter, so the matrix is folded at compile time and every XOR of three
 * terms becomes one v_bitop3_b32 (LUT 0x96); no tables are read at run time.
 */
#ifndef EC_MI355X_GF8_H
#define EC_MI355X_GF8_H

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ec_gf8_asm.h"
#include "ec_gf8_prog.h"

namespace ecgf {

typedef uint32_t u32;

/* Carry-less multiply modulo x^8+x^4+x^3+x^2+1 (EC_GF_MOD 0x11D). */
constexpr u32 mul(u32 a, u32 b)
{
    u32 r = 0;
    for (int i = 0; i < 8; ++i) {
        if (b & 1u)
            r ^= a;
        b >>= 1;
        a <<= 1;
        if (a & 0x100u)
            a ^= 0x11Du;
    }
    return r & 0xFFu;
}

/* Bit b of rowmask(C, p): output plane p of C*x depends on input plane b. */
constexpr u32 rowmask(u32 c, int p)
{
    u32 m = 0;
    for (int b = 0; b < 8; ++b)
        if ((mul(c, 1u << b) >> p) & 1u)
            m |= 1u << b;
    return m;
}

__device__ __forceinline__ u32 xor3(u32 a, u32 b, u32 c)
{
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

/* out[p] = base[p] ^ (C * src)[p] with each plane's own XOR3 chain and no
 * sharing between planes: 18.07 instructions per multiply-accumulate on
 * average (round-1 form, kept for A/B runs in tools/kbench).  `out` may
 * alias `base`, but must not alias `src`. */
template <u32 C, int W>
__device__ __forceinline__ void mul_xor_naive(u32 (&out)[8][W], const u32 (&base)[8][W],
                                              const u32 (&src)[8][W])
{
#pragma unroll
    for (int p = 0; p < 8; ++p) {
#pragma unroll
        for (int w = 0; w < W; ++w) {
            u32 t = base[p][w];
            u32 pend = 0;
            bool has = false;
#pragma unroll
            for (int b = 0; b < 8; ++b) {
                if ((rowmask(C, p) >> b) & 1u) {
                    if (has) {
                        t = xor3(t, pend, src[b][w]);
                        has = false;
                    } else {
                        pend = src[b][w];
                        has = true;
                    }
                }
            }
            if (has)
                t ^= pend;
            out[p][w] = t;
        }
    }
}

/* acc ^= C * x by the searched program of ec_gf8_prog.h (tools/gen): shared
 * temporaries across the 8 output planes, 12.85 v_bitop3/v_xor per
 * multiply-accumulate per dword on average (the reference's own searched
 * programs, ec-gf8.c, average 12.8 XOR2 for the multiply alone, before the
 * 8 accumulating XORs: ec-implementation.md:516-519). */
template <u32 C>
struct Prog;

#define ECGF_X(b) x[b][w]
#define ECGF_TV(j) t##j
#define ECGF_T2(j, s1, s2) const u32 t##j = (s1) ^ (s2);
#define ECGF_T3(j, s1, s2, s3) const u32 t##j = xor3(s1, s2, s3);
#define ECGF_A1(p, s1) a[p][w] ^= (s1);
#define ECGF_A2(p, s1, s2) a[p][w] = xor3(a[p][w], s1, s2);
#define ECGF_DEF(c)                                                            \
    template <>                                                                \
    struct Prog<c> {                                                           \
        template <int W>                                                       \
        __device__ __forceinline__ static void run(u32 (&a)[8][W],            \
                                                   const u32 (&x)[8][W])      \
        {                                                                      \
            _Pragma("unroll") for (int w = 0; w < W; ++w) { ECGF_PROG_##c }   \
        }                                                                      \
    };
ECGF_FOR_EACH(ECGF_DEF)
#undef ECGF_DEF
#undef ECGF_A2
#undef ECGF_A1
#undef ECGF_T3
#undef ECGF_T2
#undef ECGF_TV
#undef ECGF_X

/* out[p] = base[p] ^ (C * src)[p].  `out` may alias `base`, but must not
 * alias `src`. */
template <u32 C, int W, bool CSE = true>
__device__ __forceinline__ void mul_xor(u32 (&out)[8][W], const u32 (&base)[8][W],
                                        const u32 (&src)[8][W])
{
    if constexpr (!CSE) {
        mul_xor_naive<C, W>(out, base, src);
    } else {
#pragma unroll
        for (int p = 0; p < 8; ++p)
#pragma unroll
            for (int w = 0; w < W; ++w)
                out[p][w] = base[p][w];
        Prog<C>::template run<W>(out, src);
    }
}

/* Horner step acc = C*acc ^ d  (ec-code-c.c:11647-11657 inner statement). */
template <u32 C, int W, bool CSE = true>
__device__ __forceinline__ void horner(u32 (&acc)[8][W], const u32 (&d)[8][W])
{
    u32 t[8][W];
    mul_xor<C, W, CSE>(t, d, acc);
#pragma unroll
    for (int p = 0; p < 8; ++p)
#pragma unroll
        for (int w = 0; w < W; ++w)
            acc[p][w] = t[p][w];
}

/* acc ^= c*x for a wave-uniform run-time constant c.  The switch lowers to
 * a scalar compare tree (no divergence: c lives in an SGPR); c == 0 adds
 * nothing, matching the zero-skipping of ec_code_c_interleaved
 * (ec-code-c.c:11666-11676). */
template <int W, bool CSE = true>
__device__ __forceinline__ void mul_xor_rt(u32 c, u32 (&acc)[8][W], const u32 (&x)[8][W])
{
    switch (c) {
#define ECGF_CASE(n)                                                           \
    case n:                                                                    \
        mul_xor<n, W, CSE>(acc, acc, x);                                       \
        break;
#define ECGF_CASE16(h)                                                         \
    ECGF_CASE(h * 16 + 0) ECGF_CASE(h * 16 + 1) ECGF_CASE(h * 16 + 2)          \
    ECGF_CASE(h * 16 + 3) ECGF_CASE(h * 16 + 4) ECGF_CASE(h * 16 + 5)          \
    ECGF_CASE(h * 16 + 6) ECGF_CASE(h * 16 + 7) ECGF_CASE(h * 16 + 8)          \
    ECGF_CASE(h * 16 + 9) ECGF_CASE(h * 16 + 10) ECGF_CASE(h * 16 + 11)        \
    ECGF_CASE(h * 16 + 12) ECGF_CASE(h * 16 + 13) ECGF_CASE(h * 16 + 14)       \
    ECGF_CASE(h * 16 + 15)
        ECGF_CASE(1) ECGF_CASE(2) ECGF_CASE(3) ECGF_CASE(4) ECGF_CASE(5)
        ECGF_CASE(6) ECGF_CASE(7) ECGF_CASE(8) ECGF_CASE(9) ECGF_CASE(10)
        ECGF_CASE(11) ECGF_CASE(12) ECGF_CASE(13) ECGF_CASE(14) ECGF_CASE(15)
        ECGF_CASE16(1) ECGF_CASE16(2) ECGF_CASE16(3) ECGF_CASE16(4)
        ECGF_CASE16(5) ECGF_CASE16(6) ECGF_CASE16(7) ECGF_CASE16(8)
        ECGF_CASE16(9) ECGF_CASE16(10) ECGF_CASE16(11) ECGF_CASE16(12)
        ECGF_CASE16(13) ECGF_CASE16(14) ECGF_CASE16(15)
#undef ECGF_CASE16
#undef ECGF_CASE
    default:
        break;
    }
}

/* acc ^= c * x for a wave-uniform run-time c in 1..255, 2 dwords per plane
 * per lane: a jump through a PC-relative table into the searched program
 * for c (ec_gf8_asm.h, generated).  Replaces the switch above where the
 * compare tree's scalar work bounds the kernel. */
template <int W>
__device__ __forceinline__ void mul_xor_jt(u32 c, u32 (&acc)[8][W], const u32 (&x)[8][W])
{
    static_assert(W == 1 || W == 2, "the assembly bodies are generated for 1 or 2 dwords");
    u32 t[ECGF_ASM_TEMPS][W];
    if constexpr (W == 2)
        ECGF_ASM_DISPATCH_W2(acc, x, t, c);
    else
        ECGF_ASM_DISPATCH_W1(acc, x, t, c);
}

} // namespace ecgf

#endif
