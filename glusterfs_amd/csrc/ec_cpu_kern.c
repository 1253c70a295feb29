/*
 * ec_cpu_kern.c -- per-ISA kernels of the CPU engine (ec_cpu.h).
 *
 * Compiled once per ISA level by the Makefile with -DECC_SFX=base / avx2 /
 * avx512 and the matching -m flags; ec_cpu.c picks one at run time
 * (__builtin_cpu_supports).  A plane of a chunk (64 bytes) is one GCC vector
 * of 8 x u64, so the same source becomes zmm code with AVX-512, ymm pairs
 * with AVX2 and xmm quads otherwise.  Three-input XORs use vpternlogq (0x96)
 * on AVX-512.
 *
 * Primitives generated from ec_gf8_prog.h, each on 512-byte chunks and
 * called through per-constant tables:
 *   mul_c    dst  = c * x                     (first term of a row)
 *   mac_c    acc ^= c * x                     (ec_code_c_interleaved step,
 *                                              ec-code-c.c:11660-11679)
 *   row_v    a whole encode row, acc = v * acc ^ D_j over the k chunks of a
 *            stripe with acc in registers (gf8_muladd_XX, ec-code-c.c:
 *            20-11571, as ec_code_c_linear chains it, :11647-11657), v <= 31
 *
 * Built with -O2: GCC 11 at -O3 miscompiled the AVX2 build of two rows
 * (v = 15 and 25 came out wrong, found by tests/test_cpu_engine.py).
 */
#include <stdint.h>
#include <string.h>

#include "ec_cpu.h"
#include "ec_gf8_prog.h"

#ifndef ECC_SFX
#error "compile with -DECC_SFX=base|avx2|avx512"
#endif
#define ECC_CAT2(a, b) a##_##b
#define ECC_CAT(a, b) ECC_CAT2(a, b)
#define ECC_NAME(n) ECC_CAT(n, ECC_SFX)

typedef uint64_t ecc_v __attribute__((vector_size(64)));

#if defined(__AVX512F__)
#include <immintrin.h>
static inline ecc_v xor3(ecc_v a, ecc_v b, ecc_v c)
{
    return (ecc_v)_mm512_ternarylogic_epi64((__m512i)a, (__m512i)b, (__m512i)c, 0x96);
}
#else
static inline ecc_v xor3(ecc_v a, ecc_v b, ecc_v c)
{
    return a ^ b ^ c;
}
#endif

/* unaligned, aliasing view of a plane (caller buffers are only 16-byte
 * aligned on the device-mapped paths) */
typedef uint64_t ecc_vu __attribute__((vector_size(64), aligned(1), may_alias));

static inline ecc_v ld(const uint8_t *p)
{
    return *(const ecc_vu *)p;
}

static inline void st(uint8_t *p, ecc_v v)
{
    *(ecc_vu *)p = v;
}

/* Streaming store of a finished plane (nt: the call's outputs exceed the
 * caches, and every output base is 64-byte aligned): a regular store of a
 * line that is not in cache first reads it (read-for-ownership), so a
 * DRAM-bound call moved its outputs twice.  The caller fences (ecc_nt_fence)
 * before it returns. */
static inline void stv(uint8_t *p, ecc_v v, int nt)
{
#if defined(__AVX512F__)
    if (nt) {
        _mm512_stream_si512((__m512i *)(void *)p, (__m512i)v);
        return;
    }
#endif
    st(p, v);
}

/* ECC_NT_BYTES: outputs of at least this many bytes per call are streamed */
#define ECC_NT_BYTES (16u << 20)

static void nt_fence(int nt)
{
#if defined(__AVX512F__)
    if (nt)
        _mm_sfence();
#else
    (void)nt;
#endif
}

static int nt_ok(uint8_t *const *out, uint32_t n, uint64_t bytes)
{
#if defined(__AVX512F__)
    if (bytes < ECC_NT_BYTES)
        return 0;
    for (uint32_t i = 0; i < n; i++)
        if ((uintptr_t)out[i] & 63)
            return 0;
    return 1;
#else
    (void)out;
    (void)n;
    (void)bytes;
    return 0;
#endif
}

typedef void (*ecc_fn)(uint8_t *dst, const uint8_t *src);

#define ECGF_X(b) x[b]
#define ECGF_TV(j) t##j
#define ECGF_T2(j, s1, s2) const ecc_v t##j = (s1) ^ (s2);
#define ECGF_T3(j, s1, s2, s3) const ecc_v t##j = xor3(s1, s2, s3);
#define ECGF_A1(p, s1) a[p] ^= (s1);
#define ECGF_A2(p, s1, s2) a[p] = xor3(a[p], s1, s2);

/* dst = c * src */
#define ECC_DEF_MUL(c)                                                         \
    static void mul_##c(uint8_t *dst, const uint8_t *src)                      \
    {                                                                          \
        ecc_v x[8], a[8];                                                      \
        _Pragma("GCC unroll 8") for (int i = 0; i < 8; i++) {                  \
            x[i] = ld(src + 64 * i);                                           \
            a[i] = (ecc_v){0};                                                 \
        }                                                                      \
        ECGF_PROG_##c                                                          \
        _Pragma("GCC unroll 8") for (int i = 0; i < 8; i++)                    \
            st(dst + 64 * i, a[i]);                                            \
    }
/* acc ^= c * src */
#define ECC_DEF_MAC(c)                                                         \
    static void mac_##c(uint8_t *acc, const uint8_t *src)                      \
    {                                                                          \
        ecc_v x[8], a[8];                                                      \
        _Pragma("GCC unroll 8") for (int i = 0; i < 8; i++) {                  \
            x[i] = ld(src + 64 * i);                                           \
            a[i] = ld(acc + 64 * i);                                           \
        }                                                                      \
        ECGF_PROG_##c                                                          \
        _Pragma("GCC unroll 8") for (int i = 0; i < 8; i++)                    \
            st(acc + 64 * i, a[i]);                                            \
    }
/* a whole encode row with v = c, the accumulator kept in registers:
 * out = Horner over the k chunks of one stripe (ec_code_c_linear) */
#define ECC_DEF_ROW(c)                                                         \
    static void row_##c(uint8_t *out, const uint8_t *in, uint32_t k, int nt)   \
    {                                                                          \
        ecc_v x[8], a[8];                                                      \
        _Pragma("GCC unroll 8") for (int i = 0; i < 8; i++)                    \
            x[i] = ld(in + 64 * i);                                            \
        for (uint32_t j = 1; j < k; j++) {                                     \
            const uint8_t *d = in + (uint64_t)j * 512u;                        \
            _Pragma("GCC unroll 8") for (int i = 0; i < 8; i++)                \
                a[i] = ld(d + 64 * i);                                         \
            ECGF_PROG_##c                                                      \
            _Pragma("GCC unroll 8") for (int i = 0; i < 8; i++)                \
                x[i] = a[i];                                                   \
        }                                                                      \
        _Pragma("GCC unroll 8") for (int i = 0; i < 8; i++)                    \
            stv(out + 64 * i, x[i], nt);                                       \
    }
ECGF_FOR_EACH(ECC_DEF_MUL)
ECGF_FOR_EACH(ECC_DEF_MAC)
#define ECC_ROWS(M) M(1) M(2) M(3) M(4) M(5) M(6) M(7) M(8) M(9) M(10) M(11) M(12) M(13)    \
    M(14) M(15) M(16) M(17) M(18) M(19) M(20) M(21) M(22) M(23) M(24) M(25) M(26) M(27) \
    M(28) M(29) M(30) M(31)
ECC_ROWS(ECC_DEF_ROW)

#define ECC_ENTRY_MUL(c) [c] = mul_##c,
#define ECC_ENTRY_MAC(c) [c] = mac_##c,
static const ecc_fn mul_tab[256] = {ECGF_FOR_EACH(ECC_ENTRY_MUL)};
static const ecc_fn mac_tab[256] = {ECGF_FOR_EACH(ECC_ENTRY_MAC)};
typedef void (*ecc_row_fn)(uint8_t *out, const uint8_t *in, uint32_t k, int nt);
#define ECC_ENTRY_ROW(c) [c] = row_##c,
/* rows of volumes up to EC_MAX_NODES = 31 bricks (ec.h:27-32) */
static const ecc_row_fn row_tab[32] = {ECC_ROWS(ECC_ENTRY_ROW)};

/* Row i of stripe t: acc = D_0; acc = (i+1) * acc ^ D_j for j = 1..k-1
 * (ec_method_matrix_normal rows with ec_code_c_prepare's Horner ratios,
 * all equal to v = i + 1, ec-method.c:22-36, ec-code-c.c:11632-11644). */
void ECC_NAME(ecc_encode)(uint32_t k, uint32_t n, uint64_t nstripes, const uint8_t *in,
                          uint64_t in_stride, uint8_t *const *out, uint64_t out_off)
{
    const int nt = nt_ok(out, n, nstripes * 512u * n);
    for (uint64_t t = 0; t < nstripes; t++) {
        const uint8_t *s = in + t * in_stride;
        for (uint32_t i = 0; i < n; i++) {
            uint8_t *o = out[i] + (out_off + t) * 512u;
            row_tab[i + 1](o, s, k, nt); /* n <= 31: ec_method_init */
        }
    }
    nt_fence(nt);
}

#if defined(__AVX512F__)
/* One output chunk o = sum_p coef[p] * x_p (zero coefficients skipped) with
 * the accumulator in registers: the multiply is a switch over the 255
 * programs inside this function, so the 8 accumulator planes stay in zmm
 * registers across the inputs (32 zmm hold the accumulator, the input and
 * the program temporaries), where the mac_tab calls load and store the
 * accumulator once per input.  AVX-512 only: AVX2 / base would spill. */
#define ECC_CASE(c)                                                            \
    case c: {                                                                  \
        ECGF_PROG_##c                                                          \
    } break;
static void combine_row_reg(uint8_t *o, const uint8_t *const *xp, const uint8_t *coef,
                            uint32_t k, int nt)
{
    ecc_v a[8] = {{0}};
    for (uint32_t p = 0; p < k; p++) {
        const uint8_t c = coef[p];
        if (c == 0)
            continue;
        ecc_v x[8];
        _Pragma("GCC unroll 8") for (int i = 0; i < 8; i++)
            x[i] = ld(xp[p] + 64 * i);
        switch (c) {
            ECGF_FOR_EACH(ECC_CASE)
        }
    }
    _Pragma("GCC unroll 8") for (int i = 0; i < 8; i++)
        stv(o + 64 * i, a[i], nt);
}
#undef ECC_CASE
#endif

/* ecd_combine_desc_t semantics (ec_device.h) over stripes [s0, s1); `pats`
 * = the packed patterns {src[k], coef[rows][k]}; zero coefficients are
 * skipped (ec-code-c.c:11666-11676). */
void ECC_NAME(ecc_combine)(const ecd_combine_desc_t *d, const uint8_t *pats, uint64_t s0,
                           uint64_t s1)
{
    const uint32_t k = d->k;
#if defined(__AVX512F__)
    const int nt = nt_ok((uint8_t *const *)d->out_base, d->rows,
                         (s1 - s0) * 512u * d->rows) && !(d->out_stride & 63);
#endif
    for (uint64_t t = s0; t < s1; t++) {
        uint32_t q = 0;
        if (d->group_pattern) {
            q = d->group_pattern[t >> d->group_shift];
            if (q >= d->npatterns)
                q = d->npatterns - 1; /* clamp, as the kernels do */
        }
        const uint8_t *pat = pats + (size_t)q * d->pat_bytes;
#if defined(__AVX512F__)
        const uint8_t *xs[ECD_MAX_ROWS];
        for (uint32_t p = 0; p < k; p++)
            xs[p] = (const uint8_t *)d->in_base[pat[p]] + t * d->in_stride;
        for (uint32_t r = 0; r < d->rows; r++)
            combine_row_reg((uint8_t *)d->out_base[r] + t * d->out_stride, xs,
                            pat + k + (size_t)r * k, k, nt);
        continue;
#endif
        for (uint32_t r = 0; r < d->rows; r++) {
            uint8_t *o = (uint8_t *)d->out_base[r] + t * d->out_stride;
            const uint8_t *coef = pat + k + (size_t)r * k;
            int first = 1;
            for (uint32_t p = 0; p < k; p++) {
                const uint8_t c = coef[p];
                if (c == 0)
                    continue;
                const uint8_t *x = (const uint8_t *)d->in_base[pat[p]] + t * d->in_stride;
                if (first)
                    mul_tab[c](o, x);
                else
                    mac_tab[c](o, x);
                first = 0;
            }
            if (first)
                memset(o, 0, 512);
        }
    }
#if defined(__AVX512F__)
    nt_fence(nt);
#endif
}
