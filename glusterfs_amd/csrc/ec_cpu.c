/*
 * ec_cpu.c -- CPU engine dispatch (see ec_cpu.h): ISA selection, argument
 * checks, and the gathered encode of partial-stripe writes.
 */
#define _GNU_SOURCE
#include <errno.h>
#include <stdlib.h>
#include <string.h>

#include "ec_cpu.h"

int
ecc_isa_max(void)
{
#if defined(__x86_64__)
    __builtin_cpu_init();
    if (__builtin_cpu_supports("avx512f"))
        return ECC_ISA_AVX512;
    if (__builtin_cpu_supports("avx2"))
        return ECC_ISA_AVX2;
#endif
    return ECC_ISA_BASE;
}

const char *
ecc_isa_name(int isa)
{
    switch (isa) {
    case ECC_ISA_AVX512:
        return "avx512";
    case ECC_ISA_AVX2:
        return "avx2";
    default:
        return "x86-64";
    }
}

static int
clamp_isa(int isa)
{
    const int m = ecc_isa_max();
    return isa > m ? m : (isa < 0 ? 0 : isa);
}

void
ecc_encode(int isa, uint32_t k, uint32_t n, uint64_t nstripes, const uint8_t *in,
           uint8_t *const *out)
{
    const uint64_t stride = (uint64_t)k * ECD_CHUNK;
    switch (clamp_isa(isa)) {
#if defined(__x86_64__)
    case ECC_ISA_AVX512:
        ecc_encode_avx512(k, n, nstripes, in, stride, out, 0);
        return;
    case ECC_ISA_AVX2:
        ecc_encode_avx2(k, n, nstripes, in, stride, out, 0);
        return;
#endif
    default:
        ecc_encode_base(k, n, nstripes, in, stride, out, 0);
    }
}

static void
encode_one(int isa, uint32_t k, uint32_t n, const uint8_t *in, uint8_t *const *out,
           uint64_t stripe)
{
    const uint64_t stride = (uint64_t)k * ECD_CHUNK;
    switch (isa) {
#if defined(__x86_64__)
    case ECC_ISA_AVX512:
        ecc_encode_avx512(k, n, 1, in, stride, out, stripe);
        return;
    case ECC_ISA_AVX2:
        ecc_encode_avx2(k, n, 1, in, stride, out, stripe);
        return;
#endif
    default:
        ecc_encode_base(k, n, 1, in, stride, out, stripe);
    }
}

int
ecc_encode_gather(int isa, uint32_t k, uint32_t n, uint64_t nstripes, uint32_t nsegs,
                  const void *const *seg_ptr, const uint64_t *seg_len, uint8_t *const *out)
{
    const uint64_t S = (uint64_t)k * ECD_CHUNK;
    uint8_t buf[ECD_MAX_K * ECD_CHUNK] __attribute__((aligned(64)));
    uint64_t total = 0, base = 0;
    uint32_t seg = 0;

    for (uint32_t i = 0; i < nsegs; i++)
        total += seg_len[i];
    if (total != nstripes * S || k > ECD_MAX_K)
        return -EINVAL;
    isa = clamp_isa(isa);
    for (uint64_t t = 0; t < nstripes; t++) {
        const uint64_t v0 = t * S, v1 = v0 + S;
        while (seg < nsegs && base + seg_len[seg] <= v0) /* skip segments before v0 */
            base += seg_len[seg++];
        if (seg < nsegs && seg_ptr[seg] && base + seg_len[seg] >= v1) {
            /* the whole stripe lies in one caller segment: code it in place */
            encode_one(isa, k, n, (const uint8_t *)seg_ptr[seg] + (v0 - base), out, t);
            continue;
        }
        uint64_t b = base;
        for (uint32_t s = seg; s < nsegs && b < v1; b += seg_len[s++]) {
            const uint64_t lo = b > v0 ? b : v0;
            const uint64_t hi = b + seg_len[s] < v1 ? b + seg_len[s] : v1;
            if (lo >= hi)
                continue;
            if (seg_ptr[s])
                memcpy(buf + (lo - v0), (const uint8_t *)seg_ptr[s] + (lo - b), hi - lo);
            else
                memset(buf + (lo - v0), 0, hi - lo);
        }
        encode_one(isa, k, n, buf, out, t);
    }
    return 0;
}

int
ecc_combine(int isa, const ecd_combine_desc_t *d)
{
    const uint8_t *pats = d->pat_ext ? d->pat_ext : d->pat;

    if (d->k == 0 || d->k > ECD_MAX_K || d->rows == 0 || d->rows > ECD_MAX_ROWS ||
        d->npatterns == 0 || d->npatterns > ECD_MAX_PATTERNS ||
        d->pat_bytes < d->k + d->rows * d->k || (d->group_pattern && d->group_shift > 63))
        return -EINVAL;
    if (!d->pat_ext && (uint64_t)d->npatterns * d->pat_bytes > ECD_MAX_PAT_BYTES)
        return -EINVAL;
    switch (clamp_isa(isa)) {
#if defined(__x86_64__)
    case ECC_ISA_AVX512:
        ecc_combine_avx512(d, pats, 0, d->nstripes);
        break;
    case ECC_ISA_AVX2:
        ecc_combine_avx2(d, pats, 0, d->nstripes);
        break;
#endif
    default:
        ecc_combine_base(d, pats, 0, d->nstripes);
    }
    return 0;
}
