/*
 * ec_kernels_impl.h -- gfx950 kernel templates of the disperse coding path.
 * Included by ec_kernels.hip (the product launchers) and by the development
 * harness tools/kbench/kbench.hip, so tuning measures the shipped code.
 *
 * Two kernels, both working directly on ec's bit-sliced chunk layout
 * (512-byte chunks = 8 planes x 64 bytes, ec-method.h:27-29):
 *
 *  ec_encode_vander<K, N, W, NTS>   reference: ec_method_encode
 *      (ec-method.c:394-408) with the per-row Horner kernels ec_code_c_linear
 *      (ec-code-c.c:11647).  Fragment i of stripe t = Horner over the k data
 *      chunks with the row's evaluation point v = i + 1 (ec-method.c:22-36,
 *      284-286).  K, N and therefore every v are compile-time constants, so
 *      each Horner step is a straight-line XOR tree (ec_gf8.h) -- the gfx950
 *      counterpart of the reference's JIT'ed row routines (ec-code.c:722).
 *      A lane owns W dwords of all 8 planes of one chunk column (L = 16/W
 *      lanes per chunk); its k input chunks stay in VGPRs, so HBM is read once.
 *
 *  ec_combine<K, TS, NW, MIXED, NTS>  reference: ec_method_decode
 *      (ec-method.c:411-433) with ec_code_c_interleaved (ec-code-c.c:11660).
 *      Output row r of stripe t = XOR_p coef[r][p] * input_p(t) for a run-time
 *      coefficient matrix held in the kernel-argument segment (constant
 *      memory, scalar loads).  One block = one tile of T = 8*TS stripes: the
 *      k input chunks of the tile are staged into LDS by LDS-DMA (16 bytes
 *      per lane, no VGPRs), then each wave computes whole output rows (8 stripes x
 *      8 lanes x 2 dwords per plane) walking the inputs with a run-time index
 *      so a single multiply dispatch serves every coefficient: the
 *      wave-uniform coefficient selects one of 255 compile-time XOR trees
 *      through a scalar compare tree, zero coefficients are skipped.  MIXED
 *      picks a pattern (erasure mask -> sources + inverse) per stripe group.
 *
 * Tuning knobs measured with tools/kbench (profiles/kbench_*.log): one tile
 * per block beats a persistent grid with register prefetch (vmcnt also counts
 * the stores of the previous tile, which serialises the prefetch);
 * non-temporal loads lose; staging the output tile through LDS, a split
 * 16+16-case dispatch, register staging, prefetching the next input's LDS
 * reads, ping-pong accumulators (2 switch copies: i-cache misses x3.6),
 * 64-bit accumulators (v_mov_b64 join copies: +-10 % depending on the
 * coefficient matrix), grouped input staging for k = 16 and an explicit
 * binary compare tree measured equal or worse and were removed; NTS
 * (non-temporal stores), the tile size TS and the block size NW remain
 * knobs.
 */
#ifndef EC_MI355X_KERNELS_IMPL_H
#define EC_MI355X_KERNELS_IMPL_H

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <utility>

#include "ec_device.h"
#include "ec_gf8.h"

namespace ecdev {

using ecgf::u32;
typedef u32 v2u __attribute__((ext_vector_type(2)));
typedef u32 v4u __attribute__((ext_vector_type(4)));

constexpr int kBlock = 256;

/* Cache policy of the LDS-DMA staging loads: the aux operand of
 * global_load_lds, 0 = default, 2 = non-temporal.  The kernels take it as a
 * template parameter LA (default 0, the policy of the 8-stripe ec_encode_tile
 * and the zero-copy kernels); the launchers pick it per call by input size
 * (ec_kernels.hip nt_staging). */
constexpr int kLdsDmaDefault = 0, kLdsDmaNT = 2;

/* Compile-time loop: f(std::integral_constant<int, I>) for I in [B, E). */
template <int B, int E, typename F>
__device__ __forceinline__ void static_for(F &&f)
{
    if constexpr (B < E) {
        f(std::integral_constant<int, B>{});
        static_for<B + 1, E>(f);
    }
}

template <int W>
__device__ __forceinline__ void load_plane(const uint8_t *p, u32 (&d)[W])
{
    if constexpr (W == 1) {
        d[0] = *reinterpret_cast<const u32 *>(p);
    } else if constexpr (W == 2) {
        const uint2 v = *reinterpret_cast<const uint2 *>(p);
        d[0] = v.x;
        d[1] = v.y;
    } else {
        const uint4 v = *reinterpret_cast<const uint4 *>(p);
        d[0] = v.x;
        d[1] = v.y;
        d[2] = v.z;
        d[3] = v.w;
    }
}

template <int W, bool NT>
__device__ __forceinline__ void store_plane(uint8_t *p, const u32 (&d)[W])
{
    if constexpr (NT) {
        if constexpr (W == 1) {
            __builtin_nontemporal_store(d[0], reinterpret_cast<u32 *>(p));
        } else if constexpr (W == 2) {
            const v2u v = {d[0], d[1]};
            __builtin_nontemporal_store(v, reinterpret_cast<v2u *>(p));
        } else {
            const v4u v = {d[0], d[1], d[2], d[3]};
            __builtin_nontemporal_store(v, reinterpret_cast<v4u *>(p));
        }
    } else {
        if constexpr (W == 1)
            *reinterpret_cast<u32 *>(p) = d[0];
        else if constexpr (W == 2)
            *reinterpret_cast<uint2 *>(p) = make_uint2(d[0], d[1]);
        else
            *reinterpret_cast<uint4 *>(p) = make_uint4(d[0], d[1], d[2], d[3]);
    }
}

template <int W>
__device__ __forceinline__ void load_chunk(const uint8_t *p, u32 (&d)[8][W])
{
#pragma unroll
    for (int b = 0; b < 8; ++b)
        load_plane<W>(p + b * 64, d[b]);
}

template <int W, bool NT>
__device__ __forceinline__ void store_chunk(uint8_t *p, const u32 (&d)[8][W])
{
#pragma unroll
    for (int b = 0; b < 8; ++b)
        store_plane<W, NT>(p + b * 64, d[b]);
}

/* ------------------------------------------------ specialised encoder */

struct FragPtrs {
    uint8_t *p[ECD_MAX_ROWS];
};

/* Row I (evaluation point v = I + 1) of the reversed Vandermonde matrix. */
template <int K, int W, int I, bool CSE = true>
__device__ __forceinline__ void encode_row_acc(const u32 (&x)[K][8][W], u32 (&acc)[8][W])
{
    constexpr u32 v = I + 1;
    if constexpr (v == 1) {
        /* row 0 = XOR of all data chunks, as XOR3 chains */
#pragma unroll
        for (int b = 0; b < 8; ++b)
#pragma unroll
            for (int w = 0; w < W; ++w) {
                u32 t = x[0][b][w];
                int j = 1;
#pragma unroll
                for (; j + 1 < K; j += 2)
                    t = ecgf::xor3(t, x[j][b][w], x[j + 1][b][w]);
                if (j < K)
                    t ^= x[j][b][w];
                acc[b][w] = t;
            }
    } else {
#pragma unroll
        for (int b = 0; b < 8; ++b)
#pragma unroll
            for (int w = 0; w < W; ++w)
                acc[b][w] = x[0][b][w];
#pragma unroll
        for (int j = 1; j < K; ++j)
            ecgf::horner<v, W, CSE>(acc, x[j]);
    }
}

template <int K, int W, int I, bool NTS, bool CSE = true>
__device__ __forceinline__ void encode_row(const u32 (&x)[K][8][W], uint8_t *dst)
{
    u32 acc[8][W];
    encode_row_acc<K, W, I, CSE>(x, acc);
    store_chunk<W, NTS>(dst, acc);
}

template <int K, int W, bool NTS, bool CSE, int... I>
__device__ __forceinline__ void encode_rows(std::integer_sequence<int, I...>,
                                            const u32 (&x)[K][8][W], const FragPtrs &out,
                                            uint64_t off)
{
    (encode_row<K, W, I, NTS, CSE>(x, out.p[I] + off), ...);
}

/* CSE: multiply by the searched programs of ec_gf8_prog.h (false: the
 * round-1 per-plane trees, for A/B runs) */
template <int K, int N, int W, bool NTS, bool CSE = true>
__global__ __launch_bounds__(kBlock) void ec_encode_vander(const uint8_t *__restrict__ in,
                                                           const FragPtrs out,
                                                           uint64_t nstripes)
{
    constexpr int L = 16 / W;
    const uint64_t gtid = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    const uint64_t stripe = gtid / L;
    if (stripe >= nstripes)
        return;
    const u32 colb = (u32)(gtid % L) * (4 * W);

    u32 x[K][8][W];
    const uint8_t *s = in + stripe * (uint64_t)(K * ECD_CHUNK) + colb;
#pragma unroll
    for (int j = 0; j < K; ++j)
        load_chunk<W>(s + j * ECD_CHUNK, x[j]);

    encode_rows<K, W, NTS, CSE>(std::make_integer_sequence<int, N>{}, x, out,
                                stripe * (uint64_t)ECD_CHUNK + colb);
}

/* Tile encoder: the data of 8 stripes is staged in LDS by LDS-DMA
 * (global_load_lds_dwordx4, no VGPRs on the read path) into the plane-major
 * tile of ec_combine -- input chunk p, plane b, stripe s at
 * ((p * 8 + b) * 8 + s) * 64 -- and every wave then computes whole rows
 * (fragments) for the 8 stripes by Horner with the row's compile-time
 * constant v = r + 1 (ec-code-c.c:11647-11657), reading each input chunk
 * back from LDS.  The row index is wave-uniform, so the dispatch is a
 * scalar branch to one of N specialised rows.  Where the rows are cheap
 * (4+2) this beats the register-resident encoder: the LDS-DMA read path
 * leaves the VGPRs and the vector memory pipe to the stores.
 * Grid: one block per 8 stripes; LDS = K * 4 KiB. */
/* GF(2^8) power at compile time (poly 0x11D) */
constexpr u32 gf_mul_c(u32 a, u32 b)
{
    u32 r = 0;
    for (int i = 0; i < 8; ++i) {
        if (b & 1u)
            r ^= a;
        a = ((a << 1) ^ ((a & 0x80u) ? 0x1Du : 0u)) & 0xFFu;
        b >>= 1;
    }
    return r;
}
constexpr u32 gf_pow_c(u32 v, int e)
{
    return e == 0 ? 1u : gf_mul_c(v, gf_pow_c(v, e - 1));
}

/* DIRECT = false: Horner, acc = v*acc ^ x_j (a serial chain through acc);
 * true: acc ^= v^(K-1-j) * x_j, independent products (more ILP, dearer
 * constants). CW: dwords per plane per lane (2: 8 stripes per wave item,
 * 1: 4 stripes, two items per row). */
template <int K, int I, bool NTS, bool DIRECT, int CW>
__device__ __forceinline__ void encode_tile_row(const uint8_t *col, uint8_t *dst)
{
    constexpr u32 T = 8;
    constexpr u32 v = I + 1;
    u32 acc[8][CW], y[8][CW];
    if constexpr (DIRECT && v != 1) {
#pragma unroll
        for (int b = 0; b < 8; ++b)
#pragma unroll
            for (int w = 0; w < CW; ++w)
                acc[b][w] = 0;
        static_for<0, K>([&](auto J) {
            constexpr int j = decltype(J)::value;
            const uint8_t *src = col + (u32)j * (T * ECD_CHUNK);
#pragma unroll
            for (int b = 0; b < 8; ++b)
                load_plane<CW>(src + (u32)b * (T * 64u), y[b]);
            ecgf::mul_xor<gf_pow_c(v, K - 1 - j), CW, true>(acc, acc, y);
        });
    } else {
#pragma unroll
        for (int b = 0; b < 8; ++b)
            load_plane<CW>(col + (u32)b * (T * 64u), acc[b]);
#pragma unroll
        for (int j = 1; j < K; ++j) {
            const uint8_t *src = col + (u32)j * (T * ECD_CHUNK);
#pragma unroll
            for (int b = 0; b < 8; ++b)
                load_plane<CW>(src + (u32)b * (T * 64u), y[b]);
            if constexpr (v == 1) {
#pragma unroll
                for (int b = 0; b < 8; ++b)
#pragma unroll
                    for (int w = 0; w < CW; ++w)
                        acc[b][w] ^= y[b][w];
            } else {
                ecgf::horner<v, CW, true>(acc, y);
            }
        }
    }
    store_chunk<CW, NTS>(dst, acc);
}

template <int K, int N, int NW, bool NTS, bool DIRECT = false, int CW = 2>
__global__ __launch_bounds__(NW * 64) void ec_encode_tile(const uint8_t *__restrict__ in,
                                                          const FragPtrs out, uint64_t nstripes)
{
    constexpr u32 T = 8;
    constexpr uint64_t S = (uint64_t)K * ECD_CHUNK;
    constexpr u32 NI = K * T * 32 / 64;      /* LDS-DMA wave instructions per tile */
    constexpr u32 LPS = 16 / CW, SPI = 64 / LPS, IPR = T / SPI;
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const u32 tid = threadIdx.x;
    const uint64_t t0 = (uint64_t)blockIdx.x * T;
    const u32 wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const u32 lane = tid & 63u;

    /* stage: instruction ins = planes b, b+1 of input p for the 8 stripes */
#pragma unroll
    for (u32 j = 0; j < (NI + NW - 1) / NW; ++j) {
        const u32 ins = j * NW + wave;
        if (ins >= NI)
            break;
        const u32 p = ins / (T / 2);
        const u32 el = (ins * 64 + lane) % (T * 32);
        const u32 s = (el >> 2) % T;
        const uint64_t st = t0 + s;
        if (st < nstripes) {
            const uint8_t *g = in + st * S + p * ECD_CHUNK + ((el >> 2) / T) * 64u + (el & 3u) * 16u;
            __builtin_amdgcn_global_load_lds(
                (const __attribute__((address_space(1))) void *)g,
                (__attribute__((address_space(3))) void *)(lds + ins * 1024u), 16, 0, kLdsDmaDefault);
        }
    }
    __syncthreads();

    const u32 cs = lane / LPS, cc = lane % LPS;
    for (u32 it = wave; it < (u32)N * IPR; it += NW) {
        const u32 r = __builtin_amdgcn_readfirstlane(it / IPR);
        const u32 s = (it % IPR) * SPI + cs;
        const uint64_t ost = t0 + s;
        const uint8_t *col = lds + s * 64u + cc * (4u * CW);
        uint8_t *dst = out.p[r] + ost * ECD_CHUNK + cc * (4u * CW);
        if (ost < nstripes)
            static_for<0, N>([&](auto I) {
                if (r == (u32)decltype(I)::value)
                    encode_tile_row<K, decltype(I)::value, NTS, DIRECT, CW>(col, dst);
            });
    }
}

/* Narrow-tile encoder (r03): T = 4 or 8 stripes per block, one wave item
 * per fragment row (CW = T / 4 dwords per plane per lane, so an item covers
 * the tile's T stripes), NW waves per block.  At k = 16 the 8-stripe tile is
 * 64 KiB of LDS and only two blocks fit a CU, whose load / compute / store
 * phases then line up; T = 4 halves the tile so up to five blocks share a
 * CU.  WOT: each wave assembles its row's T chunks in a private LDS slice
 * and stores them as one contiguous T * 512-byte run (16 B per lane), not as
 * 64-B plane segments at a 512-B stride (PMC: 1.06-1.10x write bytes for
 * the segment stores of the 8+4 encoder). */
template <int K, int I, bool DIRECT, int CW, int T>
__device__ __forceinline__ void encode_tile_acc(const uint8_t *col, u32 (&acc)[8][CW])
{
    constexpr u32 v = I + 1;
    u32 y[8][CW];
    if constexpr (DIRECT && v != 1) {
#pragma unroll
        for (int b = 0; b < 8; ++b)
#pragma unroll
            for (int w = 0; w < CW; ++w)
                acc[b][w] = 0;
        static_for<0, K>([&](auto J) {
            constexpr int j = decltype(J)::value;
            const uint8_t *src = col + (u32)j * (T * ECD_CHUNK);
#pragma unroll
            for (int b = 0; b < 8; ++b)
                load_plane<CW>(src + (u32)b * (T * 64u), y[b]);
            ecgf::mul_xor<gf_pow_c(v, K - 1 - j), CW, true>(acc, acc, y);
        });
    } else {
        /* software-pipelined by hand: input j+1's planes are read while the
         * Horner step of input j runs, and no further (scheduling barriers):
         * left alone the scheduler issued all k x 8 reads of a row first,
         * 88-136 VGPRs, 3-5 waves per SIMD */
        u32 nx[8][CW];
#pragma unroll
        for (int b = 0; b < 8; ++b)
            load_plane<CW>(col + (u32)b * (T * 64u), acc[b]);
#pragma unroll
        for (int b = 0; b < 8; ++b)
            load_plane<CW>(col + (u32)(T * ECD_CHUNK) + (u32)b * (T * 64u), nx[b]);
#pragma unroll
        for (int j = 1; j < K; ++j) {
#pragma unroll
            for (int b = 0; b < 8; ++b)
#pragma unroll
                for (int w = 0; w < CW; ++w)
                    y[b][w] = nx[b][w];
            if (j + 1 < K) {
                const uint8_t *src = col + (u32)(j + 1) * (T * ECD_CHUNK);
#pragma unroll
                for (int b = 0; b < 8; ++b)
                    load_plane<CW>(src + (u32)b * (T * 64u), nx[b]);
            }
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (v == 1) {
#pragma unroll
                for (int b = 0; b < 8; ++b)
#pragma unroll
                    for (int w = 0; w < CW; ++w)
                        acc[b][w] ^= y[b][w];
            } else {
                ecgf::horner<v, CW, true>(acc, y);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
    }
}

/* Stage the tile's k input chunks (stripes t0 .. t0+T-1, any that exist) into
 * the plane-major LDS tile by LDS-DMA: input p, plane b, stripe s at
 * ((p * 8 + b) * T + s) * 64; a wave instruction fills 1 KiB. */
template <int T, int NW, int LA = kLdsDmaDefault, typename A>
__device__ __forceinline__ void stage_tile(uint8_t *lds, A chunk, u32 k, uint64_t t0,
                                           uint64_t nstripes, u32 wave, u32 lane)
{
    /* chunk(p, st): address of input p's chunk of stripe st, nullptr for
     * none (a padding slot); p is wave-uniform -- a computed address, not an
     * indexed pointer array, which would live in VGPRs or scratch */
    constexpr u32 PER = T / 2;                 /* wave instructions per input */
    const u32 ni = k * PER;
    for (u32 ins = wave; ins < ni; ins += NW) {
        const u32 p = ins / PER;
        const u32 el = (ins % PER) * 64 + lane;  /* 16-B piece within input p */
        const u32 seg = el >> 2;
        const uint64_t st = t0 + seg % T;
        const uint8_t *c = st < nstripes ? chunk(p, st) : nullptr;
        if (c) {
            const uint8_t *g = c + (seg / T) * 64u + (el & 3u) * 16u;
            __builtin_amdgcn_global_load_lds(
                (const __attribute__((address_space(1))) void *)g,
                (__attribute__((address_space(3))) void *)(lds + ins * 1024u), 16, 0, LA);
        }
    }
}

constexpr u32 kNoStripe = 0xFFFFFFFFu;        /* padding slot            */
constexpr uint64_t kNoSlot = ~0ull;            /* "no stripe here" in tiles */

/* wave-local LDS hand-off (the slice is private to the wave) */
__device__ __forceinline__ void wave_lds_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

/* Input of the tile encoders: stripe t of the data at in + t * S, at any
 * byte alignment (LDS-DMA honours any source address:
 * tools/kbench/ldsdma_align.hip, profiles/r03/ldsdma_align.log).  With
 * `edge` set this is the partial-stripe write of
 * ec_method_writev_encode_device: stripes 0 and nstripes - 1 (the boundary
 * stripes merged with the old head / tail content, gathered by
 * ec_rmw_gather) come from edge + 0 and edge + S, every interior stripe t
 * from the caller's buffer at in + t * S (in = user - head), so the interior
 * is never copied. */
struct EncSrc {
    const uint8_t *in;
    const uint8_t *edge;
};

/* The tile of this block.  XR = false: tile b.  XR = true (only the 16+4
 * encoder of >= 4 GiB calls is built this way, ec_kernels.hip
 * kXcdTilesBytes): blocks go round-robin to the 8 XCDs, so XCD x (blocks
 * b = x mod 8) walks its own contiguous eighth of the tiles.  A compile-time
 * choice: round 5 carried it as a run-time field of EncSrc, and the branch
 * and the wider kernel argument cost the partial-write encoder 8 % (VERDICT
 * r05). */
template <bool XR>
__device__ __forceinline__ uint64_t enc_tile()
{
    if constexpr (!XR) {
        return blockIdx.x;
    } else {
        const uint64_t g = gridDim.x, q = g / 8, r = g % 8, x = blockIdx.x % 8;
        return x * q + (x < r ? x : r) + blockIdx.x / 8;
    }
}

/* RA staging: the same plane-major tile as stage_tile, through registers --
 * piece i (16 B) = ((p * 8 + b) * T + s) * 4 + q is 16 bytes at
 * src(stripe) + (p * 8 + b) * 64 + q * 16, read as the dword-aligned dwords
 * that cover it (4, or 5 when the source is not dword-aligned: the fifth
 * holds the last wanted byte, so no load touches a page the range does not)
 * and funnel-shifted by v_alignbyte_b32, then one ds_write_b128.  (Round 3
 * measured LDS-DMA itself at every source alignment -- it honours any byte
 * address, tools/kbench/ldsdma_align.hip -- so the shipped kernels stage
 * misaligned inputs by LDS-DMA; SM = 2 is kept for the kb3 A/B.) */
template <int K, int T, int NW>
__device__ __forceinline__ void stage_tile_realign(uint8_t *lds, const EncSrc src, uint64_t t0,
                                                   uint64_t nstripes, u32 wave, u32 lane)
{
    constexpr u32 S = K * ECD_CHUNK;
    constexpr u32 NP = K * 8 * T * 4;                      /* 16-byte pieces */
    constexpr u32 IT = (NP + NW * 64 - 1) / (NW * 64);
    const u32 sh_in = (u32)(uintptr_t)src.in & 3u;         /* the interior's shift */
    u32 d[IT][4];
    bool ok[IT];
#pragma unroll
    for (u32 it = 0; it < IT; ++it) {
        const u32 i = it * (NW * 64) + wave * 64 + lane;
        const u32 q = i & 3u, sl = (i >> 2) % T, pb = (i >> 2) / T;
        const uint64_t st = t0 + sl;
        ok[it] = i < NP && st < nstripes;
        if (!ok[it])
            continue;
        const bool edge = src.edge && (st == 0 || st == nstripes - 1);
        const uint8_t *a = edge ? src.edge + (st == 0 ? 0u : S) : src.in + st * S;
        a += pb * 64u + q * 16u;
        const u32 sh = edge ? 0u : sh_in;
        const u32 *al = reinterpret_cast<const u32 *>(__builtin_assume_aligned(a - sh, 4));
        if (sh == 0) {
            const v4u v = *reinterpret_cast<const v4u *>(al);
            d[it][0] = v.x;
            d[it][1] = v.y;
            d[it][2] = v.z;
            d[it][3] = v.w;
        } else {
            u32 t[5];
            __builtin_memcpy(t, al, 20);
#pragma unroll
            for (int w = 0; w < 4; ++w)
                d[it][w] = __builtin_amdgcn_alignbyte(t[w + 1], t[w], sh);
        }
    }
#pragma unroll
    for (u32 it = 0; it < IT; ++it)
        if (ok[it])
            *reinterpret_cast<v4u *>(lds + (it * (NW * 64) + wave * 64 + lane) * 16u) =
                v4u{d[it][0], d[it][1], d[it][2], d[it][3]};
}

/* SM = 3 (r05): the same tile, staged through registers from dword-aligned
 * loads.  A 16-byte LDS-DMA load at a byte-misaligned address is not
 * coalesced: PMC of the 16+4 partial write (interior 777 bytes off) against
 * the aligned 16+4 encode, same instruction counts, per 1 GiB launch -- L1
 * (TCP) cache accesses 1.05e8 vs 3.78e7 (the reads alone 5x), UTCL1
 * requests 8.9e7 vs 3.8e7, TA busy 85 % vs 69 % of its cycles,
 * profiles/r05/pmc_rmw16/.  Here each lane loads one 16-byte piece of the
 * tile in memory order from the dword at or below it (dword-aligned: these
 * coalesce), takes the first dword of the next piece from the next lane
 * (which loaded it), funnel-shifts by v_alignbyte_b32 and writes the piece
 * to its plane-major slot.  A lane whose next piece is not the next 16
 * bytes of the same buffer (the wave's last lane, a stripe's last piece)
 * loads that dword itself; it holds the last wanted byte, so no load
 * touches a page the range does not.  Edge stripes (edge buffer) are
 * aligned and take no shift. */
template <int K, int T, int NW, int P0 = 0, bool NTL = false>
__device__ __forceinline__ void stage_tile_shift(uint8_t *lds, const EncSrc src, uint64_t t0,
                                                 uint64_t nstripes, u32 wave, u32 lane)
{
    constexpr u32 S = K * ECD_CHUNK;
    constexpr u32 PS = (K - P0) * 32u;                     /* pieces per stripe, inputs >= P0 */
    constexpr u32 NP = T * PS;                             /* 16-byte pieces */
    constexpr u32 IT = (NP + NW * 64 - 1) / (NW * 64);
    const u32 r_in = (u32)(uintptr_t)src.in & 3u;          /* the interior's shift */
    u32 d[IT][5], dst[IT], sh[IT];
    bool own[IT];
#pragma unroll
    for (u32 it = 0; it < IT; ++it) {
        const u32 m = it * (NW * 64) + wave * 64 + lane;   /* piece, memory order */
        const u32 s = m / PS, o = P0 * ECD_CHUNK + m % PS * 16u;
        const uint64_t st = t0 + s;
        dst[it] = ~0u;
        sh[it] = 0;
        /* the next 16 bytes are not the next lane's (DPP rows are 16 lanes) */
        own[it] = (lane & 15u) == 15u || o + 16u == S;
#pragma unroll
        for (int w = 0; w < 5; ++w)
            d[it][w] = 0;
        if (m < NP && st < nstripes) {
            const u32 p = o / ECD_CHUNK, b = o % ECD_CHUNK / 64u, q = o % 64u / 16u;
            dst[it] = ((p * 8 + b) * T + s) * 64u + q * 16u;
            const bool edge = src.edge && (st == 0 || st == nstripes - 1);
            const uint8_t *a = edge ? src.edge + (st == 0 ? 0u : S) + o : src.in + st * S + o;
            sh[it] = edge ? 0u : r_in;
            const u32 *al = reinterpret_cast<const u32 *>(__builtin_assume_aligned(a - sh[it], 4));
            v4u v;
            if constexpr (NTL)
                v = __builtin_nontemporal_load(reinterpret_cast<const v4u *>(al));
            else
                v = *reinterpret_cast<const v4u *>(al);
            d[it][0] = v.x;
            d[it][1] = v.y;
            d[it][2] = v.z;
            d[it][3] = v.w;
            if (sh[it] && own[it])
                d[it][4] = al[4];
        }
    }
#pragma unroll
    for (u32 it = 0; it < IT; ++it) {
        /* the next lane's first dword: DPP row_shl:1 (lane i reads lane i + 1
         * of its 16-lane row) */
        const u32 nx = (u32)__builtin_amdgcn_update_dpp(0, (int)d[it][0], 0x101, 0xF, 0xF, false);
        if (dst[it] != ~0u) {
            const u32 t4 = own[it] ? d[it][4] : nx;
            const v4u v = {__builtin_amdgcn_alignbyte(d[it][1], d[it][0], sh[it]),
                           __builtin_amdgcn_alignbyte(d[it][2], d[it][1], sh[it]),
                           __builtin_amdgcn_alignbyte(d[it][3], d[it][2], sh[it]),
                           __builtin_amdgcn_alignbyte(t4, d[it][3], sh[it])};
            *reinterpret_cast<v4u *>(lds + dst[it]) = v;
        }
    }
}

/* SM = 8 (r06, kb3 A/B only, measured slower): as SM = 3, but every
 * 16-byte load at the 16-byte boundary at or below the piece, so a
 * quarter-wave's 256 bytes never straddle a third 128-byte line; the piece
 * is funnel-shifted out of the lane's 4 dwords and the next lane's 4 (DPP
 * row_shl:1 each) by the interior's shift r = 4 dq + sb (uniform: one scalar
 * switch on dq).  Bit-exact, but 1 / 7 / 16 % slower than SM = 3 for 4+2 /
 * 8+4 / 16+4 at interior shifts 3, 7 and 13 (profiles/r06/r06zb_kb3_rmw.log):
 * the 8 staged dwords per piece and 4 DPPs cost more than the straddled
 * lines, which were not what held the partial writes back. */
template <int K, int T, int NW>
__device__ __forceinline__ void stage_tile_shift16(uint8_t *lds, const EncSrc src, uint64_t t0,
                                                   uint64_t nstripes, u32 wave, u32 lane)
{
    constexpr u32 S = K * ECD_CHUNK;
    constexpr u32 PS = K * 32u;                            /* pieces per stripe */
    constexpr u32 NP = T * PS;
    constexpr u32 IT = (NP + NW * 64 - 1) / (NW * 64);
    const u32 r16 = (u32)(uintptr_t)src.in & 15u;          /* the interior's shift */
    u32 d[IT][8], dst[IT];
    bool own[IT], edg[IT];
#pragma unroll
    for (u32 it = 0; it < IT; ++it) {
        const u32 m = it * (NW * 64) + wave * 64 + lane;   /* piece, memory order */
        const u32 s = m / PS, o = m % PS * 16u;
        const uint64_t st = t0 + s;
        dst[it] = ~0u;
        own[it] = (lane & 15u) == 15u || o + 16u == S;
        edg[it] = false;
#pragma unroll
        for (int w = 0; w < 8; ++w)
            d[it][w] = 0;
        if (m < NP && st < nstripes) {
            const u32 p = o / ECD_CHUNK, b = o % ECD_CHUNK / 64u, q = o % 64u / 16u;
            dst[it] = ((p * 8 + b) * T + s) * 64u + q * 16u;
            edg[it] = src.edge && (st == 0 || st == nstripes - 1);
            const uint8_t *a = edg[it] ? src.edge + (st == 0 ? 0u : S) + o : src.in + st * S + o;
            const u32 r = edg[it] ? 0u : r16;
            const v4u *al = reinterpret_cast<const v4u *>(__builtin_assume_aligned(a - r, 16));
            const v4u v = al[0];
            d[it][0] = v.x;
            d[it][1] = v.y;
            d[it][2] = v.z;
            d[it][3] = v.w;
            if (r && own[it]) {
                const v4u e = al[1];            /* holds the last wanted byte */
                d[it][4] = e.x;
                d[it][5] = e.y;
                d[it][6] = e.z;
                d[it][7] = e.w;
            }
        }
    }
    const u32 dq = r16 >> 2, sb = r16 & 3u;
#pragma unroll
    for (u32 it = 0; it < IT; ++it) {
        u32 f[8];
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            f[w] = d[it][w];
            const u32 nx = (u32)__builtin_amdgcn_update_dpp(0, (int)d[it][w], 0x101, 0xF, 0xF, false);
            f[w + 4] = own[it] ? d[it][w + 4] : nx;
        }
        if (dst[it] == ~0u)
            continue;
        v4u v;
        if (edg[it] || r16 == 0) {
            v = v4u{f[0], f[1], f[2], f[3]};
        } else {
            switch (dq) {              /* uniform */
            case 0:
                v = v4u{__builtin_amdgcn_alignbyte(f[1], f[0], sb), __builtin_amdgcn_alignbyte(f[2], f[1], sb),
                        __builtin_amdgcn_alignbyte(f[3], f[2], sb), __builtin_amdgcn_alignbyte(f[4], f[3], sb)};
                break;
            case 1:
                v = v4u{__builtin_amdgcn_alignbyte(f[2], f[1], sb), __builtin_amdgcn_alignbyte(f[3], f[2], sb),
                        __builtin_amdgcn_alignbyte(f[4], f[3], sb), __builtin_amdgcn_alignbyte(f[5], f[4], sb)};
                break;
            case 2:
                v = v4u{__builtin_amdgcn_alignbyte(f[3], f[2], sb), __builtin_amdgcn_alignbyte(f[4], f[3], sb),
                        __builtin_amdgcn_alignbyte(f[5], f[4], sb), __builtin_amdgcn_alignbyte(f[6], f[5], sb)};
                break;
            default:
                v = v4u{__builtin_amdgcn_alignbyte(f[4], f[3], sb), __builtin_amdgcn_alignbyte(f[5], f[4], sb),
                        __builtin_amdgcn_alignbyte(f[6], f[5], sb), __builtin_amdgcn_alignbyte(f[7], f[6], sb)};
                break;
            }
        }
        *reinterpret_cast<v4u *>(lds + dst[it]) = v;
    }
}

/* SM (staging mode): 0 = LDS-DMA from in; 1 = LDS-DMA, stripes 0 and
 * nstripes - 1 from edge (partial-stripe writes); 2 = through registers
 * (stage_tile_realign, r03 A/B: slower than LDS-DMA at every alignment);
 * 3 = dword-aligned loads through registers (stage_tile_shift, r05);
 * 8 = 16-byte-aligned loads through registers (stage_tile_shift16, r06;
 * kb3 A/B, slower) */
template <int K, int T, int NW, int SM, int LA = kLdsDmaDefault>
__device__ __forceinline__ void stage_encode_tile(uint8_t *lds, const EncSrc src, uint64_t t0,
                                                  uint64_t nstripes, u32 wave, u32 lane)
{
    constexpr uint64_t S = (uint64_t)K * ECD_CHUNK;
    if constexpr (SM == 2) {
        stage_tile_realign<K, T, NW>(lds, src, t0, nstripes, wave, lane);
    } else if constexpr (SM == 3) {
        stage_tile_shift<K, T, NW>(lds, src, t0, nstripes, wave, lane);
    } else if constexpr (SM == 8) {
        stage_tile_shift16<K, T, NW>(lds, src, t0, nstripes, wave, lane);
    } else if constexpr (SM == 7) {
        /* kb3 A/B: shift staging with non-temporal loads */
        stage_tile_shift<K, T, NW, 0, true>(lds, src, t0, nstripes, wave, lane);
    } else if constexpr (SM >= 4 && SM <= 6) {
        /* split (kb3 A/B): inputs below KD by LDS-DMA at the caller's
         * alignment (TA-bound), the rest shifted through registers (LDS
         * write-bound): the k = 16 encoder is short of LDS cycles */
        constexpr int KD = SM == 4 ? K / 2 : SM == 5 ? 3 * K / 4 : K / 4;
        stage_tile<T, NW, LA>(lds, [&](u32 p, uint64_t st) {
            const uint8_t *b = st == 0 ? src.edge : st == nstripes - 1 ? src.edge + S
                                                                       : src.in + st * S;
            return b + p * ECD_CHUNK;
        }, KD, t0, nstripes, wave, lane);
        stage_tile_shift<K, T, NW, KD>(lds, src, t0, nstripes, wave, lane);
    } else if constexpr (SM == 1) {
        stage_tile<T, NW, LA>(lds, [&](u32 p, uint64_t st) {
            const uint8_t *b = st == 0 ? src.edge : st == nstripes - 1 ? src.edge + S
                                                                       : src.in + st * S;
            return b + p * ECD_CHUNK;
        }, K, t0, nstripes, wave, lane);
    } else {
        stage_tile<T, NW, LA>(lds, [&](u32 p, uint64_t st) {
            return src.in + st * S + p * ECD_CHUNK;
        }, K, t0, nstripes, wave, lane);
    }
}

/* Write the wave's T chunks (lane (cs, cc) holds column cc of stripe cs, CW
 * dwords per plane) through its LDS slice as contiguous 16-B lane pieces:
 * chunk s goes to dst(s) + [0, 512).  dst(s) = nullptr: no stripe. */
/* H passes: the slice holds T / H chunks (H = 2 halves the LDS a wave
 * needs, for the k = 16 tiles where LDS decides how many blocks fit). */
template <int T, int CW, bool NTS, int H = 1, typename D>
__device__ __forceinline__ void store_chunks_via_lds(uint8_t *slice, const u32 (&acc)[8][CW],
                                                     u32 cs, u32 cc, u32 lane, D dst)
{
    constexpr u32 SP = T / H;                  /* chunks per pass */
#pragma unroll
    for (u32 h = 0; h < (u32)H; ++h) {
        if (H == 1 || cs / SP == h) {
            uint8_t *o = slice + (cs % SP) * ECD_CHUNK + cc * (4u * CW);
#pragma unroll
            for (int b = 0; b < 8; ++b) {
                if constexpr (CW == 1)
                    *reinterpret_cast<u32 *>(o + b * 64) = acc[b][0];
                else
                    *reinterpret_cast<uint2 *>(o + b * 64) = make_uint2(acc[b][0], acc[b][1]);
            }
        }
        wave_lds_sync();
#pragma unroll
        for (u32 j = 0; j < SP * ECD_CHUNK / 1024; ++j) {
            const u32 off = (j * 64 + lane) * 16;
            uint8_t *d = dst(h * SP + off / ECD_CHUNK);
            if (d) {
                const v4u v = *reinterpret_cast<const v4u *>(slice + off);
                if constexpr (NTS)
                    __builtin_nontemporal_store(v, reinterpret_cast<v4u *>(d + off % ECD_CHUNK));
                else
                    *reinterpret_cast<v4u *>(d + off % ECD_CHUNK) = v;
            }
        }
        wave_lds_sync();
    }
}

/* One fragment row of the narrow tile. */
template <int K, int I, int T, bool NTS, bool DIRECT, bool WOT>
__device__ __forceinline__ void encode_tile_item(const uint8_t *col, uint8_t *slice,
                                                           uint8_t *row, uint64_t t0,
                                                           uint64_t nstripes, u32 cs, u32 cc,
                                                           u32 lane)
{
    constexpr int CW = T / 4;
    u32 acc[8][CW];
    encode_tile_acc<K, I, DIRECT, CW, T>(col, acc);
    if constexpr (WOT) {
        store_chunks_via_lds<T, CW, NTS>(slice, acc, cs, cc, lane, [&](u32 s) {
            return t0 + s < nstripes ? row + (t0 + s) * ECD_CHUNK : nullptr;
        });
    } else if (t0 + cs < nstripes) {
        store_chunk<CW, NTS>(row + (t0 + cs) * ECD_CHUNK + cc * (4u * CW), acc);
    }
}

template <int K, int N, int T, int NW, bool NTS, bool DIRECT, bool WOT, int SM = 0,
          int LA = kLdsDmaDefault, bool XR = false>
__global__ __launch_bounds__(NW * 64) void ec_encode_tile_t(const EncSrc src, const FragPtrs out,
                                                            uint64_t nstripes)
{
    static_assert(T == 4 || T == 8, "4- or 8-stripe tiles");
    constexpr int CW = T / 4;
    constexpr u32 LPS = 16 / CW;               /* lanes per stripe */
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const u32 tid = threadIdx.x;
    const uint64_t t0 = enc_tile<XR>() * T;
    const u32 wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const u32 lane = tid & 63u;
    stage_encode_tile<K, T, NW, SM, LA>(lds, src, t0, nstripes, wave, lane);
    __syncthreads();
    const u32 cs = lane / LPS, cc = lane % LPS;
    const uint8_t *col = lds + cs * 64u + cc * (4u * CW);
    uint8_t *slice = lds + K * T * ECD_CHUNK + wave * T * ECD_CHUNK;
    for (u32 r = wave; r < (u32)N; r += NW) {
        const u32 ru = __builtin_amdgcn_readfirstlane(r);
        /* the row's fragment base by a run-time index (scalar load): with
         * out.p[I] per branch, the compiler hoisted all N per-lane store
         * addresses out of the loop, 2 VGPRs each (173 VGPRs at 16+4) */
        uint8_t *row = out.p[ru];
        static_for<0, N>([&](auto I) {
            if (ru == (u32)decltype(I)::value)
                encode_tile_item<K, decltype(I)::value, T, NTS, DIRECT, WOT>(
                    col, slice, row, t0, nstripes, cs, cc, lane);
        });
    }
}

template <int T, int NW, bool WOT>
constexpr size_t encode_tile_t_lds(int k)
{
    return (size_t)k * T * ECD_CHUNK + (WOT ? (size_t)NW * T * ECD_CHUNK : 0);
}

/* Row-group encoder (r03, for 16+4): one wave item = RB consecutive rows
 * (v = I0 + 1 .. I0 + RB) for 4 stripes, one dword per plane per lane.  The
 * item walks the k inputs once and every input plane read from LDS feeds RB
 * Horner chains, so the tile is read N / RB times instead of N times (the
 * one-row items of ec_encode_tile read it 20 times at 16+4, PMC: LDS array
 * ~81 % busy).  Input j + 1 is read while the RB steps of input j run, and
 * no further (scheduling barriers), which keeps the item at ~8 * (RB + 3)
 * VGPRs. */
template <int K, int I0, int RB, int T>
__device__ __forceinline__ void encode_group_acc(const uint8_t *col, u32 (&acc)[RB][8][1])
{
    u32 y[8][1], nx[8][1];
#pragma unroll
    for (int b = 0; b < 8; ++b)
        y[b][0] = *reinterpret_cast<const u32 *>(col + (u32)b * (T * 64u));
#pragma unroll
    for (int q = 0; q < RB; ++q)
#pragma unroll
        for (int b = 0; b < 8; ++b)
            acc[q][b][0] = y[b][0];
#pragma unroll
    for (int b = 0; b < 8; ++b)
        nx[b][0] = *reinterpret_cast<const u32 *>(col + (u32)(T * ECD_CHUNK) + (u32)b * (T * 64u));
#pragma unroll
    for (int j = 1; j < K; ++j) {
#pragma unroll
        for (int b = 0; b < 8; ++b)
            y[b][0] = nx[b][0];
        if (j + 1 < K) {
            const uint8_t *src = col + (u32)(j + 1) * (T * ECD_CHUNK);
#pragma unroll
            for (int b = 0; b < 8; ++b)
                nx[b][0] = *reinterpret_cast<const u32 *>(src + (u32)b * (T * 64u));
        }
        __builtin_amdgcn_sched_barrier(0);
        static_for<0, RB>([&](auto Q) {
            constexpr int q = decltype(Q)::value;
            constexpr u32 v = I0 + q + 1;
            if constexpr (v == 1) {
#pragma unroll
                for (int b = 0; b < 8; ++b)
                    acc[q][b][0] ^= y[b][0];
            } else {
                ecgf::horner<v, 1, true>(acc[q], y);
            }
        });
        __builtin_amdgcn_sched_barrier(0);
    }
}

/* T = 4 or 8 stripes per tile (SUB = T / 4 four-stripe sub-tiles), N / RB
 * row groups, one item per wave: NW = (N / RB) * SUB.  WOT: each row leaves
 * through the wave's 2 KiB LDS slice as one contiguous 2 KiB run. */
template <int K, int N, int T, int RB, bool NTS, bool WOT, int SM = 0, int LA = kLdsDmaDefault,
          bool XR = false>
__global__ __launch_bounds__((N / RB) * (T / 4) * 64) void ec_encode_tile_rb(
    const EncSrc src, const FragPtrs out, uint64_t nstripes)
{
    static_assert(N % RB == 0 && (T == 4 || T == 8), "RB | N, 4- or 8-stripe tiles");
    constexpr u32 SUB = T / 4, NW = (N / RB) * SUB;
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const u32 tid = threadIdx.x;
    const uint64_t t0 = enc_tile<XR>() * T;
    const u32 wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const u32 lane = tid & 63u;
    stage_encode_tile<K, T, NW, SM, LA>(lds, src, t0, nstripes, wave, lane);
    __syncthreads();
    const u32 g = wave / SUB, sub = wave % SUB;
    const u32 cs = lane >> 4, cc = lane & 15u;
    const uint64_t s0 = t0 + sub * 4u;          /* first stripe of the sub-tile */
    const uint8_t *col = lds + (sub * 4u + cs) * 64u + cc * 4u;
    uint8_t *slice = lds + K * T * ECD_CHUNK + wave * 4u * ECD_CHUNK;
    static_for<0, N / RB>([&](auto G) {
        constexpr int I0 = decltype(G)::value * RB;
        if (g == (u32)decltype(G)::value) {
            u32 acc[RB][8][1];
            encode_group_acc<K, I0, RB, T>(col, acc);
            static_for<0, RB>([&](auto Q) {
                constexpr int q = decltype(Q)::value;
                /* the row base by a run-time index: see ec_encode_tile_t */
                uint8_t *row = out.p[__builtin_amdgcn_readfirstlane(g * RB + q)];
                if constexpr (WOT) {
                    store_chunks_via_lds<4, 1, NTS>(slice, acc[q], cs, cc, lane, [&](u32 s) {
                        return s0 + s < nstripes ? row + (s0 + s) * ECD_CHUNK : nullptr;
                    });
                } else if (s0 + cs < nstripes) {
                    store_chunk<1, NTS>(row + (s0 + cs) * ECD_CHUNK + cc * 4u, acc[q]);
                }
            });
        }
    });
}

template <int N, int T, int RB, bool WOT>
constexpr size_t encode_tile_rb_lds(int k)
{
    return (size_t)k * T * ECD_CHUNK + (WOT ? (size_t)(N / RB) * (T / 4) * 4 * ECD_CHUNK : 0);
}

template <int W>
inline uint64_t vander_grid(uint64_t nstripes)
{
    return (nstripes * (16 / W) + kBlock - 1) / kBlock;
}

/* Zero-copy variant for buffers in pinned host memory, read and written by
 * the CUs over PCIe.  In ec_encode_vander every resident wave loads, then
 * stores, so a grid that fits the chip at once (any call below ~64 MiB)
 * uses the link in one direction at a time: a 4 MiB 4+2 call took 189 us =
 * 4 MiB in at ~56 GB/s, then 6 MiB out at ~55 GB/s (profiles/smallcalls_r01).
 * Here a smaller grid strides over the stripes and each thread prefetches
 * its next stripe before it computes and stores the current one, so the
 * reads of one stripe overlap the writes of the previous one and the link
 * runs both directions at once (~45 GB/s each way, tools/kbench/zerocopy).
 * The SW = 64/L consecutive stripes of a wave form one contiguous run of
 * SW*512 bytes in every fragment; each output row is assembled in the
 * wave's LDS slice and written back as 16-byte lanes, i.e. 1 KiB requests
 * instead of 64-byte plane segments (the request shape is what the link
 * charges for, see ec_combine_zc).  Loops and exits are wave-uniform so
 * every lane of a run takes part in its write-back. */
template <int K, int N, int W, int BS = kBlock>
__global__ __launch_bounds__(BS) void ec_encode_vander_zc(const uint8_t *__restrict__ in,
                                                          const FragPtrs out, uint64_t nstripes)
{
    constexpr int L = 16 / W;             /* lanes per stripe        */
    constexpr u32 SW = 64 / L;            /* stripes per wave        */
    constexpr u32 RUN = SW * ECD_CHUNK;   /* bytes per fragment run  */
    __shared__ __attribute__((aligned(16))) uint8_t lds[BS / 64][RUN];
    const u32 lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    const uint64_t gtid = (uint64_t)blockIdx.x * BS + threadIdx.x;
    const uint64_t step = (uint64_t)gridDim.x * (BS / L);
    const u32 colb = (u32)(gtid % L) * (4 * W);
    const u32 sl = lane / L;
    uint64_t stripe = gtid / L;
    uint64_t wfirst = stripe - sl;        /* wave-uniform */
    if (wfirst >= nstripes)
        return;
    uint8_t *slice = lds[wv];

    u32 x[K][8][W];
    auto load = [&](uint64_t st, u32 (&d)[K][8][W]) {
        if (st < nstripes) {
            const uint8_t *sp = in + st * (uint64_t)(K * ECD_CHUNK) + colb;
#pragma unroll
            for (int j = 0; j < K; ++j)
                load_chunk<W>(sp + j * ECD_CHUNK, d[j]);
        }
    };
    load(stripe, x);
    for (;;) {
        const uint64_t nxt = stripe + step, wnext = wfirst + step;
        u32 y[K][8][W];
        if (wnext < nstripes)
            load(nxt, y);
        static_for<0, N>([&](auto I) {
            u32 acc[8][W];
            encode_row_acc<K, W, decltype(I)::value>(x, acc);
            store_chunk<W, false>(slice + sl * ECD_CHUNK + colb, acc);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            uint8_t *dst = out.p[decltype(I)::value] + wfirst * ECD_CHUNK;
#pragma unroll
            for (u32 j = 0; j < RUN / 1024; ++j) {
                const u32 off = (j * 64 + lane) * 16;
                if (wfirst + off / ECD_CHUNK < nstripes)
                    *reinterpret_cast<uint4 *>(dst + off) =
                        *reinterpret_cast<const uint4 *>(slice + off);
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        });
        if (wnext >= nstripes)
            break;
        stripe = nxt;
        wfirst = wnext;
#pragma unroll
        for (int j = 0; j < K; ++j)
#pragma unroll
            for (int b = 0; b < 8; ++b)
#pragma unroll
                for (int w = 0; w < W; ++w)
                    x[j][b][w] = y[j][b][w];
    }
}

/* Zero-copy grid (tools/kbench/zcenc, profiles/zcenc_r01.log): 32 blocks
 * keep far more bytes in flight than the link's bandwidth-delay product;
 * 16 MiB / 64 MiB 4+2 calls ran 619 / 2206 us against 730 / 2446 us one-pass
 * (+11-18 %).  At <= 4 MiB the prefetch cannot desynchronise enough waves
 * and the one-pass kernel is as fast or faster, so it is used there. */
constexpr uint64_t kZcBlocks = 32;

template <int W>
inline bool vander_use_zc(uint64_t nstripes)
{
    return nstripes * (16 / W) > 4 * kZcBlocks * kBlock;
}

/* ------------------------------------------------- generic combination */

constexpr int kPatWords = 512; /* kernel-argument pattern space (2 KiB) */

/* Kernel arguments: ecd_combine_desc_t with the patterns re-laid out in
 * 32-bit words (src[] then one word-aligned row per output, ceil(k/4) words
 * each) so every coefficient is fetched by a scalar s_load_dword -- a byte
 * load from the argument segment would be a vector load followed by a
 * vmcnt(0) wait that also drains all outstanding stores. */
struct CombineArgs {
    const uint8_t *in_base[ECD_MAX_ROWS];
    uint8_t *out_base[ECD_MAX_ROWS];
    uint64_t in_stride, out_stride, nstripes;
    const uint8_t *group_pattern;
    const u32 *patg;        /* pattern table in device memory (PG kernels) */
    /* sorted slots (SLOTS kernels): slot i holds stripe slot_stripe[i] or
     * kNoStripe; every 8-slot tile is one pattern's; *slot_count slots */
    const u32 *slot_stripe, *slot_count;
    u32 k, kw, rows, group_shift, pwords, npatterns;
    u32 pat[kPatWords];
};

constexpr u32 kMaxPatWords = 128; /* one pattern: kw * (1 + rows) <= 4 * 32 */

/* A wave-uniform dword of read-only global memory by a scalar load (constant
 * address space: s_load_dword through the scalar cache).  As a vector load
 * it was global_load + s_waitcnt vmcnt(0) at the head of every block, before
 * its first staging load could issue (the group map byte of a mixed call and
 * the src[] words of a PG pattern: a full memory round trip, serialised,
 * per 4-stripe tile; r04). */
__device__ __forceinline__ u32 scalar_load_u32(const void *p)
{
    const uintptr_t a = (uintptr_t)p;
    return *reinterpret_cast<const __attribute__((address_space(4))) u32 *>(a);
}

/* The words of the block's pattern (src[] then one row of coefficients per
 * output).  PG = false: the kernel-argument segment, read by scalar loads.
 * PG = true (mixed calls with more patterns than the 2 KiB argument space
 * holds, e.g. > 7 erasure masks of a 16+4 volume): the pattern table in
 * device memory -- the per-call cache of decode matrices -- read the same
 * way, by scalar loads through the scalar cache: the src[] words once per
 * block (the staging addresses need them first), a row's coefficient words
 * when the row starts.
 * (r04-r06 loaded the whole pattern by vector loads and parked it in LDS
 * after the tile, a coefficient word then one broadcast ds_read: the k = 16
 * kernel's tile grew past 64 KiB and every wave issued the pattern loads
 * beside its staging, 3 % slower than the same patterns from the argument
 * segment, profiles/r06/r06r_kb3_mixed.log.  A vector load per coefficient
 * would need a vmcnt(0) wait that also drains the outstanding stores, and
 * the words in VGPRs cost the k = 16 kernel its second block per CU.) */
template <bool PG>
struct PatWords {
    u32 pb;
    u32 s0, s1, s2, s3;          /* PG: the src[] words */
    const u32 *t;                /* PG: the pattern in the device table */
    __device__ __forceinline__ PatWords(const CombineArgs &a, u32 pat)
    {
        pb = pat * a.pwords;
        if constexpr (PG) {
            t = a.patg + pb;
            /* the src[] words by one scalar load (pwords >= 2 kw, so 4 words
             * stay in the pattern when kw >= 2, 2 when kw = 1) */
            if (a.kw >= 2) {
                const v4u q = *reinterpret_cast<const __attribute__((address_space(4))) v4u *>(
                    (uintptr_t)t);
                s0 = q.x;
                s1 = q.y;
                s2 = a.kw > 2 ? q.z : 0u;
                s3 = a.kw > 3 ? q.w : 0u;
            } else {
                const v2u q = *reinterpret_cast<const __attribute__((address_space(4))) v2u *>(
                    (uintptr_t)t);
                s0 = q.x;
                s1 = s2 = s3 = 0u;
            }
        }
    }
    /* (the argument struct is passed in, not held: holding a reference to
     * the kernel argument made the compiler copy all 2.6 KiB to scratch) */
    __device__ __forceinline__ u32 word(const CombineArgs &a, u32 rel) const
    {
        if constexpr (PG)
            return scalar_load_u32(t + rel);
        else
            return a.pat[pb + rel];
    }
    __device__ __forceinline__ u32 byte(const CombineArgs &a, u32 idx) const
    {
        u32 w;
        if constexpr (PG) {
            /* branch-free pick (a select chain over the members became a
             * load through a selected address, i.e. a scratch alloca) */
            const u32 q = idx >> 2;
            w = (s0 & (0u - (u32)(q == 0))) | (s1 & (0u - (u32)(q == 1))) |
                (s2 & (0u - (u32)(q == 2))) | (s3 & (0u - (u32)(q == 3)));
        } else {
            w = a.pat[pb + (idx >> 2)];
        }
        return __builtin_amdgcn_readfirstlane((w >> ((idx & 3u) * 8u)) & 0xFFu);
    }
};


/* pattern id of the tile starting at stripe t0 (ids past the table clamp to
 * the last pattern: a bad caller map must not fault the device) */
template <bool MIXED>
__device__ __forceinline__ u32 tile_pattern(const CombineArgs &a, uint64_t t0)
{
    if constexpr (!MIXED)
        return 0u;
    /* the aligned dword holding the byte, by a scalar load (an aligned dword
     * never crosses a page, so it is mapped wherever the byte is) */
    const uintptr_t ba = (uintptr_t)(a.group_pattern + (t0 >> a.group_shift));
    const u32 w = scalar_load_u32(reinterpret_cast<const void *>(ba & ~(uintptr_t)3));
    const u32 id = (w >> ((u32)(ba & 3u) * 8u)) & 0xFFu;
    return id < a.npatterns ? id : a.npatterns - 1u;
}

/* Stripe of tile slot `slot`: the slot itself, or (SLOTS) the sorted list's
 * entry -- kNoSlot past the data or in a run's padding. */
template <bool SLOTS>
__device__ __forceinline__ uint64_t slot_stripe(const CombineArgs &a, uint64_t slot,
                                                u32 nslots)
{
    if constexpr (!SLOTS) {
        (void)nslots;
        return slot < a.nstripes ? slot : kNoSlot;
    } else {
        if (slot >= nslots)
            return kNoSlot;
        const u32 v = a.slot_stripe[slot];
        return v == kNoStripe ? kNoSlot : (uint64_t)v;
    }
}

/* The 8 planes of one input of an 8-stripe tile (CW = 2: 8 bytes per plane
 * per lane, planes 512 B apart) as 8 single ds_read_b64 -- 2 LDS cycles
 * each, where the ds_read2st64_b64 pairs the compiler forms cost 8 (MI355X
 * LDS table): the k = 16 combine's compute phase is LDS-read bound (r03
 * probe, profiles/r03/kb3_r03u_probe16.log: compute alone 0.274 -> 0.204 ms
 * per GiB).  Inline asm, so the compiler neither pairs them nor puts a
 * vmcnt(0) for pending LDS-DMA in front (the tile is complete: barrier). */
__device__ __forceinline__ void lds_read_planes_b64(const uint8_t *src, u32 (&y)[8][2])
{
    const u32 ad = (u32)(uintptr_t)src;
    v2u q[8];
    asm volatile("ds_read_b64 %0, %8\n\t"
                 "ds_read_b64 %1, %8 offset:512\n\t"
                 "ds_read_b64 %2, %8 offset:1024\n\t"
                 "ds_read_b64 %3, %8 offset:1536\n\t"
                 "ds_read_b64 %4, %8 offset:2048\n\t"
                 "ds_read_b64 %5, %8 offset:2560\n\t"
                 "ds_read_b64 %6, %8 offset:3072\n\t"
                 "ds_read_b64 %7, %8 offset:3584\n\t"
                 "s_waitcnt lgkmcnt(0)"
                 : "=&v"(q[0]), "=&v"(q[1]), "=&v"(q[2]), "=&v"(q[3]), "=&v"(q[4]), "=&v"(q[5]),
                   "=&v"(q[6]), "=&v"(q[7])
                 : "v"(ad)
                 : "memory");
#pragma unroll
    for (int b = 0; b < 8; ++b) {
        y[b][0] = q[b].x;
        y[b][1] = q[b].y;
    }
}

/* Store one chunk held as CW = 2 (lane cc holds bytes [8cc, 8cc + 8) of every
 * plane): lane pairs (cc, cc ^ 1) swap halves by DPP so the even lane holds
 * 16 contiguous bytes of plane b and the odd lane of plane b + 1, and the
 * chunk leaves in four 16-byte stores per lane instead of eight 8-byte ones
 * (the store issue of the k = 16 combine: r03 probe, with the reads above
 * 0.399 -> 0.378 ms per GiB).  Every lane runs the exchange; `ok` (the same
 * for both lanes of a pair: one stripe) predicates the stores only. */
template <bool NT>
__device__ __forceinline__ void store_chunk_pairs(uint8_t *chunk, u32 cc, const u32 (&acc)[8][2],
                                                  bool ok)
{
    const bool odd = cc & 1u;
    uint8_t *o = chunk + (cc & ~1u) * 8u + (odd ? 64u : 0u);
#pragma unroll
    for (int b = 0; b < 8; b += 2) {
        const u32 s0 = odd ? acc[b][0] : acc[b + 1][0];
        const u32 s1 = odd ? acc[b][1] : acc[b + 1][1];
        const u32 r0 = __builtin_amdgcn_mov_dpp(s0, 0xB1, 0xF, 0xF, false); /* quad_perm 1,0,3,2 */
        const u32 r1 = __builtin_amdgcn_mov_dpp(s1, 0xB1, 0xF, 0xF, false);
        const v4u v = odd ? v4u{r0, r1, acc[b + 1][0], acc[b + 1][1]}
                          : v4u{acc[b][0], acc[b][1], r0, r1};
        if (ok) {
            if constexpr (NT)
                __builtin_nontemporal_store(v, reinterpret_cast<v4u *>(o + b * 64));
            else
                *reinterpret_cast<v4u *>(o + b * 64) = v;
        }
    }
}

/* K: max inputs (k <= K); TS: tile = 8*TS stripes; NW: waves per block.
 *
 * LDS tile, plane-major: input p, plane b, tile stripe s, 64-byte segment at
 * ((p * 8 + b) * T + s) * 64.  The half wave that reads plane b of 4 stripes
 * with ds_read_b64 then touches 256 consecutive bytes (conflict-free), and
 * one lane address serves all 8 planes of an input (ds_read2st64_b64 with
 * immediate plane offsets) -- the earlier chunk-major tile needed an
 * XOR-rotated plane slot, hence 5 address VALUs per input. */
/* JT: 0 = the compiler's switch, 1 = the jump table of ec_gf8_asm.h.
 * (Retired, with their A/B logs in DESIGN.md 3.4: the whole-row asm block
 * and grouped staging waits (r02z, commit 87d127c), the software-pipelined
 * loop over <= 4-temporary programs (JT = 4) and the output tiles (OT) for
 * fragment outputs and k >= 8 (r02, commit 1c377cb); the narrow kernels
 * below took over every k <= 8 call in r03.)
 * SLOTS: mixed patterns with groups below a tile (1, 2, 4 stripes): the
 * stripes were sorted by pattern into 8-slot tiles (ec_slots_* kernels), and
 * the block reads its tile's stripes from the slot list. */
template <int K, int TS, int NW, bool MIXED, bool NTS, int CW = 2, bool PG = false,
          bool CSE = true, int JT = 0, bool SLOTS = false, int PU = 1, int LA = kLdsDmaDefault>
__global__ __launch_bounds__(NW * 64) void ec_combine(const CombineArgs a)
{
    constexpr u32 T = 8 * TS;            /* stripes per tile                   */
    /* CW: dwords per plane per lane in the compute phase; a wave item covers
     * SPI = 4*CW stripes of one output row */
    constexpr u32 LPS = 16 / CW, SPI = 64 / LPS, IPT = T / SPI;
    constexpr u32 NI = K * T * 32 / 64;  /* LDS-DMA wave instructions per tile */
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const u32 tid = threadIdx.x;
    const u32 k = a.k;
    const uint64_t t0 = (uint64_t)blockIdx.x * T;
    const u32 wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const u32 lane = tid & 63u;
    u32 nslots = 0;
    if constexpr (SLOTS) {
        nslots = scalar_load_u32(a.slot_count);
        if (t0 >= nslots)
            return;             /* the grid is sized for the worst padding */
    }
    /* a sorted tile is one pattern's: take it from the tile's first stripe
     * (never padding: runs are padded at their end, to 8 slots) */
    const uint64_t tp = SLOTS ? slot_stripe<SLOTS>(a, t0, nslots) : t0;
    const PatWords<PG> pw(a, tile_pattern<MIXED>(a, tp));

    /* stage: every wave instruction (global_load_lds_dwordx4) fills 1 KiB of
     * LDS linearly = planes b, b+1 of input p for the tile's 8 stripes (T=8)
     * or plane b for 16 (T=16); lane i fetches 16-byte piece i, so the tile
     * layout above is produced by the per-lane source address alone */
#pragma unroll
    for (u32 j = 0; j < (NI + NW - 1) / NW; ++j) {
        const u32 ins = j * NW + wave;           /* wave-uniform */
        if (ins >= NI)
            break;
        const u32 p = ins / (T / 2);
        if (p >= k)
            break;
        const u32 el = (ins * 64 + lane) % (T * 32); /* piece within input p */
        const u32 s = (el >> 2) % T;
        const uint64_t st = slot_stripe<SLOTS>(a, t0 + s, nslots);
        if (st != kNoSlot) {
            const u32 src = pw.byte(a, p);
            const uint8_t *g = a.in_base[src] + st * a.in_stride + ((el >> 2) / T) * 64u +
                               (el & 3u) * 16u;
            __builtin_amdgcn_global_load_lds(
                (const __attribute__((address_space(1))) void *)g,
                (__attribute__((address_space(3))) void *)(lds + ins * 1024u), 16, 0, LA);
        }
    }
    __syncthreads();

    /* compute: (row, 8-stripe subtile) items spread over the NW waves */
    const u32 cs = lane / LPS, cc = lane % LPS;
    const u32 items = a.rows * IPT;
    for (u32 it = wave; it < items; it += NW) {
        const u32 r = it / IPT, s = (it % IPT) * SPI + cs;
        const uint8_t *col = lds + s * 64u + cc * (4u * CW);
        /* the row's coefficients: up to 4 words, loaded once into SGPRs */
        const u32 rw = a.kw * (1 + r);
        const u32 w0 = pw.word(a, rw);
        const u32 w1 = K > 4 ? pw.word(a, rw + 1) : 0u;
        const u32 w2 = K > 8 ? pw.word(a, rw + 2) : 0u;
        const u32 w3 = K > 12 ? pw.word(a, rw + 3) : 0u;
        u32 acc[8][CW], y[8][CW];
#pragma unroll
        for (int b = 0; b < 8; ++b)
#pragma unroll
            for (int w = 0; w < CW; ++w)
                acc[b][w] = 0;
        /* the row's coefficients as a 128-bit scalar shift register: one
         * byte per input, 4 SALU per step instead of a select chain */
        uint64_t cl = (uint64_t)w0 | ((uint64_t)w1 << 32);
        uint64_t ch = (uint64_t)w2 | ((uint64_t)w3 << 32);
        /* PU = 1: not unrolled, as every copy of the body is a copy of the
         * 255 multiply programs (~54 KiB of code) */
#pragma unroll PU
        for (u32 p = 0; p < k; ++p) {
            const u32 c = __builtin_amdgcn_readfirstlane((u32)cl & 0xFFu);
            cl = (cl >> 8) | (ch << 56);
            ch >>= 8;
            if (c == 0)                  /* ec-code-c.c:11666-11676 */
                continue;
            const uint8_t *src = col + p * (T * ECD_CHUNK);
            if constexpr (CW == 2 && T == 8) {
                lds_read_planes_b64(src, y);
            } else {
#pragma unroll
                for (int b = 0; b < 8; ++b)
                    load_plane<CW>(src + (u32)b * (T * 64u), y[b]);
            }
            if constexpr (JT && CW == 2)
                ecgf::mul_xor_jt<CW>(c, acc, y);
            else
                ecgf::mul_xor_rt<CW, CSE>(c, acc, y);
        }
        const uint64_t ost = slot_stripe<SLOTS>(a, t0 + s, nslots);
        if constexpr (CW == 2) {
            store_chunk_pairs<NTS>(a.out_base[r] + (ost != kNoSlot ? ost : 0) * a.out_stride, cc, acc,
                                   ost != kNoSlot);
        } else if (ost != kNoSlot) {
            store_chunk<CW, NTS>(a.out_base[r] + ost * a.out_stride + cc * (4u * CW), acc);
        }
    }
}

/* Narrow-tile combine (r03): ec_combine's decode / heal / mixed kernel with
 * T = 4 stripes per block and one dword per plane per lane (16 lanes per
 * stripe), so a k = 16 tile is 32 KiB and four 8-wave blocks share a CU.
 * Each wave item is one output row for the 4 stripes; the multiply jumps
 * into the one-dword bodies of ec_gf8_asm.h.  WOT as in ec_encode_tile_t:
 * the row's 4 chunks leave through the wave's LDS slice in 512-B runs (WOT
 * = 2: a half slice, two passes).  PG and SLOTS as in ec_combine (device
 * pattern table; sorted slots, whose runs are padded to 8 and so to 4). */
template <int K, int NW, bool MIXED, bool NTS, int WOT, bool PG = false, bool SLOTS = false,
          int RB = 1, int LA = kLdsDmaDefault>
__global__ __launch_bounds__(NW * 64) void ec_combine_n(const CombineArgs a)
{
    constexpr u32 T = 4;
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const u32 tid = threadIdx.x;
    const u32 k = a.k;
    const uint64_t t0 = (uint64_t)blockIdx.x * T;
    const u32 wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const u32 lane = tid & 63u;
    u32 nslots = 0;
    if constexpr (SLOTS) {
        nslots = scalar_load_u32(a.slot_count);
        if (t0 >= nslots)
            return;             /* the grid is sized for the worst padding */
    }
    /* a sorted tile is one pattern's: take it from the tile's first slot.
     * Runs are padded to 8 slots, so a 4-slot tile can be all padding
     * (a run of 1-3 stripes): nothing to do, and no pattern to look up */
    const uint64_t tp = SLOTS ? slot_stripe<SLOTS>(a, t0, nslots) : t0;
    if (SLOTS && tp == kNoSlot)
        return;
    constexpr u32 SLICE = WOT ? (T / WOT) * ECD_CHUNK : 0;
    /* LDS: the k-input tile, then NW output slices */
    const PatWords<PG> pw(a, tile_pattern<MIXED>(a, tp));
    stage_tile<T, NW, LA>(lds, [&](u32 p, uint64_t slot) -> const uint8_t * {
        const uint64_t st = slot_stripe<SLOTS>(a, slot, nslots);
        return st != kNoSlot ? a.in_base[pw.byte(a, p)] + st * a.in_stride : nullptr;
    }, k, t0, SLOTS ? (uint64_t)nslots : a.nstripes, wave, lane);
    __syncthreads();
    const u32 cs = lane >> 4, cc = lane & 15u;
    const uint8_t *col = lds + cs * 64u + cc * 4u;
    uint8_t *slice = lds + k * T * ECD_CHUNK + wave * SLICE;
    const uint64_t ost = slot_stripe<SLOTS>(a, t0 + cs, nslots);
    /* RB rows per wave item (RB = 2: each input read from LDS feeds two
     * rows, two copies of the one-dword jump table) */
    for (u32 r = wave * RB; r < a.rows; r += NW * RB) {
        uint64_t cl[RB], ch[RB];
        u32 acc[RB][8][1], y[8][1];
#pragma unroll
        for (int q = 0; q < RB; ++q) {
            const u32 rq = r + q;
            const bool has = q == 0 || rq < a.rows;     /* wave-uniform */
            const u32 rw = a.kw * (1 + (has ? rq : r));
            const u32 w0 = has ? pw.word(a, rw) : 0u;
            const u32 w1 = K > 4 && has ? pw.word(a, rw + 1) : 0u;
            const u32 w2 = K > 8 && has ? pw.word(a, rw + 2) : 0u;
            const u32 w3 = K > 12 && has ? pw.word(a, rw + 3) : 0u;
            cl[q] = (uint64_t)w0 | ((uint64_t)w1 << 32);
            ch[q] = (uint64_t)w2 | ((uint64_t)w3 << 32);
#pragma unroll
            for (int b = 0; b < 8; ++b)
                acc[q][b][0] = 0;
        }
        auto next_c = [&](int q) {
            const u32 c = __builtin_amdgcn_readfirstlane((u32)cl[q] & 0xFFu);
            cl[q] = (cl[q] >> 8) | (ch[q] << 56);
            ch[q] >>= 8;
            return c;
        };
        auto load_in = [&](u32 p, u32 (&d)[8][1]) {
            const uint8_t *src = col + p * (T * ECD_CHUNK);
#pragma unroll
            for (int b = 0; b < 8; ++b)
                d[b][0] = *reinterpret_cast<const u32 *>(src + (u32)b * (T * 64u));
        };
        /* (r03 also timed a software-pipelined form: the loop unrolled by
         * two over two input buffers, input p + 1's reads issued before
         * input p's multiply; it tied or lost at every k, kb3_r03g.log) */
#pragma unroll 1
        for (u32 p = 0; p < k; ++p) {
            if constexpr (RB == 1) {
                const u32 c = next_c(0);
                if (c == 0)              /* ec-code-c.c:11666-11676 */
                    continue;
                load_in(p, y);
                ecgf::mul_xor_jt<1>(c, acc[0], y);
            } else {
                const u32 c0 = next_c(0), c1 = next_c(1);
                if ((c0 | c1) == 0)
                    continue;
                load_in(p, y);
                if (c0)
                    ecgf::mul_xor_jt<1>(c0, acc[0], y);
                if (c1)
                    ecgf::mul_xor_jt<1>(c1, acc[1], y);
            }
        }
#pragma unroll
        for (int q = 0; q < RB; ++q) {
            const u32 rq = r + q;
            if (q > 0 && rq >= a.rows)
                break;
            if constexpr (WOT) {
                store_chunks_via_lds<T, 1, NTS, WOT>(slice, acc[q], cs, cc, lane, [&](u32 s) {
                    const uint64_t o = s == cs ? ost : slot_stripe<SLOTS>(a, t0 + s, nslots);
                    return o != kNoSlot ? a.out_base[rq] + o * a.out_stride : nullptr;
                });
            } else if (ost != kNoSlot) {
                store_chunk<1, NTS>(a.out_base[rq] + ost * a.out_stride + cc * 4u, acc[q]);
            }
        }
    }
}

/* dynamic LDS of an ec_combine_n launch for k inputs */
template <int NW, int WOT>
constexpr size_t combine_n_lds(int k)
{
    return (size_t)k * 4 * ECD_CHUNK + (WOT ? (size_t)NW * (4 / WOT) * ECD_CHUNK : 0);
}

/* Zero-copy variant for the host-buffer path, where every input and output
 * lives in pinned host memory and the CUs read and write it over PCIe
 * (ec_device.hip run_pipeline).  There the link, not HBM or the VALU, is the
 * bound, and what matters is the request shape: ec_combine moves 64-byte
 * plane segments (stripe-strided reads, 8-byte-per-lane stores), which cost
 * ~25 % of the link against whole-line streams (tools/kbench/kbench2 KB_ZC,
 * profiles/kbench_r01_zc.log).  Here both directions are contiguous runs:
 *  - staging: piece e (16 B) of input p of the tile is byte (e % 32) * 16 of
 *    stripe e / 32, so with in_stride = 512 (fragments) one wave instruction
 *    reads 1 KiB of consecutive host memory; the LDS tile is chunk-major
 *    (input p, stripe s at (p * 8 + s) * 512), which LDS-DMA writes linearly;
 *  - compute as in ec_combine (8 stripes x 8 lanes x 2 dwords per plane);
 *    bank conflicts of the chunk-major reads are hidden by the link;
 *  - output: rows are assembled in a second LDS tile and written back with
 *    16-byte lanes in the order of the destination (stripe-major data when
 *    out_stride = rows * 512, otherwise row buffers), i.e. 1 KiB runs.
 * LDS = (k + rows) * 4 KiB, so the launcher uses it for k + rows <= 32. */
template <int K, int NW, bool MIXED>
__global__ __launch_bounds__(NW * 64) void ec_combine_zc(const CombineArgs a)
{
    constexpr u32 T = 8;
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const u32 tid = threadIdx.x;
    const u32 k = a.k, rows = a.rows;
    const uint64_t t0 = (uint64_t)blockIdx.x * T;
    const u32 wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const u32 lane = tid & 63u;
    uint8_t *otile = lds + k * (T * ECD_CHUNK);

    const PatWords<false> pw(a, tile_pattern<MIXED>(a, t0));

    /* stage: wave instruction ins = 1 KiB = stripes 2q, 2q+1 of input p */
    const u32 ni = k * (T / 2);
    for (u32 ins = wave; ins < ni; ins += NW) {
        const u32 p = ins / (T / 2);
        const u32 e = (ins % (T / 2)) * 64 + lane;   /* piece within input p */
        const uint64_t st = t0 + e / 32;
        if (st < a.nstripes) {
            const u32 src = pw.byte(a, p);
            const uint8_t *g = a.in_base[src] + st * a.in_stride + (e % 32) * 16u;
            __builtin_amdgcn_global_load_lds(
                (const __attribute__((address_space(1))) void *)g,
                (__attribute__((address_space(3))) void *)(lds + ins * 1024u), 16, 0, kLdsDmaDefault);
        }
    }
    __syncthreads();

    const u32 cs = lane >> 3, cc = lane & 7u;
    for (u32 r = wave; r < rows; r += NW) {
        const uint8_t *col = lds + cs * ECD_CHUNK + cc * 8u;
        const u32 rw = a.kw * (1 + r);
        const u32 w0 = pw.word(a, rw);
        const u32 w1 = K > 4 ? pw.word(a, rw + 1) : 0u;
        const u32 w2 = K > 8 ? pw.word(a, rw + 2) : 0u;
        const u32 w3 = K > 12 ? pw.word(a, rw + 3) : 0u;
        u32 acc[8][2], y[8][2];
#pragma unroll
        for (int b = 0; b < 8; ++b)
            acc[b][0] = acc[b][1] = 0;
        /* the row's coefficients as a 128-bit scalar shift register: one
         * byte per input, 4 SALU per step instead of a select chain */
        uint64_t cl = (uint64_t)w0 | ((uint64_t)w1 << 32);
        uint64_t ch = (uint64_t)w2 | ((uint64_t)w3 << 32);
        /* PU = 1: not unrolled, as every copy of the body is a copy of the
         * 255 multiply programs (~54 KiB of code) */
#pragma unroll 1
        for (u32 p = 0; p < k; ++p) {
            const u32 c = __builtin_amdgcn_readfirstlane((u32)cl & 0xFFu);
            cl = (cl >> 8) | (ch << 56);
            ch >>= 8;
            if (c == 0)                  /* ec-code-c.c:11666-11676 */
                continue;
            const uint8_t *src = col + p * (T * ECD_CHUNK);
#pragma unroll
            for (int b = 0; b < 8; ++b)
                load_plane<2>(src + (u32)b * 64u, y[b]);
            ecgf::mul_xor_rt<2>(c, acc, y);
        }
        uint8_t *o = otile + (r * T + cs) * ECD_CHUNK + cc * 8u;
#pragma unroll
        for (int b = 0; b < 8; ++b)
            *reinterpret_cast<uint2 *>(o + b * 64) = make_uint2(acc[b][0], acc[b][1]);
    }
    __syncthreads();

    /* write back: 16-byte pieces in destination order */
    const bool stripe_major = a.out_stride == (uint64_t)rows * ECD_CHUNK;
    const u32 np = rows * T * 32;
    for (u32 idx = tid; idx < np; idx += NW * 64) {
        const u32 w = idx % 32;
        u32 s, r;
        if (stripe_major) {
            s = idx / (rows * 32);
            r = (idx / 32) % rows;
        } else {
            r = idx / (T * 32);
            s = (idx / 32) % T;
        }
        const uint64_t ost = t0 + s;
        if (ost < a.nstripes)
            *reinterpret_cast<uint4 *>(a.out_base[r] + ost * a.out_stride + w * 16u) =
                *reinterpret_cast<const uint4 *>(otile + (r * T + s) * ECD_CHUNK + w * 16u);
    }
}

/* Zero-copy combine, persistent and double-buffered (r03): the same tiles,
 * request shapes and output order as ec_combine_zc, but each block walks
 * tiles blockIdx.x, + gridDim.x, ... and issues the staging loads of its
 * next tile right before the stores of the current one, so reads from and
 * writes to host memory are in flight together.  In ec_combine_zc every
 * block of a small call (a 4 MiB 8+4 heal window is 128 tiles, one block
 * each, all resident at once) reads, then computes, then writes in
 * lockstep, and the full-duplex link carries one direction at a time.
 * Per iteration: compute tile i from buf[i & 1] into otile; barrier; stage
 * tile i + 1 into buf[(i + 1) & 1] (last read in iteration i - 1, before
 * its barrier); store tile i; wait for both; barrier.  The otile reads are
 * inline asm: the compiler would otherwise put a vmcnt(0) for the pending
 * LDS-DMA in front of them and serialise the two directions again.  Raw
 * s_barrier with explicit waits (no fences: __syncthreads() adds a
 * vmcnt(0) per barrier, which is wanted only at the end of an iteration).
 * The row bases live in LDS: a lane-indexed out_base[r] is a vector load
 * from the kernel arguments, whose vmcnt(0) would wait for the staging too.
 * LDS = (2k + rows) * 4 KiB + 8 * ECD_MAX_ROWS: k <= 8 any rows up to 16,
 * k = 16 (r04) up to 7 rows in the CU's 160 KiB -- the heal and the
 * row-masked encode of a 16+4 volume, not its 16-row decode. */
__device__ __forceinline__ uint64_t lds_read_u64(const uint8_t *p)
{
    uint64_t v;
    asm volatile("ds_read_b64 %0, %1\n\ts_waitcnt lgkmcnt(0)"
                 : "=v"(v)
                 : "v"((u32)(uintptr_t)p)
                 : "memory");
    return v;
}

__device__ __forceinline__ v4u lds_read_b128(const uint8_t *p)
{
    v4u v;
    asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)"
                 : "=v"(v)
                 : "v"((u32)(uintptr_t)p)
                 : "memory");
    return v;
}

template <int K, int NW, bool MIXED, int TT = 8>
__global__ __launch_bounds__(NW * 64) void ec_combine_zc_db(const CombineArgs a)
{
    /* TT stripes per tile: 8 (lanes hold 2 dwords of a plane), or 4 for the
     * 16-row decode of a 16+4 volume, whose two 8-stripe input tiles and
     * output tile would not fit the CU's LDS (lanes hold 1 dword) */
    constexpr u32 T = TT, CW = TT / 4, LPS = 64 / TT;   /* lanes per stripe */
    static_assert(TT == 4 || TT == 8, "4- or 8-stripe tiles");
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const u32 tid = threadIdx.x;
    const u32 k = a.k, rows = a.rows;
    const u32 wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const u32 lane = tid & 63u;
    const u32 tb = k * (T * ECD_CHUNK);
    uint8_t *otile = lds + 2u * tb;
    const uint64_t ntiles = (a.nstripes + T - 1) / T;
    const bool stripe_major = a.out_stride == (uint64_t)rows * ECD_CHUNK;

    /* stage tile t into buffer b: wave instruction ins = 1 KiB = stripes
     * 2q, 2q + 1 of input p (as ec_combine_zc) */
    auto stage = [&](uint64_t t, u32 b) {
        const uint64_t t0 = t * T;
        const PatWords<false> pw(a, tile_pattern<MIXED>(a, t0));
        uint8_t *buf = lds + b * tb;
        const u32 ni = k * (T / 2);
        for (u32 ins = wave; ins < ni; ins += NW) {
            const u32 p = ins / (T / 2);
            const u32 e = (ins % (T / 2)) * 64 + lane;
            const uint64_t st = t0 + e / 32;
            if (st < a.nstripes) {
                const uint8_t *g = a.in_base[pw.byte(a, p)] + st * a.in_stride + (e % 32) * 16u;
                __builtin_amdgcn_global_load_lds(
                    (const __attribute__((address_space(1))) void *)g,
                    (__attribute__((address_space(3))) void *)(buf + ins * 1024u), 16, 0,
                    kLdsDmaDefault);
            }
        }
    };

    uint8_t *obase = otile + rows * (T * ECD_CHUNK);   /* row bases, 8 B each */
    uint64_t t = blockIdx.x;
    if (t >= ntiles)
        return;                 /* block-uniform: every wave leaves together */
    if (tid < rows)
        *reinterpret_cast<uint64_t *>(obase + tid * 8u) = (uint64_t)(uintptr_t)a.out_base[tid];
    stage(t, 0);
    /* the builtins below are IntrNoMem to LLVM: a compiler-only barrier keeps
     * the plain C++ LDS writes (row bases, otile) on their side of them */
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_waitcnt(0x0070);        /* vmcnt(0) lgkmcnt(0) */
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    const u32 cs = lane / LPS, cc = lane % LPS;
    for (u32 i = 0;; ++i) {
        const uint64_t t0 = t * T;
        const uint8_t *buf = lds + (i & 1u) * tb;
        {
            const PatWords<false> pw(a, tile_pattern<MIXED>(a, t0));
            for (u32 r = wave; r < rows; r += NW) {
                const uint8_t *col = buf + cs * ECD_CHUNK + cc * (4u * CW);
                const u32 rw = a.kw * (1 + r);
                const u32 w0 = pw.word(a, rw);
                const u32 w1 = K > 4 ? pw.word(a, rw + 1) : 0u;
                const u32 w2 = K > 8 ? pw.word(a, rw + 2) : 0u;
                const u32 w3 = K > 12 ? pw.word(a, rw + 3) : 0u;
                u32 acc[8][CW], y[8][CW];
#pragma unroll
                for (int b = 0; b < 8; ++b)
#pragma unroll
                    for (u32 w = 0; w < CW; ++w)
                        acc[b][w] = 0;
                /* one coefficient byte per input, shifted out of a 64-bit
                 * (K <= 8) or 128-bit (K = 16) scalar register pair */
                uint64_t cl = (uint64_t)w0 | ((uint64_t)w1 << 32);
                uint64_t ch = (uint64_t)w2 | ((uint64_t)w3 << 32);
#pragma unroll 1
                for (u32 p = 0; p < k; ++p) {
                    const u32 c = __builtin_amdgcn_readfirstlane((u32)cl & 0xFFu);
                    cl = (cl >> 8) | (ch << 56);
                    ch >>= 8;
                    if (c == 0)          /* ec-code-c.c:11666-11676 */
                        continue;
                    const uint8_t *src = col + p * (T * ECD_CHUNK);
#pragma unroll
                    for (int b = 0; b < 8; ++b)
                        load_plane<CW>(src + (u32)b * 64u, y[b]);
                    ecgf::mul_xor_rt<CW>(c, acc, y);
                }
                uint8_t *o = otile + (r * T + cs) * ECD_CHUNK + cc * (4u * CW);
#pragma unroll
                for (int b = 0; b < 8; ++b) {
                    if constexpr (CW == 2)
                        *reinterpret_cast<uint2 *>(o + b * 64) = make_uint2(acc[b][0], acc[b][1]);
                    else
                        *reinterpret_cast<u32 *>(o + b * 64) = acc[b][0];
                }
            }
        }
        asm volatile("" ::: "memory");
        __builtin_amdgcn_s_waitcnt(0xC07F);    /* lgkmcnt(0): otile written */
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        const uint64_t tn = t + gridDim.x;
        if (tn < ntiles)
            stage(tn, (i + 1u) & 1u);
        const u32 np = rows * T * 32;
        for (u32 idx = tid; idx < np; idx += NW * 64) {
            const u32 w = idx % 32;
            u32 s, r;
            if (stripe_major) {
                s = idx / (rows * 32);
                r = (idx / 32) % rows;
            } else {
                r = idx / (T * 32);
                s = (idx / 32) % T;
            }
            const uint64_t ost = t0 + s;
            const v4u v = lds_read_b128(otile + (r * T + s) * ECD_CHUNK + w * 16u);
            uint8_t *ob = reinterpret_cast<uint8_t *>(lds_read_u64(obase + r * 8u));
            /* a global (not flat) store: a flat one would count in lgkmcnt
             * as well, and the next ds_read's wait would drain it */
            if (ost < a.nstripes)
                *(__attribute__((address_space(1))) v4u *)(ob + ost * a.out_stride + w * 16u) = v;
        }
        asm volatile("" ::: "memory");
        __builtin_amdgcn_s_waitcnt(0x0F70);    /* vmcnt(0): tile i + 1 landed, stores out */
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (tn >= ntiles)
            break;
        t = tn;
    }
}

/* Counting sort of the stripes of a mixed call by pattern id, for pattern
 * groups of 1, 2 or 4 stripes, so the tile kernel gets 8 stripes of one
 * pattern per tile.  Each pattern's run is padded to a multiple of 8 slots
 * (kNoStripe), so tiles never straddle two patterns:
 *   ec_slots_count    per-pattern stripe counts (LDS histogram per block)
 *   ec_slots_scan     padded run offsets, the slot total (one block)
 *   ec_slots_scatter  slot of every stripe (LDS ranks + one global atomic
 *                     per block and pattern)
 * Order within a run follows the blocks' atomics; any order decodes the same
 * bytes.  Workspace: counts[256], cursors[256], total, slots. */
constexpr u32 kSlotBlock = 256, kSlotPerThread = 8;

__device__ __forceinline__ u32 clamp_pattern(const CombineArgs &a, uint64_t st)
{
    const u32 id = a.group_pattern[st >> a.group_shift];
    return id < a.npatterns ? id : a.npatterns - 1u;
}

__global__ __launch_bounds__(kSlotBlock) void ec_slots_count(const CombineArgs a, u32 *counts)
{
    __shared__ u32 h[256];
    h[threadIdx.x] = 0;
    __syncthreads();
    const uint64_t base = (uint64_t)blockIdx.x * kSlotBlock * kSlotPerThread;
    for (u32 i = 0; i < kSlotPerThread; ++i) {
        const uint64_t st = base + i * kSlotBlock + threadIdx.x;
        if (st < a.nstripes)
            atomicAdd(&h[clamp_pattern(a, st)], 1u);
    }
    __syncthreads();
    if (h[threadIdx.x])
        atomicAdd(&counts[threadIdx.x], h[threadIdx.x]);
}

__global__ __launch_bounds__(256) void ec_slots_scan(const u32 *counts, u32 *cursors, u32 *total)
{
    __shared__ u32 v[256];
    const u32 t = threadIdx.x;
    v[t] = (counts[t] + 7u) & ~7u;
    __syncthreads();
    for (u32 o = 1; o < 256; o <<= 1) {     /* Hillis-Steele inclusive scan */
        const u32 x = t >= o ? v[t - o] : 0u;
        __syncthreads();
        v[t] += x;
        __syncthreads();
    }
    cursors[t] = v[t] - ((counts[t] + 7u) & ~7u);
    if (t == 255)
        *total = v[255];
}

__global__ __launch_bounds__(kSlotBlock) void ec_slots_scatter(const CombineArgs a, u32 *cursors,
                                                               u32 *slots)
{
    __shared__ u32 h[256], basep[256];
    h[threadIdx.x] = 0;
    __syncthreads();
    const uint64_t base = (uint64_t)blockIdx.x * kSlotBlock * kSlotPerThread;
    u32 pat[kSlotPerThread], rank[kSlotPerThread];
#pragma unroll
    for (u32 i = 0; i < kSlotPerThread; ++i) {
        const uint64_t st = base + i * kSlotBlock + threadIdx.x;
        pat[i] = st < a.nstripes ? clamp_pattern(a, st) : 256u;
        rank[i] = pat[i] < 256u ? atomicAdd(&h[pat[i]], 1u) : 0u;
    }
    __syncthreads();
    if (h[threadIdx.x])
        basep[threadIdx.x] = atomicAdd(&cursors[threadIdx.x], h[threadIdx.x]);
    __syncthreads();
#pragma unroll
    for (u32 i = 0; i < kSlotPerThread; ++i)
        if (pat[i] < 256u)
            slots[basep[pat[i]] + rank[i]] = (u32)(base + i * kSlotBlock + threadIdx.x);
}

template <int TS>
inline uint64_t combine_grid(uint64_t nstripes)
{
    return (nstripes + 8 * TS - 1) / (8 * TS);
}

template <int TS>
inline size_t combine_lds(u32 k)
{
    return (size_t)k * 8 * TS * ECD_CHUNK;
}

/* ------------------------------------------- partial-stripe writes (RMW) */

/* The padded write buffer of ec_writev_prepare_buffers (ec-inode-write.c:
 * 1825-1848) merged with the old head / tail stripe (ec_merge_stripe_head /
 * _tail_locked, :1883-1908), described instead of materialised: byte v of
 * the virtual input is seg[0] for v < b1 (old head bytes, nullptr = zeros),
 * user[v - b1] for b1 <= v < b2, and seg[2][v - b2] after (old tail bytes or
 * zeros).  `user` has arbitrary byte alignment. */
struct RmwSrc {
    const uint8_t *head, *user, *tail;
    uint64_t b1, b2;
};

__device__ __forceinline__ uint8_t rmw_byte(const RmwSrc &v, uint64_t o)
{
    if (o < v.b1)
        return v.head ? v.head[o] : 0;
    if (o < v.b2)
        return v.user[o - v.b1];
    return v.tail ? v.tail[o - v.b2] : 0;
}

/* W dwords of `p`, which may have any byte alignment.  ROCm runs gfx950 in
 * unaligned access mode, so this is one global_load_dwordx{1,2,4} at the
 * byte address (it touches exactly [p, p + 4W): no over-read into a page
 * the range does not cover).  Round 1's realignment issued W + 1 separate
 * dword loads per plane (0.51 of HBM peak, profiles/bench_r01_i.log); the
 * one-instruction form below (load_plane_realign) beats both. */
template <int W>
__device__ __forceinline__ void load_plane_unaligned(const uint8_t *p, u32 (&d)[W])
{
    if constexpr (W == 1) {
        __builtin_memcpy(&d[0], p, 4);
    } else if constexpr (W == 2) {
        uint2 v;
        __builtin_memcpy(&v, p, 8);
        d[0] = v.x;
        d[1] = v.y;
    } else {
        uint4 v;
        __builtin_memcpy(&v, p, 16);
        d[0] = v.x;
        d[1] = v.y;
        d[2] = v.z;
        d[3] = v.w;
    }
}

/* W dwords starting at `a + sh` bytes, from W + 1 dword-aligned dwords at
 * `a` funnel-shifted by v_alignbyte_b32 (one global_load_dwordx{2,3,5}).
 * The extra dword is the one holding the last wanted byte, so the load
 * never touches a page the wanted range does not. */
template <int W>
__device__ __forceinline__ void load_plane_realign(const uint8_t *a, u32 sh, u32 (&d)[W])
{
    u32 t[W + 1];
    __builtin_memcpy(t, __builtin_assume_aligned(a, 4), 4 * (W + 1));
#pragma unroll
    for (int i = 0; i < W; ++i)
        d[i] = __builtin_amdgcn_alignbyte(t[i + 1], t[i], sh);
}

/* Materialise bytes [o0, o0 + n) of the virtual input into dst (16 bytes
 * per thread; n a multiple of 16).  Interior pieces take the realigned
 * dword path, the <= 2 pieces that straddle a segment boundary go byte by
 * byte. */
__global__ __launch_bounds__(kBlock) void ec_rmw_gather(const RmwSrc v, uint64_t o0, uint64_t n,
                                                        uint8_t *__restrict__ dst)
{
    const uint64_t i = ((uint64_t)blockIdx.x * kBlock + threadIdx.x) * 16;
    if (i >= n)
        return;
    const uint64_t o = o0 + i;
    u32 d[4];
    if (o >= v.b1 && o + 16 <= v.b2) {
        load_plane_unaligned<4>(v.user + (o - v.b1), d);
    } else {
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            u32 x = 0;
#pragma unroll
            for (int b = 0; b < 4; ++b)
                x |= (u32)rmw_byte(v, o + 4 * w + b) << (8 * b);
            d[w] = x;
        }
    }
    *reinterpret_cast<uint4 *>(dst + i) = make_uint4(d[0], d[1], d[2], d[3]);
}

/* Fused partial-stripe encode for the compile-time Vandermonde geometries:
 * stripe 0 and stripe nst-1 (the merged boundary stripes, gathered into
 * `edge` by ec_rmw_gather: edge + 0 and edge + (nedge-1)*stripe) are read
 * aligned; every interior stripe t is read straight from the caller's
 * buffer at user + t*stripe - head, so the interior is never copied (the
 * reference memcpy's the whole write first, ec-inode-write.c:1844).
 * (Gathering the two boundary stripes inside this kernel instead, byte-wise
 * through RmwSrc, put the 16+4 instance's inputs in scratch: 316 VGPRs and
 * 528 B of private memory, 6.9 ms per GiB.)
 * LM: 0 = byte-address loads (load_plane_unaligned), 1 = dword-aligned loads
 * funnel-shifted (load_plane_realign); the launcher picks per geometry. */
template <int K, int N, int W, int LM = 0>
__global__ __launch_bounds__(kBlock) void ec_encode_vander_rmw(const uint8_t *__restrict__ edge,
                                                               const uint8_t *user_shift,
                                                               const FragPtrs out,
                                                               uint64_t nstripes)
{
    constexpr int L = 16 / W;
    constexpr uint64_t S = (uint64_t)K * ECD_CHUNK;
    const uint64_t gtid = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    const uint64_t stripe = gtid / L;
    if (stripe >= nstripes)
        return;
    const u32 colb = (u32)(gtid % L) * (4 * W);
    u32 x[K][8][W];
    if (stripe == 0 || stripe == nstripes - 1) {
        const uint8_t *s = edge + (stripe == 0 ? 0 : (nstripes > 1 ? S : 0)) + colb;
#pragma unroll
        for (int j = 0; j < K; ++j)
            load_chunk<W>(s + j * ECD_CHUNK, x[j]);
    } else {
        /* user_shift = user - head: the virtual offset of user byte 0 is head */
        const uint8_t *s = user_shift + stripe * S + colb;
        if constexpr (LM == 0) {
#pragma unroll
            for (int j = 0; j < K; ++j)
#pragma unroll
                for (int b = 0; b < 8; ++b)
                    load_plane_unaligned<W>(s + j * ECD_CHUNK + b * 64, x[j][b]);
        } else {
            /* every plane of every stripe has the same misalignment */
            const u32 sh = (u32)(uintptr_t)user_shift & 3u;
            const uint8_t *al = s - sh;
#pragma unroll
            for (int j = 0; j < K; ++j)
#pragma unroll
                for (int b = 0; b < 8; ++b)
                    load_plane_realign<W>(al + j * ECD_CHUNK + b * 64, sh, x[j][b]);
        }
    }
    encode_rows<K, W, false, true>(std::make_integer_sequence<int, N>{}, x, out,
                                   stripe * (uint64_t)ECD_CHUNK + colb);
}

} // namespace ecdev

#endif
