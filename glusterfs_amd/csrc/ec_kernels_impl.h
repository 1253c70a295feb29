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
 *  ec_combine<K, TS, MIXED, NTS>    reference: ec_method_decode
 *      (ec-method.c:411-433) with ec_code_c_interleaved (ec-code-c.c:11660).
 *      Output row r of stripe t = XOR_p coef[r][p] * input_p(t) for a run-time
 *      coefficient matrix held in the kernel-argument segment (constant
 *      memory, scalar loads).  One block = one tile of T = 8*TS stripes: the
 *      k input chunks of the tile are staged through LDS with coalesced
 *      16-byte loads, then each wave computes whole output rows (8 stripes x
 *      8 lanes x 2 dwords per plane) walking the inputs with a run-time index
 *      so a single multiply dispatch serves every coefficient: the
 *      wave-uniform coefficient selects one of 255 compile-time XOR trees
 *      through a scalar compare tree, zero coefficients are skipped.  MIXED
 *      picks a pattern (erasure mask -> sources + inverse) per stripe group.
 *
 * Tuning knobs measured with tools/kbench (profiles/kbench_*.log): one tile
 * per block beats a persistent grid with register prefetch (vmcnt also counts
 * the stores of the previous tile, which serialises the prefetch);
 * non-temporal loads lose; staging the output tile through LDS and a split
 * 16+16-case dispatch measured equal or worse and were removed; NTS
 * (non-temporal stores) and the block size NW remain knobs.
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
template <int K, int W, int I, bool NTS>
__device__ __forceinline__ void encode_row(const u32 (&x)[K][8][W], uint8_t *dst)
{
    constexpr u32 v = I + 1;
    u32 acc[8][W];
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
            ecgf::horner<v, W>(acc, x[j]);
    }
    store_chunk<W, NTS>(dst, acc);
}

template <int K, int W, bool NTS, int... I>
__device__ __forceinline__ void encode_rows(std::integer_sequence<int, I...>,
                                            const u32 (&x)[K][8][W], const FragPtrs &out,
                                            uint64_t off)
{
    (encode_row<K, W, I, NTS>(x, out.p[I] + off), ...);
}

template <int K, int N, int W, bool NTS>
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

    encode_rows<K, W, NTS>(std::make_integer_sequence<int, N>{}, x, out,
                           stripe * (uint64_t)ECD_CHUNK + colb);
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
 * runs both directions at once (~45 GB/s each way, tools/kbench/zerocopy). */
template <int K, int N, int W, int BS = kBlock>
__global__ __launch_bounds__(BS) void ec_encode_vander_zc(const uint8_t *__restrict__ in,
                                                          const FragPtrs out, uint64_t nstripes)
{
    constexpr int L = 16 / W;
    const uint64_t gtid = (uint64_t)blockIdx.x * BS + threadIdx.x;
    const uint64_t step = (uint64_t)gridDim.x * (BS / L);
    const u32 colb = (u32)(gtid % L) * (4 * W);
    uint64_t stripe = gtid / L;
    if (stripe >= nstripes)
        return;

    u32 x[K][8][W];
    const uint8_t *s = in + stripe * (uint64_t)(K * ECD_CHUNK) + colb;
#pragma unroll
    for (int j = 0; j < K; ++j)
        load_chunk<W>(s + j * ECD_CHUNK, x[j]);
    for (;;) {
        const uint64_t nxt = stripe + step;
        u32 y[K][8][W];
        if (nxt < nstripes) {
            const uint8_t *sn = in + nxt * (uint64_t)(K * ECD_CHUNK) + colb;
#pragma unroll
            for (int j = 0; j < K; ++j)
                load_chunk<W>(sn + j * ECD_CHUNK, y[j]);
        }
        encode_rows<K, W, false>(std::make_integer_sequence<int, N>{}, x, out,
                                 stripe * (uint64_t)ECD_CHUNK + colb);
        if (nxt >= nstripes)
            break;
        stripe = nxt;
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
    u32 k, kw, rows, group_shift, pwords;
    u32 pat[kPatWords];
};

/* LDS byte offset of 16-byte piece q (0..31) of the chunk of input p, tile
 * stripe s, tile of T stripes.  Plane slots are XOR-rotated by s&3 so the 4
 * stripes a half wave reads with ds_read_b64 hit 4 different 64-byte bank
 * windows (conflict-free), and a ds_write_b128 group of 8 lanes (2 planes of
 * one chunk) covers one full 128-byte bank row. */
__device__ __forceinline__ u32 lds_piece(u32 p, u32 s, u32 q, u32 T)
{
    return (p * T + s) * ECD_CHUNK + ((((q >> 2) ^ (s & 3u)) << 6) | ((q & 3u) << 4));
}

__device__ __forceinline__ u32 pat_byte(const CombineArgs &a, u32 word, u32 idx)
{
    const u32 w = a.pat[word + (idx >> 2)];
    return __builtin_amdgcn_readfirstlane((w >> ((idx & 3u) * 8u)) & 0xFFu);
}

/* K: max inputs (k <= K); TS: tile = 8*TS stripes; NW: waves per block;
 * GLDS: stage the tile with LDS-DMA (global_load_lds_dwordx4, no VGPRs)
 * instead of global_load + ds_write; PF: issue the next input's LDS reads
 * before each multiply. */
template <int K, int TS, int NW, bool MIXED, bool NTS, bool GLDS = false, bool PF = false,
          bool PP = false>
__global__ __launch_bounds__(NW * 64) void ec_combine(const CombineArgs a)
{
    constexpr u32 T = 8 * TS;            /* stripes per tile                   */
    constexpr u32 NT = NW * 64;          /* threads per block                  */
    constexpr u32 PER = (K * T * 32 + NT - 1) / NT; /* staged pieces per thread */
    constexpr int CW = 2;                /* dwords per plane per lane (compute) */
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const u32 tid = threadIdx.x;
    const u32 k = a.k;
    const uint64_t t0 = (uint64_t)blockIdx.x * T;
    const u32 wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const u32 lane = tid & 63u;

    u32 pb = 0;
    if constexpr (MIXED)
        pb = __builtin_amdgcn_readfirstlane(a.group_pattern[t0 >> a.group_shift]) * a.pwords;

    if constexpr (GLDS) {
        /* every wave instruction fills 1 KiB of LDS linearly (2 chunks of one
         * input); the XOR plane rotation is applied to the per-lane source
         * address instead of the destination */
        constexpr u32 NI = K * T * 32 / 64; /* wave instructions per tile */
#pragma unroll
        for (u32 j = 0; j < (NI + NW - 1) / NW; ++j) {
            const u32 ins = j * NW + wave;           /* wave-uniform */
            if (ins >= NI)
                break;
            const u32 p = ins / (T / 2);
            if (p >= k)
                break;
            const u32 e = ins * 64 + lane;            /* LDS piece */
            const u32 s = (e / 32) % T, slot = e & 31u;
            const uint64_t st = t0 + s;
            if (st < a.nstripes) {
                const u32 src = pat_byte(a, pb, p);
                const uint8_t *g = a.in_base[src] + st * a.in_stride +
                                   ((((slot >> 2) ^ (s & 3u)) << 6) | ((slot & 3u) << 4));
                __builtin_amdgcn_global_load_lds(
                    (const __attribute__((address_space(1))) void *)g,
                    (__attribute__((address_space(3))) void *)(lds + ins * 1024u), 16, 0, 0);
            }
        }
    } else {
        /* stage: 16-byte pieces e = (input p, stripe s, piece q), coalesced */
        uint4 v[PER];
#pragma unroll
        for (u32 j = 0; j < PER; ++j) {
            const u32 e = tid + j * NT;
            const u32 p = e / (T * 32), s = (e / 32) % T, q = e & 31u;
            const uint64_t st = t0 + s;
            v[j] = make_uint4(0, 0, 0, 0);
            if (p < k && st < a.nstripes) {
                const u32 src = pat_byte(a, pb, p);
                v[j] = *reinterpret_cast<const uint4 *>(a.in_base[src] + st * a.in_stride +
                                                        q * 16u);
            }
        }
#pragma unroll
        for (u32 j = 0; j < PER; ++j) {
            const u32 e = tid + j * NT;
            const u32 p = e / (T * 32), s = (e / 32) % T, q = e & 31u;
            if (p < k)
                *reinterpret_cast<uint4 *>(lds + lds_piece(p, s, q, T)) = v[j];
        }
    }
    __syncthreads();

    /* compute: (row, 8-stripe subtile) items spread over the NW waves */
    const u32 cs = lane >> 3, cc = lane & 7u;
    const u32 items = a.rows * TS;
    for (u32 it = wave; it < items; it += NW) {
        const u32 r = it / TS, s = (it % TS) * 8u + cs;
        const u32 rot = (s & 3u) << 6;
        const uint8_t *col = lds + s * ECD_CHUNK + cc * 8u;
        /* the row's coefficients: up to 4 words, loaded once into SGPRs */
        const u32 rw = pb + a.kw * (1 + r);
        const u32 w0 = a.pat[rw];
        const u32 w1 = K > 4 ? a.pat[rw + 1] : 0u;
        const u32 w2 = K > 8 ? a.pat[rw + 2] : 0u;
        const u32 w3 = K > 12 ? a.pat[rw + 3] : 0u;
        u32 acc[8][CW], y[8][CW];
#pragma unroll
        for (int b = 0; b < 8; ++b)
#pragma unroll
            for (int w = 0; w < CW; ++w)
                acc[b][w] = 0;
        auto read_input = [&](u32 p, u32 (&d)[8][CW]) {
            const uint8_t *src = col + p * (T * ECD_CHUNK);
#pragma unroll
            for (int b = 0; b < 8; ++b) {
                const uint2 t = *reinterpret_cast<const uint2 *>(src + (((u32)b << 6) ^ rot));
                d[b][0] = t.x;
                d[b][1] = t.y;
            }
        };
        auto coef = [&](u32 p) {
            const u32 wsel = p < 4 ? w0 : p < 8 ? w1 : p < 12 ? w2 : w3;
            return __builtin_amdgcn_readfirstlane((wsel >> ((p & 3u) * 8u)) & 0xFFu);
        };
        if constexpr (PP) {
            /* ping-pong accumulators (ecgf::mul_xor_rt_pp): acc -> y2 -> acc */
            u32 acc2[8][CW];
            for (u32 p = 0; p < k; p += 2) {
                const u32 c0 = coef(p);
                if (c0)
                    read_input(p, y);
                ecgf::mul_xor_rt_pp<CW>(c0, acc, acc2, y);
                const u32 c1 = p + 1 < k ? coef(p + 1) : 0u;
                if (c1)
                    read_input(p + 1, y);
                ecgf::mul_xor_rt_pp<CW>(c1, acc2, acc, y);
            }
        } else {
            if constexpr (PF)
                read_input(0, y);
            for (u32 p = 0; p < k; ++p) {
                const u32 c = coef(p);
                if constexpr (PF) {
                    /* issue the next input's LDS reads before this multiply */
                    u32 yn[8][CW];
                    read_input(p + 1 < k ? p + 1 : p, yn);
                    ecgf::mul_xor_rt<CW>(c, acc, y);
#pragma unroll
                    for (int b = 0; b < 8; ++b)
#pragma unroll
                        for (int w = 0; w < CW; ++w)
                            y[b][w] = yn[b][w];
                } else {
                    if (c == 0)
                        continue;
                    read_input(p, y);
                    ecgf::mul_xor_rt<CW>(c, acc, y);
                }
            }
        }
        const uint64_t ost = t0 + s;
        if (ost < a.nstripes)
            store_chunk<CW, NTS>(a.out_base[r] + ost * a.out_stride + cc * 8u, acc);
    }
}

/* ec_combine for wide codes (k > G): the tile's inputs are staged and
 * consumed in groups of G fragments through one G-input LDS buffer, the
 * output rows accumulating in VGPRs across groups (wave w owns items w,
 * w + NW, ...; at most IPW each).  LDS per block drops from k to G inputs,
 * so more blocks share a CU and one block's XOR-heavy compute phase overlaps
 * other blocks' loads and stores -- at k = 16 the single-phase kernel holds
 * 2 blocks per CU and runs its memory and VALU phases nearly back to back. */
template <int K, int G, int NW, int IPW, bool MIXED, bool NTS>
__global__ __launch_bounds__(NW * 64) void ec_combine_grouped(const CombineArgs a)
{
    constexpr u32 T = 8;                 /* stripes per tile                   */
    constexpr int CW = 2;
    constexpr u32 NI = G * T * 32 / 64;  /* LDS-DMA wave instructions / group */
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const u32 tid = threadIdx.x;
    const u32 k = a.k;
    const uint64_t t0 = (uint64_t)blockIdx.x * T;
    const u32 wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const u32 lane = tid & 63u;
    const u32 cs = lane >> 3, cc = lane & 7u;
    const u32 rot = (cs & 3u) << 6;
    const uint8_t *col = lds + cs * ECD_CHUNK + cc * 8u;

    u32 pb = 0;
    if constexpr (MIXED)
        pb = __builtin_amdgcn_readfirstlane(a.group_pattern[t0 >> a.group_shift]) * a.pwords;

    u32 acc[IPW][8][CW];
#pragma unroll
    for (int j = 0; j < IPW; ++j)
#pragma unroll
        for (int b = 0; b < 8; ++b)
#pragma unroll
            for (int w = 0; w < CW; ++w)
                acc[j][b][w] = 0;

    for (u32 g0 = 0; g0 < k; g0 += G) {
        if (g0)
            __syncthreads();             /* everyone is done with the buffer */
#pragma unroll
        for (u32 j = 0; j < (NI + NW - 1) / NW; ++j) {
            const u32 ins = j * NW + wave;
            if (ins >= NI)
                break;
            const u32 p = g0 + ins / (T / 2);
            if (p >= k)
                break;
            const u32 e = ins * 64 + lane;
            const u32 s = (e / 32) % T, slot = e & 31u;
            const uint64_t st = t0 + s;
            if (st < a.nstripes) {
                const u32 src = pat_byte(a, pb, p);
                const uint8_t *gp = a.in_base[src] + st * a.in_stride +
                                    ((((slot >> 2) ^ (s & 3u)) << 6) | ((slot & 3u) << 4));
                __builtin_amdgcn_global_load_lds(
                    (const __attribute__((address_space(1))) void *)gp,
                    (__attribute__((address_space(3))) void *)(lds + ins * 1024u), 16, 0, 0);
            }
        }
        __syncthreads();
        const u32 ng = k - g0 < (u32)G ? k - g0 : (u32)G;
        /* the items' coefficient words for this group (<= 2 words each) */
        u32 cw[IPW][2];
        static_for<0, IPW>([&](auto jj) {
            constexpr int j = decltype(jj)::value;
            const u32 r = wave + (u32)j * NW;
            const u32 rw = pb + a.kw * (1 + (r < a.rows ? r : 0)) + (g0 >> 2);
            cw[j][0] = a.pat[rw];
            cw[j][1] = G > 4 ? a.pat[rw + 1] : 0u;
        });
        for (u32 q = 0; q < ng; ++q) {
            /* one LDS read of input q serves all of this wave's rows */
            u32 y[8][CW];
            const uint8_t *src = col + q * (T * ECD_CHUNK);
#pragma unroll
            for (int b = 0; b < 8; ++b) {
                const uint2 t = *reinterpret_cast<const uint2 *>(src + (((u32)b << 6) ^ rot));
                y[b][0] = t.x;
                y[b][1] = t.y;
            }
            static_for<0, IPW>([&](auto jj) {
                constexpr int j = decltype(jj)::value;
                const u32 wsel = q < 4 ? cw[j][0] : cw[j][1];
                u32 c = __builtin_amdgcn_readfirstlane((wsel >> ((q & 3u) * 8u)) & 0xFFu);
                if (wave + (u32)j * NW >= a.rows)
                    c = 0;
                ecgf::mul_xor_rt<CW>(c, acc[j], y);
            });
        }
    }
    const uint64_t ost = t0 + cs;
    if (ost < a.nstripes) {
        static_for<0, IPW>([&](auto jj) {
            constexpr int j = decltype(jj)::value;
            const u32 r = wave + (u32)j * NW;
            if (r < a.rows)
                store_chunk<CW, NTS>(a.out_base[r] + ost * a.out_stride + cc * 8u, acc[j]);
        });
    }
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

/* W dwords of `p`, which may have any byte alignment: the aligned dwords
 * that cover [p, p + 4W) are loaded and funnel-shifted with v_alignbyte_b32.
 * Every loaded dword holds at least one byte of the range, so no load can
 * cross into a page the range does not touch. */
template <int W>
__device__ __forceinline__ void load_plane_unaligned(const uint8_t *p, u32 (&d)[W])
{
    const u32 mis = (u32)((uintptr_t)p & 3u);
    const u32 *a = reinterpret_cast<const u32 *>((uintptr_t)p & ~(uintptr_t)3);
    if (mis == 0) {
#pragma unroll
        for (int w = 0; w < W; ++w)
            d[w] = a[w];
        return;
    }
    u32 t[W + 1];
#pragma unroll
    for (int w = 0; w <= W; ++w)
        t[w] = a[w];
#pragma unroll
    for (int w = 0; w < W; ++w)
        d[w] = __builtin_amdgcn_alignbyte(t[w + 1], t[w], mis);
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
 * buffer at user + t*stripe - head with realigned loads, so the interior is
 * never copied (the reference memcpy's the whole write first,
 * ec-inode-write.c:1844). */
template <int K, int N, int W>
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
#pragma unroll
        for (int j = 0; j < K; ++j)
#pragma unroll
            for (int b = 0; b < 8; ++b)
                load_plane_unaligned<W>(s + j * ECD_CHUNK + b * 64, x[j][b]);
    }
    encode_rows<K, W, false>(std::make_integer_sequence<int, N>{}, x, out,
                             stripe * (uint64_t)ECD_CHUNK + colb);
}

} // namespace ecdev

#endif
