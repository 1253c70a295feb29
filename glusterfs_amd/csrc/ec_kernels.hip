/*
 * ec_kernels.hip -- gfx950 kernels for the GlusterFS disperse coding path.
 *
 * Two kernels, both working directly on ec's bit-sliced chunk layout
 * (512-byte chunks = 8 planes x 64 bytes, ec-method.h:27-29):
 *
 *  ec_encode_vander<K, N, W>   reference: ec_method_encode (ec-method.c:394-408)
 *      with the per-row Horner kernels ec_code_c_linear (ec-code-c.c:11647).
 *      Fragment i of stripe t = Horner over the k data chunks with the row's
 *      evaluation point v = i + 1 (ec-method.c:22-36, 284-286).  K, N and
 *      therefore every v are compile-time constants, so each Horner step is a
 *      straight-line XOR tree (ec_gf8.h) -- the gfx950 counterpart of the
 *      reference's JIT'ed x64/SSE/AVX row routines (ec-code.c:722-752).
 *
 *  ec_combine<K, W, MIXED>     reference: ec_method_decode (ec-method.c:411-433)
 *      with ec_code_c_interleaved (ec-code-c.c:11660-11679).  Output row r of
 *      stripe t = XOR_p coef[r][p] * input_p(t) for a run-time k x k (or n x k)
 *      coefficient matrix held in the kernel-argument segment (constant
 *      memory, read with scalar loads).  Each coefficient is wave-uniform, so
 *      the multiply dispatches through a scalar compare tree into one of 255
 *      compile-time XOR trees; zero coefficients are skipped.  MIXED selects a
 *      pattern (erasure mask -> sources + inverse) per group of stripes.
 *
 * Work decomposition (both kernels): a lane owns W consecutive dwords of all
 * 8 planes of one chunk column, i.e. L = 16/W lanes cover a chunk; a 64-lane
 * wave covers 4W consecutive stripes and a 256-thread block 16W stripes.
 * Every load/store is a W-dword vector access; one wave instruction touches
 * 4W fully used 64-byte plane segments.  All k input chunks of the lane's
 * column stay in VGPRs, so HBM is read once and written once: the kernels are
 * HBM-bound streaming kernels (no MFMA: this is GF(2) XOR algebra).
 */
#include <hip/hip_runtime.h>
#include <errno.h>
#include <stdint.h>
#include <utility>

#include "ec_device.h"
#include "ec_gf8.h"
#include "ec_kernels.h"

using ecgf::u32;

namespace {

constexpr int kBlock = 256;

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

template <int W>
__device__ __forceinline__ void store_plane(uint8_t *p, const u32 (&d)[W])
{
    if constexpr (W == 1) {
        *reinterpret_cast<u32 *>(p) = d[0];
    } else if constexpr (W == 2) {
        *reinterpret_cast<uint2 *>(p) = make_uint2(d[0], d[1]);
    } else {
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

template <int W>
__device__ __forceinline__ void store_chunk(uint8_t *p, const u32 (&d)[8][W])
{
#pragma unroll
    for (int b = 0; b < 8; ++b)
        store_plane<W>(p + b * 64, d[b]);
}

/* Compile-time loop: f(std::integral_constant<int, I>) for I in [B, E). */
template <int B, int E, typename F>
__device__ __forceinline__ void static_for(F &&f)
{
    if constexpr (B < E) {
        f(std::integral_constant<int, B>{});
        static_for<B + 1, E>(f);
    }
}

/* ------------------------------------------------ specialised encoder */

struct FragPtrs {
    uint8_t *p[ECD_MAX_ROWS];
};

/* Row I (evaluation point v = I + 1) of the reversed Vandermonde matrix. */
template <int K, int W, int I>
__device__ __forceinline__ void encode_row(const u32 (&x)[K][8][W], uint8_t *dst)
{
    constexpr u32 v = I + 1;
    u32 acc[8][W];
    if constexpr (v == 1) {
        /* row 0 = XOR of all data chunks: XOR3 chains */
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
    store_chunk<W>(dst, acc);
}

template <int K, int W, int... I>
__device__ __forceinline__ void encode_rows(std::integer_sequence<int, I...>,
                                            const u32 (&x)[K][8][W],
                                            const FragPtrs &out, uint64_t off)
{
    (encode_row<K, W, I>(x, out.p[I] + off), ...);
}

template <int K, int N, int W>
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

    encode_rows<K, W>(std::make_integer_sequence<int, N>{}, x, out,
                      stripe * (uint64_t)ECD_CHUNK + colb);
}

/* ------------------------------------------------- generic combination */

/* Tile geometry of ec_combine: a tile is T = 8 consecutive stripes; a wave
 * computes one output row of the whole tile (8 stripes x 8 lanes, W = 2
 * dwords of every plane per lane), the 4 waves of a block take rows
 * w, w+4, ...  The tile's k input chunks are staged in LDS so that a lane can
 * walk the inputs with a run-time index (one shared multiply dispatch). */
constexpr int kTile = 8;                 /* stripes per tile                */
constexpr int kCW = 2;                   /* dwords per plane per lane       */

/* LDS byte offset of 16-byte piece q (0..31) of the chunk of input p, tile
 * stripe s.  Plane slots are XOR-rotated by s&3 so that the 4 stripes a half
 * wave reads with ds_read_b64 fall on 4 different 64-byte bank windows. */
__device__ __forceinline__ u32 lds_piece(u32 p, u32 s, u32 q)
{
    return (p * kTile + s) * ECD_CHUNK + ((((q >> 2) ^ (s & 3u)) << 6) | ((q & 3u) << 4));
}

template <int K, bool MIXED>
__global__ __launch_bounds__(kBlock) void ec_combine(const ecd_combine_desc_t d)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const u32 tid = threadIdx.x;
    const u32 k = d.k;
    const uint64_t ntiles = (d.nstripes + kTile - 1) / kTile;

    /* staging role: thread loads piece q of stripe s for every input p */
    const u32 ls = tid >> 5, lq = tid & 31u;
    /* compute role: wave w, lane -> (stripe cs, column pair cc) */
    const u32 wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const u32 lane = tid & 63u;
    const u32 cs = lane >> 3, cc = lane & 7u;

    for (uint64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const uint64_t t0 = tile * kTile;
        u32 pbase = 0;
        if constexpr (MIXED)
            pbase = __builtin_amdgcn_readfirstlane(d.group_pattern[t0 >> d.group_shift]) *
                    d.pat_bytes;

        /* stage: global -> registers -> LDS (16-B pieces, coalesced) */
        {
            const uint64_t st = t0 + ls;
            uint4 v[K];
#pragma unroll
            for (int p = 0; p < K; ++p) {
                v[p] = make_uint4(0, 0, 0, 0);
                if ((u32)p < k && st < d.nstripes) {
                    const u32 src = __builtin_amdgcn_readfirstlane(d.pat[pbase + p]);
                    const uint8_t *g = static_cast<const uint8_t *>(d.in_base[src]) +
                                       st * d.in_stride + lq * 16u;
                    v[p] = *reinterpret_cast<const uint4 *>(g);
                }
            }
#pragma unroll
            for (int p = 0; p < K; ++p)
                if ((u32)p < k)
                    *reinterpret_cast<uint4 *>(lds + lds_piece(p, ls, lq)) = v[p];
        }
        __syncthreads();

        /* compute: one output row per wave at a time */
        const uint64_t ost = t0 + cs;
        const u32 cbase = pbase + k;
        for (u32 r = wave; r < d.rows; r += kBlock / 64) {
            u32 acc[8][kCW];
#pragma unroll
            for (int b = 0; b < 8; ++b)
#pragma unroll
                for (int w = 0; w < kCW; ++w)
                    acc[b][w] = 0;
            for (u32 p = 0; p < k; ++p) {
                const u32 c = __builtin_amdgcn_readfirstlane(d.pat[cbase + r * k + p]);
                if (c == 0)
                    continue;
                u32 y[8][kCW];
                const uint8_t *src = lds + (p * kTile + cs) * ECD_CHUNK + cc * 8u;
#pragma unroll
                for (int b = 0; b < 8; ++b) {
                    const uint2 t = *reinterpret_cast<const uint2 *>(
                        src + (((u32)b ^ (cs & 3u)) << 6));
                    y[b][0] = t.x;
                    y[b][1] = t.y;
                }
                ecgf::mul_xor_rt<kCW>(c, acc, y);
            }
            if (ost < d.nstripes) {
                uint8_t *dst = static_cast<uint8_t *>(d.out_base[r]) + ost * d.out_stride +
                               cc * 8u;
                store_chunk<kCW>(dst, acc);
            }
        }
        __syncthreads();
    }
}

/* ------------------------------------------------------------ launchers */

template <int W>
inline uint64_t grid_for(uint64_t nstripes)
{
    return (nstripes * (16 / W) + kBlock - 1) / kBlock;
}

template <int K, int N, int W>
int launch_vander(hipStream_t s, uint64_t nstripes, const void *in, void *const *out)
{
    FragPtrs f;
    for (int i = 0; i < N; ++i)
        f.p[i] = static_cast<uint8_t *>(out[i]);
    const uint64_t g = grid_for<W>(nstripes);
    if (g == 0)
        return 0;
    if (g > 0x7fffffffull)
        return -EINVAL;
    hipLaunchKernelGGL((ec_encode_vander<K, N, W>), dim3((u32)g), dim3(kBlock), 0, s,
                       static_cast<const uint8_t *>(in), f, nstripes);
    return hipGetLastError() == hipSuccess ? 0 : -EIO;
}

template <int K>
int launch_combine(hipStream_t s, const ecd_combine_desc_t *d)
{
    const uint64_t ntiles = (d->nstripes + kTile - 1) / kTile;
    if (ntiles == 0)
        return 0;
    const u32 grid = (u32)(ntiles < 4096 ? ntiles : 4096);
    const size_t lds = (size_t)d->k * kTile * ECD_CHUNK;
    if (d->group_pattern)
        hipLaunchKernelGGL((ec_combine<K, true>), dim3(grid), dim3(kBlock), lds, s, *d);
    else
        hipLaunchKernelGGL((ec_combine<K, false>), dim3(grid), dim3(kBlock), lds, s, *d);
    return hipGetLastError() == hipSuccess ? 0 : -EIO;
}

} // namespace

int ecdk_has_vander(uint32_t k, uint32_t n)
{
    return (k == 2 && n == 3) || (k == 4 && n == 6) || (k == 8 && n == 12) ||
           (k == 16 && n == 20);
}

int ecdk_encode_vander(hipStream_t s, uint32_t k, uint32_t n, uint64_t nstripes,
                       const void *in, void *const *out)
{
    if (k == 2 && n == 3)
        return launch_vander<2, 3, 4>(s, nstripes, in, out);
    if (k == 4 && n == 6)
        return launch_vander<4, 6, 2>(s, nstripes, in, out);
    if (k == 8 && n == 12)
        return launch_vander<8, 12, 2>(s, nstripes, in, out);
    if (k == 16 && n == 20)
        return launch_vander<16, 20, 1>(s, nstripes, in, out);
    return -ENOTSUP;
}

int ecdk_combine(hipStream_t s, const ecd_combine_desc_t *d)
{
    if (d->k == 0 || d->k > ECD_MAX_K || d->rows == 0 || d->rows > ECD_MAX_ROWS)
        return -EINVAL;
    if ((uint64_t)d->npatterns * d->pat_bytes > ECD_MAX_PAT_BYTES ||
        d->pat_bytes < d->k + d->rows * d->k)
        return -EINVAL;
    if (d->group_pattern && d->group_shift < 3)
        return -EINVAL;
    if (d->k <= 4)
        return launch_combine<4>(s, d);
    if (d->k <= 8)
        return launch_combine<8>(s, d);
    return launch_combine<16>(s, d);
}
