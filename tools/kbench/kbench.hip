/*
 * kbench.hip -- development harness (not product): A/B the shipped kernel
 * templates of glusterfs_amd/csrc/ec_kernels_impl.h over their tuning knobs,
 * next to HBM calibration kernels, in ONE process with interleaved rounds and
 * the median of rounds (cdna_hip_programming.md 5.4 rule 24).  Each variant's
 * output is compared with the group's first variant.
 *
 *   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I glusterfs_amd/csrc \
 *         tools/kbench/kbench.hip -o tools/kbench/kbench
 *   tools/kbench/kbench [GiB=1] [rounds=7]
 */
#include "../../glusterfs_amd/csrc/ec_kernels.hip"
#include "ec_gf8_asm_t4.h"   /* the <= 4-temporary programs (kb_combine_pf) */

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#define CHK(x)                                                                             \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__);  \
            exit(1);                                                                       \
        }                                                                                  \
    } while (0)

/* ---------------------------------------------------------- calibration */
__global__ void k_copy(const uint4 *__restrict__ a, uint4 *__restrict__ b, size_t n)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
         i += (size_t)gridDim.x * blockDim.x)
        b[i] = a[i];
}

__global__ void k_copy_nt(const uint4 *__restrict__ a, uint4 *__restrict__ b, size_t n)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
         i += (size_t)gridDim.x * blockDim.x) {
        const v4u v = __builtin_nontemporal_load(reinterpret_cast<const v4u *>(a + i));
        __builtin_nontemporal_store(v, reinterpret_cast<v4u *>(b + i));
    }
}

__global__ void k_read(const uint4 *__restrict__ a, size_t n, u32 *sink)
{
    u32 x = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
         i += (size_t)gridDim.x * blockDim.x) {
        const uint4 v = a[i];
        x ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (x == 0x12345678u)
        sink[0] = x;
}

__global__ void k_write(uint4 *__restrict__ b, size_t n)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
         i += (size_t)gridDim.x * blockDim.x)
        b[i] = make_uint4((u32)i, (u32)i, (u32)i, (u32)i);
}

/* our access shape: 8 lanes x 8 B cover one 64-B plane segment, a wave
 * instruction covers 8 stripes' segments at a 512-B stride */
__global__ void k_write_seg(uint8_t *__restrict__ b, size_t nchunks)
{
    const size_t gt = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    const size_t ch = gt / 8;
    if (ch >= nchunks)
        return;
    const u32 c = (gt % 8) * 8;
#pragma unroll
    for (int p = 0; p < 8; ++p)
        *reinterpret_cast<uint2 *>(b + ch * 512 + p * 64 + c) = make_uint2((u32)gt, p);
}

__global__ void k_read_seg(const uint8_t *__restrict__ a, size_t nchunks, u32 *sink)
{
    const size_t gt = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    const size_t ch = gt / 8;
    if (ch >= nchunks)
        return;
    const u32 c = (gt % 8) * 8;
    u32 x = 0;
#pragma unroll
    for (int p = 0; p < 8; ++p) {
        const uint2 v = *reinterpret_cast<const uint2 *>(a + ch * 512 + p * 64 + c);
        x ^= v.x ^ v.y;
    }
    if (x == 0x12345678u)
        sink[0] = x;
}

struct Variant {
    std::string name;
    double bytes;                  /* algorithmic bytes per launch */
    std::function<void(hipStream_t)> fn;
    uint8_t *out;                  /* checked region (nullptr: no check) */
    size_t out_bytes;
};

static void fill(uint8_t *d, size_t n, uint32_t seed)
{
    std::vector<uint32_t> h(n / 4);
    uint32_t x = seed | 1;
    for (auto &w : h) {
        x ^= x << 13;
        x ^= x >> 17;
        x ^= x << 5;
        w = x;
    }
    CHK(hipMemcpy(d, h.data(), n, hipMemcpyHostToDevice));
}

static void run_group(const char *title, std::vector<Variant> &vars, int rounds, int iters,
                      hipStream_t s)
{
    std::vector<uint8_t> ref, cur;
    for (size_t v = 0; v < vars.size(); ++v) {
        if (!vars[v].out)
            continue;
        CHK(hipMemset(vars[v].out, 0, vars[v].out_bytes));
        vars[v].fn(s);
        CHK(hipStreamSynchronize(s));
        cur.resize(vars[v].out_bytes);
        CHK(hipMemcpy(cur.data(), vars[v].out, vars[v].out_bytes, hipMemcpyDeviceToHost));
        if (ref.empty())
            ref = cur;
        else if (cur != ref)
            printf("  MISMATCH %s\n", vars[v].name.c_str());
    }
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    std::vector<std::vector<double>> t(vars.size());
    for (int rd = 0; rd < rounds; ++rd)
        for (size_t v = 0; v < vars.size(); ++v) {
            vars[v].fn(s);
            vars[v].fn(s);
            CHK(hipEventRecord(e0, s));
            for (int i = 0; i < iters; ++i)
                vars[v].fn(s);
            CHK(hipEventRecord(e1, s));
            CHK(hipEventSynchronize(e1));
            float ms;
            CHK(hipEventElapsedTime(&ms, e0, e1));
            t[v].push_back(ms / iters);
        }
    printf("== %s\n%-34s %9s %9s %9s %7s\n", title, "variant", "ms(med)", "ms(min)", "GB/s",
           "frac8T");
    for (size_t v = 0; v < vars.size(); ++v) {
        std::sort(t[v].begin(), t[v].end());
        const double med = t[v][t[v].size() / 2];
        printf("%-34s %9.4f %9.4f %9.1f %7.3f\n", vars[v].name.c_str(), med, t[v][0],
               vars[v].bytes / med / 1e6, vars[v].bytes / med / 1e6 / 8000.0);
    }
    fflush(stdout);
}

/* Candidate multiply without the 255-way compare tree:
 * a wave takes R output rows at one dword per lane (16 lanes per stripe, 4
 * stripes per item), forms the doublings F*2^i (i < 8) of each staged input
 * once -- 3 XORs each in bit-sliced form (poly 0x11D), the rest renaming --
 * and for every row adds the doublings its coefficient selects, two bits at
 * a time: one XOR or XOR3 per plane per bit pair behind a uniform 4-way
 * branch.  Staging is ec_combine's (plane-major LDS tile, 8 stripes). */
__device__ __forceinline__ void kb_dbl(const u32 (&x)[8], u32 (&y)[8])
{
    y[0] = x[7];
    y[1] = x[0];
    y[2] = x[1] ^ x[7];
    y[3] = x[2] ^ x[7];
    y[4] = x[3] ^ x[7];
    y[5] = x[4];
    y[6] = x[5];
    y[7] = x[6];
}

template <int K, int NW, int R, bool NTS>
__global__ __launch_bounds__(NW * 64) void kb_combine_bp(const CombineArgs a)
{
    constexpr u32 T = 8;
    constexpr u32 NI = K * T * 32 / 64;
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const u32 tid = threadIdx.x;
    const u32 k = a.k;
    const uint64_t t0 = (uint64_t)blockIdx.x * T;
    const u32 wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const u32 lane = tid & 63u;
#pragma unroll
    for (u32 j = 0; j < (NI + NW - 1) / NW; ++j) {
        const u32 ins = j * NW + wave;
        if (ins >= NI)
            break;
        const u32 p = ins / (T / 2);
        if (p >= k)
            break;
        const u32 el = (ins * 64 + lane) % (T * 32);
        const u32 s = (el >> 2) % T;
        const uint64_t st = t0 + s;
        if (st < a.nstripes) {
            const u32 src = __builtin_amdgcn_readfirstlane((a.pat[p >> 2] >> ((p & 3u) * 8u)) & 0xFFu);
            const uint8_t *g = a.in_base[src] + st * a.in_stride + ((el >> 2) / T) * 64u +
                               (el & 3u) * 16u;
            __builtin_amdgcn_global_load_lds(
                (const __attribute__((address_space(1))) void *)g,
                (__attribute__((address_space(3))) void *)(lds + ins * 1024u), 16, 0, 0);
        }
    }
    __syncthreads();

    const u32 cs = lane >> 4, cc = lane & 15u;
    const u32 items = ((a.rows + R - 1) / R) * 2;
    for (u32 it = wave; it < items; it += NW) {
        const u32 r0 = (it >> 1) * R, s = (it & 1u) * 4u + cs;
        const uint8_t *col = lds + s * 64u + cc * 4u;
        u32 acc[R][8];
#pragma unroll
        for (int j = 0; j < R; ++j)
#pragma unroll
            for (int b = 0; b < 8; ++b)
                acc[j][b] = 0;
        for (u32 p = 0; p < k; ++p) {
            u32 d[8][8];
            const uint8_t *src = col + p * (T * ECD_CHUNK);
#pragma unroll
            for (int b = 0; b < 8; ++b)
                d[0][b] = *reinterpret_cast<const u32 *>(src + (u32)b * (T * 64u));
#pragma unroll
            for (int i = 1; i < 8; ++i)
                kb_dbl(d[i - 1], d[i]);
#pragma unroll
            for (int j = 0; j < R; ++j) {
                if (r0 + j >= a.rows)
                    break;
                const u32 c = __builtin_amdgcn_readfirstlane(
                    (a.pat[a.kw * (1 + r0 + j) + (p >> 2)] >> ((p & 3u) * 8u)) & 0xFFu);
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const u32 sel = (c >> (2 * q)) & 3u;
                    if (sel == 1) {
#pragma unroll
                        for (int b = 0; b < 8; ++b)
                            acc[j][b] ^= d[2 * q][b];
                    } else if (sel == 2) {
#pragma unroll
                        for (int b = 0; b < 8; ++b)
                            acc[j][b] ^= d[2 * q + 1][b];
                    } else if (sel == 3) {
#pragma unroll
                        for (int b = 0; b < 8; ++b)
                            acc[j][b] = ecgf::xor3(acc[j][b], d[2 * q][b], d[2 * q + 1][b]);
                    }
                }
            }
        }
        const uint64_t ost = t0 + s;
        if (ost < a.nstripes) {
#pragma unroll
            for (int j = 0; j < R; ++j)
                if (r0 + j < a.rows) {
                    uint8_t *o = a.out_base[r0 + j] + ost * a.out_stride + cc * 4u;
#pragma unroll
                    for (int b = 0; b < 8; ++b)
                        __builtin_nontemporal_store(acc[j][b], reinterpret_cast<u32 *>(o + b * 64));
                }
        }
    }
}

/* Candidate (r02z): persistent blocks with a double-buffered LDS tile.
 * ec_combine stages a tile, waits, computes and stores, so a CU's memory
 * pipe idles whenever its resident blocks all compute at once; at k = 16
 * only two 64 KiB tiles fit a CU.  Here one block per CU loops over tiles
 * t, t + grid, ...: the LDS-DMA loads of tile t+2G are issued into the
 * buffer tile t has just released, so every compute phase runs with the
 * next tile's loads (and this tile's stores) in flight.  The wait for tile
 * t's loads counts only what this wave issued after them (the stores of the
 * previous tile and the loads of the next): vector memory operations
 * complete in issue order on gfx9, so vmcnt(N) with N <= that count means
 * tile t has landed. */
__device__ __forceinline__ void kb_wait_vm_atmost(u32 n)
{
    /* s_waitcnt takes an immediate: pick the largest encodable bound <= n */
#define KB_VM(N) (((N) & 15) | (((N) >> 4) << 14) | (0x7 << 4) | (0xF << 8))
    if (n >= 24)
        __builtin_amdgcn_s_waitcnt(KB_VM(24));
    else if (n >= 16)
        __builtin_amdgcn_s_waitcnt(KB_VM(16));
    else if (n >= 12)
        __builtin_amdgcn_s_waitcnt(KB_VM(12));
    else if (n >= 8)
        __builtin_amdgcn_s_waitcnt(KB_VM(8));
    else if (n >= 4)
        __builtin_amdgcn_s_waitcnt(KB_VM(4));
    else if (n >= 2)
        __builtin_amdgcn_s_waitcnt(KB_VM(2));
    else
        __builtin_amdgcn_s_waitcnt(KB_VM(0));
#undef KB_VM
}

template <int K, int NW, bool NTS>
__global__ __launch_bounds__(NW * 64) void kb_combine_db(const CombineArgs a)
{
    constexpr u32 T = 8;
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const u32 tid = threadIdx.x;
    const u32 k = a.k;
    const u32 wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const u32 lane = tid & 63u;
    const u32 tile_bytes = k * T * ECD_CHUNK;
    const uint64_t ntiles = (a.nstripes + T - 1) / T;
    const u32 ni = k * (T / 2);                       /* wave instructions per tile */
    const PatWords<false> pw(a, 0u, lane, nullptr);
    /* stage tile `tl` into buffer `bf`; returns this wave's instruction count */
    auto stage = [&](uint64_t tl, u32 bf) -> u32 {
        u32 n = 0;
        for (u32 ins = wave; ins < ni; ins += NW) {
            const u32 p = ins / (T / 2);
            const u32 el = (ins * 64 + lane) % (T * 32);
            const u32 s = (el >> 2) % T;
            const uint64_t st = tl * T + s;
            /* past the data: re-read the last stripe (keeps the count uniform) */
            const uint64_t sc = st < a.nstripes ? st : a.nstripes - 1;
            const uint8_t *g = a.in_base[pw.byte(a, p)] + sc * a.in_stride +
                               ((el >> 2) / T) * 64u + (el & 3u) * 16u;
            __builtin_amdgcn_global_load_lds(
                (const __attribute__((address_space(1))) void *)g,
                (__attribute__((address_space(3))) void *)(lds + bf * tile_bytes + ins * 1024u),
                16, 0, 0);
            ++n;
        }
        return n;
    };
    uint64_t t = blockIdx.x;
    if (t >= ntiles)
        return;
    u32 after = 0;                                  /* ops issued after tile t's loads */
    stage(t, 0);
    if (t + gridDim.x < ntiles)
        after = stage(t + gridDim.x, 1);
    const u32 cs = lane >> 3, cc = lane & 7u;
    const u32 items = a.rows;
    for (u32 bf = 0; t < ntiles; t += gridDim.x, bf ^= 1u) {
        kb_wait_vm_atmost(after);
        __syncthreads();
        const uint8_t *base = lds + bf * tile_bytes;
        u32 nst = 0;
        for (u32 r = wave; r < items; r += NW) {
            const uint8_t *col = base + cs * 64u + cc * 8u;
            const u32 rw = a.kw * (1 + r);
            const u32 w0 = pw.word(a, rw);
            const u32 w1 = K > 4 ? pw.word(a, rw + 1) : 0u;
            const u32 w2 = K > 8 ? pw.word(a, rw + 2) : 0u;
            const u32 w3 = K > 12 ? pw.word(a, rw + 3) : 0u;
            u32 acc[8][2], y[8][2];
#pragma unroll
            for (int b = 0; b < 8; ++b)
                acc[b][0] = acc[b][1] = 0;
            uint64_t cl = (uint64_t)w0 | ((uint64_t)w1 << 32);
            uint64_t ch = (uint64_t)w2 | ((uint64_t)w3 << 32);
#pragma unroll 1
            for (u32 p = 0; p < k; ++p) {
                const u32 c = __builtin_amdgcn_readfirstlane((u32)cl & 0xFFu);
                cl = (cl >> 8) | (ch << 56);
                ch >>= 8;
                if (c == 0)
                    continue;
                const uint8_t *src = col + p * (T * ECD_CHUNK);
#pragma unroll
                for (int b = 0; b < 8; ++b)
                    load_plane<2>(src + (u32)b * (T * 64u), y[b]);
                ecgf::mul_xor_jt<2>(c, acc, y);
            }
            const uint64_t ost = t * T + cs;
            if (ost < a.nstripes)
                store_chunk<2, NTS>(a.out_base[r] + ost * a.out_stride + cc * 8u, acc);
            nst += 8;                                /* stores counted per wave */
        }
        __syncthreads();                             /* buffer bf is free */
        u32 nl = 0;
        if (t + 2ull * gridDim.x < ntiles)
            nl = stage(t + 2ull * gridDim.x, bf);
        /* next iteration waits for tile t+G, issued before these stores and loads */
        after = nst + nl;
    }
}

/* Candidate (r02z): ec_combine with the next input's LDS reads issued before
 * the current multiply (software pipelining), so the LDS latency overlaps
 * the dispatch and the body instead of heading every multiply.  The second
 * 16-VGPR input buffer fits the 64-VGPR budget (two 16-wave blocks per CU)
 * only with programs of at most 4 temporaries (gf8_asm_t4.h).  Zero
 * coefficients go through table entry 0 (a no-op body).  (Now also
 * ec_combine JT = 4.) */
template <int K, int NW, bool NTS>
__global__ __launch_bounds__(NW * 64) void kb_combine_pf(const CombineArgs a)
{
    constexpr u32 T = 8;
    constexpr u32 NI = K * T * 32 / 64;
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const u32 tid = threadIdx.x;
    const u32 k = a.k;
    const uint64_t t0 = (uint64_t)blockIdx.x * T;
    const u32 wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const u32 lane = tid & 63u;
    const PatWords<false> pw(a, 0u, lane, nullptr);
#pragma unroll
    for (u32 j = 0; j < (NI + NW - 1) / NW; ++j) {
        const u32 ins = j * NW + wave;
        if (ins >= NI)
            break;
        const u32 p = ins / (T / 2);
        if (p >= k)
            break;
        const u32 el = (ins * 64 + lane) % (T * 32);
        const u32 s = (el >> 2) % T;
        const uint64_t st = t0 + s;
        if (st < a.nstripes) {
            const uint8_t *g = a.in_base[pw.byte(a, p)] + st * a.in_stride +
                               ((el >> 2) / T) * 64u + (el & 3u) * 16u;
            __builtin_amdgcn_global_load_lds(
                (const __attribute__((address_space(1))) void *)g,
                (__attribute__((address_space(3))) void *)(lds + ins * 1024u), 16, 0, 0);
        }
    }
    __syncthreads();
    const u32 cs = lane >> 3, cc = lane & 7u;
    for (u32 r = wave; r < a.rows; r += NW) {
        const uint8_t *col = lds + cs * 64u + cc * 8u;
        const u32 rw = a.kw * (1 + r);
        const u32 w0 = pw.word(a, rw);
        const u32 w1 = K > 4 ? pw.word(a, rw + 1) : 0u;
        const u32 w2 = K > 8 ? pw.word(a, rw + 2) : 0u;
        const u32 w3 = K > 12 ? pw.word(a, rw + 3) : 0u;
        u32 acc[8][2], ya[8][2], yb[8][2], t[ECGF_ASM_TEMPS_T4][2];
#pragma unroll
        for (int b = 0; b < 8; ++b) {
            acc[b][0] = acc[b][1] = 0;
            load_plane<2>(col + (u32)b * (T * 64u), ya[b]);
        }
        uint64_t cl = (uint64_t)w0 | ((uint64_t)w1 << 32);
        uint64_t ch = (uint64_t)w2 | ((uint64_t)w3 << 32);
#pragma unroll 1
        for (u32 p = 0; p < k; ++p) {
            const u32 c = __builtin_amdgcn_readfirstlane((u32)cl & 0xFFu);
            cl = (cl >> 8) | (ch << 56);
            ch >>= 8;
            const uint8_t *nx = col + (p + 1 < k ? p + 1 : p) * (T * ECD_CHUNK);
#pragma unroll
            for (int b = 0; b < 8; ++b)
                load_plane<2>(nx + (u32)b * (T * 64u), yb[b]);
            ECGF_ASM_DISPATCH_W2_T4(acc, ya, t, c);
#pragma unroll
            for (int b = 0; b < 8; ++b) {
                ya[b][0] = yb[b][0];
                ya[b][1] = yb[b][1];
            }
        }
        const uint64_t ost = t0 + cs;
        if (ost < a.nstripes)
            store_chunk<2, NTS>(a.out_base[r] + ost * a.out_stride + cc * 8u, acc);
    }
}

/* Candidate (r02z): decode output assembled in LDS and written as the
 * tile's contiguous stripe-major run (8 stripes x k chunks, 16 B per lane,
 * 1 KiB per wave instruction) instead of 64-B plane segments at a k*512-B
 * stride straight from the registers (PMC: the headline decode writes ~4 %
 * more HBM bytes than it produces).  Needs out_stride == rows * 512 and
 * out_base[r] = out + r * 512 (a full decode), single pattern. */
template <int K, int NW, bool NTS>
__global__ __launch_bounds__(NW * 64) void kb_combine_ot(const CombineArgs a)
{
    constexpr u32 T = 8;
    constexpr u32 NI = K * T * 32 / 64;
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const u32 tid = threadIdx.x;
    const u32 k = a.k;
    const uint64_t t0 = (uint64_t)blockIdx.x * T;
    const u32 wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const u32 lane = tid & 63u;
    uint8_t *otile = lds + k * (T * ECD_CHUNK);      /* [stripe][row][512 B] */
    const PatWords<false> pw(a, 0u, lane, nullptr);
#pragma unroll
    for (u32 j = 0; j < (NI + NW - 1) / NW; ++j) {
        const u32 ins = j * NW + wave;
        if (ins >= NI)
            break;
        const u32 p = ins / (T / 2);
        if (p >= k)
            break;
        const u32 el = (ins * 64 + lane) % (T * 32);
        const u32 s = (el >> 2) % T;
        const uint64_t st = t0 + s;
        if (st < a.nstripes) {
            const uint8_t *g = a.in_base[pw.byte(a, p)] + st * a.in_stride +
                               ((el >> 2) / T) * 64u + (el & 3u) * 16u;
            __builtin_amdgcn_global_load_lds(
                (const __attribute__((address_space(1))) void *)g,
                (__attribute__((address_space(3))) void *)(lds + ins * 1024u), 16, 0, 0);
        }
    }
    __syncthreads();
    const u32 cs = lane >> 3, cc = lane & 7u;
    const u32 rows = a.rows;
    for (u32 r = wave; r < rows; r += NW) {
        const uint8_t *col = lds + cs * 64u + cc * 8u;
        const u32 rw = a.kw * (1 + r);
        const u32 w0 = pw.word(a, rw);
        const u32 w1 = K > 4 ? pw.word(a, rw + 1) : 0u;
        const u32 w2 = K > 8 ? pw.word(a, rw + 2) : 0u;
        const u32 w3 = K > 12 ? pw.word(a, rw + 3) : 0u;
        u32 acc[8][2], y[8][2];
#pragma unroll
        for (int b = 0; b < 8; ++b)
            acc[b][0] = acc[b][1] = 0;
        uint64_t cl = (uint64_t)w0 | ((uint64_t)w1 << 32);
        uint64_t ch = (uint64_t)w2 | ((uint64_t)w3 << 32);
#pragma unroll 1
        for (u32 p = 0; p < k; ++p) {
            const u32 c = __builtin_amdgcn_readfirstlane((u32)cl & 0xFFu);
            cl = (cl >> 8) | (ch << 56);
            ch >>= 8;
            if (c == 0)
                continue;
            const uint8_t *src = col + p * (T * ECD_CHUNK);
#pragma unroll
            for (int b = 0; b < 8; ++b)
                load_plane<2>(src + (u32)b * (T * 64u), y[b]);
            ecgf::mul_xor_jt<2>(c, acc, y);
        }
        uint8_t *o = otile + (cs * rows + r) * ECD_CHUNK + cc * 8u;
#pragma unroll
        for (int b = 0; b < 8; ++b)
            *reinterpret_cast<uint2 *>(o + b * 64) = make_uint2(acc[b][0], acc[b][1]);
    }
    __syncthreads();
    /* the tile's 8 stripes are one contiguous run of the output */
    const uint64_t nst = a.nstripes - t0 < T ? a.nstripes - t0 : T;
    const u32 pieces = (u32)nst * rows * (ECD_CHUNK / 16);
    uint8_t *dst = a.out_base[0] + t0 * a.out_stride;
    for (u32 i = tid; i < pieces; i += NW * 64) {
        const v4u v = *reinterpret_cast<const v4u *>(otile + i * 16u);
        if constexpr (NTS)
            __builtin_nontemporal_store(v, reinterpret_cast<v4u *>(dst + i * 16u));
        else
            *reinterpret_cast<v4u *>(dst + i * 16u) = v;
    }
}

/* decode k+r with the first r bricks missing, coefficients from the host
 * inverse (a dense k x k matrix is all we need for timing; correctness of
 * the math is covered by the parity tests -- here variants are compared
 * with each other). */
template <int K>
static void add_decode(std::vector<Variant> &vars, uint64_t nst, uint8_t *const *frags,
                       uint8_t *out, const uint8_t *coef)
{
    ecd_combine_desc_t d;
    memset(&d, 0, sizeof(d));
    d.k = K;
    d.rows = K;
    d.nstripes = nst;
    d.in_stride = ECD_CHUNK;
    d.out_stride = (uint64_t)K * ECD_CHUNK;
    for (int p = 0; p < K; ++p) {
        d.in_base[p] = frags[p];
        d.pat[p] = (uint8_t)p;
    }
    for (int r = 0; r < K; ++r)
        d.out_base[r] = out + (uint64_t)r * ECD_CHUNK;
    memcpy(d.pat + K, coef, K * K);
    d.npatterns = 1;
    d.pat_bytes = K + K * K;
    static CombineArgs a;
    if (ecdk_pack_args(&d, &a))
        exit(2);
    const double bytes = 2.0 * nst * K * ECD_CHUNK;
    const size_t ob = (size_t)nst * K * ECD_CHUNK;
    auto add = [&](const char *nm, auto kern, int ts, int nw) {
        const size_t lds = (size_t)K * 8 * ts * ECD_CHUNK;
        const uint64_t g = (nst + 8 * ts - 1) / (8 * ts);
        vars.push_back({nm, bytes, [=](hipStream_t s) {
                            hipLaunchKernelGGL(kern, dim3((u32)g), dim3(64 * nw), lds, s, a);
                        }, out, ob});
    };
    /* (GLDS / PF / register staging were measured here in r01a-c and
     * removed; the shipped kernel stages by LDS-DMA into a plane-major tile.
     * r02: the searched multiply programs of ec_gf8_prog.h ("CSE", the
     * default) against the round-1 per-plane trees ("naive"); the bit-pair
     * candidate kb_combine_bp lost in r01 and is no longer timed) */
    /* r02 (kbench_r02t.log and earlier): switch / naive / aligned / unrolled
     * variants retired; r02z: the whole-row asm block ("row") and grouped
     * waits ("split") were timed here (kbench_r02z_row.log, _split.log; code
     * in commit 87d127c) and retired */
    add("TS1 NW4 NTS jt", ec_combine<K, 1, 4, false, true, 2, false, true, 1>, 1, 4);
    add("TS1 NW8 NTS jt", ec_combine<K, 1, 8, false, true, 2, false, true, 1>, 1, 8);
    add("TS1 NW16 NTS jt", ec_combine<K, 1, 16, false, true, 2, false, true, 1>, 1, 16);
    /* r02z: output assembled in LDS, written as one contiguous run */
    auto addot = [&](const char *nm, auto kern, int nw) {
        const size_t lds = 2 * (size_t)K * 8 * ECD_CHUNK;
        CHK(hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)lds));
        const uint64_t g = (nst + 7) / 8;
        vars.push_back({nm, bytes, [=](hipStream_t s) {
                            hipLaunchKernelGGL(kern, dim3((u32)g), dim3(64 * nw), lds, s, a);
                        }, out, ob});
    };
    addot("TS1 NW8 NTS ot", kb_combine_ot<K, 8, true>, 8);
    addot("TS1 NW16 NTS ot", kb_combine_ot<K, 16, true>, 16);
    addot("TS1 NW8 ot (default stores)", kb_combine_ot<K, 8, false>, 8);
    /* r02z: next input's LDS reads issued before the current multiply */
    add("TS1 NW8 NTS pf", kb_combine_pf<K, 8, true>, 1, 8);
    add("TS1 NW16 NTS pf", kb_combine_pf<K, 16, true>, 1, 16);
    /* persistent double-buffered tiles: `bpc` blocks per CU */
    auto adddb = [&](const char *nm, auto kern, int nw, int bpc) {
        const size_t lds = 2 * (size_t)K * 8 * ECD_CHUNK;
        CHK(hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)lds));
        const uint64_t tiles = (nst + 7) / 8;
        const uint64_t g = std::min<uint64_t>(tiles, 256ull * bpc);
        vars.push_back({nm, bytes, [=](hipStream_t s) {
                            hipLaunchKernelGGL(kern, dim3((u32)g), dim3(64 * nw), lds, s, a);
                        }, out, ob});
    };
    if (K == 16) {
        adddb("db NW16 x1", kb_combine_db<K, 16, true>, 16, 1);
        adddb("db NW8 x1", kb_combine_db<K, 8, true>, 8, 1);
        adddb("db NW16 x2", kb_combine_db<K, 16, true>, 16, 2);
    } else if (K == 8) {
        adddb("db NW16 x1", kb_combine_db<K, 16, true>, 16, 1);
        adddb("db NW8 x2", kb_combine_db<K, 8, true>, 8, 2);
        adddb("db NW16 x2", kb_combine_db<K, 16, true>, 16, 2);
    } else {
        adddb("db NW8 x2", kb_combine_db<K, 8, true>, 8, 2);
        adddb("db NW8 x4", kb_combine_db<K, 8, true>, 8, 4);
        adddb("db NW16 x2", kb_combine_db<K, 16, true>, 16, 2);
    }
}

template <int K, int N, typename KF>
static void add_encode_w(std::vector<Variant> &vars, const char *nm, uint64_t nst,
                         const uint8_t *in, const FragPtrs &f, KF kern, int W)
{
    const double bytes = (double)nst * (K + N) * ECD_CHUNK;
    const uint64_t g = (nst * (16 / W) + kBlock - 1) / kBlock;
    vars.push_back({nm, bytes, [=](hipStream_t s) {
                        hipLaunchKernelGGL(kern, dim3((u32)g), dim3(kBlock), 0, s, in, f, nst);
                    }, f.p[N - 1], (size_t)nst * ECD_CHUNK});
}

/* GF(2^8) product, poly 0x11D (host side, for building coefficient rows) */
static uint8_t kb_gmul(uint8_t a, uint8_t b)
{
    uint8_t r = 0;
    while (b) {
        if (b & 1)
            r ^= a;
        a = (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1D : 0));
        b >>= 1;
    }
    return r;
}

/* Encode through the generic tile kernel (LDS-DMA staging, NT stores):
 * rows = n, coefficient (i+1)^(k-1-j) for input j (ec-method.c:22-36). */
template <int K, int N, int NW, bool NTS, bool DIRECT = false, int CW = 2>
static void add_encode_tile(std::vector<Variant> &vars, const char *nm, uint64_t nst,
                            const uint8_t *in, const FragPtrs &f)
{
    const size_t lds = (size_t)K * 8 * ECD_CHUNK;
    const uint64_t g = (nst + 7) / 8;
    vars.push_back({nm, (double)nst * (K + N) * ECD_CHUNK, [=](hipStream_t st) {
                        hipLaunchKernelGGL((ec_encode_tile<K, N, NW, NTS, DIRECT, CW>), dim3((u32)g),
                                           dim3(64 * NW), lds, st, in, f, nst);
                    }, f.p[N - 1], (size_t)nst * ECD_CHUNK});
}

template <int K, int NW, int JT>
static void add_encode_combine(std::vector<Variant> &vars, const char *nm, int n, uint64_t nst,
                               const uint8_t *in, const FragPtrs &f)
{
    ecd_combine_desc_t d;
    memset(&d, 0, sizeof(d));
    d.k = K;
    d.rows = n;
    d.nstripes = nst;
    d.in_stride = (uint64_t)K * ECD_CHUNK;
    d.out_stride = ECD_CHUNK;
    for (int p = 0; p < K; ++p) {
        d.in_base[p] = in + (uint64_t)p * ECD_CHUNK;
        d.pat[p] = (uint8_t)p;
    }
    for (int r = 0; r < n; ++r) {
        d.out_base[r] = f.p[r];
        uint8_t v = 1;
        for (int j = K - 1; j >= 0; --j) {      /* v = (r+1)^(K-1-j) */
            d.pat[K + r * K + j] = v;
            v = kb_gmul(v, (uint8_t)(r + 1));
        }
    }
    d.npatterns = 1;
    d.pat_bytes = K + n * K;
    CombineArgs *a = new CombineArgs;            /* kept for the process */
    if (ecdk_pack_args(&d, a))
        exit(5);
    const size_t lds = (size_t)K * 8 * ECD_CHUNK;
    const uint64_t g = (nst + 7) / 8;
    const CombineArgs *ap = a;
    vars.push_back({nm, (double)nst * (K + n) * ECD_CHUNK, [=](hipStream_t st) {
                        hipLaunchKernelGGL((ec_combine<K, 1, NW, false, true, 2, false, true, JT>),
                                           dim3((u32)g), dim3(64 * NW), lds, st, *ap);
                    }, f.p[n - 1], (size_t)nst * ECD_CHUNK});
}

int main(int argc, char **argv)
{
    const double gib = argc > 1 ? atof(argv[1]) : 1.0;
    const int rounds = argc > 2 ? atoi(argv[2]) : 7;
    const int iters = 10;
    hipDeviceProp_t prop;
    CHK(hipGetDeviceProperties(&prop, 0));
    printf("device %s CUs %d, %.2f GiB user data per launch\n", prop.gcnArchName,
           prop.multiProcessorCount, gib);
    hipStream_t s;
    CHK(hipStreamCreate(&s));
    const uint64_t user = (uint64_t)(gib * (1ull << 30));
    uint8_t *bufA, *bufB;
    CHK(hipMalloc(&bufA, user * 3));   /* inputs / fragments */
    CHK(hipMalloc(&bufB, user * 3));   /* outputs */
    fill(bufA, user * 3, 12345);

    {   /* calibration */
        std::vector<Variant> v;
        const size_t n16 = user / 16;
        const int grid = prop.multiProcessorCount * 8;
        u32 *sink = reinterpret_cast<u32 *>(bufB + user * 3 - 64);
        v.push_back({"copy uint4", 2.0 * user, [=](hipStream_t st) {
                         hipLaunchKernelGGL(k_copy, dim3(grid), dim3(256), 0, st,
                                            (const uint4 *)bufA, (uint4 *)bufB, n16);
                     }, nullptr, 0});
        v.push_back({"copy uint4 NT", 2.0 * user, [=](hipStream_t st) {
                         hipLaunchKernelGGL(k_copy_nt, dim3(grid), dim3(256), 0, st,
                                            (const uint4 *)bufA, (uint4 *)bufB, n16);
                     }, nullptr, 0});
        v.push_back({"read-only", 1.0 * user, [=](hipStream_t st) {
                         hipLaunchKernelGGL(k_read, dim3(grid), dim3(256), 0, st,
                                            (const uint4 *)bufA, n16, sink);
                     }, nullptr, 0});
        v.push_back({"write-only", 1.0 * user, [=](hipStream_t st) {
                         hipLaunchKernelGGL(k_write, dim3(grid), dim3(256), 0, st, (uint4 *)bufB,
                                            n16);
                     }, nullptr, 0});
        const size_t nch = user / 512;
        const u32 sg = (u32)((nch * 8 + 255) / 256);
        v.push_back({"read-only 64B segs", 1.0 * user, [=](hipStream_t st) {
                         hipLaunchKernelGGL(k_read_seg, dim3(sg), dim3(256), 0, st,
                                            (const uint8_t *)bufA, nch, sink);
                     }, nullptr, 0});
        v.push_back({"write-only 64B segs", 1.0 * user, [=](hipStream_t st) {
                         hipLaunchKernelGGL(k_write_seg, dim3(sg), dim3(256), 0, st, bufB, nch);
                     }, nullptr, 0});
        run_group("HBM calibration", v, rounds, iters, s);
    }
    if (!getenv("KB_NO_DECODE")) {   /* 4+2 decode */
        const uint64_t nst = user / (4 * ECD_CHUNK);
        uint8_t *fr[4];
        for (int p = 0; p < 4; ++p)
            fr[p] = bufA + (uint64_t)p * nst * ECD_CHUNK;
        const uint8_t inv[16] = {0xcb, 0x5d, 0xdd, 0x4b, 0x4b, 0x00, 0xdd, 0x96,
                                 0xa7, 0x8c, 0x03, 0x28, 0xd2, 0xd5, 0x04, 0x02};
        std::vector<Variant> v;
        add_decode<4>(v, nst, fr, bufB, inv);
        run_group("decode 4+2 mask 0x3C", v, rounds, iters, s);
    }
    if (!getenv("KB_NO_DECODE")) {   /* 8+4 decode: a dense pseudo-random nonzero matrix */
        const uint64_t nst = user / (8 * ECD_CHUNK);
        uint8_t *fr[8];
        for (int p = 0; p < 8; ++p)
            fr[p] = bufA + (uint64_t)p * nst * ECD_CHUNK;
        uint8_t c[64];
        for (int i = 0; i < 64; ++i)
            c[i] = (uint8_t)(1 + (i * 97 + 31) % 255);
        std::vector<Variant> v;
        add_decode<8>(v, nst, fr, bufB, c);
        run_group("decode 8+4 dense", v, rounds, iters, s);
    }
    if (!getenv("KB_NO_DECODE")) {   /* 8+4 fused heal shape: k = 8 inputs, 4 output rows */
        const int K = 8, RW = 4;
        const uint64_t nst = user / (K * ECD_CHUNK);
        ecd_combine_desc_t d;
        memset(&d, 0, sizeof(d));
        d.k = K;
        d.rows = RW;
        d.nstripes = nst;
        d.in_stride = ECD_CHUNK;
        d.out_stride = ECD_CHUNK;
        for (int p = 0; p < K; ++p) {
            d.in_base[p] = bufA + (uint64_t)p * nst * ECD_CHUNK;
            d.pat[p] = (uint8_t)p;
        }
        for (int r = 0; r < RW; ++r)
            d.out_base[r] = bufB + (uint64_t)r * nst * ECD_CHUNK;
        for (int i = 0; i < RW * K; ++i)
            d.pat[K + i] = (uint8_t)(1 + (i * 97 + 31) % 255);
        d.npatterns = 1;
        d.pat_bytes = K + RW * K;
        static CombineArgs a;
        if (ecdk_pack_args(&d, &a))
            exit(4);
        const double bytes = (double)nst * (K + RW) * ECD_CHUNK;
        const size_t lds = (size_t)K * 8 * ECD_CHUNK;
        const uint64_t g = (nst + 7) / 8;
        std::vector<Variant> v;
        auto addh = [&](const char *nm, auto kern, int nw) {
            v.push_back({nm, bytes, [=](hipStream_t st) {
                             hipLaunchKernelGGL(kern, dim3((u32)g), dim3(64 * nw), lds, st, a);
                         }, bufB, (size_t)nst * RW * ECD_CHUNK});
        };
        addh("heal NW4 NTS", ec_combine<K, 1, 4, false, true>, 4);
        addh("heal NW4 NTS naive", ec_combine<K, 1, 4, false, true, 2, false, false>, 4);
        addh("heal NW4 NTS jt", ec_combine<K, 1, 4, false, true, 2, false, true, 1>, 4);
        addh("heal NW8 NTS", ec_combine<K, 1, 8, false, true>, 8);
        addh("heal NW16 NTS", ec_combine<K, 1, 16, false, true>, 16);
        run_group("heal 8+4 (regenerate 4 rows)", v, rounds, iters, s);
    }
    if (!getenv("KB_NO_DECODE")) {   /* 16+4 decode, dense */
        const uint64_t nst = user / (16 * ECD_CHUNK);
        uint8_t *fr[16];
        for (int p = 0; p < 16; ++p)
            fr[p] = bufA + (uint64_t)p * nst * ECD_CHUNK;
        uint8_t c[256];
        for (int i = 0; i < 256; ++i)
            c[i] = (uint8_t)(1 + (i * 173 + 11) % 255);
        std::vector<Variant> v;
        add_decode<16>(v, nst, fr, bufB, c);
        run_group("decode 16+4 dense", v, rounds, iters, s);
    }
    if (!getenv("KB_NO_DECODE")) {   /* 8+4 mixed: 16 random dense patterns over 12 fragments, 1024-stripe groups */
        const int K = 8, N = 12, NP = 16;
        const uint64_t nst = user / (K * ECD_CHUNK);
        ecd_combine_desc_t d;
        memset(&d, 0, sizeof(d));
        d.k = K;
        d.rows = K;
        d.nstripes = nst;
        d.in_stride = ECD_CHUNK;
        d.out_stride = (uint64_t)K * ECD_CHUNK;
        for (int f = 0; f < N; ++f)
            d.in_base[f] = bufA + (uint64_t)f * nst * ECD_CHUNK * 2 / 3;
        for (int r = 0; r < K; ++r)
            d.out_base[r] = bufB + (uint64_t)r * ECD_CHUNK;
        d.npatterns = NP;
        d.pat_bytes = K + K * K;
        uint32_t x = 7;
        for (int q = 0; q < NP; ++q) {
            uint8_t *pp = d.pat + q * d.pat_bytes;
            int used = 0;
            for (int f = 0; f < N && used < K; ++f) {        /* k of the n bricks */
                x = x * 1103515245u + 12345u;
                if ((int)((x >> 16) % (N - f)) < K - used)
                    pp[used++] = (uint8_t)f;
            }
            for (int i = 0; i < K * K; ++i) {
                x = x * 1103515245u + 12345u;
                pp[K + i] = (uint8_t)(1 + (x >> 16) % 255);
            }
        }
        const uint64_t ngroups = (nst + 1023) / 1024;
        std::vector<uint8_t> gp(ngroups);
        for (auto &g : gp) {
            x = x * 1103515245u + 12345u;
            g = (uint8_t)((x >> 16) % NP);
        }
        uint8_t *dgp;
        CHK(hipMalloc(&dgp, ngroups));
        CHK(hipMemcpy(dgp, gp.data(), ngroups, hipMemcpyHostToDevice));
        d.group_pattern = dgp;
        d.group_shift = 10;
        static CombineArgs a;
        if (ecdk_pack_args(&d, &a))
            exit(3);
        const double bytes = 2.0 * nst * K * ECD_CHUNK;
        std::vector<Variant> v;
        const size_t lds = (size_t)K * 8 * ECD_CHUNK;
        const uint64_t g = (nst + 7) / 8;
        auto addm = [&](const char *nm, auto kern, int nw) {
            v.push_back({nm, bytes, [=](hipStream_t st) {
                             hipLaunchKernelGGL(kern, dim3((u32)g), dim3(64 * nw), lds, st, a);
                         }, bufB, (size_t)nst * K * ECD_CHUNK});
        };
        addm("mixed TS1 NW4 NTS", ec_combine<K, 1, 4, true, true>, 4);
        addm("mixed TS1 NW8 NTS naive", ec_combine<K, 1, 8, true, true, 2, false, false>, 8);
        addm("mixed TS1 NW8 NTS jt", ec_combine<K, 1, 8, true, true, 2, false, true, 1>, 8);
        addm("mixed TS1 NW4 NTS jt", ec_combine<K, 1, 4, true, true, 2, false, true, 1>, 4);
        addm("mixed TS1 NW8 NTS", ec_combine<K, 1, 8, true, true>, 8);
        addm("mixed TS1 NW16 NTS", ec_combine<K, 1, 16, true, true>, 16);
        run_group("decode 8+4 mixed (16 patterns, 1024-stripe groups)", v, rounds, iters, s);
    }
    if (!getenv("KB_NO_ENCODE")) {   /* encode 4+2, 8+4, 16+4: shipped W/NTS, CSE vs naive */
        auto frag_ptrs = [&](uint64_t nst, int n) {
            FragPtrs f;
            for (int i = 0; i < n; ++i)
                f.p[i] = bufB + (uint64_t)i * nst * ECD_CHUNK;
            return f;
        };
        std::vector<Variant> v;
        uint64_t nst = user / (4 * ECD_CHUNK);
        FragPtrs f = frag_ptrs(nst, 6);
        add_encode_w<4, 6>(v, "enc 4+2 W2", nst, bufA, f, ec_encode_vander<4, 6, 2, false>, 2);
        add_encode_w<4, 6>(v, "enc 4+2 W2 naive", nst, bufA, f,
                           ec_encode_vander<4, 6, 2, false, false>, 2);
        add_encode_w<4, 6>(v, "enc 4+2 W2 NTS", nst, bufA, f, ec_encode_vander<4, 6, 2, true>, 2);
        add_encode_combine<4, 8, 1>(v, "enc 4+2 tile NW8 jt", 6, nst, bufA, f);
        add_encode_combine<4, 16, 1>(v, "enc 4+2 tile NW16 jt", 6, nst, bufA, f);
        add_encode_tile<4, 6, 16, true>(v, "enc 4+2 vtile NW16 NTS", nst, bufA, f);
        add_encode_tile<4, 6, 16, true, true>(v, "enc 4+2 vtile NW16 NTS direct", nst, bufA, f);
        add_encode_tile<4, 6, 16, true, false, 1>(v, "enc 4+2 vtile NW16 NTS CW1", nst, bufA, f);
        add_encode_tile<4, 6, 16, true, true, 1>(v, "enc 4+2 vtile NW16 NTS direct CW1", nst, bufA, f);
        add_encode_tile<4, 6, 8, true, true, 1>(v, "enc 4+2 vtile NW8 NTS direct CW1", nst, bufA, f);
        run_group("encode 4+2", v, rounds, iters, s);
        v.clear();
        nst = user / (8 * ECD_CHUNK);
        f = frag_ptrs(nst, 12);
        add_encode_w<8, 12>(v, "enc 8+4 W1 NTS", nst, bufA, f, ec_encode_vander<8, 12, 1, true>, 1);
        add_encode_w<8, 12>(v, "enc 8+4 W1 NTS naive", nst, bufA, f,
                            ec_encode_vander<8, 12, 1, true, false>, 1);
        add_encode_w<8, 12>(v, "enc 8+4 W2 NTS", nst, bufA, f, ec_encode_vander<8, 12, 2, true>, 2);
        add_encode_combine<8, 8, 1>(v, "enc 8+4 tile NW8 jt", 12, nst, bufA, f);
        add_encode_combine<8, 16, 1>(v, "enc 8+4 tile NW16 jt", 12, nst, bufA, f);
        add_encode_tile<8, 12, 16, true>(v, "enc 8+4 vtile NW16 NTS", nst, bufA, f);
        add_encode_tile<8, 12, 16, true, true>(v, "enc 8+4 vtile NW16 NTS direct", nst, bufA, f);
        add_encode_tile<8, 12, 16, true, false, 1>(v, "enc 8+4 vtile NW16 NTS CW1", nst, bufA, f);
        add_encode_tile<8, 12, 16, true, true, 1>(v, "enc 8+4 vtile NW16 NTS direct CW1", nst, bufA, f);
        run_group("encode 8+4", v, rounds, iters, s);
        v.clear();
        {   /* configs[2]: one 64K-stripe batch */
            const uint64_t n64 = 65536;
            add_encode_w<8, 12>(v, "enc 8+4 64K W1 NTS", n64, bufA, f,
                                ec_encode_vander<8, 12, 1, true>, 1);
            add_encode_combine<8, 16, 1>(v, "enc 8+4 64K tile NW16 jt", 12, n64, bufA, f);
            add_encode_combine<8, 8, 1>(v, "enc 8+4 64K tile NW8 jt", 12, n64, bufA, f);
            add_encode_tile<8, 12, 16, true, true, 2>(v, "enc 8+4 64K vtile NW16 NTS direct", n64, bufA, f);
            add_encode_tile<8, 12, 16, true, true, 1>(v, "enc 8+4 64K vtile NW16 NTS direct CW1", n64, bufA, f);
            run_group("encode 8+4, 64K stripes", v, rounds, iters, s);
        }
        v.clear();
        nst = user / (16 * ECD_CHUNK);
        f = frag_ptrs(nst, 20);
        add_encode_w<16, 20>(v, "enc 16+4 W1 NTS", nst, bufA, f, ec_encode_vander<16, 20, 1, true>, 1);
        add_encode_w<16, 20>(v, "enc 16+4 W1 NTS naive", nst, bufA, f,
                             ec_encode_vander<16, 20, 1, true, false>, 1);
        add_encode_combine<16, 16, 1>(v, "enc 16+4 tile NW16 jt", 20, nst, bufA, f);
        add_encode_tile<16, 20, 10, true>(v, "enc 16+4 vtile NW10 NTS", nst, bufA, f);
        add_encode_tile<16, 20, 10, true, true>(v, "enc 16+4 vtile NW10 NTS direct", nst, bufA, f);
        add_encode_tile<16, 20, 10, true, false, 1>(v, "enc 16+4 vtile NW10 NTS CW1", nst, bufA, f);
        add_encode_tile<16, 20, 16, true, false, 1>(v, "enc 16+4 vtile NW16 NTS CW1", nst, bufA, f);
        add_encode_tile<16, 20, 16, true, true, 1>(v, "enc 16+4 vtile NW16 NTS direct CW1", nst, bufA, f);
        add_encode_tile<16, 20, 16, true, true, 2>(v, "enc 16+4 vtile NW16 NTS direct", nst, bufA, f);
        /* r02z: single ds_read_b64 per plane (256 B/clk) instead of read2 (128)
         * was timed here and retired: kbench_r02z_b64.log, commit 2a288b0 */
        /* r02z: row groups (RB rows per wave item sharing each LDS read) were
         * timed here and retired: kbench_r02z_rb.log, code in commit 822a197 */
        run_group("encode 16+4", v, rounds, iters, s);
    }
    if (!getenv("KB_NO_RMW")) {   /* partial-stripe write: interior stripes read at an odd address */
        std::vector<Variant> v;
        const uint64_t nst = user / (4 * ECD_CHUNK);
        FragPtrs f;
        for (int i = 0; i < 6; ++i)
            f.p[i] = bufB + (uint64_t)i * nst * ECD_CHUNK;
        const uint8_t *edge = bufA + 2 * user;
        const uint8_t *ush = bufA + 777;
        const double bytes = (double)nst * (4 + 6) * ECD_CHUNK;
        const uint64_t g = (nst * 8 + kBlock - 1) / kBlock;
        auto addr = [&](const char *nm, auto kern) {
            v.push_back({nm, bytes, [=](hipStream_t st) {
                             hipLaunchKernelGGL(kern, dim3((u32)g), dim3(kBlock), 0, st, edge, ush,
                                                f, nst);
                         }, f.p[5], (size_t)nst * ECD_CHUNK});
        };
        addr("rmw 4+2 W2 unaligned x2", ec_encode_vander_rmw<4, 6, 2, 0>);
        addr("rmw 4+2 W2 realign x3", ec_encode_vander_rmw<4, 6, 2, 1>);
        /* (different input bytes: reported as a MISMATCH, timing only) */
        add_encode_w<4, 6>(v, "enc 4+2 W2 (aligned input)", nst, bufA, f,
                           ec_encode_vander<4, 6, 2, false>, 2);
        run_group("partial write 4+2 (odd address)", v, rounds, iters, s);
    }
    if (!getenv("KB_NO_RMW")) {   /* the same for 8+4 and 16+4 (W = 1: one dword per plane per lane) */
        auto wide = [&](auto kk, auto nn, const char *title, auto k0, auto k1) {
            constexpr int K = decltype(kk)::value, N = decltype(nn)::value;
            std::vector<Variant> v;
            const uint64_t nst = user / (K * ECD_CHUNK);
            FragPtrs f;
            for (int i = 0; i < N; ++i)
                f.p[i] = bufB + (uint64_t)i * nst * ECD_CHUNK;
            const uint8_t *edge = bufA + 2 * user;
            const uint8_t *ush = bufA + 777;
            const double bytes = (double)nst * (K + N) * ECD_CHUNK;
            const uint64_t g = (nst * 16 + kBlock - 1) / kBlock;
            auto addr = [&](const char *nm, auto kern) {
                v.push_back({nm, bytes, [=](hipStream_t st) {
                                 hipLaunchKernelGGL(kern, dim3((u32)g), dim3(kBlock), 0, st, edge,
                                                    ush, f, nst);
                             }, f.p[N - 1], (size_t)nst * ECD_CHUNK});
            };
            addr("rmw W1 unaligned x1", k0);
            addr("rmw W1 realign x2", k1);
            run_group(title, v, rounds, iters, s);
        };
        wide(std::integral_constant<int, 8>{}, std::integral_constant<int, 12>{},
             "partial write 8+4 (odd address)", ec_encode_vander_rmw<8, 12, 1, 0>,
             ec_encode_vander_rmw<8, 12, 1, 1>);
        wide(std::integral_constant<int, 16>{}, std::integral_constant<int, 20>{},
             "partial write 16+4 (odd address)", ec_encode_vander_rmw<16, 20, 1, 0>,
             ec_encode_vander_rmw<16, 20, 1, 1>);
    }
    return 0;
}
