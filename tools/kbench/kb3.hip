/*
 * kb3.hip -- round-3 development harness (not product): A/B of the
 * narrow-tile kernels (ec_encode_tile_t, ec_combine_n) against the shipped
 * instantiations, in ONE process with interleaved rounds and the median of
 * rounds; every variant's output is compared with its group's first.
 *
 *   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I glusterfs_amd/csrc \
 *         tools/kbench/kb3.hip -o tools/kbench/kb3
 *   tools/kbench/kb3 [GiB=1] [rounds=7] [groups=all|enc16,enc8,...]
 */
#include "../../glusterfs_amd/csrc/ec_kernels.hip"

/* ec_device.hip's error record, which the launchers call (not linked here) */
extern "C" int ecd_hip_fail(const char *, int) { return -EIO; }
#ifdef KB3_WITH_JIT
extern "C" int ecj_lds_pad_kb;
#else
/* the run-time compiled kernels (ec_jit.hip) are not part of this harness
 * unless it is built with them (-DKB3_WITH_JIT ../../glusterfs_amd/csrc/ec_jit.hip -ldl) */
extern "C" int ecj_eligible(const ecd_combine_desc_t *) { return 0; }
extern "C" int ecj_launch(hipStream_t, const ecd_combine_desc_t *, int) { return -EAGAIN; }
#endif

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

struct Variant {
    std::string name;
    double bytes;
    std::function<void(hipStream_t)> fn;
    uint8_t *out;
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
            for (int i = 0; i < 3; ++i)
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
    printf("== %s\n%-40s %9s %9s %9s %7s\n", title, "variant", "ms(med)", "ms(min)", "GB/s",
           "frac8T");
    for (size_t v = 0; v < vars.size(); ++v) {
        std::sort(t[v].begin(), t[v].end());
        const double med = t[v][t[v].size() / 2];
        printf("%-40s %9.4f %9.4f %9.1f %7.3f\n", vars[v].name.c_str(), med, t[v][0],
               vars[v].bytes / med / 1e6, vars[v].bytes / med / 1e6 / 8000.0);
    }
    fflush(stdout);
    CHK(hipEventDestroy(e0));
    CHK(hipEventDestroy(e1));
}

static bool want(const char *groups, const char *g)
{
    if (!groups || !strcmp(groups, "all"))
        return true;
    std::string s = std::string(",") + groups + ",";
    return s.find(std::string(",") + g + ",") != std::string::npos;
}

static void lds_attr(const void *kern, size_t bytes)
{
    if (bytes > (64u << 10))
        CHK(hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes));
}

static FragPtrs frag_ptrs(uint8_t *b, uint64_t nst, int n)
{
    FragPtrs f;
    for (int i = 0; i < n; ++i)
        f.p[i] = b + (uint64_t)i * nst * ECD_CHUNK;
    return f;
}

/* The round-2 baselines these kernels were first timed against (the 8-stripe
 * encoders / ec_combine dispatch) left the library when the narrow kernels
 * shipped; their numbers are in profiles/kb3_r03d.log.  "shipped" below is
 * the library's current dispatch. */
static int encode_shipped(hipStream_t st, int k, int n, uint64_t nst, const uint8_t *in,
                          void *const *o)
{
    return ecdk_encode_vander(st, k, n, nst, in, o, false);
}

static void add_shipped_encode(std::vector<Variant> &v, const char *nm, int k, int n,
                               uint64_t nst, const uint8_t *in, FragPtrs f)
{
    v.push_back({nm, (double)nst * (k + n) * ECD_CHUNK, [=](hipStream_t st) {
                     void *o[ECD_MAX_ROWS];
                     for (int i = 0; i < n; ++i)
                         o[i] = f.p[i];
                     if (encode_shipped(st, k, n, nst, in, o))
                         exit(7);
                 }, f.p[n - 1], (size_t)nst * ECD_CHUNK});
}

template <int K, int N, int T, int NW, bool DIRECT, bool WOT>
static void add_tile_t(std::vector<Variant> &v, const char *nm, uint64_t nst, const uint8_t *in,
                       FragPtrs f)
{
    auto kern = ec_encode_tile_t<K, N, T, NW, true, DIRECT, WOT>;
    const size_t lds = encode_tile_t_lds<T, NW, WOT>(K);
    lds_attr((const void *)kern, lds);
    const uint64_t g = (nst + T - 1) / T;
    v.push_back({nm, (double)nst * (K + N) * ECD_CHUNK, [=](hipStream_t st) {
                     hipLaunchKernelGGL(kern, dim3((u32)g), dim3(64 * NW), lds, st, EncSrc{in, nullptr}, f, nst);
                 }, f.p[N - 1], (size_t)nst * ECD_CHUNK});
}

template <int K, int N, int T, int RB, bool WOT>
static void add_tile_rb(std::vector<Variant> &v, const char *nm, uint64_t nst, const uint8_t *in,
                        FragPtrs f)
{
    auto kern = ec_encode_tile_rb<K, N, T, RB, true, WOT>;
    const size_t lds = encode_tile_rb_lds<N, T, RB, WOT>(K);
    lds_attr((const void *)kern, lds);
    const uint64_t g = (nst + T - 1) / T;
    constexpr int NW = (N / RB) * (T / 4);
    v.push_back({nm, (double)nst * (K + N) * ECD_CHUNK, [=](hipStream_t st) {
                     hipLaunchKernelGGL(kern, dim3((u32)g), dim3(64 * NW), lds, st, EncSrc{in, nullptr}, f, nst);
                 }, f.p[N - 1], (size_t)nst * ECD_CHUNK});
}

/* Compile-time decode matrix (the kb3 dense coefficients below, c = 1 + (i *
 * 173 + 11) % 255 for i = r * K + p): how fast would a combine be without the
 * run-time multiply dispatch (a per-matrix JIT kernel)?  T stripes per tile,
 * CW = T / 4 dwords per plane per lane, one row per wave item. */
constexpr u32 ct_coef(int i) { return (u32)(1 + (i * 173 + 11) % 255); }

template <int K, int R, int T>
__device__ __forceinline__ void ct_row(const uint8_t *col, u32 (&acc)[8][T / 4])
{
    constexpr int CW = T / 4;
    u32 y[8][CW], nx[8][CW];
#pragma unroll
    for (int b = 0; b < 8; ++b)
#pragma unroll
        for (int w = 0; w < CW; ++w)
            acc[b][w] = 0;
#pragma unroll
    for (int b = 0; b < 8; ++b)
        load_plane<CW>(col + (u32)b * (T * 64u), nx[b]);
    static_for<0, K>([&](auto P) {
        constexpr int p = decltype(P)::value;
#pragma unroll
        for (int b = 0; b < 8; ++b)
#pragma unroll
            for (int w = 0; w < CW; ++w)
                y[b][w] = nx[b][w];
        if constexpr (p + 1 < K) {
#pragma unroll
            for (int b = 0; b < 8; ++b)
                load_plane<CW>(col + (u32)(p + 1) * (T * ECD_CHUNK) + (u32)b * (T * 64u), nx[b]);
        }
        __builtin_amdgcn_sched_barrier(0);
        ecgf::mul_xor<ct_coef(R * K + p), CW, true>(acc, acc, y);
        __builtin_amdgcn_sched_barrier(0);
    });
}

template <int K, int T, int NW, bool WOT>
__global__ __launch_bounds__(NW * 64) void kb_combine_ct(const CombineArgs a)
{
    constexpr int CW = T / 4;
    constexpr u32 LPS = 16 / CW;
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const u32 tid = threadIdx.x;
    const uint64_t t0 = (uint64_t)blockIdx.x * T;
    const u32 wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const u32 lane = tid & 63u;
    stage_tile<T, NW>(lds, [&](u32 p, uint64_t st) {
        return a.in_base[p] + st * a.in_stride;
    }, K, t0, a.nstripes, wave, lane);
    __syncthreads();
    const u32 cs = lane / LPS, cc = lane % LPS;
    const uint8_t *col = lds + cs * 64u + cc * (4u * CW);
    uint8_t *slice = lds + K * T * ECD_CHUNK + wave * T * ECD_CHUNK;
    for (u32 r = wave; r < (u32)K; r += NW) {
        const u32 ru = __builtin_amdgcn_readfirstlane(r);
        static_for<0, K>([&](auto R) {
            if (ru == (u32)decltype(R)::value) {
                u32 acc[8][CW];
                ct_row<K, decltype(R)::value, T>(col, acc);
                uint8_t *row = a.out_base[ru];
                if constexpr (WOT) {
                    store_chunks_via_lds<T, CW, true>(slice, acc, cs, cc, lane, [&](u32 s) {
                        return t0 + s < a.nstripes ? row + (t0 + s) * a.out_stride : nullptr;
                    });
                } else if (t0 + cs < a.nstripes) {
                    store_chunk<CW, true>(row + (t0 + cs) * a.out_stride + cc * (4u * CW), acc);
                }
            }
        });
    }
}

template <int K, int T, int NW, bool WOT>
static void add_combine_ct(std::vector<Variant> &v, const char *nm, const CombineArgs *a,
                           double bytes, uint8_t *out, size_t ob)
{
    auto kern = kb_combine_ct<K, T, NW, WOT>;
    const size_t lds = (size_t)K * T * ECD_CHUNK + (WOT ? (size_t)NW * T * ECD_CHUNK : 0);
    lds_attr((const void *)kern, lds);
    const uint64_t g = (a->nstripes + T - 1) / T;
    v.push_back({nm, bytes, [=](hipStream_t st) {
                     hipLaunchKernelGGL(kern, dim3((u32)g), dim3(64 * NW), lds, st, *a);
                 }, out, ob});
}

/* r06: the whole-matrix program of ONE fixed 16 x 16
 * decode matrix (kb3's dense ct_coef matrix), four-Russians over 4-plane
 * groups with the sub-sums shared by all 128 output planes
 * (tools/gen/gen_wm16.py -> kb_wm16.h: 2381 instructions per dword column
 * against 3290 for the row-by-row programs).  One 4-stripe tile per block
 * (32 KiB of LDS, staged by LDS-DMA like the shipped kernels); each lane
 * owns one dword column of the 4 stripes.  NWV = 1: one wave runs all 16
 * rows (128 accumulators); NWV = 2: two waves run 8 rows each (the tables
 * built twice, 2725 instructions).  The outputs of a full decode are one
 * contiguous 32 KiB run per tile (stripe-major), so they go back through
 * the tile's LDS and leave as 16-byte lane stores.  MODE 1: compute only
 * (no staging, no stores) -- the time of the program itself. */
#include "kb_wm16.h"

template <int NWV, int MODE, int LA>
__global__ __launch_bounds__(NWV * 64) void kb_combine_wm(const CombineArgs a)
{
    constexpr int T = 4;
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const u32 tid = threadIdx.x;
    const uint64_t t0 = (uint64_t)blockIdx.x * T;
    const u32 wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const u32 lane = tid & 63u;
    if constexpr (MODE == 0)
        stage_tile<T, NWV, LA>(lds, [&](u32 p, uint64_t st) {
            return a.in_base[p] + st * a.in_stride;
        }, 16, t0, a.nstripes, wave, lane);
    __syncthreads();
    const u32 cs = lane >> 4, cc = lane & 15u;
    const uint8_t *col = lds + cs * 64u + cc * 4u;
    uint8_t *ob = lds + cs * 8192u + cc * 4u;
    if constexpr (NWV == 1) {
        u32 acc[128];
        wm16_rows16<T>(col, acc);
        if constexpr (MODE == 1) {
            u32 x = 0;
#pragma unroll
            for (int o = 0; o < 128; ++o)
                x ^= acc[o];
            if (x == 0x9E3779B9u)             /* keeps the program live */
                *reinterpret_cast<u32 *>(a.out_base[0]) = x;
            return;
        }
        /* LDS operations of one wave run in order: the input tile is read
         * before it is overwritten */
#pragma unroll
        for (int o = 0; o < 128; ++o)
            *reinterpret_cast<u32 *>(ob + (o >> 3) * 512u + (o & 7) * 64u) = acc[o];
    } else {
        u32 acc[64];
        if (wave == 0)
            wm16_rows_lo<T>(col, acc);
        else
            wm16_rows_hi<T>(col, acc);
        if constexpr (MODE == 1) {
            u32 x = 0;
#pragma unroll
            for (int o = 0; o < 64; ++o)
                x ^= acc[o];
            if (x == 0x9E3779B9u)
                *reinterpret_cast<u32 *>(a.out_base[0]) = x;
            return;
        }
        __syncthreads();                       /* both waves done reading */
#pragma unroll
        for (int o = 0; o < 64; ++o)
            *reinterpret_cast<u32 *>(ob + (wave * 8 + (o >> 3)) * 512u + (o & 7) * 64u) = acc[o];
    }
    __syncthreads();
    uint8_t *o = a.out_base[0] + t0 * a.out_stride;
    const uint64_t left = a.nstripes - t0;
    const u32 nbytes = (u32)(left < T ? left : T) * 8192u;
#pragma unroll 4
    for (u32 i = tid * 16u; i < (u32)T * 8192u; i += NWV * 64u * 16u)
        if (i < nbytes)
            __builtin_nontemporal_store(*reinterpret_cast<const v4u *>(lds + i),
                                        reinterpret_cast<v4u *>(o + i));
}

template <int NWV, int MODE>
static void add_combine_wm(std::vector<Variant> &v, const char *nm, const CombineArgs *a,
                           double bytes, uint8_t *out, size_t ob)
{
    const bool nt = nt_staging(a->nstripes * 16 * ECD_CHUNK);
    const void *kern = nt ? (const void *)kb_combine_wm<NWV, MODE, kLdsDmaNT>
                          : (const void *)kb_combine_wm<NWV, MODE, kLdsDmaDefault>;
    const uint64_t g = (a->nstripes + 3) / 4;
    v.push_back({nm, bytes, [=](hipStream_t st) {
                     void *args[] = {(void *)a};
                     CHK(hipLaunchKernel(kern, dim3((u32)g), dim3(64 * NWV), args, 32u << 10, st));
                 }, MODE == 0 ? out : nullptr, ob});
}

/* r06: the run-time four-Russians combine (tools/gen/gen_fr_asm.py ->
 * kb_fr16.h): the decode matrix is a run-time argument, as in the shipped
 * kernel, but each wave runs 8 rows at once -- per input, the 22 XOR
 * combinations of its two 4-plane groups are built once into registers and
 * every row's multiply-accumulate is an 8-instruction body (a jump per row
 * and input, GPR-indexed to the row's accumulators) instead of a 12.85-
 * instruction program that re-reads the input's planes from LDS.  One
 * 4-stripe tile per block, two waves (rows 0-7, 8-15).  w.cw[p * 4 + q]:
 * the coefficients of input p for rows 4q .. 4q + 3, one byte each. */
#include "kb_fr16.h"
struct FRW {
    u32 cw[64];
};

template <int LA>
__global__ __launch_bounds__(128) void kb_combine_fr(const CombineArgs a, const FRW w)
{
    constexpr int T = 4;
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const u32 tid = threadIdx.x;
    const uint64_t t0 = (uint64_t)blockIdx.x * T;
    const u32 wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const u32 lane = tid & 63u;
    stage_tile<T, 2, LA>(lds, [&](u32 p, uint64_t st) {
        return a.in_base[p] + st * a.in_stride;
    }, 16, t0, a.nstripes, wave, lane);
    __syncthreads();
    const u32 cs = lane >> 4, cc = lane & 15u;
    const uint8_t *col = lds + cs * 64u + cc * 4u;
    u32 acc[64];
#pragma unroll
    for (int o = 0; o < 64; ++o)
        acc[o] = 0;
#pragma unroll 1
    for (u32 p = 0; p < 16; ++p) {
        u32 x[8];
#pragma unroll
        for (int b = 0; b < 8; ++b)
            x[b] = *reinterpret_cast<const u32 *>(col + (p * 8 + b) * (T * 64u));
        const u32 cw0 = __builtin_amdgcn_readfirstlane(w.cw[p * 4 + wave * 2]);
        const u32 cw1 = __builtin_amdgcn_readfirstlane(w.cw[p * 4 + wave * 2 + 1]);
        FR_ASM_ROWS8(x, cw0, cw1, acc);
    }
    __syncthreads();
    uint8_t *ob = lds + cs * 8192u + cc * 4u + wave * 4096u;
#pragma unroll
    for (int o = 0; o < 64; ++o)
        *reinterpret_cast<u32 *>(ob + (o >> 3) * 512u + (o & 7) * 64u) = acc[o];
    __syncthreads();
    uint8_t *o = a.out_base[0] + t0 * a.out_stride;
    const uint64_t left = a.nstripes - t0;
    const u32 nbytes = (u32)(left < T ? left : T) * 8192u;
    for (u32 i = tid * 16u; i < (u32)T * 8192u; i += 128u * 16u)
        if (i < nbytes)
            __builtin_nontemporal_store(*reinterpret_cast<const v4u *>(lds + i),
                                        reinterpret_cast<v4u *>(o + i));
}

static void add_combine_fr(std::vector<Variant> &v, const char *nm, const CombineArgs *a,
                           const uint8_t *coef, double bytes, uint8_t *out, size_t ob)
{
    FRW *w = new FRW;
    memset(w, 0, sizeof(*w));
    for (int p = 0; p < 16; ++p)
        for (int r = 0; r < 16; ++r)
            w->cw[p * 4 + r / 4] |= (u32)coef[r * 16 + p] << (8 * (r % 4));
    const bool nt = nt_staging(a->nstripes * 16 * ECD_CHUNK);
    const void *kern = nt ? (const void *)kb_combine_fr<kLdsDmaNT>
                          : (const void *)kb_combine_fr<kLdsDmaDefault>;
    const uint64_t g = (a->nstripes + 3) / 4;
    v.push_back({nm, bytes, [=](hipStream_t st) {
                     void *args[] = {(void *)a, (void *)w};
                     CHK(hipLaunchKernel(kern, dim3((u32)g), dim3(128), args, 32u << 10, st));
                 }, out, ob});
}

/* Double-buffered persistent combine for k = 16 (r03 candidate, measured slower: DESIGN.md 3.3.1).  The 8-stripe
 * tile of ec_combine is split into two 32 KiB halves (inputs 0-7, 8-15) that
 * stay within the 64 KiB of one block, so two blocks still share a CU, and
 * the halves are staged one phase ahead of the reads: inputs 8-15 of tile t
 * land while inputs 0-7 are multiplied, inputs 0-7 of the block's next tile
 * while inputs 8-15 are.  Synchronisation by counted vmcnt and raw
 * s_barrier (cdna_hip_programming.md "Pipelining across barriers"): every
 * wave issues exactly 2 LDS-DMA instructions per half (addresses of missing
 * stripes are clamped, never skipped) and 8 stores per tile when it has a
 * row, so
 *   top of tile t:   outstanding A(t), S(t-1)       -> vmcnt(S) retires A(t)
 *   after inputs 0-7: outstanding S(t-1), B(t), A(t') -> vmcnt(2 or 0)
 * and the LDS reads are inline asm (opaque to the compiler, which would
 * otherwise wait vmcnt(0) before any ds_read behind a pending LDS-DMA).
 * One p-loop with the half switch at p = 8, so the jump table exists once. */
template <int NW, bool NTS>
__global__ __launch_bounds__(NW * 64) void ec_combine_db(const CombineArgs a)
{
    static_assert(NW == 16, "16 waves: 2 LDS-DMA instructions per wave per half");
    constexpr u32 T = 8, K = 16;
    constexpr u32 HALF = 8 * T * ECD_CHUNK;          /* 32 KiB */
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const u32 tid = threadIdx.x;
    const u32 wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const u32 lane = tid & 63u;
    const uint64_t ntiles = (a.nstripes + T - 1) / T;
    uint64_t t = blockIdx.x;
    if (t >= ntiles)
        return;
    const uint64_t last = a.nstripes - 1;
    const PatWords<false> pw(a, 0u);
    /* half h of tile `tile`: input p = 8h + ins / 4, 1 KiB per instruction */
    auto stage = [&](uint64_t tile, u32 h) {
#pragma unroll
        for (u32 j = 0; j < 2; ++j) {
            const u32 ins = j * NW + wave;
            const u32 p = h * 8 + ins / 4;
            const u32 el = (ins % 4) * 64 + lane;
            const u32 seg = el >> 2;
            uint64_t st = tile * T + seg % T;
            st = st < last ? st : last;
            const uint8_t *g = a.in_base[pw.byte(a, p)] + st * a.in_stride + (seg / T) * 64u +
                               (el & 3u) * 16u;
            __builtin_amdgcn_global_load_lds(
                (const __attribute__((address_space(1))) void *)g,
                (__attribute__((address_space(3))) void *)(lds + h * HALF + ins * 1024u), 16, 0, 0);
        }
    };
    const u32 r = wave;
    const bool has = r < a.rows;                     /* wave-uniform */
    u32 w[4] = {0u, 0u, 0u, 0u};
    if (has) {
        const u32 rw = a.kw * (1 + r);
#pragma unroll
        for (int i = 0; i < 4; ++i)
            w[i] = pw.word(a, rw + i);
    }
    const u32 cs = lane >> 3, cc = lane & 7u;
    const u32 col = (u32)(uintptr_t)lds + cs * 64u + cc * 8u;   /* LDS byte address */
    stage(t, 0);
    bool stored = false;
    for (;;) {
        if (stored)
            asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        else
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        stage(t, 1);
        const uint64_t tn = t + gridDim.x;
        const bool more = tn < ntiles;
        u32 acc[8][2], y[8][2];
#pragma unroll
        for (int b = 0; b < 8; ++b)
            acc[b][0] = acc[b][1] = 0;
        uint64_t cl = (uint64_t)w[0] | ((uint64_t)w[1] << 32);
        uint64_t ch = (uint64_t)w[2] | ((uint64_t)w[3] << 32);
#pragma unroll 1
        for (u32 p = 0; p < K; ++p) {
            if (p == 8) {
                __builtin_amdgcn_s_barrier();        /* inputs 0-7 read by all */
                if (more) {
                    stage(tn, 0);
                    asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
                } else {
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                }
                __builtin_amdgcn_s_barrier();        /* inputs 8-15 landed */
            }
            const u32 c = __builtin_amdgcn_readfirstlane((u32)cl & 0xFFu);
            cl = (cl >> 8) | (ch << 56);
            ch >>= 8;
            if (c == 0)                              /* ec-code-c.c:11666-11676 */
                continue;
            v4u q0, q1, q2, q3;
            const u32 addr = col + p * (T * ECD_CHUNK);
            asm volatile("ds_read2st64_b64 %0, %4 offset1:1\n\t"
                         "ds_read2st64_b64 %1, %4 offset0:2 offset1:3\n\t"
                         "ds_read2st64_b64 %2, %4 offset0:4 offset1:5\n\t"
                         "ds_read2st64_b64 %3, %4 offset0:6 offset1:7\n\t"
                         "s_waitcnt lgkmcnt(0)"
                         : "=&v"(q0), "=&v"(q1), "=&v"(q2), "=&v"(q3)
                         : "v"(addr)
                         : "memory");
            y[0][0] = q0.x; y[0][1] = q0.y; y[1][0] = q0.z; y[1][1] = q0.w;
            y[2][0] = q1.x; y[2][1] = q1.y; y[3][0] = q1.z; y[3][1] = q1.w;
            y[4][0] = q2.x; y[4][1] = q2.y; y[5][0] = q2.z; y[5][1] = q2.w;
            y[6][0] = q3.x; y[6][1] = q3.y; y[7][0] = q3.z; y[7][1] = q3.w;
            ecgf::mul_xor_jt<2>(c, acc, y);
        }
        const uint64_t ost = t * T + cs;
        /* every tile but the grid's last is whole, so a wave with a row
         * issues its 8 stores (the count the next tile's vmcnt assumes);
         * lanes of missing stripes (last tile only) store nothing */
        if (has && ost < a.nstripes)
            store_chunk<2, NTS>(a.out_base[r] + ost * a.out_stride + cc * 8u, acc);
        stored = has;
        if (!more)
            break;
        t = tn;
    }
}

/* Persistent k = 16 combine with deferred stores (r04 candidate, VERDICT r03
 * #5: the compute phase and the HBM phases add up instead of overlapping).
 * One 64 KiB tile per block, as ec_combine (so two blocks still share a CU),
 * but each block walks tiles blockIdx.x, + gridDim.x, ... and, once every
 * wave has read tile t (barrier), issues the staging of tile t + 1 into the
 * same LDS and only then the stores of tile t's row from its registers: the
 * block's reads and writes are in flight together, and the stores drain
 * under the next tile's compute.  Waits are counted: per wave 4 LDS-DMA
 * instructions (missing stripes' addresses clamped, never skipped), then 4
 * 16-byte stores (a full tile: every tile but the grid's last), so
 * vmcnt(4) retires exactly the staging.  LDS reads in asm (the compiler
 * would put vmcnt(0) before a ds_read behind pending LDS-DMA). MIX = the
 * tile's pattern from the group map (kernel-argument patterns). */
template <bool NTS, int LA, bool MIX = false>
__global__ __launch_bounds__(16 * 64) void ec_combine_pd(const CombineArgs a)
{
    constexpr u32 T = 8, K = 16, NW = 16;
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const u32 tid = threadIdx.x;
    const u32 wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const u32 lane = tid & 63u;
    const uint64_t ntiles = (a.nstripes + T - 1) / T;
    uint64_t t = blockIdx.x;
    if (t >= ntiles)
        return;
    const uint64_t last = a.nstripes - 1;
    auto stage = [&](uint64_t tile) {
        const PatWords<false> pw(a, tile_pattern<MIX>(a, tile * T));
#pragma unroll
        for (u32 j = 0; j < 4; ++j) {
            const u32 ins = j * NW + wave;
            const u32 p = ins / (T / 2);
            const u32 el = (ins * 64 + lane) % (T * 32);
            uint64_t st = tile * T + (el >> 2) % T;
            st = st < last ? st : last;
            const uint8_t *g = a.in_base[pw.byte(a, p)] + st * a.in_stride + ((el >> 2) / T) * 64u +
                               (el & 3u) * 16u;
            __builtin_amdgcn_global_load_lds(
                (const __attribute__((address_space(1))) void *)g,
                (__attribute__((address_space(3))) void *)(lds + ins * 1024u), 16, 0, LA);
        }
    };
    const u32 r = wave;
    const bool has = r < a.rows;                     /* wave-uniform */
    const u32 cs = lane >> 3, cc = lane & 7u;
    const uint8_t *col = lds + cs * 64u + cc * 8u;
    stage(t);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    for (;;) {
        u32 acc[8][2], y[8][2];
#pragma unroll
        for (int b = 0; b < 8; ++b)
            acc[b][0] = acc[b][1] = 0;
        if (has) {
            const PatWords<false> pw(a, tile_pattern<MIX>(a, t * T));
            const u32 rw = a.kw * (1 + r);
            uint64_t cl = (uint64_t)pw.word(a, rw) | ((uint64_t)pw.word(a, rw + 1) << 32);
            uint64_t ch = (uint64_t)pw.word(a, rw + 2) | ((uint64_t)pw.word(a, rw + 3) << 32);
#pragma unroll 1
            for (u32 p = 0; p < K; ++p) {
                const u32 c = __builtin_amdgcn_readfirstlane((u32)cl & 0xFFu);
                cl = (cl >> 8) | (ch << 56);
                ch >>= 8;
                if (c == 0)                          /* ec-code-c.c:11666-11676 */
                    continue;
                lds_read_planes_b64(col + p * (T * ECD_CHUNK), y);
                ecgf::mul_xor_jt<2>(c, acc, y);
            }
        }
        asm volatile("" ::: "memory");
        __builtin_amdgcn_s_barrier();                /* tile t read by every wave */
        asm volatile("" ::: "memory");
        const uint64_t tn = t + gridDim.x;
        const bool more = tn < ntiles;
        if (more)
            stage(tn);
        const uint64_t ost = t * T + cs;
        if (has)
            store_chunk_pairs<NTS>(a.out_base[r] + (ost < a.nstripes ? ost : 0) * a.out_stride, cc,
                                   acc, ost < a.nstripes);
        if (!more)
            break;
        if (has)
            asm volatile("s_waitcnt vmcnt(4)" ::: "memory");   /* staging in, stores may fly */
        else
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();                /* tile t + 1 in LDS */
        asm volatile("" ::: "memory");
        t = tn;
    }
}

/* Where does the k = 16 decode's time go?  A copy of ec_combine's single-
 * pattern k = 16 path (8-stripe tile, 16 waves, CW = 2, jump table) with
 * the HBM sides removable: MODE bit 0 = no staging loads (compute on
 * whatever the LDS holds), bit 1 = no stores (kept live by an impossible
 * run-time condition). */
template <int MODE>
__global__ __launch_bounds__(16 * 64) void kb_combine_probe(const CombineArgs a)
{
    constexpr u32 T = 8, NW = 16, CW = 2, NI = 16 * T * 32 / 64;
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const u32 tid = threadIdx.x;
    const uint64_t t0 = (uint64_t)blockIdx.x * T;
    const u32 wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const u32 lane = tid & 63u;
    const PatWords<false> pw(a, 0u);
    if constexpr (!(MODE & 1)) {
#pragma unroll
        for (u32 j = 0; j < NI / NW; ++j) {
            const u32 ins = j * NW + wave;
            const u32 p = ins / (T / 2);
            const u32 el = (ins * 64 + lane) % (T * 32);
            const u32 s = (el >> 2) % T;
            const uint64_t st = t0 + s;
            if (st < a.nstripes) {
                const uint8_t *g = a.in_base[pw.byte(a, p)] + st * a.in_stride + ((el >> 2) / T) * 64u +
                                   (el & 3u) * 16u;
                __builtin_amdgcn_global_load_lds(
                    (const __attribute__((address_space(1))) void *)g,
                    (__attribute__((address_space(3))) void *)(lds + ins * 1024u), 16, 0, 0);
            }
        }
    }
    __syncthreads();
    const u32 cs = lane / 8, cc = lane % 8;
    const u32 r = wave;
    const uint8_t *col = lds + cs * 64u + cc * 8u;
    const u32 rw = a.kw * (1 + r);
    uint64_t cl = (uint64_t)pw.word(a, rw) | ((uint64_t)pw.word(a, rw + 1) << 32);
    uint64_t ch = (uint64_t)pw.word(a, rw + 2) | ((uint64_t)pw.word(a, rw + 3) << 32);
    u32 acc[8][CW], y[8][CW];
#pragma unroll
    for (int b = 0; b < 8; ++b)
        acc[b][0] = acc[b][1] = 0;
#pragma unroll 1
    for (u32 p = 0; p < 16; ++p) {
        const u32 c = __builtin_amdgcn_readfirstlane((u32)cl & 0xFFu);
        cl = (cl >> 8) | (ch << 56);
        ch >>= 8;
        if (c == 0)
            continue;
        const uint8_t *src = col + p * (T * ECD_CHUNK);
        if constexpr (MODE & 4) {
            /* 8 single ds_read_b64 (2 LDS cycles each) instead of the 4
             * ds_read2st64_b64 (8 each) the compiler pairs them into */
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
                         : "=&v"(q[0]), "=&v"(q[1]), "=&v"(q[2]), "=&v"(q[3]), "=&v"(q[4]),
                           "=&v"(q[5]), "=&v"(q[6]), "=&v"(q[7])
                         : "v"(ad)
                         : "memory");
#pragma unroll
            for (int b = 0; b < 8; ++b) {
                y[b][0] = q[b].x;
                y[b][1] = q[b].y;
            }
        } else {
#pragma unroll
            for (int b = 0; b < 8; ++b)
                load_plane<CW>(src + (u32)b * (T * 64u), y[b]);
        }
        ecgf::mul_xor_jt<CW>(c, acc, y);
    }
    const uint64_t ost = t0 + cs;
    const bool st_ok = (MODE & 2) ? a.nstripes == 0x123456789ull : ost < a.nstripes;
    if constexpr (MODE & 8) {
        /* 16-byte stores: lane pairs (cc, cc ^ 1) swap halves so the even
         * lane holds 16 B of plane b, the odd lane 16 B of plane b + 1 */
        const bool odd = cc & 1u;
        uint8_t *o = a.out_base[r] + ost * a.out_stride + (cc & ~1u) * 8u;
#pragma unroll
        for (int b = 0; b < 8; b += 2) {
            const u32 s0 = odd ? acc[b][0] : acc[b + 1][0];
            const u32 s1 = odd ? acc[b][1] : acc[b + 1][1];
            const u32 r0 = __builtin_amdgcn_mov_dpp(s0, 0xB1, 0xF, 0xF, false);
            const u32 r1 = __builtin_amdgcn_mov_dpp(s1, 0xB1, 0xF, 0xF, false);
            const v4u out = odd ? v4u{r0, r1, acc[b + 1][0], acc[b + 1][1]}
                                : v4u{acc[b][0], acc[b][1], r0, r1};
            if (st_ok)
                __builtin_nontemporal_store(out, reinterpret_cast<v4u *>(o + (b + (odd ? 1 : 0)) * 64));
        }
    } else if (st_ok) {
        store_chunk<CW, true>(a.out_base[r] + ost * a.out_stride + cc * 8u, acc);
    }
}

/* decode desc: k inputs (fragments), `rows` outputs, dense coefficients */
static CombineArgs *make_args(int k, int rows, uint64_t nst, uint8_t *const *frags, uint8_t *out,
                              bool stripe_major, const uint8_t *coef)
{
    ecd_combine_desc_t d;
    memset(&d, 0, sizeof(d));
    d.k = k;
    d.rows = rows;
    d.nstripes = nst;
    d.in_stride = ECD_CHUNK;
    d.out_stride = stripe_major ? (uint64_t)rows * ECD_CHUNK : ECD_CHUNK;
    for (int p = 0; p < k; ++p) {
        d.in_base[p] = frags[p];
        d.pat[p] = (uint8_t)p;
    }
    for (int r = 0; r < rows; ++r)
        d.out_base[r] = stripe_major ? out + (uint64_t)r * ECD_CHUNK : out + (uint64_t)r * nst * ECD_CHUNK;
    memcpy(d.pat + k, coef, (size_t)rows * k);
    d.npatterns = 1;
    d.pat_bytes = k + rows * k;
    CombineArgs *a = new CombineArgs;
    if (ecdk_pack_args(&d, a))
        exit(2);
    return a;
}

static void add_shipped_combine(std::vector<Variant> &v, const char *nm, const CombineArgs *a,
                                double bytes, uint8_t *out, size_t ob)
{
    v.push_back({nm, bytes, [=](hipStream_t st) {
                     const int rc = nt_staging(a->nstripes * a->k * ECD_CHUNK)
                                        ? launch_combine_k<true, kLdsDmaNT>(st, *a)
                                        : launch_combine_k<true, kLdsDmaDefault>(st, *a);
                     if (rc)
                         exit(8);
                 }, out, ob});
}

template <int K, int NW, int WOT, int RB = 1>
static void add_combine_n(std::vector<Variant> &v, const char *nm, const CombineArgs *a,
                          double bytes, uint8_t *out, size_t ob)
{
    auto kern = ec_combine_n<K, NW, false, true, WOT, false, false, RB>;
    const size_t lds = combine_n_lds<NW, WOT>(K);
    lds_attr((const void *)kern, lds);
    const uint64_t g = (a->nstripes + 3) / 4;
    v.push_back({nm, bytes, [=](hipStream_t st) {
                     hipLaunchKernelGGL(kern, dim3((u32)g), dim3(64 * NW), lds, st, *a);
                 }, out, ob});
}

int main(int argc, char **argv)
{
    const double gib = argc > 1 ? atof(argv[1]) : 1.0;
    const int rounds = argc > 2 ? atoi(argv[2]) : 7;
    const char *groups = argc > 3 ? argv[3] : "all";
    const int iters = 10;
    hipDeviceProp_t prop;
    CHK(hipGetDeviceProperties(&prop, 0));
    printf("device %s CUs %d, %.2f GiB user data per launch\n", prop.gcnArchName,
           prop.multiProcessorCount, gib);
    hipStream_t s;
    CHK(hipStreamCreate(&s));
    const uint64_t user = (uint64_t)(gib * (1ull << 30));
    uint8_t *bufA, *bufB;
    CHK(hipMalloc(&bufA, user * 2));
    CHK(hipMalloc(&bufB, user * 2));
    fill(bufA, user * 2, 12345);
    std::vector<Variant> v;

    if (want(groups, "enc16")) {
        const uint64_t nst = user / (16 * ECD_CHUNK);
        FragPtrs f = frag_ptrs(bufB, nst, 20);
        add_shipped_encode(v, "shipped (tile T8 CW1 NW16)", 16, 20, nst, bufA, f);
        add_tile_t<16, 20, 4, 4, false, true>(v, "T4 NW4 WOT", nst, bufA, f);
        add_tile_t<16, 20, 4, 5, false, true>(v, "T4 NW5 WOT", nst, bufA, f);
        add_tile_t<16, 20, 4, 10, false, true>(v, "T4 NW10 WOT", nst, bufA, f);
        add_tile_t<16, 20, 4, 16, false, true>(v, "T4 NW16 WOT", nst, bufA, f);
        add_tile_t<16, 20, 4, 5, true, true>(v, "T4 NW5 direct WOT", nst, bufA, f);
        run_group("encode 16+4", v, rounds, iters, s);
        v.clear();
    }
    /* partial-stripe writes (ecdk_encode_vander_rmw): interior read in place
     * at a 3-byte misalignment, edges from an aligned scratch: round-2
     * register kernel against the tile encoders with register staging */
    auto rmw_group = [&](auto kk, auto nn, auto ww, const char *title) {
        constexpr int K = decltype(kk)::value, N = decltype(nn)::value, W = decltype(ww)::value;
        const uint64_t nst = user / (K * ECD_CHUNK);
        FragPtrs f = frag_ptrs(bufB, nst, N);
        const uint8_t *edge = bufA + user + 4096;        /* 2 stripes, aligned */
        const uint8_t *ushift = bufA + 3;                 /* interior at +3 bytes */
        const double bytes = (double)nst * (K + N) * ECD_CHUNK;
        v.push_back({"round-2 register kernel (LM=1)", bytes, [=](hipStream_t st) {
                         hipLaunchKernelGGL((ec_encode_vander_rmw<K, N, W, 1>), dim3((u32)vander_grid<W>(nst)),
                                            dim3(kBlock), 0, st, edge, ushift, f, nst);
                     }, f.p[N - 1], (size_t)nst * ECD_CHUNK});
        if constexpr (K == 16) {
            auto kern = ec_encode_tile_rb<16, 20, 4, 2, true, true, 2>;
            auto kern3 = ec_encode_tile_rb<16, 20, 4, 2, true, true, 3>;
            const size_t lds = encode_tile_rb_lds<20, 4, 2, true>(16);
            v.push_back({"tile encoder, register staging (SM=2)", bytes, [=](hipStream_t st) {
                             hipLaunchKernelGGL(kern, dim3((u32)((nst + 3) / 4)), dim3(640), lds, st,
                                                EncSrc{ushift, edge}, f, nst);
                         }, f.p[N - 1], (size_t)nst * ECD_CHUNK});
            v.push_back({"tile encoder, dword-aligned shift staging (SM=3)", bytes, [=](hipStream_t st) {
                             hipLaunchKernelGGL(kern3, dim3((u32)((nst + 3) / 4)), dim3(640), lds, st,
                                                EncSrc{ushift, edge}, f, nst);
                         }, f.p[N - 1], (size_t)nst * ECD_CHUNK});
            auto kern8 = ec_encode_tile_rb<16, 20, 4, 2, true, true, 8>;
            v.push_back({"16-byte-aligned shift staging (SM=8)", bytes, [=](hipStream_t st) {
                             hipLaunchKernelGGL(kern8, dim3((u32)((nst + 3) / 4)), dim3(640), lds, st,
                                                EncSrc{ushift, edge}, f, nst);
                         }, f.p[N - 1], (size_t)nst * ECD_CHUNK});
            for (u32 sh : {7u, 13u}) {   /* dword shifts 1 and 3 (timing only) */
                const uint8_t *us = bufA + sh;
                v.push_back({std::string("SM=3 at +") + std::to_string(sh), bytes, [=](hipStream_t st) {
                                 hipLaunchKernelGGL(kern3, dim3((u32)((nst + 3) / 4)), dim3(640), lds, st,
                                                    EncSrc{us, edge}, f, nst);
                             }, nullptr, 0});
                v.push_back({std::string("SM=8 at +") + std::to_string(sh), bytes, [=](hipStream_t st) {
                                 hipLaunchKernelGGL(kern8, dim3((u32)((nst + 3) / 4)), dim3(640), lds, st,
                                                    EncSrc{us, edge}, f, nst);
                             }, nullptr, 0});
            }
            auto kern4 = ec_encode_tile_rb<16, 20, 4, 2, true, true, 4>;
            auto kern5 = ec_encode_tile_rb<16, 20, 4, 2, true, true, 5>;
            auto kern6 = ec_encode_tile_rb<16, 20, 4, 2, true, true, 6>;
            auto kern7 = ec_encode_tile_rb<16, 20, 4, 2, true, true, 7>;
            v.push_back({"shift staging, non-temporal loads (SM=7)", bytes, [=](hipStream_t st) {
                             hipLaunchKernelGGL(kern7, dim3((u32)((nst + 3) / 4)), dim3(640), lds, st,
                                                EncSrc{ushift, edge}, f, nst);
                         }, f.p[N - 1], (size_t)nst * ECD_CHUNK});
            v.push_back({"split: 8 inputs LDS-DMA, 8 shifted (SM=4)", bytes, [=](hipStream_t st) {
                             hipLaunchKernelGGL(kern4, dim3((u32)((nst + 3) / 4)), dim3(640), lds, st,
                                                EncSrc{ushift, edge}, f, nst);
                         }, f.p[N - 1], (size_t)nst * ECD_CHUNK});
            v.push_back({"split: 12 inputs LDS-DMA, 4 shifted (SM=5)", bytes, [=](hipStream_t st) {
                             hipLaunchKernelGGL(kern5, dim3((u32)((nst + 3) / 4)), dim3(640), lds, st,
                                                EncSrc{ushift, edge}, f, nst);
                         }, f.p[N - 1], (size_t)nst * ECD_CHUNK});
            v.push_back({"split: 4 inputs LDS-DMA, 12 shifted (SM=6)", bytes, [=](hipStream_t st) {
                             hipLaunchKernelGGL(kern6, dim3((u32)((nst + 3) / 4)), dim3(640), lds, st,
                                                EncSrc{ushift, edge}, f, nst);
                         }, f.p[N - 1], (size_t)nst * ECD_CHUNK});
        } else {
            constexpr int NW = N;
            auto kern = ec_encode_tile_t<K, N, 4, NW, true, (K == 4), true, 2>;
            auto kern3 = ec_encode_tile_t<K, N, 4, NW, true, (K == 4), true, 3>;
            const size_t lds = encode_tile_t_lds<4, NW, true>(K);
            v.push_back({"tile encoder, register staging (SM=2)", bytes, [=](hipStream_t st) {
                             hipLaunchKernelGGL(kern, dim3((u32)((nst + 3) / 4)), dim3(64 * NW), lds, st,
                                                EncSrc{ushift, edge}, f, nst);
                         }, f.p[N - 1], (size_t)nst * ECD_CHUNK});
            v.push_back({"tile encoder, dword-aligned shift staging (SM=3)", bytes, [=](hipStream_t st) {
                             hipLaunchKernelGGL(kern3, dim3((u32)((nst + 3) / 4)), dim3(64 * NW), lds, st,
                                                EncSrc{ushift, edge}, f, nst);
                         }, f.p[N - 1], (size_t)nst * ECD_CHUNK});
            auto kern8 = ec_encode_tile_t<K, N, 4, NW, true, (K == 4), true, 8>;
            v.push_back({"16-byte-aligned shift staging (SM=8)", bytes, [=](hipStream_t st) {
                             hipLaunchKernelGGL(kern8, dim3((u32)((nst + 3) / 4)), dim3(64 * NW), lds, st,
                                                EncSrc{ushift, edge}, f, nst);
                         }, f.p[N - 1], (size_t)nst * ECD_CHUNK});
            for (u32 sh : {7u, 13u}) {   /* dword shifts 1 and 3 (timing only) */
                const uint8_t *us = bufA + sh;
                v.push_back({std::string("SM=3 at +") + std::to_string(sh), bytes, [=](hipStream_t st) {
                                 hipLaunchKernelGGL(kern3, dim3((u32)((nst + 3) / 4)), dim3(64 * NW), lds, st,
                                                    EncSrc{us, edge}, f, nst);
                             }, nullptr, 0});
                v.push_back({std::string("SM=8 at +") + std::to_string(sh), bytes, [=](hipStream_t st) {
                                 hipLaunchKernelGGL(kern8, dim3((u32)((nst + 3) / 4)), dim3(64 * NW), lds, st,
                                                    EncSrc{us, edge}, f, nst);
                             }, nullptr, 0});
            }
            auto kern7 = ec_encode_tile_t<K, N, 4, NW, true, (K == 4), true, 7>;
            v.push_back({"shift staging, non-temporal loads (SM=7)", bytes, [=](hipStream_t st) {
                             hipLaunchKernelGGL(kern7, dim3((u32)((nst + 3) / 4)), dim3(64 * NW), lds, st,
                                                EncSrc{ushift, edge}, f, nst);
                         }, f.p[N - 1], (size_t)nst * ECD_CHUNK});
        }
        v.push_back({"shipped (tile encoder, LDS-DMA at +3 bytes)", bytes, [=](hipStream_t st) {
                         void *o[ECD_MAX_ROWS];
                         for (int i = 0; i < N; ++i)
                             o[i] = f.p[i];
                         if (ecdk_encode_vander_rmw(st, K, N, nst, edge, ushift, o))
                             exit(9);
                     }, f.p[N - 1], (size_t)nst * ECD_CHUNK});
        v.push_back({"aligned encode (shipped, reference point)", bytes, [=](hipStream_t st) {
                         void *o[ECD_MAX_ROWS];
                         for (int i = 0; i < N; ++i)
                             o[i] = f.p[i];
                         if (ecdk_encode_vander(st, K, N, nst, bufA, o, false))
                             exit(9);
                     }, nullptr, 0});
        run_group(title, v, rounds, iters, s);
        v.clear();
    };
    if (want(groups, "rmw"))
        rmw_group(std::integral_constant<int, 4>{}, std::integral_constant<int, 6>{},
                  std::integral_constant<int, 2>{}, "partial write 4+2, interior +3 bytes");
    if (want(groups, "rmw"))
        rmw_group(std::integral_constant<int, 8>{}, std::integral_constant<int, 12>{},
                  std::integral_constant<int, 1>{}, "partial write 8+4, interior +3 bytes");
    if (want(groups, "rmw"))
        rmw_group(std::integral_constant<int, 16>{}, std::integral_constant<int, 20>{},
                  std::integral_constant<int, 1>{}, "partial write 16+4, interior +3 bytes");
    if (want(groups, "enc16rb")) {
        for (int big = 0; big < 2; ++big) {
            const uint64_t nst = big ? user / (16 * ECD_CHUNK) : 32768;
            FragPtrs f = frag_ptrs(bufB, nst, 20);
            add_shipped_encode(v, "shipped (tile T8 CW1 NW16)", 16, 20, nst, bufA, f);
            add_tile_rb<16, 20, 4, 5, true>(v, "RB5 T4 WOT (4 waves)", nst, bufA, f);
            add_tile_rb<16, 20, 4, 5, false>(v, "RB5 T4 (4 waves)", nst, bufA, f);
            add_tile_rb<16, 20, 4, 4, true>(v, "RB4 T4 WOT (5 waves)", nst, bufA, f);
            add_tile_rb<16, 20, 4, 4, false>(v, "RB4 T4 (5 waves)", nst, bufA, f);
            add_tile_rb<16, 20, 4, 2, true>(v, "RB2 T4 WOT (10 waves)", nst, bufA, f);
            add_tile_rb<16, 20, 8, 5, true>(v, "RB5 T8 WOT (8 waves)", nst, bufA, f);
            add_tile_rb<16, 20, 8, 5, false>(v, "RB5 T8 (8 waves)", nst, bufA, f);
            add_tile_rb<16, 20, 8, 10, false>(v, "RB10 T8 (4 waves)", nst, bufA, f);
            run_group(big ? "encode 16+4 row groups (size = GiB arg)" : "encode 16+4 row groups, 32K stripes",
                      v, rounds, iters, s);
            v.clear();
        }
    }
    if (want(groups, "enc8")) {
        for (int big = 0; big < 2; ++big) {
            const uint64_t nst = big ? user / (8 * ECD_CHUNK) : 65536;
            FragPtrs f = frag_ptrs(bufB, nst, 12);
            add_shipped_encode(v, "shipped (narrow T4 NW12)",
                               8, 12, nst, bufA, f);
            add_tile_t<8, 12, 8, 12, true, true>(v, "T8 NW12 direct WOT", nst, bufA, f);
            add_tile_t<8, 12, 4, 4, true, true>(v, "T4 NW4 direct WOT", nst, bufA, f);
            add_tile_t<8, 12, 4, 6, true, true>(v, "T4 NW6 direct WOT", nst, bufA, f);
            add_tile_t<8, 12, 4, 6, false, true>(v, "T4 NW6 WOT", nst, bufA, f);
            add_tile_t<8, 12, 4, 4, false, true>(v, "T4 NW4 WOT", nst, bufA, f);
            add_tile_t<8, 12, 4, 12, false, true>(v, "T4 NW12 WOT", nst, bufA, f);
            add_tile_rb<8, 12, 4, 2, true>(v, "RB2 T4 WOT (6 waves)", nst, bufA, f);
            add_tile_rb<8, 12, 4, 3, true>(v, "RB3 T4 WOT (4 waves)", nst, bufA, f);
            add_tile_rb<8, 12, 4, 4, true>(v, "RB4 T4 WOT (3 waves)", nst, bufA, f);
            add_tile_rb<8, 12, 8, 3, true>(v, "RB3 T8 WOT (8 waves)", nst, bufA, f);
            run_group(big ? "encode 8+4 (size = GiB arg)" : "encode 8+4, 64K stripes", v, rounds,
                      iters, s);
            v.clear();
        }
    }
    if (want(groups, "enc4")) {
        const uint64_t nst = user / (4 * ECD_CHUNK);
        FragPtrs f = frag_ptrs(bufB, nst, 6);
        add_shipped_encode(v, "shipped (narrow T4 NW6 direct)", 4, 6, nst, bufA, f);
        add_tile_t<4, 6, 8, 6, true, true>(v, "T8 NW6 direct WOT", nst, bufA, f);
        add_tile_t<4, 6, 4, 6, true, true>(v, "T4 NW6 direct WOT", nst, bufA, f);
        add_tile_t<4, 6, 4, 6, false, true>(v, "T4 NW6 WOT", nst, bufA, f);
        add_tile_t<4, 6, 4, 3, true, true>(v, "T4 NW3 direct WOT", nst, bufA, f);
        add_tile_t<4, 6, 4, 3, false, true>(v, "T4 NW3 WOT", nst, bufA, f);
        add_tile_rb<4, 6, 4, 2, true>(v, "RB2 T4 WOT (3 waves)", nst, bufA, f);
        add_tile_rb<4, 6, 4, 3, true>(v, "RB3 T4 WOT (2 waves)", nst, bufA, f);
        add_tile_rb<4, 6, 8, 2, true>(v, "RB2 T8 WOT (6 waves)", nst, bufA, f);
        run_group("encode 4+2", v, rounds, iters, s);
        v.clear();
    }
    auto decode_group = [&](auto kk, const char *title, bool heal) {
        constexpr int K = decltype(kk)::value;
        const int rows = heal ? 4 : K;
        const uint64_t nst = user / (K * ECD_CHUNK);
        uint8_t *fr[16];
        for (int p = 0; p < K; ++p)
            fr[p] = bufA + (uint64_t)p * nst * ECD_CHUNK;
        uint8_t c[256];
        for (int i = 0; i < 256; ++i)
            c[i] = (uint8_t)(1 + (i * 173 + 11) % 255);
        const CombineArgs *a = make_args(K, rows, nst, fr, bufB, !heal, c);
        const double bytes = (double)nst * (K + rows) * ECD_CHUNK;
        const size_t ob = (size_t)nst * rows * ECD_CHUNK;
        add_shipped_combine(v, "shipped", a, bytes, bufB, ob);
        add_combine_n<K, 8, 0>(v, "narrow NW8", a, bytes, bufB, ob);
        if constexpr (K == 16) {
            auto kern = ec_combine_db<16, true>;
            lds_attr((const void *)kern, 64u << 10);
            const uint64_t ntiles = (a->nstripes + 7) / 8;
            for (int per = 1; per <= 3; per += 2) {
                const uint64_t g = std::min<uint64_t>(ntiles, (uint64_t)per * prop.multiProcessorCount * 2);
                v.push_back({per == 1 ? "double-buffered halves, 2 blocks/CU" : "double-buffered halves, grid 6/CU",
                             bytes, [=](hipStream_t st) {
                                 hipLaunchKernelGGL(kern, dim3((u32)g), dim3(64 * 16), 64u << 10, st, *a);
                             }, bufB, ob});
            }
        }
        add_combine_n<K, 8, 1>(v, "narrow NW8 WOT", a, bytes, bufB, ob);
        add_combine_n<K, 4, 1>(v, "narrow NW4 WOT", a, bytes, bufB, ob);
        add_combine_n<K, 8, 1, 2>(v, "narrow NW8 WOT RB2", a, bytes, bufB, ob);
        add_combine_n<K, 4, 1, 2>(v, "narrow NW4 WOT RB2", a, bytes, bufB, ob);
        add_combine_n<K, 2, 1, 2>(v, "narrow NW2 WOT RB2", a, bytes, bufB, ob);
        add_combine_n<K, 8, 0, 2>(v, "narrow NW8 RB2", a, bytes, bufB, ob);
        run_group(title, v, rounds, iters, s);
        v.clear();
    };
    if (want(groups, "dec16"))
        decode_group(std::integral_constant<int, 16>{}, "decode 16+4 dense", false);
    /* r04: the persistent deferred-store k = 16 combine against the shipped
     * one, grids of 1 / 2 / 3 / 4 blocks per CU (two are resident) */
    if (want(groups, "dec16pd")) {
        constexpr int K = 16;
        const uint64_t nst = user / (K * ECD_CHUNK);
        uint8_t *fr[16];
        for (int p = 0; p < K; ++p)
            fr[p] = bufA + (uint64_t)p * nst * ECD_CHUNK;
        uint8_t c[256];
        for (int i = 0; i < 256; ++i)
            c[i] = (uint8_t)(1 + (i * 173 + 11) % 255);
        const CombineArgs *a = make_args(K, K, nst, fr, bufB, true, c);
        const double bytes = (double)nst * 2 * K * ECD_CHUNK;
        const size_t ob = (size_t)nst * K * ECD_CHUNK;
        const bool nt = nt_staging(nst * K * ECD_CHUNK);
        add_shipped_combine(v, "shipped", a, bytes, bufB, ob);
        const uint64_t ntiles = (nst + 7) / 8;
        for (int per : {2, 4, 8}) {
            const uint64_t g = std::min<uint64_t>(ntiles, (uint64_t)per * prop.multiProcessorCount);
            static char nm[3][64];
            char *n = nm[per == 2 ? 0 : per == 4 ? 1 : 2];
            snprintf(n, 64, "persistent deferred stores, grid %d/CU", per);
            if (nt) {
                auto kern = ec_combine_pd<true, kLdsDmaNT>;
                lds_attr((const void *)kern, 64u << 10);
                v.push_back({n, bytes, [=](hipStream_t st) {
                                 hipLaunchKernelGGL(kern, dim3((u32)g), dim3(64 * 16), 64u << 10, st, *a);
                             }, bufB, ob});
            } else {
                auto kern = ec_combine_pd<true, kLdsDmaDefault>;
                lds_attr((const void *)kern, 64u << 10);
                v.push_back({n, bytes, [=](hipStream_t st) {
                                 hipLaunchKernelGGL(kern, dim3((u32)g), dim3(64 * 16), 64u << 10, st, *a);
                             }, bufB, ob});
            }
        }
        run_group("decode 16+4, persistent deferred stores (r04)", v, rounds, iters, s);
        v.clear();
    }
    /* Placement of the fragments: contiguous in one allocation (64 MiB apart
     * at 1 GiB), staggered by p * 4 KiB + p * 64 B, or one hipMalloc each
     * (as torch tensors are) -- the bench's k >= 8 decodes ran ~8-10 %
     * slower than kb3's, its 4+2 decode did not. */
    auto layout_group = [&](auto kk, const char *title) {
        constexpr int K = decltype(kk)::value;
        const uint64_t nst = user / (K * ECD_CHUNK);
        const uint64_t fb = nst * ECD_CHUNK;
        uint8_t c[256];
        for (int i = 0; i < 256; ++i)
            c[i] = (uint8_t)ct_coef(i);
        const double bytes = 2.0 * nst * K * ECD_CHUNK;
        const size_t ob = (size_t)nst * K * ECD_CHUNK;
        uint8_t *fr[16];
        for (int p = 0; p < K; ++p)
            fr[p] = bufA + (uint64_t)p * fb;
        add_shipped_combine(v, "contiguous (64 MiB apart at 16+4)", make_args(K, K, nst, fr, bufB, true, c),
                            bytes, bufB, ob);
        uint8_t *fs[16];
        for (int p = 0; p < K; ++p)
            fs[p] = bufA + (uint64_t)p * fb + (uint64_t)p * (4096 + 64) * 4;
        add_shipped_combine(v, "staggered by p * 16.25 KiB", make_args(K, K, nst, fs, bufB, true, c),
                            bytes, bufB, ob);
        static uint8_t *sep[16];
        for (int p = 0; p < K; ++p) {
            CHK(hipMalloc(&sep[p], fb));
            CHK(hipMemcpy(sep[p], fr[p], fb, hipMemcpyDeviceToDevice));
        }
        add_shipped_combine(v, "one hipMalloc per fragment", make_args(K, K, nst, sep, bufB, true, c),
                            bytes, bufB, ob);
        run_group(title, v, rounds, iters, s);
        v.clear();
        for (int p = 0; p < K; ++p)
            CHK(hipFree(sep[p]));
    };
    /* fragments at an odd address: read in place by LDS-DMA (r03) */
    auto misdec_group = [&](auto kk, const char *title) {
        constexpr int K = decltype(kk)::value;
        const uint64_t nst = user / (K * ECD_CHUNK);
        const uint64_t fb = nst * ECD_CHUNK + 64;
        uint8_t c[256];
        for (int i = 0; i < 256; ++i)
            c[i] = (uint8_t)ct_coef(i);
        const double bytes = 2.0 * nst * K * ECD_CHUNK;
        const size_t ob = (size_t)nst * K * ECD_CHUNK;
        for (int off : {0, 3, 8}) {
            uint8_t *fr[16];
            for (int p = 0; p < K; ++p)
                fr[p] = bufA + (uint64_t)p * fb + off;
            static char nm[3][48];
            snprintf(nm[off == 0 ? 0 : off == 3 ? 1 : 2], 48, "fragments at +%d bytes", off);
            add_shipped_combine(v, nm[off == 0 ? 0 : off == 3 ? 1 : 2],
                                make_args(K, K, nst, fr, bufB, true, c), bytes, nullptr, ob);
        }
        run_group(title, v, rounds, iters, s);
        v.clear();
    };
    if (want(groups, "misdec")) {
        misdec_group(std::integral_constant<int, 4>{}, "decode 4+2, fragment alignment");
        misdec_group(std::integral_constant<int, 8>{}, "decode 8+4, fragment alignment");
        misdec_group(std::integral_constant<int, 16>{}, "decode 16+4, fragment alignment");
    }
    if (want(groups, "layout16"))
        layout_group(std::integral_constant<int, 16>{}, "decode 16+4 dense, fragment placement");
    if (want(groups, "layout8"))
        layout_group(std::integral_constant<int, 8>{}, "decode 8+4 dense, fragment placement");
    if (want(groups, "layout4"))
        layout_group(std::integral_constant<int, 4>{}, "decode 4+2 dense, fragment placement");
    if (want(groups, "probe16")) {   /* k = 16 decode with its HBM sides removed */
        constexpr int K = 16;
        const uint64_t nst = user / (K * ECD_CHUNK);
        uint8_t *fr[16];
        for (int p = 0; p < K; ++p)
            fr[p] = bufA + (uint64_t)p * nst * ECD_CHUNK;
        uint8_t c[256];
        for (int i = 0; i < 256; ++i)
            c[i] = (uint8_t)(1 + (i * 173 + 11) % 255);
        const CombineArgs *a = make_args(K, K, nst, fr, bufB, true, c);
        const double bytes = 2.0 * nst * K * ECD_CHUNK;
        const size_t ob = (size_t)nst * K * ECD_CHUNK;
        add_shipped_combine(v, "shipped", a, bytes, bufB, ob);
        {
            static const char *pn[10] = {"probe: full (= shipped)", "probe: no staging loads",
                                        "probe: no stores", "probe: compute only",
                                        "probe: ds_read_b64 x8", "probe: ds_read_b64 x8, compute only",
                                        "probe: 16-B stores (DPP pairs)", "probe: b64 reads + 16-B stores",
                                        "probe: b64 reads, no stores", "probe: 16-B stores, no loads"};
            const void *kerns[10] = {(const void *)kb_combine_probe<0>, (const void *)kb_combine_probe<1>,
                                    (const void *)kb_combine_probe<2>, (const void *)kb_combine_probe<3>,
                                    (const void *)kb_combine_probe<4>, (const void *)kb_combine_probe<7>,
                                    (const void *)kb_combine_probe<8>, (const void *)kb_combine_probe<12>,
                                    (const void *)kb_combine_probe<6>, (const void *)kb_combine_probe<9>};
            for (int m = 0; m < 10; ++m) {
                const uint64_t g = (a->nstripes + 7) / 8;
                const void *kern = kerns[m];
                v.push_back({pn[m], bytes, [=](hipStream_t st) {
                                 void *args[] = {(void *)a};
                                 CHK(hipLaunchKernel(kern, dim3((u32)g), dim3(1024), args, 64u << 10, st));
                             }, (m == 0 || m == 4 || m == 6 || m == 7) ? bufB : nullptr, ob});
            }
        }
        run_group("decode 16+4 dense, probes", v, rounds, iters, s);
        v.clear();
    }
    if (want(groups, "dec16ct")) {  /* compile-time matrix: the JIT question */
        constexpr int K = 16;
        const uint64_t nst = user / (K * ECD_CHUNK);
        uint8_t *fr[16];
        for (int p = 0; p < K; ++p)
            fr[p] = bufA + (uint64_t)p * nst * ECD_CHUNK;
        uint8_t c[256];
        for (int i = 0; i < 256; ++i)
            c[i] = (uint8_t)ct_coef(i);
        const CombineArgs *a = make_args(K, K, nst, fr, bufB, true, c);
        const double bytes = 2.0 * nst * K * ECD_CHUNK;
        const size_t ob = (size_t)nst * K * ECD_CHUNK;
        add_shipped_combine(v, "shipped (run-time matrix)", a, bytes, bufB, ob);
        add_combine_ct<K, 8, 16, false>(v, "ct T8 NW16", a, bytes, bufB, ob);
        add_combine_ct<K, 8, 8, false>(v, "ct T8 NW8", a, bytes, bufB, ob);
        add_combine_ct<K, 4, 8, true>(v, "ct T4 NW8 WOT", a, bytes, bufB, ob);
        add_combine_ct<K, 4, 4, true>(v, "ct T4 NW4 WOT", a, bytes, bufB, ob);
        add_combine_ct<K, 4, 8, false>(v, "ct T4 NW8", a, bytes, bufB, ob);
        run_group("decode 16+4 dense, compile-time matrix", v, rounds, iters, s);
        v.clear();
    }
    if (want(groups, "dec16wm")) {  /* whole-matrix program (r06) */
        constexpr int K = 16;
        const uint64_t nst = user / (K * ECD_CHUNK);
        uint8_t *fr[16];
        for (int p = 0; p < K; ++p)
            fr[p] = bufA + (uint64_t)p * nst * ECD_CHUNK;
        uint8_t c[256];
        for (int i = 0; i < 256; ++i)
            c[i] = (uint8_t)ct_coef(i);
        const CombineArgs *a = make_args(K, K, nst, fr, bufB, true, c);
        const double bytes = 2.0 * nst * K * ECD_CHUNK;
        const size_t ob = (size_t)nst * K * ECD_CHUNK;
        printf("instructions per dword column: row by row %d, whole matrix %d, two halves %d\n",
               WM16_OPS_ROWWISE, WM16_OPS_FULL, WM16_OPS_HALVES);
        add_shipped_combine(v, "shipped (run-time matrix)", a, bytes, bufB, ob);
        add_combine_wm<1, 0>(v, "whole matrix, 1 wave x 16 rows", a, bytes, bufB, ob);
        add_combine_wm<2, 0>(v, "whole matrix, 2 waves x 8 rows", a, bytes, bufB, ob);
        add_combine_ct<K, 4, 4, true>(v, "ct row-wise T4 NW4 WOT", a, bytes, bufB, ob);
#ifdef KB3_WITH_JIT
        {
            /* the library's path: ecdk_combine -> the hiprtc-compiled kernel
             * of this matrix (EC_MI355X_JIT_SYNC=1: compiled at first call) */
            ecd_combine_desc_t *d = new ecd_combine_desc_t;
            memset(d, 0, sizeof(*d));
            d->k = K;
            d->rows = K;
            d->nstripes = nst;
            d->in_stride = ECD_CHUNK;
            d->out_stride = (uint64_t)K * ECD_CHUNK;
            for (int p = 0; p < K; ++p) {
                d->in_base[p] = fr[p];
                d->pat[p] = (uint8_t)p;
                d->out_base[p] = bufB + (uint64_t)p * ECD_CHUNK;
            }
            memcpy(d->pat + K, c, (size_t)K * K);
            d->npatterns = 1;
            d->pat_bytes = K + K * K;
            v.push_back({"library JIT (hiprtc)", bytes, [=](hipStream_t st) {
                             ecj_lds_pad_kb = 0;
                             if (ecdk_combine(st, d))
                                 exit(9);
                         }, bufB, ob});
            /* 4 blocks per CU (8 waves) as the kb3 kernel's 204 VGPRs allow,
             * instead of the 5 its 32 KiB tile allows */
            v.push_back({"library JIT, 40 KiB LDS (4 blocks/CU)", bytes, [=](hipStream_t st) {
                             ecj_lds_pad_kb = 8;
                             if (ecdk_combine(st, d))
                                 exit(9);
                             ecj_lds_pad_kb = 0;
                         }, bufB, ob});
            v.push_back({"library JIT, 54 KiB LDS (2 blocks/CU)", bytes, [=](hipStream_t st) {
                             ecj_lds_pad_kb = 22;
                             if (ecdk_combine(st, d))
                                 exit(9);
                             ecj_lds_pad_kb = 0;
                         }, bufB, ob});
        }
#endif
        add_combine_fr(v, "run-time four-Russians (8 rows per wave)", a, c, bytes, bufB, ob);
        add_combine_wm<1, 1>(v, "whole matrix 16 rows, compute only", a, bytes, bufB, ob);
        add_combine_wm<2, 1>(v, "whole matrix 2 x 8 rows, compute only", a, bytes, bufB, ob);
        {
            const uint64_t g = (a->nstripes + 7) / 8;
            const void *kern = (const void *)kb_combine_probe<7>;
            v.push_back({"shipped, compute only (probe 7)", bytes, [=](hipStream_t st) {
                             void *args[] = {(void *)a};
                             CHK(hipLaunchKernel(kern, dim3((u32)g), dim3(1024), args, 64u << 10, st));
                         }, nullptr, ob});
        }
        run_group("decode 16+4 dense, whole-matrix program (r06)", v, rounds, iters, s);
        v.clear();
        /* the same with every fragment and the output in an allocation of its
         * own, as torch tensors are (bench.py): placement moves multi-stream
         * kernels */
        static uint8_t *sep[17];
        for (int p = 0; p < K; ++p) {
            CHK(hipMalloc(&sep[p], nst * ECD_CHUNK));
            CHK(hipMemcpy(sep[p], fr[p], nst * ECD_CHUNK, hipMemcpyDeviceToDevice));
        }
        CHK(hipMalloc(&sep[16], ob));
        const CombineArgs *a2 = make_args(K, K, nst, sep, sep[16], true, c);
        add_shipped_combine(v, "shipped, separate allocations", a2, bytes, sep[16], ob);
        add_combine_wm<2, 0>(v, "whole matrix 2 x 8, separate allocations", a2, bytes, sep[16], ob);
#ifdef KB3_WITH_JIT
        {
            ecd_combine_desc_t *d = new ecd_combine_desc_t;
            memset(d, 0, sizeof(*d));
            d->k = K;
            d->rows = K;
            d->nstripes = nst;
            d->in_stride = ECD_CHUNK;
            d->out_stride = (uint64_t)K * ECD_CHUNK;
            for (int p = 0; p < K; ++p) {
                d->in_base[p] = sep[p];
                d->pat[p] = (uint8_t)p;
                d->out_base[p] = sep[16] + (uint64_t)p * ECD_CHUNK;
            }
            memcpy(d->pat + K, c, (size_t)K * K);
            d->npatterns = 1;
            d->pat_bytes = K + K * K;
            v.push_back({"library JIT, separate allocations", bytes, [=](hipStream_t st) {
                             if (ecdk_combine(st, d))
                                 exit(9);
                         }, sep[16], ob});
        }
#endif
        run_group("decode 16+4 dense, separate allocations (r06)", v, rounds, iters, s);
        v.clear();
        for (int p = 0; p < 17; ++p)
            CHK(hipFree(sep[p]));
    }
    if (want(groups, "dec8"))
        decode_group(std::integral_constant<int, 8>{}, "decode 8+4 dense", false);
    if (want(groups, "heal8"))
        decode_group(std::integral_constant<int, 8>{}, "heal 8+4 (4 rows)", true);
    if (want(groups, "dec4"))
        decode_group(std::integral_constant<int, 4>{}, "decode 4+2 dense", false);
    if (want(groups, "dec8b")) {   /* configs[2]: one 64K-stripe batch, 8+4 decode */
        constexpr int K = 8;
        const uint64_t nst = 65536;
        uint8_t *fr[8];
        for (int p = 0; p < K; ++p)
            fr[p] = bufA + (uint64_t)p * nst * ECD_CHUNK;
        uint8_t c[64];
        for (int i = 0; i < 64; ++i)
            c[i] = (uint8_t)(1 + (i * 173 + 11) % 255);
        const CombineArgs *a = make_args(K, K, nst, fr, bufB, true, c);
        const double bytes = 2.0 * nst * K * ECD_CHUNK;
        const size_t ob = (size_t)nst * K * ECD_CHUNK;
        add_shipped_combine(v, "shipped", a, bytes, bufB, ob);
        add_combine_n<K, 8, 1>(v, "narrow NW8 WOT", a, bytes, bufB, ob);
        run_group("decode 8+4, 64K stripes", v, rounds, iters, s);
        v.clear();
    }
    auto mixed_group = [&](auto kk, int n, int np, const char *title, bool spaced = false) {
        /* np random dense patterns over n fragments, 1024-stripe groups.
         * spaced (r06): fragment f at f * nst * 512 (disjoint, as the dense
         * decode groups lay them), else at f * nst * 512 * K / n (overlapping:
         * the pre-r06 layout, kept for comparison) */
        constexpr int K = decltype(kk)::value;
        const uint64_t nst = user / (K * ECD_CHUNK);
        ecd_combine_desc_t d;
        memset(&d, 0, sizeof(d));
        d.k = K;
        d.rows = K;
        d.nstripes = nst;
        d.in_stride = ECD_CHUNK;
        d.out_stride = (uint64_t)K * ECD_CHUNK;
        for (int f = 0; f < n; ++f)
            d.in_base[f] = bufA + (spaced ? (uint64_t)f * nst * ECD_CHUNK
                                          : (uint64_t)f * nst * ECD_CHUNK * K / n);
        for (int r = 0; r < K; ++r)
            d.out_base[r] = bufB + (uint64_t)r * ECD_CHUNK;
        d.npatterns = np;
        d.pat_bytes = K + K * K;
        std::vector<uint8_t> pats((size_t)np * d.pat_bytes);
        uint32_t x = 7;
        for (int q = 0; q < np; ++q) {
            uint8_t *pp = pats.data() + q * d.pat_bytes;
            int used = 0;
            for (int f = 0; f < n && used < K; ++f) {
                x = x * 1103515245u + 12345u;
                if ((int)((x >> 16) % (n - f)) < K - used)
                    pp[used++] = (uint8_t)f;
            }
            for (int i = 0; i < K * K; ++i) {
                x = x * 1103515245u + 12345u;
                pp[K + i] = (uint8_t)(1 + (x >> 16) % 255);
            }
        }
        d.pat_ext = pats.data();
        const uint64_t ngroups = (nst + 1023) / 1024;
        std::vector<uint8_t> gp(ngroups);
        for (auto &g : gp) {
            x = x * 1103515245u + 12345u;
            g = (uint8_t)((x >> 16) % np);
        }
        uint8_t *dgp;
        CHK(hipMalloc(&dgp, ngroups));
        CHK(hipMemcpy(dgp, gp.data(), ngroups, hipMemcpyHostToDevice));
        d.group_pattern = dgp;
        d.group_shift = 10;
        CombineArgs *a = new CombineArgs;
        const double bytes = 2.0 * nst * K * ECD_CHUNK;
        const size_t ob = (size_t)nst * K * ECD_CHUNK;
        {
            /* the library's device entry: packs, uploads the pattern table
             * when the patterns exceed the argument space (bench's 64-mask
             * 16+4 call), launches */
            ecd_combine_desc_t *dl = new ecd_combine_desc_t(d);
            v.push_back({"library (ecdk_combine)", bytes, [=](hipStream_t st) {
                             if (ecdk_combine(st, dl))
                                 exit(9);
                         }, bufB, ob});
        }
        if (ecdk_pack_args(&d, a) != 0) {
            /* the device-table case: the library variant, and the same
             * kernel with the table uploaded once (no per-call host work) */
            std::vector<u32> w((size_t)a->pwords * a->npatterns, 0u);
            pack_words(&d, a->kw, a->pwords, w.data());
            u32 *tab;
            CHK(hipMalloc(&tab, w.size() * 4));
            CHK(hipMemcpy(tab, w.data(), w.size() * 4, hipMemcpyHostToDevice));
            a->patg = tab;
            add_shipped_combine(v, "device-table kernel, table resident", a, bytes, bufB, ob);
            /* the library's per-call ordering steps around that kernel: a
             * stream wait on the (long complete) upload event before it, a
             * reader event recorded after it */
            hipEvent_t *evs = new hipEvent_t[2];
            CHK(hipEventCreateWithFlags(&evs[0], hipEventDisableTiming));
            CHK(hipEventCreateWithFlags(&evs[1], hipEventDisableTiming));
            CHK(hipEventRecord(evs[0], s));
            CHK(hipStreamSynchronize(s));
            v.push_back({"resident + wait on a complete event", bytes, [=](hipStream_t st) {
                             CHK(hipStreamWaitEvent(st, evs[0], 0));
                             if (launch_combine_k<true, kLdsDmaNT>(st, *a))
                                 exit(8);
                         }, bufB, ob});
            v.push_back({"resident + reader event record", bytes, [=](hipStream_t st) {
                             if (launch_combine_k<true, kLdsDmaNT>(st, *a))
                                 exit(8);
                             CHK(hipEventRecord(evs[1], st));
                         }, bufB, ob});
            run_group(title, v, rounds, iters, s);
            v.clear();
            return;
        }
        add_shipped_combine(v, "shipped", a, bytes, bufB, ob);
        {
            /* the same patterns read from a device table (the kernel the
             * library runs past the argument space), table resident */
            CombineArgs *ap = new CombineArgs(*a);
            std::vector<u32> w((size_t)a->pwords * a->npatterns, 0u);
            pack_words(&d, a->kw, a->pwords, w.data());
            u32 *tab;
            CHK(hipMalloc(&tab, w.size() * 4));
            CHK(hipMemcpy(tab, w.data(), w.size() * 4, hipMemcpyHostToDevice));
            ap->patg = tab;
            add_shipped_combine(v, "device-table kernel, same patterns", ap, bytes, bufB, ob);
        }
        /* controls (r06): the mixed mechanism with every group on pattern 0,
         * and pattern 0 as a plain single-pattern call */
        {
            uint8_t *dz;
            CHK(hipMalloc(&dz, ngroups));
            CHK(hipMemset(dz, 0, ngroups));
            ecd_combine_desc_t dz_d = d;
            dz_d.group_pattern = dz;
            CombineArgs *az = new CombineArgs;
            ecd_combine_desc_t d1 = d;
            d1.npatterns = 1;
            d1.group_pattern = nullptr;
            d1.group_shift = 0;
            CombineArgs *a1 = new CombineArgs;
            if (ecdk_pack_args(&dz_d, az) == 0)
                add_shipped_combine(v, "shipped, map all pattern 0", az, bytes, bufB, ob);
            if (ecdk_pack_args(&d1, a1) == 0)
                add_shipped_combine(v, "shipped, pattern 0 single (not mixed)", a1, bytes, bufB, ob);
        }
        auto addm = [&](const char *nm, auto kern, int nw, size_t lds) {
            lds_attr((const void *)kern, lds);
            const uint64_t g = (nst + 3) / 4;
            v.push_back({nm, bytes, [=](hipStream_t st) {
                             hipLaunchKernelGGL(kern, dim3((u32)g), dim3(64 * nw), lds, st, *a);
                         }, bufB, ob});
        };
        addm("narrow NW4 WOT", ec_combine_n<K, 4, true, true, 1>, 4, combine_n_lds<4, 1>(K));
        addm("narrow NW8", ec_combine_n<K, 8, true, true, 0>, 8, combine_n_lds<8, 0>(K));
        addm("narrow NW8 WOT RB2", ec_combine_n<K, 8, true, true, 1, false, false, 2>, 8,
             combine_n_lds<8, 1>(K));
        addm("narrow NW4 WOT RB2", ec_combine_n<K, 4, true, true, 1, false, false, 2>, 4,
             combine_n_lds<4, 1>(K));
        run_group(title, v, rounds, iters, s);
        v.clear();
    };
    if (want(groups, "mixed8"))
        mixed_group(std::integral_constant<int, 8>{}, 12, 16, "mixed 8+4, 16 patterns, 1024-stripe groups");
    if (want(groups, "mixed16"))
        mixed_group(std::integral_constant<int, 16>{}, 20, 7, "mixed 16+4, 7 patterns, 1024-stripe groups");
    /* r06: disjoint fragments; 64 masks of 16+4 (the bench's configs[4] call,
     * device pattern table) */
    if (want(groups, "mixed8s"))
        mixed_group(std::integral_constant<int, 8>{}, 12, 16, "mixed 8+4, 16 patterns, disjoint fragments",
                    true);
    if (want(groups, "mixed16s")) {
        mixed_group(std::integral_constant<int, 16>{}, 20, 7, "mixed 16+4, 7 patterns, disjoint fragments",
                    true);
        mixed_group(std::integral_constant<int, 16>{}, 20, 64,
                    "mixed 16+4, 64 patterns, disjoint fragments", true);
    }
    /* LDS-DMA staging policy (r03): the shipped choice by input size against
     * the default and the non-temporal policy at every size, same process;
     * bytes up to the GiB argument */
    if (want(groups, "ldsnt")) {
        auto policies = [&](const char *title, std::function<void(hipStream_t)> fn, double bytes,
                            uint8_t *out, size_t ob) {
            static const char *nm[3] = {"shipped (policy by size)", "default policy always",
                                        "non-temporal always"};
            const int ov[3] = {-1, kLdsDmaDefault, kLdsDmaNT};
            for (int i = 0; i < 3; ++i) {
                const int o = ov[i];
                v.push_back({nm[i], bytes, [=](hipStream_t st) {
                                 ecdk_ldsnt_override = o;
                                 fn(st);
                             }, out, ob});
            }
            run_group(title, v, rounds, iters, s);
            v.clear();
            ecdk_ldsnt_override = -1;
        };
        uint8_t c[256];
        for (int i = 0; i < 256; ++i)
            c[i] = (uint8_t)(1 + (i * 173 + 11) % 255);
        static char title[64][96];
        int nt = 0;
        const char *szs = getenv("KB3_LDSNT_MIB");      /* e.g. "256,384,512,1024" */
        std::vector<uint64_t> sizes;
        for (const char *q = szs ? szs : "32,128,256,1024"; *q; q += (*q == ',')) {
            sizes.push_back(strtoull(q, const_cast<char **>(&q), 10));
        }
        for (uint64_t mib : sizes) {
            if ((mib << 20) > user)
                continue;
            for (int K : {4, 8, 16}) {
                const uint64_t nst = (mib << 20) / (K * ECD_CHUNK);
                uint8_t *fr[16];
                for (int p = 0; p < K; ++p)
                    fr[p] = bufA + (uint64_t)p * nst * ECD_CHUNK;
                const CombineArgs *a = make_args(K, K, nst, fr, bufB, true, c);
                snprintf(title[nt], 96, "staging policy: decode %d+%d, %llu MiB", K, K == 4 ? 2 : 4,
                         (unsigned long long)mib);
                policies(title[nt++], [=](hipStream_t st) {
                    const int rc = nt_staging(a->nstripes * a->k * ECD_CHUNK)
                                       ? launch_combine_k<true, kLdsDmaNT>(st, *a)
                                       : launch_combine_k<true, kLdsDmaDefault>(st, *a);
                    if (rc)
                        exit(8);
                }, 2.0 * nst * K * ECD_CHUNK, bufB, (size_t)nst * K * ECD_CHUNK);
                const int N = K == 4 ? 6 : K == 8 ? 12 : 20;
                FragPtrs f = frag_ptrs(bufB, nst, N);
                snprintf(title[nt], 96, "staging policy: encode %d+%d, %llu MiB", K, N - K,
                         (unsigned long long)mib);
                policies(title[nt++], [=](hipStream_t st) {
                    void *o[ECD_MAX_ROWS];
                    for (int i = 0; i < N; ++i)
                        o[i] = f.p[i];
                    if (ecdk_encode_vander(st, K, N, nst, bufA, o, false))
                        exit(7);
                }, (double)nst * (K + N) * ECD_CHUNK, f.p[N - 1], (size_t)nst * ECD_CHUNK);
                /* partial-stripe write: interior 3 bytes off, edges from scratch */
                const uint8_t *edge = bufA + user + 4096;
                const uint8_t *ushift = bufA + 3;
                snprintf(title[nt], 96, "staging policy: partial write %d+%d (+3 B), %llu MiB", K,
                         N - K, (unsigned long long)mib);
                policies(title[nt++], [=](hipStream_t st) {
                    void *o[ECD_MAX_ROWS];
                    for (int i = 0; i < N; ++i)
                        o[i] = f.p[i];
                    if (ecdk_encode_vander_rmw(st, K, N, nst, edge, ushift, o))
                        exit(9);
                }, (double)nst * (K + N) * ECD_CHUNK, f.p[N - 1], (size_t)nst * ECD_CHUNK);
            }
        }
    }
    CHK(hipFree(bufA));
    CHK(hipFree(bufB));
    return 0;
}
