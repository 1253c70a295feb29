/*
 * kbench2.hip -- development harness (not product): decode experiments.
 *   A) 4+2 decode, mask 0x3C: shipped ec_combine vs a register-resident
 *      decode whose inverse is folded at compile time (ec_decode_static).
 *
 *   hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/kbench/kbench2.hip -o tools/kbench/kbench2
 */
#include "../../glusterfs_amd/csrc/ec_kernels.hip"

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

namespace proto {

struct Mat {
    u32 m[16][16];
};

constexpr u32 gpow(u32 v, int e)
{
    u32 r = 1;
    for (int i = 0; i < e; ++i)
        r = ecgf::mul(r, v);
    return r;
}

constexpr u32 ginv(u32 a)
{
    for (u32 b = 1; b < 256; ++b)
        if (ecgf::mul(a, b) == 1)
            return b;
    return 0;
}

/* decode matrix for the k bricks set in MASK (ascending) */
template <int K, uint32_t MASK>
constexpr Mat decode_matrix()
{
    Mat a{}, inv{};
    int p = 0;
    for (int b = 0; b < 32 && p < K; ++b)
        if ((MASK >> b) & 1u) {
            for (int j = 0; j < K; ++j)
                a.m[p][j] = gpow((u32)b + 1, K - 1 - j);
            ++p;
        }
    for (int i = 0; i < K; ++i)
        inv.m[i][i] = 1;
    for (int c = 0; c < K; ++c) {
        int piv = c;
        while (a.m[piv][c] == 0)
            ++piv;
        for (int j = 0; j < K; ++j) {
            u32 t = a.m[c][j]; a.m[c][j] = a.m[piv][j]; a.m[piv][j] = t;
            t = inv.m[c][j]; inv.m[c][j] = inv.m[piv][j]; inv.m[piv][j] = t;
        }
        const u32 d = ginv(a.m[c][c]);
        for (int j = 0; j < K; ++j) {
            a.m[c][j] = ecgf::mul(a.m[c][j], d);
            inv.m[c][j] = ecgf::mul(inv.m[c][j], d);
        }
        for (int r = 0; r < K; ++r)
            if (r != c && a.m[r][c]) {
                const u32 f = a.m[r][c];
                for (int j = 0; j < K; ++j) {
                    a.m[r][j] ^= ecgf::mul(f, a.m[c][j]);
                    inv.m[r][j] ^= ecgf::mul(f, inv.m[c][j]);
                }
            }
    }
    return inv;
}

struct InPtrs {
    const uint8_t *p[16];
};

template <int K, uint32_t MASK, int W, int R, bool NTS = false>
__device__ __forceinline__ void decode_row(const u32 (&x)[K][8][W], uint8_t *dst)
{
    constexpr Mat M = decode_matrix<K, MASK>();
    u32 acc[8][W];
#pragma unroll
    for (int b = 0; b < 8; ++b)
#pragma unroll
        for (int w = 0; w < W; ++w)
            acc[b][w] = 0;
    static_for<0, K>([&](auto p) {
        constexpr u32 c = M.m[R][decltype(p)::value];
        if constexpr (c != 0)
            ecgf::mul_xor<c, W>(acc, acc, x[decltype(p)::value]);
    });
    store_chunk<W, NTS>(dst, acc);
}

template <int K, uint32_t MASK, int W, bool NTS = false>
__global__ __launch_bounds__(kBlock) void ec_decode_static(const InPtrs in, uint8_t *out,
                                                           uint64_t nstripes)
{
    constexpr int L = 16 / W;
    const uint64_t gtid = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    const uint64_t stripe = gtid / L;
    if (stripe >= nstripes)
        return;
    const u32 colb = (u32)(gtid % L) * (4 * W);
    u32 x[K][8][W];
#pragma unroll
    for (int p = 0; p < K; ++p)
        load_chunk<W>(in.p[p] + stripe * (uint64_t)ECD_CHUNK + colb, x[p]);
    uint8_t *o = out + stripe * (uint64_t)(K * ECD_CHUNK) + colb;
    static_for<0, K>([&](auto r) {
        decode_row<K, MASK, W, decltype(r)::value, NTS>(x, o + decltype(r)::value * ECD_CHUNK);
    });
}

} // namespace proto

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

template <int K, uint32_t MASK>
static void static_group(uint8_t *bufA, uint8_t *bufB, uint64_t user, int rounds, int iters,
                         hipStream_t s)
{
        const uint64_t nst = user / (K * ECD_CHUNK);
        proto::InPtrs ip;
        ecd_combine_desc_t d;
        memset(&d, 0, sizeof(d));
        d.k = K;
        d.rows = K;
        d.nstripes = nst;
        d.in_stride = ECD_CHUNK;
        d.out_stride = (uint64_t)K * ECD_CHUNK;
        constexpr proto::Mat M = proto::decode_matrix<K, MASK>();
        printf("inv 0x%X:", MASK);
        for (int r = 0; r < K; ++r)
            for (int p = 0; p < K; ++p)
                printf(" %02x", M.m[r][p]);
        printf("\n");
        for (int p = 0; p < K; ++p) {
            ip.p[p] = bufA + (uint64_t)p * nst * ECD_CHUNK;
            d.in_base[p] = const_cast<uint8_t *>(ip.p[p]);
            d.pat[p] = (uint8_t)p;
        }
        for (int r = 0; r < K; ++r) {
            d.out_base[r] = bufB + (uint64_t)r * ECD_CHUNK;
            for (int p = 0; p < K; ++p)
                d.pat[K + r * K + p] = (uint8_t)M.m[r][p];
        }
        d.npatterns = 1;
        d.pat_bytes = K + K * K;
        static CombineArgs a;
        if (ecdk_pack_args(&d, &a))
            exit(2);
        const double bytes = 2.0 * nst * K * ECD_CHUNK;
        const size_t ob = (size_t)nst * K * ECD_CHUNK;
        std::vector<Variant> v;
        v.push_back({"combine (shipped launcher)", bytes, [=](hipStream_t st) {
                         ecdk_combine(st, &d);
                     }, bufB, ob});
        auto addst = [&](const char *nm, auto kern, int W) {
            const uint64_t g = (nst * (16 / W) + kBlock - 1) / kBlock;
            v.push_back({nm, bytes, [=](hipStream_t st) {
                             hipLaunchKernelGGL(kern, dim3((u32)g), dim3(kBlock), 0, st, ip, bufB,
                                                nst);
                         }, bufB, ob});
        };
        addst("static W1", proto::ec_decode_static<K, MASK, 1, false>, 1);
        addst("static W1 NTS", proto::ec_decode_static<K, MASK, 1, true>, 1);
        if constexpr (K <= 8) {
            addst("static W2", proto::ec_decode_static<K, MASK, 2, false>, 2);
            addst("static W2 NTS", proto::ec_decode_static<K, MASK, 2, true>, 2);
        }
        char title[64];
        snprintf(title, sizeof(title), "decode %d+x mask 0x%X", K, MASK);
        run_group(title, v, rounds, iters, s);
    }

int main(int argc, char **argv)
{
    const double gib = argc > 1 ? atof(argv[1]) : 1.0;
    const int rounds = argc > 2 ? atoi(argv[2]) : 7;
    const int iters = 10;
    hipStream_t s;
    CHK(hipStreamCreate(&s));
    const uint64_t user = (uint64_t)(gib * (1ull << 30));
    uint8_t *bufA, *bufB;
    CHK(hipMalloc(&bufA, user * 3));
    CHK(hipMalloc(&bufB, user * 3));
    fill(bufA, user * 3, 12345);

    if (getenv("KB_STATIC")) {
        static_group<4, 0x3C>(bufA, bufB, user, rounds, iters, s);
        static_group<8, 0xFF0>(bufA, bufB, user, rounds, iters, s);
        static_group<8, 0xEB5>(bufA, bufB, user, rounds, iters, s);
        static_group<16, 0xFFFF0>(bufA, bufB, user, rounds, iters, s);
    }
    if (getenv("KB_ZC")) {
    /* Z) zero-copy decode: fragments and output in pinned host memory, read
     * and written by the CUs over PCIe (the host-buffer path of
     * ec_device.hip for pinned callers) -- combine variants */
    for (const int K : {4, 8}) {
        const uint64_t nst = (512ull << 20) / (K * ECD_CHUNK);
        const proto::Mat M = K == 4 ? proto::decode_matrix<4, 0x3C>()
                                    : proto::decode_matrix<8, 0xFF0>();
        uint8_t *hin, *hout;
        CHK(hipHostMalloc((void **)&hin, (size_t)nst * K * ECD_CHUNK, hipHostMallocDefault));
        CHK(hipHostMalloc((void **)&hout, (size_t)nst * K * ECD_CHUNK, hipHostMallocDefault));
        memset(hin, 0x5a, (size_t)nst * K * ECD_CHUNK);
        ecd_combine_desc_t d;
        memset(&d, 0, sizeof(d));
        d.k = K;
        d.rows = K;
        d.nstripes = nst;
        d.in_stride = ECD_CHUNK;
        d.out_stride = (uint64_t)K * ECD_CHUNK;
        for (int p = 0; p < K; ++p) {
            d.in_base[p] = hin + (uint64_t)p * nst * ECD_CHUNK;
            d.pat[p] = (uint8_t)p;
        }
        for (int r = 0; r < K; ++r) {
            d.out_base[r] = hout + (uint64_t)r * ECD_CHUNK;
            for (int p = 0; p < K; ++p)
                d.pat[K + r * K + p] = (uint8_t)M.m[r][p];
        }
        d.npatterns = 1;
        d.pat_bytes = K + K * K;
        static CombineArgs a;
        if (ecdk_pack_args(&d, &a))
            exit(2);
        const double ub = (double)nst * K * ECD_CHUNK; /* user bytes: GB/s = user rate */
        std::vector<Variant> v;
        const size_t ob = (size_t)nst * K * ECD_CHUNK;
        auto addz = [&](const char *nm, auto kern, int ts, int nw, int ldsmul = 1) {
            v.push_back({nm, ub, [=](hipStream_t st) {
                             hipLaunchKernelGGL(kern, dim3((u32)(nst / (8 * ts))), dim3(64 * nw),
                                                (size_t)K * 8 * ts * ECD_CHUNK * ldsmul, st, a);
                         }, hout, ob});
        };
        v.push_back({"shipped device launcher", ub,
                     [=](hipStream_t st) { ecdk_combine(st, &d); }, hout, ob});
        v.push_back({"shipped host launcher", ub,
                     [=](hipStream_t st) { ecdk_combine_host(st, &d); }, hout, ob});
        if (K == 4) {
            addz("TS1 NW8 NTS", ec_combine<4, 1, 8, false, true>, 1, 8);
            addz("TS1 NW8", ec_combine<4, 1, 8, false, false>, 1, 8);
            addz("TS1 NW4", ec_combine<4, 1, 4, false, false>, 1, 4);
            addz("TS2 NW4", ec_combine<4, 2, 4, false, false>, 2, 4);
            addz("TS2 NW8", ec_combine<4, 2, 8, false, false>, 2, 8);
            addz("TS4 NW8", ec_combine<4, 4, 8, false, false>, 4, 8);
            addz("TS4 NW16", ec_combine<4, 4, 16, false, false>, 4, 16);
            addz("ZC NW4", ec_combine_zc<4, 4, false>, 1, 4, 2);
            addz("ZC NW8", ec_combine_zc<4, 8, false>, 1, 8, 2);
        } else {
            addz("TS1 NW4 NTS", ec_combine<8, 1, 4, false, true>, 1, 4);
            addz("TS1 NW4", ec_combine<8, 1, 4, false, false>, 1, 4);
            addz("TS1 NW8", ec_combine<8, 1, 8, false, false>, 1, 8);
            addz("TS2 NW8", ec_combine<8, 2, 8, false, false>, 2, 8);
            addz("TS2 NW16", ec_combine<8, 2, 16, false, false>, 2, 16);
            addz("ZC NW4", ec_combine_zc<8, 4, false>, 1, 4, 2);
            addz("ZC NW8", ec_combine_zc<8, 8, false>, 1, 8, 2);
        }
        char title[96];
        snprintf(title, sizeof title, "zero-copy decode %d+%d, 512 MiB pinned host (GB/s = user)",
                 K, K / 2);
        run_group(title, v, rounds, 3, s);
        CHK(hipHostFree(hin));
        CHK(hipHostFree(hout));
    }
    }
    if (getenv("KB_NTS")) {
    /* B) non-temporal stores vs default, at 1 GiB and at 64K-stripe batches */
    for (const double g : {gib, 0.0}) {
        for (const int K : {4, 8, 16}) {
            const uint64_t nst = g > 0 ? (uint64_t)(g * (1ull << 30)) / (K * ECD_CHUNK) : 65536;
            const int N = K == 16 ? 20 : K + K / 2;
            FragPtrs f;
            for (int i = 0; i < N; ++i)
                f.p[i] = bufB + (uint64_t)i * nst * ECD_CHUNK;
            std::vector<Variant> v;
            const double eb = (double)nst * (K + N) * ECD_CHUNK;
            auto adde = [&](const char *nm, auto kern, int W) {
                const uint64_t gr = (nst * (16 / W) + kBlock - 1) / kBlock;
                v.push_back({nm, eb, [=](hipStream_t st) {
                                 hipLaunchKernelGGL(kern, dim3((u32)gr), dim3(kBlock), 0, st,
                                                    bufA, f, nst);
                             }, f.p[N - 1], (size_t)nst * ECD_CHUNK});
            };
            if (K == 4) {
                adde("enc W2", ec_encode_vander<4, 6, 2, false>, 2);
                adde("enc W2 NTS", ec_encode_vander<4, 6, 2, true>, 2);
            } else if (K == 8) {
                adde("enc W1", ec_encode_vander<8, 12, 1, false>, 1);
                adde("enc W1 NTS", ec_encode_vander<8, 12, 1, true>, 1);
            } else {
                adde("enc W1", ec_encode_vander<16, 20, 1, false>, 1);
                adde("enc W1 NTS", ec_encode_vander<16, 20, 1, true>, 1);
            }
            char title[96];
            snprintf(title, sizeof title, "encode %d+%d, %lu stripes", K, N - K,
                     (unsigned long)nst);
            run_group(title, v, rounds, iters, s);
            v.clear();
            ecd_combine_desc_t d;
            memset(&d, 0, sizeof(d));
            d.k = K;
            d.rows = K;
            d.nstripes = nst;
            d.in_stride = ECD_CHUNK;
            d.out_stride = (uint64_t)K * ECD_CHUNK;
            for (int p = 0; p < K; ++p) {
                d.in_base[p] = bufA + (uint64_t)p * nst * ECD_CHUNK;
                d.pat[p] = (uint8_t)p;
            }
            for (int r = 0; r < K; ++r)
                d.out_base[r] = bufB + (uint64_t)r * ECD_CHUNK;
            for (int i = 0; i < K * K; ++i)
                d.pat[K + i] = (uint8_t)(1 + (i * 97 + 31) % 255);
            d.npatterns = 1;
            d.pat_bytes = K + K * K;
            static CombineArgs a;
            if (ecdk_pack_args(&d, &a))
                exit(2);
            const double db = 2.0 * nst * K * ECD_CHUNK;
            auto addd = [&](const char *nm, auto kern, int ts, int nw) {
                v.push_back({nm, db, [=](hipStream_t st) {
                                 hipLaunchKernelGGL(kern, dim3((u32)(nst / (8 * ts))),
                                                    dim3(64 * nw), (size_t)K * 8 * ts * ECD_CHUNK,
                                                    st, a);
                             }, bufB, (size_t)nst * K * ECD_CHUNK});
            };
            if (K == 4) {
                addd("dec TS2 NW4", ec_combine<4, 2, 4, false, false>, 2, 4);
                addd("dec TS2 NW4 NTS", ec_combine<4, 2, 4, false, true>, 2, 4);
            } else if (K == 8) {
                addd("dec NW8", ec_combine<8, 1, 8, false, false>, 1, 8);
                addd("dec NW8 NTS", ec_combine<8, 1, 8, false, true>, 1, 8);
            } else {
                addd("dec NW8", ec_combine<16, 1, 8, false, false>, 1, 8);
                addd("dec NW8 NTS", ec_combine<16, 1, 8, false, true>, 1, 8);
            }
            snprintf(title, sizeof title, "decode %d+%d dense, %lu stripes", K, N - K,
                     (unsigned long)nst);
            run_group(title, v, rounds, iters, s);
        }
    }
    }
    /* D) combine variants (tile, block size, NT stores) on the real decode
     * matrices of 4+2 mask 0x3C, 8+4 0xFF0 and 16+4 0xFFFF0 */
    for (const int K : {4, 8, 16}) {
        if (getenv("KB_K") && atoi(getenv("KB_K")) != K)
            continue;
        const uint64_t nst = (uint64_t)(gib * (1ull << 30)) / (K * ECD_CHUNK);
        const proto::Mat M = K == 4   ? proto::decode_matrix<4, 0x3C>()
                             : K == 8 ? proto::decode_matrix<8, 0xFF0>()
                                      : proto::decode_matrix<16, 0xFFFF0>();
        ecd_combine_desc_t d;
        memset(&d, 0, sizeof(d));
        d.k = K;
        d.rows = K;
        d.nstripes = nst;
        d.in_stride = ECD_CHUNK;
        d.out_stride = (uint64_t)K * ECD_CHUNK;
        for (int p = 0; p < K; ++p) {
            d.in_base[p] = bufA + (uint64_t)p * nst * ECD_CHUNK;
            d.pat[p] = (uint8_t)p;
        }
        for (int r = 0; r < K; ++r) {
            d.out_base[r] = bufB + (uint64_t)r * ECD_CHUNK;
            for (int p = 0; p < K; ++p)
                d.pat[K + r * K + p] = (uint8_t)M.m[r][p];
        }
        d.npatterns = 1;
        d.pat_bytes = K + K * K;
        static CombineArgs a;
        if (ecdk_pack_args(&d, &a))
            exit(2);
        const double db = 2.0 * nst * K * ECD_CHUNK;
        std::vector<Variant> v;
        auto addd = [&](const char *nm, auto kern, int ts, int nw) {
            v.push_back({nm, db, [=](hipStream_t st) {
                             hipLaunchKernelGGL(kern, dim3((u32)(nst / (8 * ts))), dim3(64 * nw),
                                                (size_t)K * 8 * ts * ECD_CHUNK, st, a);
                         }, bufB, (size_t)nst * K * ECD_CHUNK});
        };
        if (K == 4) {
            addd("TS2 NW4 (shipped)", ec_combine<4, 2, 4, false, false>, 2, 4);
            addd("TS2 NW4 NTS", ec_combine<4, 2, 4, false, true>, 2, 4);
            addd("TS2 NW8 NTS", ec_combine<4, 2, 8, false, true>, 2, 8);
            addd("TS1 NW8", ec_combine<4, 1, 8, false, false>, 1, 8);
            addd("TS1 NW8 NTS", ec_combine<4, 1, 8, false, true>, 1, 8);
        } else if (K == 8) {
            addd("NW8 NTS (shipped)", ec_combine<8, 1, 8, false, true>, 1, 8);
            addd("NW8", ec_combine<8, 1, 8, false, false>, 1, 8);
            addd("NW4 NTS", ec_combine<8, 1, 4, false, true>, 1, 4);
            addd("NW16 NTS", ec_combine<8, 1, 16, false, true>, 1, 16);
            addd("NW4 NTS CW1", ec_combine<8, 1, 4, false, true, 1>, 1, 4);
            addd("NW8 NTS CW1", ec_combine<8, 1, 8, false, true, 1>, 1, 8);
        } else {
            addd("NW8 NTS (shipped)", ec_combine<16, 1, 8, false, true>, 1, 8);
            addd("NW16 NTS", ec_combine<16, 1, 16, false, true>, 1, 16);
            addd("NW16", ec_combine<16, 1, 16, false, false>, 1, 16);
            addd("NW16 NTS CW1", ec_combine<16, 1, 16, false, true, 1>, 1, 16);
            addd("NW8 NTS CW1", ec_combine<16, 1, 8, false, true, 1>, 1, 8);
            addd("TS2 NW16 NTS CW1", ec_combine<16, 2, 16, false, true, 1>, 2, 16);
        }
        char title[96];
        snprintf(title, sizeof title, "decode %d+%d real inverse, %lu stripes", K,
                 K == 16 ? 4 : K / 2, (unsigned long)nst);
        run_group(title, v, rounds, iters, s);
    }
    return 0;
}
