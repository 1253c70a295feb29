/* zcenc.hip -- development probe (not product): kernel time of the 4+2 / 8+4
 * encoders on pinned host buffers (coded over PCIe, no copies) for call
 * sizes 128 KiB .. 64 MiB, the shipped one-pass kernel against the
 * grid-stride prefetching ec_encode_vander_zc at several grid shapes.
 *   hipcc -O3 -std=c++17 --offload-arch=gfx950 -Iglusterfs_amd/csrc \
 *       tools/kbench/zcenc.hip -o tools/kbench/zcenc */
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <functional>
#include <vector>

#include "ec_kernels_impl.h"

using namespace ecdev;

#define CHK(x)                                                                            \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess) {                                                           \
            printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);             \
            exit(1);                                                                      \
        }                                                                                 \
    } while (0)

static double time_it(const std::function<void()> &f, hipEvent_t e0, hipEvent_t e1)
{
    std::vector<double> t;
    for (int r = 0; r < 15; ++r) {
        f();
        CHK(hipEventRecord(e0, 0));
        for (int i = 0; i < 4; ++i)
            f();
        CHK(hipEventRecord(e1, 0));
        CHK(hipEventSynchronize(e1));
        float ms;
        CHK(hipEventElapsedTime(&ms, e0, e1));
        t.push_back(ms / 4);
    }
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
}

template <int K, int N, int W>
static void run(size_t bytes, hipEvent_t e0, hipEvent_t e1)
{
    const uint64_t nst = bytes / (512 * K);
    const size_t S = nst * 512 * K, F = nst * 512;
    uint8_t *in, *ref[N];
    CHK(hipHostMalloc(&in, S, hipHostMallocDefault));
    FragPtrs f, g;
    for (int i = 0; i < N; ++i) {
        CHK(hipHostMalloc(&f.p[i], F, hipHostMallocDefault));
        ref[i] = (uint8_t *)malloc(F);
    }
    for (size_t b = 0; b < S; ++b)
        in[b] = (uint8_t)(b * 2654435761u >> 11);
    const double bus = S + (double)N * F;
    auto show = [&](const char *name, int grid, int bs, double ms) {
        int bad = 0;
        for (int i = 0; i < N; ++i)
            bad |= memcmp(ref[i], f.p[i], F) != 0;
        printf("%2d+%-2d %6zu KiB  %-22s grid %5d x %3d  %8.1f us  %6.1f GB/s bus  %6.1f user %s\n",
               K, N - K, S >> 10, name, grid, bs, ms * 1e3, bus / ms / 1e6, S / ms / 1e6,
               bad ? "MISMATCH" : "");
        fflush(stdout);
    };
    const int g0 = (int)vander_grid<W>(nst);
    auto base = [&] {
        hipLaunchKernelGGL((ec_encode_vander<K, N, W, false>), dim3(g0), dim3(kBlock), 0, 0, in, f,
                           nst);
    };
    base();
    CHK(hipDeviceSynchronize());
    for (int i = 0; i < N; ++i)
        memcpy(ref[i], f.p[i], F);
    show("one-pass", g0, 256, time_it(base, e0, e1));
    for (int i = 0; i < N; ++i)
        memset(f.p[i], 0, F);
    const uint64_t thr = nst * (16 / W);
    for (int grid : {16, 64, 128, 256, 512, 1024}) {
        if ((uint64_t)grid * 256 > thr)
            continue;
        auto z = [&] {
            hipLaunchKernelGGL((ec_encode_vander_zc<K, N, W, 256>), dim3(grid), dim3(256), 0, 0,
                               in, f, nst);
        };
        show("zc", grid, 256, time_it(z, e0, e1));
    }
    for (int grid : {256, 512, 1024, 2048}) {
        if ((uint64_t)grid * 64 > thr)
            continue;
        auto z = [&] {
            hipLaunchKernelGGL((ec_encode_vander_zc<K, N, W, 64>), dim3(grid), dim3(64), 0, 0, in,
                               f, nst);
        };
        show("zc", grid, 64, time_it(z, e0, e1));
    }
    (void)g;
    CHK(hipHostFree(in));
    for (int i = 0; i < N; ++i) {
        CHK(hipHostFree(f.p[i]));
        free(ref[i]);
    }
}

int main()
{
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    for (size_t kib : {128, 1024, 4096, 16384, 65536}) {
        run<4, 6, 2>(kib << 10, e0, e1);
        run<8, 12, 1>(kib << 10, e0, e1);
    }
    return 0;
}
