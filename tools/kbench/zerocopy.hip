/* zerocopy.hip -- development probe (not product): PCIe rates when the CUs
 * themselves read / write pinned host memory (no SDMA), to size a zero-copy
 * coder that streams fragments straight between host buffers.
 *   hipcc -O3 --offload-arch=gfx950 tools/kbench/zerocopy.hip -o tools/kbench/zerocopy */
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CHK(x)                                                                            \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess) {                                                           \
            printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);             \
            exit(1);                                                                      \
        }                                                                                 \
    } while (0)

typedef unsigned v4u __attribute__((ext_vector_type(4)));

template <int U, bool NT>
__global__ __launch_bounds__(256) void copy_k(const v4u *__restrict__ in, v4u *__restrict__ out,
                                              size_t n)
{
    const size_t stride = (size_t)gridDim.x * 256 * U;
    for (size_t base = (size_t)blockIdx.x * 256 * U + threadIdx.x; base < n; base += stride) {
        v4u v[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (base + u * 256 < n)
                v[u] = NT ? __builtin_nontemporal_load(in + base + u * 256) : in[base + u * 256];
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (base + u * 256 < n) {
                if (NT)
                    __builtin_nontemporal_store(v[u], out + base + u * 256);
                else
                    out[base + u * 256] = v[u];
            }
    }
}

int main(int argc, char **argv)
{
    const size_t MB = 1 << 20, N = (argc > 1 ? atoi(argv[1]) : 512) * MB;
    void *h1, *h2, *d1, *d2;
    CHK(hipHostMalloc(&h1, N, hipHostMallocDefault));
    CHK(hipHostMalloc(&h2, N, hipHostMallocDefault));
    CHK(hipMalloc(&d1, N));
    CHK(hipMalloc(&d2, N));
    memset(h1, 1, N);
    memset(h2, 2, N);
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    const size_t n = N / 16;
    auto run = [&](const char *name, const void *src, void *dst, int grid, int u, bool nt,
                   double dirs) {
        auto launch = [&] {
            if (u == 4 && nt)
                copy_k<4, true><<<grid, 256>>>((const v4u *)src, (v4u *)dst, n);
            else if (u == 4)
                copy_k<4, false><<<grid, 256>>>((const v4u *)src, (v4u *)dst, n);
            else if (nt)
                copy_k<1, true><<<grid, 256>>>((const v4u *)src, (v4u *)dst, n);
            else
                copy_k<1, false><<<grid, 256>>>((const v4u *)src, (v4u *)dst, n);
        };
        launch();
        CHK(hipDeviceSynchronize());
        CHK(hipEventRecord(e0));
        for (int r = 0; r < 3; ++r)
            launch();
        CHK(hipEventRecord(e1));
        CHK(hipEventSynchronize(e1));
        float ms;
        CHK(hipEventElapsedTime(&ms, e0, e1));
        ms /= 3;
        printf("%-28s grid=%5d U=%d nt=%d  %8.3f ms  %7.1f GB/s per direction\n", name, grid, u,
               nt, ms, N / (ms * 1e-3) / 1e9 * (dirs > 1 ? 1 : 1));
    };
    for (int grid : {256, 1024, 4096}) {
        for (int u : {1, 4}) {
            run("kernel host->dev", h1, d1, grid, u, false, 1);
            run("kernel dev->host", d2, h2, grid, u, false, 1);
            run("kernel dev->host NT", d2, h2, grid, u, true, 1);
            run("kernel host->host", h1, h2, grid, u, false, 2);
            run("kernel host->host NT", h1, h2, grid, u, true, 2);
        }
    }
    return 0;
}
