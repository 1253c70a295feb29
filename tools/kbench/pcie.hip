/* pcie.hip -- development probe (not product): host<->device copy rates
 * with pinned buffers, one direction at a time and both at once, to size
 * the library's PCIe pipeline (ec_device.hip).
 *   hipcc -O3 --offload-arch=gfx950 tools/kbench/pcie.hip -o tools/kbench/pcie */
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

static double now()
{
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

__global__ void touch(unsigned *p)
{
    p[blockIdx.x * blockDim.x + threadIdx.x] += 1;
}

int main(int argc, char **argv)
{
    const size_t MB = 1 << 20, N = (argc > 1 ? atoi(argv[1]) : 512) * MB;
    const size_t chunk = (argc > 2 ? atoi(argv[2]) : 32) * MB;
    void *h1, *h2, *d1, *d2;
    CHK(hipHostMalloc(&h1, N, hipHostMallocDefault));
    CHK(hipHostMalloc(&h2, N, hipHostMallocDefault));
    CHK(hipMalloc(&d1, N));
    CHK(hipMalloc(&d2, N));
    memset(h1, 1, N);
    memset(h2, 2, N);
    hipStream_t s[4];
    for (auto &x : s)
        CHK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
    hipEvent_t ev[2];
    for (auto &e : ev)
        CHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    auto run = [&](const char *name, int mode) {
        for (int rep = 0; rep < 2; ++rep) {
            CHK(hipDeviceSynchronize());
            const double t0 = now();
            for (size_t off = 0; off < N; off += chunk) {
                const size_t n = off + chunk <= N ? chunk : N - off;
                if (mode == 0 || mode == 2)
                    CHK(hipMemcpyAsync((char *)d1 + off, (char *)h1 + off, n,
                                       hipMemcpyHostToDevice, s[0]));
                if (mode == 1 || mode == 2)
                    CHK(hipMemcpyAsync((char *)h2 + off, (char *)d2 + off, n,
                                       hipMemcpyDeviceToHost, s[1]));
                if (mode == 3) { /* both directions, alternating 2 streams each */
                    const int k = (off / chunk) & 1;
                    CHK(hipMemcpyAsync((char *)d1 + off, (char *)h1 + off, n,
                                       hipMemcpyHostToDevice, s[k]));
                    CHK(hipMemcpyAsync((char *)h2 + off, (char *)d2 + off, n,
                                       hipMemcpyDeviceToHost, s[2 + k]));
                }
                if (mode == 5 || mode == 6) { /* kernel -> event -> D2H on another stream */
                    const int k = (off / chunk) & 1;
                    hipEvent_t &e = ev[k];
                    touch<<<64, 256, 0, s[0]>>>((unsigned *)d2);
                    CHK(hipEventRecord(e, s[0]));
                    hipStream_t ds = mode == 5 ? s[2 + k] : s[0];
                    if (mode == 5)
                        CHK(hipStreamWaitEvent(ds, e, 0));
                    CHK(hipMemcpyAsync((char *)h2 + off, (char *)d2 + off, n,
                                       hipMemcpyDeviceToHost, ds));
                }
                if (mode == 4) /* both directions on ONE stream, in order */
                {
                    CHK(hipMemcpyAsync((char *)d1 + off, (char *)h1 + off, n,
                                       hipMemcpyHostToDevice, s[0]));
                    CHK(hipMemcpyAsync((char *)h2 + off, (char *)d2 + off, n,
                                       hipMemcpyDeviceToHost, s[0]));
                }
            }
            CHK(hipDeviceSynchronize());
            const double t = now() - t0;
            if (rep == 1) {
                const double bytes = (mode >= 2 && mode <= 4 ? 2.0 : 1.0) * N;
                printf("%-40s %8.2f ms  %7.1f GB/s total\n", name, t * 1e3, bytes / t / 1e9);
            }
        }
    };
    printf("buffer %zu MiB, chunk %zu MiB\n", N / MB, chunk / MB);
    run("H2D only", 0);
    run("D2H only", 1);
    run("H2D + D2H, separate streams", 2);
    run("H2D + D2H, 2+2 streams", 3);
    run("H2D then D2H, one stream", 4);
    run("D2H after kernel, cross-stream event", 5);
    run("D2H after kernel, same stream", 6);
    return 0;
}
