/* ptrq.hip -- development probe: cost of the HIP pointer queries the host
 * path makes per call (hipPointerGetAttributes, hipHostGetDevicePointer) on
 * pageable and pinned host memory, from 1 and 16 threads.
 *   hipcc -O2 --offload-arch=gfx950 tools/kbench/ptrq.hip -o tools/kbench/ptrq -lpthread */
#include <hip/hip_runtime.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <time.h>

static double now(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + t.tv_nsec * 1e-9;
}

struct Arg { void *p; int which; long iters; double secs; };

static void *work(void *v)
{
    Arg *a = (Arg *)v;
    double t0 = now();
    for (long i = 0; i < a->iters; ++i) {
        if (a->which == 0) {
            hipPointerAttribute_t at;
            if (hipPointerGetAttributes(&at, a->p) != hipSuccess)
                (void)hipGetLastError();
        } else {
            void *d = nullptr;
            if (hipHostGetDevicePointer(&d, a->p, 0) != hipSuccess)
                (void)hipGetLastError();
        }
    }
    a->secs = now() - t0;
    return nullptr;
}

int main()
{
    (void)hipFree(nullptr);
    void *pageable = aligned_alloc(4096, 1 << 20);
    void *pinned = nullptr;
    (void)hipHostMalloc(&pinned, 1 << 20, hipHostMallocDefault);
    const char *names[2] = {"hipPointerGetAttributes", "hipHostGetDevicePointer"};
    for (int which = 0; which < 2; ++which)
        for (int mem = 0; mem < 2; ++mem)
            for (int nt : {1, 16}) {
                pthread_t th[16];
                Arg a[16];
                for (int t = 0; t < nt; ++t) {
                    a[t] = {mem ? pinned : pageable, which, 20000, 0};
                    pthread_create(&th[t], nullptr, work, &a[t]);
                }
                double mx = 0;
                for (int t = 0; t < nt; ++t) {
                    pthread_join(th[t], nullptr);
                    mx = a[t].secs > mx ? a[t].secs : mx;
                }
                printf("%-24s %-8s %2d thr: %.3f us per call per thread\n", names[which],
                       mem ? "pinned" : "pageable", nt, mx / 20000 * 1e6);
            }
    return 0;
}
