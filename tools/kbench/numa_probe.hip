/* numa_probe.hip -- development probe: does initialising the HIP runtime
 * change the process's memory policy, CPU affinity or thread count, and
 * what happens to a 16-thread CPU loop over buffers allocated after it?
 *   hipcc -O2 --offload-arch=gfx950 tools/kbench/numa_probe.hip -o tools/kbench/numa_probe -lpthread */
#include <hip/hip_runtime.h>
#include <pthread.h>
#include <sched.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>

static void show(const char *tag)
{
    int mode = -1;
    unsigned long mask[16] = {0};
    long r = syscall(SYS_get_mempolicy, &mode, mask, 1024ul, 0ul, 0ul);
    cpu_set_t cs;
    sched_getaffinity(0, sizeof(cs), &cs);
    int nthr = 0;
    FILE *f = fopen("/proc/self/status", "r");
    char line[256];
    char mems[128] = "";
    while (f && fgets(line, sizeof line, f)) {
        if (!strncmp(line, "Threads:", 8))
            nthr = atoi(line + 8);
        if (!strncmp(line, "Mems_allowed_list:", 18))
            snprintf(mems, sizeof mems, "%s", line + 18);
    }
    if (f)
        fclose(f);
    mems[strcspn(mems, "\n")] = 0;
    printf("%-16s mempolicy rc %ld mode %d nodemask %lx | affinity %d cpus | threads %d | mems %s\n",
           tag, r, mode, mask[0], CPU_COUNT(&cs), nthr, mems);
}

static double now()
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + t.tv_nsec * 1e-9;
}

static void *loop(void *v)
{
    double *out = (double *)v;
    const size_t n = 2 << 20;
    unsigned char *a = (unsigned char *)aligned_alloc(4096, n), *b = (unsigned char *)aligned_alloc(4096, n);
    memset(a, 1, n);
    memset(b, 2, n);
    const double t0 = now();
    int it = 0;
    while (now() - t0 < 0.5) {
        for (size_t i = 0; i < n; i += 8)
            *(unsigned long *)(b + i) ^= *(unsigned long *)(a + i);
        ++it;
    }
    *out = (double)it * n * 2 / (now() - t0) / 1e9;
    free(a);
    free(b);
    return nullptr;
}

static void run(const char *tag)
{
    pthread_t th[16];
    double r[16];
    for (int i = 0; i < 16; ++i)
        pthread_create(&th[i], nullptr, loop, &r[i]);
    double s = 0;
    for (int i = 0; i < 16; ++i) {
        pthread_join(th[i], nullptr);
        s += r[i];
    }
    printf("%-16s 16-thread xor loop over 2x2 MiB per thread: %.1f GB/s\n", tag, s);
}

int main()
{
    show("before init");
    run("before init");
    (void)hipFree(nullptr);
    show("after hipFree(0)");
    run("after init");
    void *p;
    (void)hipMalloc(&p, 1 << 20);
    show("after hipMalloc");
    run("after hipMalloc");
    return 0;
}
