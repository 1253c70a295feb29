/* concur.c -- concurrency probe for the small-call batching question
 * (VERDICT r03 "do this" #4): GlusterFS codes one fop per
 * call on many threads -- self-heal runs background-heals = 8 windows of
 * 4 MiB at once (ec.c:1714-1718, ec-heal.c:2063-2068), FUSE / write-behind
 * writes are 128 KiB (fuse-bridge.c:5179, write-behind.c:3198-3200) -- and
 * each GPU-routed host call is its own launch.  A batching queue would
 * coalesce concurrent calls into one launch; its best case is ONE call
 * carrying all of their bytes.  So every scenario is timed three ways:
 *   concurrent  T threads issuing their own calls back to back (today)
 *   ceiling     one thread issuing calls T times as large (what a perfect
 *               coalescing queue would launch: same bytes, one launch)
 *   serial      one thread issuing the small calls back to back
 * per engine setting (run the binary once per setting: EC_GPU_ALWAYS=1 for
 * "gpu", gen "avx" for "cpu", default "auto") and buffer provenance (pool:
 * ec_method_buffer_get, what the integration patch gives a client; pageable:
 * plain malloc).
 *   heal   8 threads: 8+4 decode of a 4 MiB window (8 fragments) + encode
 *          of the decoded window into 12 fragments (ec-heal.c:2048-2107)
 *   write  16 threads: 8+4 encode of 128 KiB (a FUSE write)
 *   read   16 threads: 8+4 decode of 128 KiB with 4 bricks lost
 * Output: one JSON line per (scenario, provenance, way).
 *   gcc -O2 -pthread -Iinclude tools/kbench/concur.c -Lglusterfs_amd/lib \
 *       -lec_mi355x -Wl,-rpath,'$ORIGIN/../../glusterfs_amd/lib' -o tools/kbench/concur
 *   tools/kbench/concur [secs] [gen] [pool|pageable|both]
 *   (CONCUR_HEAL_THREADS: heal threads, default 8; CONCUR_SCEN=heal|write|read:
 *   that scenario only; CONCUR_WAYS=concurrent,ceiling,serial: those ways only)
 * Each line also reports the process's threads after the run (the library's
 * copy / helper threads and the HIP runtime's, plus main) and the copy
 * threads the library sized from the CPU quota.                                                   */
#define _GNU_SOURCE
#include <pthread.h>
#include <sched.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <dirent.h>
#include <time.h>

#include "ec_method.h"

/* threads of this process now (after the workers were joined: the main
 * thread plus every thread the library and the HIP runtime started) */
static int proc_threads(void)
{
    DIR *d = opendir("/proc/self/task");
    int n = 0;
    if (!d)
        return -1;
    for (struct dirent *e; (e = readdir(d));)
        n += e->d_name[0] != '.';
    closedir(d);
    return n;
}

static double now(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + t.tv_nsec * 1e-9;
}

enum { HEAL = 0, WRITE = 1, READ = 2 };
static const char *scen_name[] = {"heal_8+4_4MiB", "write_8+4_128KiB", "read_8+4_128KiB"};

typedef struct {
    ec_matrix_list_t *list;
    int scen, pool;
    size_t size;      /* user bytes per call */
    double secs;
    long calls;
    double lat_sum;
    double *lat;
    long lat_cap;
    int bad;
    pthread_barrier_t *start;   /* every thread set up before any is timed */
} worker_t;

static const uint32_t K = 8, N = 12;
static const uintptr_t MASK = 0xFF0; /* bricks 0..3 lost */

static uint8_t *get(size_t n, int pool)
{
    uint8_t *p = pool ? ec_method_buffer_get(n) : NULL;
    if (!p)
        p = aligned_alloc(4096, (n + 4095) / 4096 * 4096);
    return p;
}

static void put(uint8_t *p)
{
    if (p && ec_method_buffer_put(p) != 1)
        free(p);
}

static int cmpd(const void *a, const void *b)
{
    const double x = *(const double *)a, y = *(const double *)b;
    return x < y ? -1 : x > y;
}

/* Heal windows cycle through NWIN distinct sets of buffers per thread (a
 * heal streams a file: 8 threads x 4 x 16 MiB, past the host's L3), FUSE-sized
 * calls reuse one set (a write's data was just copied in by the kernel). */
#define NWIN 4

static void *work(void *arg)
{
    worker_t *w = arg;
    const size_t fs = w->size / K;
    const int nw = w->scen == HEAL ? NWIN : 1;
    uint8_t *in[NWIN], *out[NWIN], *fr[NWIN], *fr2[NWIN];
    void *fo[32], *fi[NWIN][32];
    uint32_t rows[32], nr = 0;
    for (int x = 0; x < nw; x++) {
        in[x] = get(w->size, w->pool);
        out[x] = get(w->size, w->pool);
        fr[x] = get(fs * N, w->pool);
        fr2[x] = get(fs * N, w->pool);
        for (size_t b = 0; b < w->size; b++)
            in[x][b] = (uint8_t)((b + x + (uintptr_t)w) * 2654435761u >> 13);
        for (uint32_t i = 0; i < N; i++)
            fo[i] = fr[x] + i * fs;
        ec_method_encode(w->list, w->size, in[x], fo);
        nr = 0;
        for (uint32_t i = 0; i < N; i++)
            if (MASK >> i & 1) {
                rows[nr] = i + 1;
                fi[x][nr++] = fr[x] + i * fs;
            }
    }
    pthread_barrier_wait(w->start);
    const double t_end = now() + w->secs;
    double t = now();
    int x = 0;
    while (t < t_end) {
        if (w->scen != WRITE &&
            ec_method_decode(w->list, fs, MASK, rows, fi[x], out[x]) != 0) {
            w->bad = 1;
            break;
        }
        if (w->scen != READ) {
            for (uint32_t i = 0; i < N; i++)
                fo[i] = fr2[x] + i * fs;
            ec_method_encode(w->list, w->size, w->scen == HEAL ? out[x] : in[x], fo);
        }
        const double t2 = now();
        if (w->calls < w->lat_cap)
            w->lat[w->calls] = t2 - t;
        w->calls++;
        t = t2;
        x = (x + 1) % nw;
    }
    for (x = 0; x < nw; x++) {
        memset(out[x], 0, w->size);
        if (ec_method_decode(w->list, fs, MASK, rows, fi[x], out[x]) != 0 ||
            memcmp(in[x], out[x], w->size))
            w->bad = 1;
        if (w->scen != READ && w->calls >= nw && memcmp(fr[x], fr2[x], fs * N))
            w->bad = 1;
        put(in[x]);
        put(out[x]);
        put(fr[x]);
        put(fr2[x]);
    }
    return NULL;
}

/* T threads of calls of `size` user bytes */
static int run(ec_matrix_list_t *list, const char *way, int scen, int pool, size_t size,
               int threads, double secs, const char *mode)
{
    worker_t w[64];
    pthread_t th[64];
    ec_method_stats_t s0, s1;
    pthread_barrier_t start;
    pthread_barrier_init(&start, NULL, threads);
    ec_method_get_stats(&s0);
    for (int i = 0; i < threads; i++) {
        memset(&w[i], 0, sizeof(w[i]));
        w[i].list = list;
        w[i].scen = scen;
        w[i].pool = pool;
        w[i].size = size;
        w[i].secs = secs;
        w[i].lat_cap = 1 << 20;
        w[i].lat = malloc(sizeof(double) * w[i].lat_cap);
        w[i].start = &start;
    }
    for (int i = 0; i < threads; i++)
        pthread_create(&th[i], NULL, work, &w[i]);
    for (int i = 0; i < threads; i++)
        pthread_join(th[i], NULL);
    ec_method_get_stats(&s1);
    pthread_barrier_destroy(&start);
    long calls = 0, nl = 0;
    int bad = 0;
    for (int i = 0; i < threads; i++) {
        calls += w[i].calls;
        bad |= w[i].bad;
    }
    double *all = malloc(sizeof(double) * (calls + 1));
    for (int i = 0; i < threads; i++) {
        const long c = w[i].calls < w[i].lat_cap ? w[i].calls : w[i].lat_cap;
        memcpy(all + nl, w[i].lat, sizeof(double) * c);
        nl += c;
        free(w[i].lat);
    }
    qsort(all, nl, sizeof(double), cmpd);
    printf("{\"scenario\": \"%s\", \"mode\": \"%s\", \"buffers\": \"%s\", \"way\": \"%s\", "
           "\"threads\": %d, \"call_KiB\": %zu, \"user_GBps\": %.2f, \"calls_per_s\": %.0f, "
           "\"p50_us\": %.1f, \"p99_us\": %.1f, \"gpu_calls\": %llu, \"cpu_calls\": %llu, "
           "\"proc_threads\": %d, \"copy_threads\": %d, \"ok\": %s}\n",
           scen_name[scen], mode, pool ? "pool" : "pageable", way, threads, size >> 10,
           (double)calls * size / secs / 1e9, calls / secs, nl ? all[nl / 2] * 1e6 : 0.0,
           nl ? all[(long)(nl * 0.99)] * 1e6 : 0.0,
           (unsigned long long)(s1.gpu_calls - s0.gpu_calls),
           (unsigned long long)(s1.cpu_calls - s0.cpu_calls), proc_threads(),
           ec_method_copy_threads(), bad ? "false" : "true");
    fflush(stdout);
    free(all);
    return bad;
}

/* Bind the process to the CPUs of the GPU's NUMA node that it may use (as
 * INTEGRATION.md advises a client and bench.py does per rank): the pool's
 * pages sit on that node, and CPU-engine threads on the other socket would
 * read them remotely.  CONCUR_BIND=0 leaves the affinity alone. */
static void bind_gpu_node(void)
{
    const char *e = getenv("CONCUR_BIND");
    if (e && *e == '0')
        return;
    const int node = ec_method_device_numa_node(0);
    if (node < 0)
        return;
    char path[96], buf[4096];
    snprintf(path, sizeof path, "/sys/devices/system/node/node%d/cpulist", node);
    FILE *f = fopen(path, "r");
    if (!f)
        return;
    if (!fgets(buf, sizeof buf, f)) {
        fclose(f);
        return;
    }
    fclose(f);
    cpu_set_t allowed, want;
    CPU_ZERO(&want);
    sched_getaffinity(0, sizeof allowed, &allowed);
    for (char *t = strtok(buf, ",\n"); t; t = strtok(NULL, ",\n")) {
        int a, b;
        if (sscanf(t, "%d-%d", &a, &b) != 2)
            b = a = atoi(t);
        for (int c = a; c <= b && c < CPU_SETSIZE; c++)
            if (CPU_ISSET(c, &allowed))
                CPU_SET(c, &want);
    }
    if (CPU_COUNT(&want) > 0 && sched_setaffinity(0, sizeof want, &want) == 0)
        fprintf(stderr, "concur: bound to %d CPUs of node %d\n", CPU_COUNT(&want), node);
}

/* CONCUR_WAYS: comma-separated ways to run (default all three) */
static int way_on(const char *way)
{
    const char *e = getenv("CONCUR_WAYS");
    return !e || !*e || strstr(e, way) != NULL;
}

int main(int argc, char **argv)
{
    bind_gpu_node();
    const double secs = argc > 1 ? atof(argv[1]) : 1.0;
    const char *gen = argc > 2 ? argv[2] : "auto";
    const char *ga = getenv("EC_GPU_ALWAYS");
    const char *mode = strcmp(gen, "auto") ? "cpu" : (ga && *ga == '1') ? "gpu" : "auto";
    ec_matrix_list_t list;
    if (ec_method_init(NULL, &list, K, N, 2 * N, gen) != 0)
        return 1;
    int bad = 0;
    const struct {
        int scen, threads;
        size_t size;
    } sc[] = {{HEAL, 8, 4u << 20}, {WRITE, 16, 128u << 10}, {READ, 16, 128u << 10}};
    const char *ht = getenv("CONCUR_HEAL_THREADS");   /* heal threads (default 8) */
    const char *only = getenv("CONCUR_SCEN");          /* heal | write | read */
    const int heal_threads = ht && atoi(ht) > 0 ? atoi(ht) : 8;
    const char *which = argc > 3 ? argv[3] : "both";   /* pool | pageable | both */
    for (int pool = 1; pool >= 0; pool--)
        for (size_t s = 0; s < sizeof(sc) / sizeof(sc[0]); s++) {
            const int threads = sc[s].scen == HEAL ? heal_threads : sc[s].threads;
            if ((pool && !strcmp(which, "pageable")) || (!pool && !strcmp(which, "pool")))
                continue;
            if (only && strncmp(scen_name[sc[s].scen], only, strlen(only)))
                continue;
            if (way_on("concurrent"))
                bad |= run(&list, "concurrent", sc[s].scen, pool, sc[s].size, threads, secs, mode);
            if (way_on("ceiling"))
                bad |= run(&list, "ceiling", sc[s].scen, pool, sc[s].size * threads, 1, secs,
                           mode);
            if (way_on("serial"))
                bad |= run(&list, "serial", sc[s].scen, pool, sc[s].size, 1, secs, mode);
        }
    ec_method_fini(&list);
    return bad;
}
