/* smallcalls.c -- development probe (not product): many client threads
 * issuing GlusterFS-sized coding calls through the drop-in ABI, the way the
 * disperse xlator does (128 KiB FUSE / write-behind
 * writes, ec-inode-write.c:2136; reads decode per fop, ec-inode-read.c:1196).
 * Every thread owns page-aligned pageable buffers (iobufs) or buffers in a
 * registered arena, calls ec_method_encode / ec_method_decode back to back
 * for `secs` seconds and checks its last decode against its input.
 *   gcc -O2 -pthread -Iinclude tools/kbench/smallcalls.c -Lglusterfs_amd/lib \
 *       -lec_mi355x -Wl,-rpath,'$ORIGIN/../../glusterfs_amd/lib' -o tools/kbench/smallcalls
 *   tools/kbench/smallcalls [secs]  -> one line per (k+r, op, buffers, size, threads) */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "ec_method.h"

static double now(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + t.tv_nsec * 1e-9;
}

typedef struct {
    ec_matrix_list_t *list;
    uint32_t k, n;
    uintptr_t mask;
    size_t size; /* user bytes per call */
    int decode, registered;
    double secs;
    uint8_t *arena; /* registered mode: this thread's slice */
    /* results */
    long calls;
    double *lat;
    long lat_cap;
    int bad;
} worker_t;

static int cmpd(const void *a, const void *b)
{
    const double x = *(const double *)a, y = *(const double *)b;
    return x < y ? -1 : x > y;
}

static void *work(void *arg)
{
    worker_t *w = arg;
    const size_t fs = w->size / w->k;
    uint8_t *in, *out, *frag[32];
    void *fo[32];
    void *fi[32];
    uint32_t rows[32], nr = 0;
    if (w->registered) {
        uint8_t *p = w->arena;
        in = p;
        p += w->size;
        out = p;
        p += w->size;
        for (uint32_t i = 0; i < w->n; i++, p += fs)
            frag[i] = p;
    } else {
        in = aligned_alloc(4096, w->size);
        out = aligned_alloc(4096, w->size);
        for (uint32_t i = 0; i < w->n; i++)
            frag[i] = aligned_alloc(4096, fs);
    }
    for (size_t b = 0; b < w->size; b++)
        in[b] = (uint8_t)((b + (uintptr_t)w) * 2654435761u >> 13);
    for (uint32_t i = 0; i < w->n; i++)
        fo[i] = frag[i];
    ec_method_encode(w->list, w->size, in, fo);
    for (uint32_t i = 0; i < w->n; i++)
        if (w->mask >> i & 1) {
            rows[nr] = i + 1;
            fi[nr++] = frag[i];
        }
    const double t_end = now() + w->secs;
    double t = now();
    while (t < t_end) {
        if (w->decode) {
            if (ec_method_decode(w->list, fs, w->mask, rows, fi, out) != 0) {
                w->bad = 1;
                break;
            }
        } else {
            for (uint32_t i = 0; i < w->n; i++)
                fo[i] = frag[i];
            ec_method_encode(w->list, w->size, in, fo);
        }
        const double t2 = now();
        if (w->calls < w->lat_cap)
            w->lat[w->calls] = t2 - t;
        w->calls++;
        t = t2;
    }
    memset(out, 0, w->size);
    if (ec_method_decode(w->list, fs, w->mask, rows, fi, out) != 0 || memcmp(in, out, w->size))
        w->bad = 1;
    if (!w->registered) {
        free(in);
        free(out);
        for (uint32_t i = 0; i < w->n; i++)
            free(frag[i]);
    }
    return NULL;
}

static int cell(ec_matrix_list_t *list, uint32_t k, uint32_t n, uintptr_t mask, size_t size,
                int decode, int registered, int threads, double secs)
{
    worker_t w[64];
    pthread_t th[64];
    const size_t per = 2 * size + n * (size / k);
    uint8_t *arena = NULL;
    if (registered) {
        arena = aligned_alloc(4096, per * threads);
        if (!arena || ec_method_host_register(arena, per * threads) != 0) {
            printf("register failed: %s\n", ec_method_last_error());
            return 1;
        }
    }
    for (int i = 0; i < threads; i++) {
        memset(&w[i], 0, sizeof(w[i]));
        w[i].list = list;
        w[i].k = k;
        w[i].n = n;
        w[i].mask = mask;
        w[i].size = size;
        w[i].decode = decode;
        w[i].registered = registered;
        w[i].secs = secs;
        w[i].arena = arena ? arena + per * i : NULL;
        w[i].lat_cap = 1 << 20;
        w[i].lat = malloc(sizeof(double) * w[i].lat_cap);
    }
    const double t0 = now();
    for (int i = 0; i < threads; i++)
        pthread_create(&th[i], NULL, work, &w[i]);
    for (int i = 0; i < threads; i++)
        pthread_join(th[i], NULL);
    const double el = now() - t0;
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
    const double busy = secs; /* each thread ran ~secs of back-to-back calls */
    (void)el;
    ec_method_stats_t st;
    ec_method_get_stats(&st);
    printf("%2u+%-2u %s %-10s %5zu KiB x %2d thr: %8.2f GB/s user  %8.0f calls/s  "
           "p50 %7.1f us  p99 %7.1f us  %s  [%s: gpu %llu cpu %llu]\n",
           k, n - k, decode ? "dec" : "enc", registered ? "registered" : "pageable", size >> 10,
           threads, (double)calls * size / busy / 1e9, calls / busy,
           nl ? all[nl / 2] * 1e6 : 0.0, nl ? all[(long)(nl * 0.99)] * 1e6 : 0.0,
           bad ? "MISMATCH" : "ok", ec_method_engine(list), (unsigned long long)st.gpu_calls,
           (unsigned long long)st.cpu_calls);
    fflush(stdout);
    free(all);
    if (registered) {
        ec_method_host_unregister(arena);
        free(arena);
    }
    return bad;
}

int main(int argc, char **argv)
{
    const double secs = argc > 1 ? atof(argv[1]) : 1.0;
    if (argc > 6) { /* one cell: secs k dec reg KiB threads [gen] */
        const uint32_t k = atoi(argv[2]), n = k == 16 ? 20 : k + k / 2;
        ec_matrix_list_t list, pre;
        /* SC_PREINIT=1: also bring up the gfx950 engine (HIP) first, to
         * separate the cost of an initialised HIP runtime from routing */
        const int preinit = getenv("SC_PREINIT") && atoi(getenv("SC_PREINIT"));
        if (preinit && ec_method_init(NULL, &pre, k, n, 2 * n, "auto") != 0)
            return 1;
        if (ec_method_init(NULL, &list, k, n, 2 * n, argc > 7 ? argv[7] : "auto") != 0)
            return 1;
        const size_t sz = ((size_t)atoi(argv[5]) << 10) / (512 * k) * (512 * k);
        const int bad = cell(&list, k, n, ((1u << n) - 1) & ~((1u << (n - k)) - 1), sz,
                             atoi(argv[3]), atoi(argv[4]), atoi(argv[6]), secs);
        ec_method_fini(&list);
        if (preinit)
            ec_method_fini(&pre);
        return bad;
    }
    const size_t sizes[] = {128 << 10, 1 << 20, 4 << 20};
    const int thr[] = {1, 4, 16};
    int bad = 0;
    struct {
        uint32_t k, n;
        uintptr_t mask;
    } geo[] = {{4, 6, 0x3C}, {8, 12, 0xFF0}};
    for (int g = 0; g < 2; g++) {
        ec_matrix_list_t list;
        if (ec_method_init(NULL, &list, geo[g].k, geo[g].n, 2 * geo[g].n, "auto") != 0) {
            printf("init failed: %s\n", ec_method_last_error());
            return 1;
        }
        for (int reg = 0; reg < 2; reg++)
            for (int dec = 0; dec < 2; dec++)
                for (size_t s = 0; s < sizeof(sizes) / sizeof(sizes[0]); s++)
                    for (size_t t = 0; t < sizeof(thr) / sizeof(thr[0]); t++) {
                        /* sizes must be whole stripes */
                        const size_t sz = sizes[s] / (512 * geo[g].k) * (512 * geo[g].k);
                        bad |= cell(&list, geo[g].k, geo[g].n, geo[g].mask, sz, dec, reg,
                                    thr[t], secs);
                    }
        ec_method_fini(&list);
    }
    return bad;
}
