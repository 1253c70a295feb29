/* Host-side stress for the sanitizer builds (tests/test_sanitizers.py):
 * ec_method.c (GF tables, matrices, the mask-keyed LRU cache of inverses,
 * config pack/unpack/check) and the CPU engine, with ec_device stubbed out.
 * 8 threads share one list whose cache holds 3 matrices while 15 masks are
 * in use (eviction under contention, ec-method.c:200-256); every decode is
 * checked against the data it was encoded from. */
#include <errno.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "ec_method.h"

enum { K = 4, N = 6, NST = 37, THREADS = 8, ITERS = 60 };
enum { K2 = 16, N2 = 20, NST2 = 16 };

static ec_matrix_list_t list, list16;
static unsigned char data[512 * K * NST], *frag[N];
static unsigned char data16[512 * K2 * NST2], *frag16[N2];
static int failures;

/* Mixed decodes on either volume (r05: the per-thread pattern-set memo is
 * shared by volumes of different k, and grows as sets grow): a set of 1-12
 * masks, drawn from a few fixed sets so calls repeat, one mask per stripe
 * group; every group checked against the data. */
static void
mixed(unsigned *seed, int wide)
{
    const uint32_t k = wide ? K2 : K, n = wide ? N2 : N, nst = wide ? NST2 : NST;
    const unsigned char *ref = wide ? data16 : data;
    unsigned char **fr = wide ? frag16 : frag;
    const uint32_t group = wide ? 2 : 4, ng = (nst + group - 1) / group;
    uintptr_t gm[64];
    unsigned char *out = malloc((size_t)512 * k * nst);
    unsigned set = rand_r(seed) % 3, sseed = set * 977u + (unsigned)wide;
    uint32_t nm = 1 + (set * 5 + (unsigned)wide) % 12, g;
    uintptr_t pool[12];

    for (uint32_t i = 0; i < nm; i++) {
        uintptr_t m = 0;
        while ((uint32_t)__builtin_popcountll(m) < k)
            m |= (uintptr_t)1 << (rand_r(&sseed) % n);
        pool[i] = m;
    }
    for (g = 0; g < ng; g++)
        gm[g] = pool[rand_r(seed) % nm];
    memset(out, 0, (size_t)512 * k * nst);
    if (ec_method_decode_mixed(wide ? &list16 : &list, nst, group, gm,
                               (const void *const *)fr, out) != 0 ||
        memcmp(out, ref, (size_t)512 * k * nst) != 0)
        __atomic_add_fetch(&failures, 1, __ATOMIC_RELAXED);
    free(out);
}

static void *
worker(void *arg)
{
    unsigned seed = (unsigned)(size_t)arg * 7919u + 1;
    unsigned char *out = malloc(sizeof(data));
    for (int it = 0; it < ITERS; it++) {
        uint32_t rows[K], m = 0, p = 0;
        void *in[K];
        while (__builtin_popcount(m) < K)
            m |= 1u << (rand_r(&seed) % N);
        for (uint32_t b = 0; b < N; b++)
            if (m >> b & 1) {
                rows[p] = b + 1;
                in[p++] = frag[b];
            }
        memset(out, 0, sizeof(data));
        if (ec_method_decode(&list, 512 * NST, m, rows, in, out) != 0 ||
            memcmp(out, data, sizeof(data)) != 0)
            __atomic_add_fetch(&failures, 1, __ATOMIC_RELAXED);
        mixed(&seed, it & 1);
        if (it % 10 == 0) {
            unsigned char *f2[N];
            void *o[N];
            for (int i = 0; i < N; i++)
                o[i] = f2[i] = malloc(512 * NST);
            ec_method_encode(&list, sizeof(data), data, o);
            for (int i = 0; i < N; i++) {
                if (memcmp(f2[i], frag[i], 512 * NST) != 0)
                    __atomic_add_fetch(&failures, 1, __ATOMIC_RELAXED);
                free(f2[i]);
            }
        }
    }
    free(out);
    return NULL;
}

/* ECD_STUB_GPU=1 (the stub's pretend device codes on the CPU engine): calls
 * of >= 1 MiB split between the device layer, on the library's helper
 * threads, and the caller (ec_method.c encode_split / decode_split) -- the
 * helper pool's hand-off under the sanitizers.  4 threads, each its own
 * 1.6 MiB 4+2 encode, decode and 16-stripe-group mixed decode. */
enum { BIG = 800 };

static void *
split_worker(void *arg)
{
    const size_t db = (size_t)512 * K * BIG, fb = (size_t)512 * BIG;
    unsigned char *d = malloc(db), *out = malloc(db), *f[N];
    void *o[N], *in[K];
    uint32_t rows[K] = {3, 4, 5, 6};
    uintptr_t gm[BIG / 16];

    for (size_t i = 0; i < db; i++)
        d[i] = (unsigned char)((i + (size_t)arg) * 2654435761u >> 11);
    for (int i = 0; i < N; i++)
        o[i] = f[i] = malloc(fb);
    for (int it = 0; it < 6; it++) {
        if (ec_method_encode_batch(&list, BIG, d, o) != 0)
            __atomic_add_fetch(&failures, 1, __ATOMIC_RELAXED);
        for (int i = 0; i < K; i++)
            in[i] = f[rows[i] - 1];
        memset(out, 0, db);
        if (ec_method_decode_batch(&list, BIG, 0x3C, rows, (const void *const *)in, out) != 0 ||
            memcmp(out, d, db) != 0)
            __atomic_add_fetch(&failures, 1, __ATOMIC_RELAXED);
        for (size_t g = 0; g < BIG / 16; g++)
            gm[g] = g & 1 ? 0x3C : 0x0F;
        memset(out, 0, db);
        if (ec_method_decode_mixed(&list, BIG, 16, gm, (const void *const *)f, out) != 0 ||
            memcmp(out, d, db) != 0)
            __atomic_add_fetch(&failures, 1, __ATOMIC_RELAXED);
    }
    for (int i = 0; i < N; i++)
        free(f[i]);
    free(d);
    free(out);
    return NULL;
}

int
main(void)
{
    pthread_t th[THREADS];
    void *o[N];
    uint8_t v[8];
    ec_config_t c, d;

    for (size_t i = 0; i < sizeof(data); i++)
        data[i] = (unsigned char)(i * 2654435761u >> 13);
    if (ec_method_init(NULL, &list, K, N, 3, "auto") != 0)
        return 2;
    for (int i = 0; i < N; i++)
        o[i] = frag[i] = malloc(512 * NST);
    ec_method_encode(&list, sizeof(data), data, o);
    {
        void *o2[N2];
        for (size_t i = 0; i < sizeof(data16); i++)
            data16[i] = (unsigned char)(i * 2246822519u >> 11);
        if (ec_method_init(NULL, &list16, K2, N2, 2 * N2, "auto") != 0)
            return 2;
        for (int i = 0; i < N2; i++)
            o2[i] = frag16[i] = malloc(512 * NST2);
        ec_method_encode(&list16, sizeof(data16), data16, o2);
    }
    for (int t = 0; t < THREADS; t++)
        pthread_create(&th[t], NULL, worker, (void *)(size_t)t);
    for (int t = 0; t < THREADS; t++)
        pthread_join(th[t], NULL);
    if (getenv("ECD_STUB_GPU")) {
        ec_method_stats_t st0, st1;
        ec_method_get_stats(&st0);
        for (int t = 0; t < 4; t++)
            pthread_create(&th[t], NULL, split_worker, (void *)(size_t)t);
        for (int t = 0; t < 4; t++)
            pthread_join(th[t], NULL);
        ec_method_get_stats(&st1);
        /* every call split: both engines counted once per call */
        if (st1.gpu_calls - st0.gpu_calls < 4 * 6 * 3 || st1.cpu_calls - st0.cpu_calls < 4 * 6 * 3)
            failures++;
        printf("split calls: gpu %llu cpu %llu\n",
               (unsigned long long)(st1.gpu_calls - st0.gpu_calls),
               (unsigned long long)(st1.cpu_calls - st0.cpu_calls));
    }
    if (list.count > 3)
        failures++;
    /* trusted.ec.config round trip and checks (ec-helpers.c:298-380) */
    ec_method_config_fill(6, 2, &c);
    if (ec_method_config_pack(&c, v) || ec_method_config_unpack(v, 8, &d) ||
        ec_method_config_check(6, 2, &d) != 0 || ec_method_config_check(6, 1, &d) != -ENOTSUP)
        failures++;
    memset(v, 0, 8);
    if (ec_method_config_unpack(v, 8, &d) != -ENODATA || ec_method_config_unpack(v, 7, &d) != -EINVAL)
        failures++;
    /* every inverse of 8+4, as the cache computes them */
    for (uint32_t m = 0; m < (1u << 12); m++) {
        uint32_t rows[8], p = 0, inv[64];
        if (__builtin_popcount(m) != 8)
            continue;
        for (uint32_t b = 0; b < 12; b++)
            if (m >> b & 1)
                rows[p++] = b + 1;
        if (ec_method_inverse_matrix(8, rows, inv) != 0)
            failures++;
    }
    ec_method_fini(&list);
    ec_method_fini(&list); /* idempotent */
    ec_method_fini(&list16);
    for (int i = 0; i < N; i++)
        free(frag[i]);
    for (int i = 0; i < N2; i++)
        free(frag16[i]);
    printf("sanitize_check failures=%d\n", failures);
    return failures != 0;
}
