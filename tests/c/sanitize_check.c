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

static ec_matrix_list_t list;
static unsigned char data[512 * K * NST], *frag[N];
static int failures;

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
    for (int t = 0; t < THREADS; t++)
        pthread_create(&th[t], NULL, worker, (void *)(size_t)t);
    for (int t = 0; t < THREADS; t++)
        pthread_join(th[t], NULL);
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
    for (int i = 0; i < N; i++)
        free(frag[i]);
    printf("sanitize_check failures=%d\n", failures);
    return failures != 0;
}
