/* e2e.c -- development probe (not product): host-buffer encode/decode rates
 * of libec_mi355x.so from a plain C process (no torch), the way the GlusterFS
 * ec xlator would call it.  Pinned (ec_method_host_alloc)
 * and pageable (malloc) buffers.
 *   gcc -O2 -Iinclude tools/kbench/e2e.c -Lglusterfs_amd/lib -lec_mi355x \
 *       -Wl,-rpath,'$ORIGIN/../../glusterfs_amd/lib' -o tools/kbench/e2e
 *   tools/kbench/e2e [MiB] [steps] */
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

static void *alloc(size_t n, int pinned)
{
    return pinned ? ec_method_host_alloc(n) : malloc(n);
}

static void release(void *p, int pinned)
{
    if (pinned)
        ec_method_host_free(p);
    else
        free(p);
}

static int run(uint32_t k, uint32_t r, uintptr_t mask, size_t mib, int steps, int pinned)
{
    const uint32_t n = k + r;
    const uint64_t nst = (mib << 20) / (512ull * k), S = nst * 512 * k;
    ec_matrix_list_t list;
    uint8_t *in = alloc(S, pinned), *out = alloc(S, pinned), *frag[32];
    void *fo[32];
    const void *fi[32];
    uint32_t rows[32];
    uint32_t i, nr = 0;
    double te, td, t0;
    int rc, s;

    if (ec_method_init(NULL, &list, k, n, 2 * n, "auto") != 0)
        return 1;
    for (uint64_t b = 0; b < S; b++)
        in[b] = (uint8_t)(b * 2654435761u >> 13);
    for (i = 0; i < n; i++)
        fo[i] = frag[i] = alloc(nst * 512, pinned);
    rc = ec_method_encode_batch(&list, nst, in, fo);
    t0 = now();
    for (s = 0; s < steps && rc == 0; s++)
        rc = ec_method_encode_batch(&list, nst, in, fo);
    te = (now() - t0) / steps;
    for (i = 0; i < n; i++)
        if (mask >> i & 1) {
            rows[nr] = i + 1;
            fi[nr++] = frag[i];
        }
    rc = rc ? rc : ec_method_decode_batch(&list, nst, mask, rows, fi, out);
    t0 = now();
    for (s = 0; s < steps && rc == 0; s++)
        rc = ec_method_decode_batch(&list, nst, mask, rows, fi, out);
    td = (now() - t0) / steps;
    printf("%u+%u %-8s enc %6.2f GB/s user (%5.1f bus)  dec %6.2f GB/s user (%5.1f bus)  %s\n",
           k, r, pinned ? "pinned" : "pageable", S / te / 1e9, S * (1.0 + (double)n / k) / te / 1e9,
           S / td / 1e9, 2.0 * S / td / 1e9,
           rc == 0 && memcmp(in, out, S) == 0 ? "ok" : "MISMATCH");
    for (i = 0; i < n; i++)
        release(frag[i], pinned);
    release(in, pinned);
    release(out, pinned);
    ec_method_fini(&list);
    return rc != 0;
}

int main(int argc, char **argv)
{
    const size_t mib = argc > 1 ? (size_t)atoi(argv[1]) : 512;
    const int steps = argc > 2 ? atoi(argv[2]) : 3;
    int bad = 0;
    for (int pinned = 1; pinned >= 0; pinned--) {
        bad |= run(4, 2, 0x3C, mib, steps, pinned);
        bad |= run(8, 4, 0xFF0, mib, steps, pinned);
    }
    return bad;
}
