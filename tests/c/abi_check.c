/* Compiled with plain gcc against include/ec_method.h and linked against
 * glusterfs_amd/lib/libec_mi355x.so, the way GlusterFS's ec xlator would
 * (INTEGRATION.md).  Checks the 120-byte ec_matrix_list_t layout of
 * ec-types.h:549-562 and exercises ec_method_init/encode/decode/fini and the
 * row-masked encode the integration patch's ec_writev_encode calls:
 * argv[1] = "gpu" requires the gfx950 engine, "cpu" the CPU engine (a node
 * without GPU, or cpu-extensions=none). */
#include <errno.h>
#include <stddef.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "ec_method.h"

int
main(int argc, char **argv)
{
    ec_matrix_list_t list;
    int rc, expect_gpu = argc > 1 && strcmp(argv[1], "gpu") == 0;

    if (sizeof(ec_matrix_list_t) != 120 || offsetof(ec_matrix_list_t, columns) != 56 ||
        offsetof(ec_matrix_list_t, rows) != 60 || offsetof(ec_matrix_list_t, max) != 64 ||
        offsetof(ec_matrix_list_t, count) != 68 || offsetof(ec_matrix_list_t, stripe) != 72 ||
        offsetof(ec_matrix_list_t, pool) != 80 || offsetof(ec_matrix_list_t, gf) != 88 ||
        offsetof(ec_matrix_list_t, code) != 96 || offsetof(ec_matrix_list_t, encode) != 104 ||
        offsetof(ec_matrix_list_t, objects) != 112) {
        printf("layout mismatch\n");
        return 2;
    }
    rc = ec_method_init(NULL, &list, 8, 4, 8, "auto"); /* k > n: -EINVAL */
    ec_method_fini(&list);                              /* safe after a failed init */
    if (rc != -EINVAL) {
        printf("bad geometry accepted: %d\n", rc);
        return 3;
    }
    rc = ec_method_init(NULL, &list, 4, 6, 12, expect_gpu ? "auto" : "none");
    if (rc != 0) {
        printf("init failed %d\n", rc);
        return 4;
    }
    printf("engine %s\n", ec_method_engine(&list));
    if (expect_gpu != (strncmp(ec_method_engine(&list), "gfx950", 6) == 0)) {
        printf("wrong engine\n");
        return 7;
    }
    {
        enum { NST = 100, K = 4, N = 6 };
        unsigned char *in = malloc(512 * K * NST), *frag[N], *dec = malloc(512 * K * NST);
        void *outs[N], *ins[K];
        uint32_t rows[K] = {3, 4, 5, 6};
        int i;

        for (i = 0; i < 512 * K * NST; i++)
            in[i] = (unsigned char)(i * 131 + 7);
        for (i = 0; i < N; i++)
            outs[i] = frag[i] = malloc(512 * NST);
        ec_method_encode(&list, 512 * K * NST, in, outs);
        if (outs[0] != frag[0] + 512 * NST) {
            printf("out[] not advanced\n");
            return 5;
        }
        for (i = 0; i < K; i++)
            ins[i] = frag[rows[i] - 1];
        rc = ec_method_decode(&list, 512 * NST, 0x3C, rows, ins, dec);
        if (rc != 0 || memcmp(in, dec, 512 * K * NST) != 0) {
            printf("decode rc=%d mismatch\n", rc);
            return 6;
        }
        {
            /* a heal write of bricks 0 and 1 (the patch's ec_writev_encode):
             * only those two fragments, equal to the full encode's */
            unsigned char *h0 = malloc(512 * NST), *h1 = malloc(512 * NST);
            void *hs[N] = {h0, h1, NULL, NULL, NULL, NULL};
            ec_method_encode_rows(&list, 512 * K * NST, in, 0x3, hs);
            if (hs[0] != h0 + 512 * NST || hs[2] != NULL ||
                memcmp(h0, frag[0], 512 * NST) != 0 || memcmp(h1, frag[1], 512 * NST) != 0) {
                printf("encode_rows mismatch\n");
                return 8;
            }
            free(h0);
            free(h1);
        }
        printf("roundtrip ok\n");
    }
    ec_method_fini(&list);
    return 0;
}
