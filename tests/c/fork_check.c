/* fork() after split calls (ec_method.c pool_atfork_child): the
 * parent's split calls start helper threads; a child forked afterwards has
 * none of them, and before the atfork handler its first split call queued
 * its GPU share for a helper that did not exist and waited forever.  Built
 * against the device-layer stub (tests/c/ecd_stub.c) with ECD_STUB_GPU=1,
 * EC_HYBRID_SHARE=450 (every >= 1 MiB call is split), so no GPU is needed.
 * The child runs split encodes under alarm(); exit 0 = both sides exact. */
#include <signal.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/wait.h>
#include <unistd.h>

#include "ec_method.h"

#define K 8
#define N 12
#define SIZE (4u << 20)

static int encode_check(ec_matrix_list_t *l, const uint8_t *in, uint8_t *fr, const uint8_t *want)
{
    void *o[N];
    for (int i = 0; i < N; i++)
        o[i] = fr + (size_t)i * (SIZE / K);
    memset(fr, 0, (size_t)SIZE / K * N);
    ec_method_encode(l, SIZE, (void *)in, o);
    return want ? memcmp(fr, want, (size_t)SIZE / K * N) != 0 : 0;
}

int main(void)
{
    ec_matrix_list_t l;
    ec_method_stats_t s0, s1;
    uint8_t *in = malloc(SIZE), *fr = malloc((size_t)SIZE / K * N), *ref = malloc((size_t)SIZE / K * N);
    for (uint32_t i = 0; i < SIZE; i++)
        in[i] = (uint8_t)(i * 2654435761u >> 11);
    if (ec_method_init(NULL, &l, K, N, 2 * N, "auto") != 0)
        return 2;
    ec_method_get_stats(&s0);
    for (int r = 0; r < 4; r++)
        encode_check(&l, in, ref, NULL);              /* starts the split helpers */
    ec_method_get_stats(&s1);
    if (s1.gpu_calls == s0.gpu_calls) {
        fprintf(stderr, "no split call in the parent\n");
        return 3;
    }
    const pid_t pid = fork();
    if (pid == 0) {
        alarm(20);                                    /* a hang ends the child */
        int bad = 0;
        for (int r = 0; r < 4; r++)
            bad |= encode_check(&l, in, fr, ref);
        ec_method_get_stats(&s0);
        _exit(bad ? 4 : s0.gpu_calls > s1.gpu_calls ? 0 : 5);
    }
    int bad = 0;
    for (int r = 0; r < 4; r++)
        bad |= encode_check(&l, in, fr, ref);
    int st = 0;
    waitpid(pid, &st, 0);
    printf("parent %s, child %s %d\n", bad ? "WRONG" : "ok",
           WIFEXITED(st) ? "exit" : "signal", WIFEXITED(st) ? WEXITSTATUS(st) : WTERMSIG(st));
    ec_method_fini(&l);
    return bad || !WIFEXITED(st) || WEXITSTATUS(st) != 0;
}
