/*
 * gf8_search.c -- search for short multiply-accumulate programs over GF(2^8)
 * bit-planes (build-time tool; its output is committed as
 * glusterfs_amd/csrc/ec_gf8_prog.h by tools/gen/gen_gf8_prog.py).
 *
 * For a constant c, "acc ^= c * x" on a bit-sliced chunk is 8 independent
 * plane updates  acc[p] ^= XOR_{b in L_p} x[b],  where L_p (an 8-bit set)
 * is row p of c's 8x8 GF(2) matrix (poly 0x11D, ec-galois.c:59-69).  The
 * machines this runs on have a 3-input XOR (gfx950 v_bitop3_b32 0x96,
 * AVX-512 vpternlog), so the cost model is: one instruction per XOR of 2
 * or 3 operands.  A program = shared temporaries t_j (each the XOR of 2 or 3
 * earlier signals: planes of x or temporaries) + per output p the fewest
 * signals whose XOR is L_p, chained into acc[p] with ceil(m_p / 2) XOR3s:
 *     cost = #temporaries + sum_p ceil(m_p / 2).
 * Without temporaries this is the naive per-plane tree (ec_gf8.h r01:
 * 18.1 instructions per multiply on average).  Beam search over the
 * temporaries (width BEAM, depth MAXT) with exact per-output minimum
 * covers (BFS over the 256 sets).
 *
 * Output, one line per constant:
 *   c cost ntemps  [t: a b c]...  |  [p: m s0 s1 ...]...
 * signals 0..7 = x planes, 8.. = temporaries in order, -1 = unused operand.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#ifndef MAXT
#define MAXT 8
#endif
#define BEAM 96
#define MAXS (8 + MAXT)

static unsigned gf_mul(unsigned a, unsigned b)
{
    unsigned r = 0;
    for (int i = 0; i < 8; i++) {
        if (b & 1)
            r ^= a;
        b >>= 1;
        a <<= 1;
        if (a & 0x100)
            a ^= 0x11D;
    }
    return r & 0xFF;
}

typedef struct {
    int ns;                 /* signals */
    uint8_t sig[MAXS];      /* set of x planes each signal is the XOR of */
    int8_t op[MAXT][3];     /* operands of temporary j (signal 8 + j) */
    int cost;
} state_t;

static uint8_t tgt[8];

/* min number of signals whose XOR is each target; fills cover choices */
static int eval(const state_t *s, int m_out[8], int pick[8][MAXS], int *npick)
{
    int dist[256], from[256], via[256];
    int q[256], qh = 0, qt = 0;
    for (int i = 0; i < 256; i++)
        dist[i] = 99;
    dist[0] = 0;
    q[qt++] = 0;
    while (qh < qt) {
        const int u = q[qh++];
        for (int j = 0; j < s->ns; j++) {
            const int v = u ^ s->sig[j];
            if (dist[v] > dist[u] + 1) {
                dist[v] = dist[u] + 1;
                from[v] = u;
                via[v] = j;
                q[qt++] = v;
            }
        }
    }
    int cost = s->ns - 8;
    for (int p = 0; p < 8; p++) {
        const int m = dist[tgt[p]];
        cost += (m + 1) / 2;
        if (m_out)
            m_out[p] = m;
        if (pick) {
            int k = 0;
            for (int v = tgt[p]; v; v = from[v])
                pick[p][k++] = via[v];
            npick[p] = k;
        }
    }
    return cost;
}

static int cmp_state(const void *a, const void *b)
{
    return ((const state_t *)a)->cost - ((const state_t *)b)->cost;
}

static int seen_sig(const state_t *s, uint8_t v)
{
    for (int i = 0; i < s->ns; i++)
        if (s->sig[i] == v)
            return 1;
    return v == 0;
}

int main(void)
{
    static state_t beam[BEAM], next[BEAM * 600];
    long total = 0, naive_total = 0;
    for (unsigned c = 1; c < 256; c++) {
        for (int p = 0; p < 8; p++) {
            tgt[p] = 0;
            for (int b = 0; b < 8; b++)
                if ((gf_mul(c, 1u << b) >> p) & 1)
                    tgt[p] |= 1u << b;
        }
        state_t s0;
        memset(&s0, 0, sizeof(s0));
        s0.ns = 8;
        for (int b = 0; b < 8; b++)
            s0.sig[b] = 1u << b;
        s0.cost = eval(&s0, NULL, NULL, NULL);
        const int naive = s0.cost;
        state_t best = s0;
        int nb = 1;
        beam[0] = s0;
        for (int depth = 0; depth < MAXT; depth++) {
            int nn = 0;
            for (int i = 0; i < nb; i++) {
                const state_t *s = &beam[i];
                for (int a = 0; a < s->ns; a++)
                    for (int b = a + 1; b < s->ns; b++)
                        for (int d = b; d <= s->ns; d++) { /* d == ns: 2 operands */
                            if (d == b)
                                continue;
                            uint8_t v = s->sig[a] ^ s->sig[b];
                            if (d < s->ns)
                                v ^= s->sig[d];
                            if (seen_sig(s, v))
                                continue;
                            state_t t = *s;
                            t.sig[t.ns] = v;
                            t.op[t.ns - 8][0] = (int8_t)a;
                            t.op[t.ns - 8][1] = (int8_t)b;
                            t.op[t.ns - 8][2] = (int8_t)(d < s->ns ? d : -1);
                            t.ns++;
                            t.cost = eval(&t, NULL, NULL, NULL);
                            if (t.cost <= s->cost + 1 && nn < BEAM * 600)
                                next[nn++] = t;
                        }
            }
            if (nn == 0)
                break;
            qsort(next, nn, sizeof(state_t), cmp_state);
            /* dedupe identical signal sets (order-insensitive would be
             * better; identical prefixes are common enough) */
            nb = 0;
            for (int i = 0; i < nn && nb < BEAM; i++) {
                int dup = 0;
                for (int j = 0; j < nb && !dup; j++)
                    dup = beam[j].cost == next[i].cost &&
                          memcmp(beam[j].sig, next[i].sig, sizeof(next[i].sig)) == 0;
                if (!dup)
                    beam[nb++] = next[i];
            }
            if (beam[0].cost < best.cost)
                best = beam[0];
        }
        /* drop temporaries no output uses (cost can only fall) */
        int m[8], pick[8][MAXS], np[8];
        best.cost = eval(&best, m, pick, np);
        total += best.cost;
        naive_total += naive;
        printf("%u %d %d", c, best.cost, best.ns - 8);
        for (int j = 0; j < best.ns - 8; j++)
            printf(" %d %d %d", best.op[j][0], best.op[j][1], best.op[j][2]);
        printf(" |");
        for (int p = 0; p < 8; p++) {
            printf(" %d", np[p]);
            for (int k = 0; k < np[p]; k++)
                printf(" %d", pick[p][k]);
        }
        printf("\n");
    }
    fprintf(stderr, "avg instructions per multiply-accumulate: %.2f (naive %.2f)\n",
            total / 255.0, naive_total / 255.0);
    return 0;
}
