/*
 * ec_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C restatement of GlusterFS's disperse (EC) coding path, used as the
 * parity checker for the MI355X implementation in glusterfs_amd/.  Only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * this library; the product library (libec_mi355x.so) never links it.
 *
 * Every function cites the reference file:line it restates (paths relative to
 * xlators/cluster/ec/src/ in zhudongmei/glusterfs):
 *
 *   GF(2^8) tables        ec-galois.c:53-70   (ec_gf_init_tables, poly 0x11D)
 *   gf mul/div/exp        ec-galois.c:123-183
 *   encode matrix         ec-method.c:22-36   (ec_method_matrix_normal)
 *   inverse matrix        ec-method.c:38-72   (ec_method_matrix_inverse)
 *   Horner ratio prepare  ec-code-c.c:11632-11644 (ec_code_c_prepare)
 *   gf8_muladd_XX         ec-code-c.c:20-11571 (out = out*X ^ in, one chunk)
 *   linear row kernel     ec-code-c.c:11647-11657 (ec_code_c_linear)
 *   interleaved row       ec-code-c.c:11660-11679 (ec_code_c_interleaved)
 *   encode stripe loop    ec-method.c:394-408 (ec_method_encode)
 *   decode chunk loop     ec-method.c:411-433 (ec_method_decode)
 *
 * Parity pinning: the reference coding sources cannot be built in this image
 * (they include libglusterfs headers that need liburcu/libuuid and a
 * configure-generated config.h), so this restatement is pinned by
 *   (1) tests/golden/gf8_muladd_ref.npz: the 256 gf8_muladd_XX XOR programs of
 *       ec-code-c.c interpreted from the reference source text (generator:
 *       tests/golden/gen_gf8_muladd.py), checked on random chunks;
 *   (2) the inverse matrices and zero-coefficient census that the survey
 *       session recorded from the compiled reference.
 *
 * The multiply-by-constant is evaluated from the 8x8 GF(2) matrix of the
 * constant (column b = X * 2^b), which is the algebraic definition the
 * reference's straight-line XOR programs implement.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define OR_GF_BITS 8
#define OR_GF_SIZE 256
#define OR_GF_MOD 0x11D
#define OR_WORD_SIZE 64                          /* EC_METHOD_WORD_SIZE */
#define OR_CHUNK_SIZE (OR_WORD_SIZE * OR_GF_BITS) /* EC_METHOD_CHUNK_SIZE = 512 */
#define OR_WIDTH (OR_WORD_SIZE / 8)              /* u64 words per plane = 8 */
#define OR_MAX_COLS 16

/* ---------------------------------------------------------------- GF(2^8) */

static uint32_t or_log[OR_GF_SIZE * 2 - 1];
static uint32_t or_pow[OR_GF_SIZE * 2 - 1];
/* rowmask[c][p]: bit b set <=> output plane p of (x * c) depends on plane b */
static uint8_t or_rowmask[OR_GF_SIZE][8];
static pthread_once_t or_once = PTHREAD_ONCE_INIT;

/* ec-galois.c:53-70 */
static void
or_tables_init(void)
{
    uint32_t i, v;

    memset(or_log, 0xff, sizeof(uint32_t) * OR_GF_SIZE);
    or_pow[0] = 1;
    or_log[0] = OR_GF_SIZE;
    or_log[1] = 0;
    for (i = 1; i < OR_GF_SIZE; i++) {
        v = or_pow[i - 1] << 1;
        if (v >= OR_GF_SIZE)
            v ^= OR_GF_MOD;
        or_pow[i] = v;
        or_pow[i + OR_GF_SIZE - 1] = v;
        or_log[v] = i;
        or_log[v + OR_GF_SIZE - 1] = i;
    }
}

uint32_t or_gf_mul(uint32_t a, uint32_t b);

static void
or_init_once(void)
{
    uint32_t c, b, p, col;

    or_tables_init();
    for (c = 0; c < OR_GF_SIZE; c++) {
        memset(or_rowmask[c], 0, 8);
        for (b = 0; b < 8; b++) {
            col = or_gf_mul(c, 1u << b);
            for (p = 0; p < 8; p++)
                if (col & (1u << p))
                    or_rowmask[c][p] |= (uint8_t)(1u << b);
        }
    }
}

void
or_init(void)
{
    pthread_once(&or_once, or_init_once);
}

/* ec-galois.c:135-147 */
uint32_t
or_gf_mul(uint32_t a, uint32_t b)
{
    if (a >= OR_GF_SIZE || b >= OR_GF_SIZE)
        return OR_GF_SIZE;
    if (a == 0 || b == 0)
        return 0;
    return or_pow[or_log[a] + or_log[b]];
}

/* ec-galois.c:149-164 */
uint32_t
or_gf_div(uint32_t a, uint32_t b)
{
    if (a >= OR_GF_SIZE || b >= OR_GF_SIZE)
        return OR_GF_SIZE;
    if (b == 0)
        return OR_GF_SIZE;
    if (a == 0)
        return 0;
    return or_pow[OR_GF_SIZE - 1 + or_log[a] - or_log[b]];
}

/* ec-galois.c:166-183 */
uint32_t
or_gf_exp(uint32_t a, uint32_t b)
{
    uint32_t r = 1;

    if (a >= OR_GF_SIZE || (a == 0 && b == 0))
        return OR_GF_SIZE;
    while (b != 0) {
        if (b & 1)
            r = or_gf_mul(r, a);
        a = or_gf_mul(a, a);
        b >>= 1;
    }
    return r;
}

/* ------------------------------------------------------------- matrices */

/* ec-method.c:22-36: row i = [v^(k-1), v^(k-2), ..., v, 1] with v = values[i] */
void
or_matrix_normal(uint32_t *matrix, uint32_t columns, const uint32_t *values,
                 uint32_t count)
{
    uint32_t i, j, v, acc;

    or_init();
    for (i = 0; i < count; i++) {
        v = values[i];
        acc = or_gf_exp(v, columns - 1);
        *matrix++ = acc;
        for (j = 1; j < columns; j++) {
            acc = or_gf_div(acc, v);
            *matrix++ = acc;
        }
    }
}

/* ec-method.c:38-72.  Same loop structure as the reference: build the
 * coefficients of prod(x + values[i]) into a[], then for every column do the
 * synthetic division by (x + values[i]) while accumulating the derivative
 * value p, writing the column bottom-up and normalising it top-down. */
void
or_matrix_inverse(uint32_t *matrix, const uint32_t *values, uint32_t count)
{
    uint32_t a[OR_MAX_COLS];
    uint32_t i, j, p, last, t;
    uint32_t *m;

    or_init();
    last = count - 1;
    for (i = 0; i < last; i++)
        a[i] = 1;
    a[last] = values[0];
    for (i = last; i > 0; i--) {
        for (j = i - 1; j < last; j++)
            a[j] = a[j + 1] ^ or_gf_mul(values[i], a[j]);
        a[last] = or_gf_mul(values[i], a[last]);
    }
    m = matrix;
    for (i = 0; i < count; i++) {
        p = a[0];
        m += count;
        t = p ^ values[i];
        *m = t;
        for (j = 1; j < last; j++) {
            m += count;
            t = a[j] ^ or_gf_mul(values[i], t);
            *m = t;
            p = t ^ or_gf_mul(values[i], p);
        }
        for (j = 0; j < last; j++) {
            *m = or_gf_div(*m, p);
            m -= count;
        }
        *m = or_gf_div(1, p);
        m++;
    }
}

/* ec-code-c.c:11632-11644: values[i] <- values[i] / next nonzero value to its
 * right (the last nonzero value is kept as is). */
void
or_prepare(uint32_t *values, uint32_t count)
{
    uint32_t i, last = 1, v;

    or_init();
    for (i = count; i > 0; i--) {
        if (values[i - 1] != 0) {
            v = values[i - 1];
            values[i - 1] = or_gf_div(v, last);
            last = v;
        }
    }
}

/* ---------------------------------------------------------- chunk kernels */

/* ec-code-c.c:20-11571 semantics: out = out * c ^ in over one 512-B chunk of
 * 8 bit-planes x 8 u64 words.  c == 0 is the reference's memcpy (:19-23).
 * The per-constant straight-line bodies are generated from the 8x8 GF(2)
 * matrix of c (oracle/gen_muladd.py -> or_muladd_gen.h), like the
 * reference's own 256 gf8_muladd_XX routines. */
#include "or_muladd_gen.h"

static inline void
or_muladd_i(void *out, const void *in, uint32_t c)
{
    or_mx[c & 0xff]((uint64_t *)out, (const uint64_t *)in);
}

void
or_muladd(void *out, const void *in, uint32_t c)
{
    or_init();
    or_muladd_i(out, in, c);
}

static const uint64_t or_zero[OR_CHUNK_SIZE / 8];

/* ec-code-c.c:11647-11657 (values already prepared, count = k) */
static void
or_linear(uint8_t *dst, const uint8_t *src, uint64_t offset,
          const uint32_t *values, uint32_t count)
{
    src += offset;
    memcpy(dst, src, OR_CHUNK_SIZE);
    while (--count > 0) {
        src += OR_CHUNK_SIZE;
        or_muladd_i(dst, src, *values);
        values++;
    }
}

/* ec-code-c.c:11660-11679 (values already prepared) */
static void
or_interleaved(uint8_t *dst, const uint8_t *const *src, uint64_t offset,
               const uint32_t *values, uint32_t count)
{
    uint32_t i = 0, last, v;

    while ((last = *values++) == 0)
        i++;
    memcpy(dst, src[i++] + offset, OR_CHUNK_SIZE);
    while (i < count) {
        v = *values++;
        if (v != 0) {
            or_muladd_i(dst, src[i] + offset, last);
            last = v;
        }
        i++;
    }
    or_muladd_i(dst, or_zero, last);
}

/* ------------------------------------------------------ encode / decode */

typedef struct {
    uint32_t k, n;
    uint32_t enc[32 * OR_MAX_COLS]; /* prepared encode rows, n x k */
} or_code_t;

static void
or_code_setup(or_code_t *c, uint32_t k, uint32_t n)
{
    uint32_t vals[32] = {0}, i;

    c->k = k;
    c->n = n;
    for (i = 0; i < n; i++)
        vals[i] = i + 1; /* ec-method.c:284-286 */
    or_matrix_normal(c->enc, k, vals, n);
    for (i = 0; i < n; i++)
        or_prepare(c->enc + i * k, k);
}

/* ec-method.c:394-408 over stripes [s0, s1).  out[i] is fragment i's base. */
static void
or_encode_range(const or_code_t *c, const uint8_t *in, uint8_t *const *out,
                uint64_t s0, uint64_t s1)
{
    uint64_t s;
    uint32_t i;
    const uint64_t stripe = (uint64_t)OR_CHUNK_SIZE * c->k;

    for (s = s0; s < s1; s++)
        for (i = 0; i < c->n; i++)
            or_linear(out[i] + s * OR_CHUNK_SIZE, in, s * stripe,
                      c->enc + i * c->k, c->k);
}

/* k, n: code geometry; size: user bytes (multiple of 512*k); out: n
 * fragment buffers of size/k bytes each. */
int
or_encode(uint32_t k, uint32_t n, uint64_t size, const void *in, void **out)
{
    or_code_t c;

    if (k < 1 || k > OR_MAX_COLS || n < k || n > 32 ||
        size % ((uint64_t)OR_CHUNK_SIZE * k) != 0)
        return -1;
    or_code_setup(&c, k, n);
    or_encode_range(&c, (const uint8_t *)in, (uint8_t *const *)out, 0,
                    size / ((uint64_t)OR_CHUNK_SIZE * k));
    return 0;
}

/* Decode matrix for the k ascending row values (brick_idx + 1), prepared. */
int
or_decode_matrix(uint32_t k, const uint32_t *rows, uint32_t *out_prepared,
                 uint32_t *out_raw)
{
    uint32_t m[OR_MAX_COLS * OR_MAX_COLS], r;

    if (k < 1 || k > OR_MAX_COLS)
        return -1;
    or_matrix_inverse(m, rows, k);
    if (out_raw)
        memcpy(out_raw, m, sizeof(uint32_t) * k * k);
    for (r = 0; r < k; r++)
        or_prepare(m + r * k, k);
    if (out_prepared)
        memcpy(out_prepared, m, sizeof(uint32_t) * k * k);
    return 0;
}

static void
or_decode_range(uint32_t k, const uint32_t *prep, const uint8_t *const *in,
                uint8_t *out, uint64_t c0, uint64_t c1)
{
    uint64_t pos;
    uint32_t r;

    for (pos = c0; pos < c1; pos++)
        for (r = 0; r < k; r++)
            or_interleaved(out + (pos * k + r) * OR_CHUNK_SIZE, in,
                           pos * OR_CHUNK_SIZE, prep + r * k, k);
}

/* ec-method.c:411-433.  size: bytes per fragment (multiple of 512); rows[p]
 * = brick index + 1 of in[p], ascending; out: size*k bytes. */
int
or_decode(uint32_t k, uint64_t size, const uint32_t *rows, const void **in,
          void *out)
{
    uint32_t prep[OR_MAX_COLS * OR_MAX_COLS];

    if (size % OR_CHUNK_SIZE != 0 || or_decode_matrix(k, rows, prep, NULL))
        return -1;
    or_decode_range(k, prep, (const uint8_t *const *)in, (uint8_t *)out, 0,
                    size / OR_CHUNK_SIZE);
    return 0;
}

/* ------------------------------------------- multi-threaded CPU baseline */

typedef struct {
    const or_code_t *code;
    const uint32_t *prep;
    const uint8_t *in;
    const uint8_t *const *ins;
    uint8_t *const *outs;
    uint8_t *out;
    uint64_t lo, hi;
} or_job_t;

static void *
or_encode_job(void *arg)
{
    or_job_t *j = (or_job_t *)arg;
    or_encode_range(j->code, j->in, j->outs, j->lo, j->hi);
    return NULL;
}

static void *
or_decode_job(void *arg)
{
    or_job_t *j = (or_job_t *)arg;
    or_decode_range(j->code->k, j->prep, j->ins, j->out, j->lo, j->hi);
    return NULL;
}

static int
or_run_jobs(or_job_t *tmpl, uint64_t units, uint32_t nthreads,
            void *(*fn)(void *))
{
    pthread_t th[256];
    or_job_t jobs[256];
    uint32_t t;

    if (nthreads < 1)
        nthreads = 1;
    if (nthreads > 256)
        nthreads = 256;
    for (t = 0; t < nthreads; t++) {
        jobs[t] = *tmpl;
        jobs[t].lo = units * t / nthreads;
        jobs[t].hi = units * (t + 1) / nthreads;
        if (pthread_create(&th[t], NULL, fn, &jobs[t]) != 0)
            return -1;
    }
    for (t = 0; t < nthreads; t++)
        pthread_join(th[t], NULL);
    return 0;
}

/* Same stripes as or_encode, split by contiguous stripe ranges. */
int
or_encode_mt(uint32_t k, uint32_t n, uint64_t size, const void *in, void **out,
             uint32_t nthreads)
{
    or_code_t c;
    or_job_t j;

    if (k < 1 || k > OR_MAX_COLS || n < k || n > 32 ||
        size % ((uint64_t)OR_CHUNK_SIZE * k) != 0)
        return -1;
    or_code_setup(&c, k, n);
    memset(&j, 0, sizeof(j));
    j.code = &c;
    j.in = (const uint8_t *)in;
    j.outs = (uint8_t *const *)out;
    return or_run_jobs(&j, size / ((uint64_t)OR_CHUNK_SIZE * k), nthreads,
                       or_encode_job);
}

int
or_decode_mt(uint32_t k, uint64_t size, const uint32_t *rows, const void **in,
             void *out, uint32_t nthreads)
{
    uint32_t prep[OR_MAX_COLS * OR_MAX_COLS];
    or_code_t c;
    or_job_t j;

    if (size % OR_CHUNK_SIZE != 0 || or_decode_matrix(k, rows, prep, NULL))
        return -1;
    memset(&j, 0, sizeof(j));
    c.k = k;
    j.code = &c;
    j.prep = prep;
    j.ins = (const uint8_t *const *)in;
    j.out = (uint8_t *)out;
    return or_run_jobs(&j, size / OR_CHUNK_SIZE, nthreads, or_decode_job);
}

/* ------------------------------------------------------ synthetic input */

/* xorshift64 (13, 7, 17), little-endian u64 stores. */
uint64_t
or_fill_xorshift(void *buf, uint64_t size, uint64_t seed)
{
    uint64_t x = seed, i, n = size / 8;
    uint64_t *p = (uint64_t *)buf;
    uint8_t *tail;

    for (i = 0; i < n; i++) {
        x ^= x << 13;
        x ^= x >> 7;
        x ^= x << 17;
        p[i] = x;
    }
    tail = (uint8_t *)buf + n * 8;
    for (i = 0; i < size % 8; i++) {
        if (i == 0) {
            x ^= x << 13;
            x ^= x >> 7;
            x ^= x << 17;
        }
        tail[i] = (uint8_t)(x >> (8 * i));
    }
    return x;
}
