/*
 * ec_method.c -- host (C) side of the MI355X disperse coder: the drop-in
 * ec_method_* API of include/ec_method.h.
 *
 * What stays on the host, as in the reference, is the O(k^2) scalar work:
 * GF(2^8) log/exp tables (ec-galois.c:53-70), the encode matrix
 * (ec-method.c:22-36), the per-mask inverse (ec-method.c:38-72) and the LRU
 * cache of inverses keyed by brick mask (ec-method.c:134-256).  The per-byte
 * work -- the reference's row kernels called from ec-method.c:401-407 and
 * :422-428 -- goes to the gfx950 kernels through ec_device.h, or to the CPU
 * engine of ec_cpu.h: on nodes without a gfx950 GPU, for cpu-extensions =
 * none / x64 / sse / avx, for host-buffer calls below the crossover or when
 * every GPU is saturated, and as the fallback when a device submission for
 * host buffers fails (the reference coder cannot fail: ec-method.c:393-408,
 * ec-code.c:1007-1013).
 *
 * Storage contract: only the 120 bytes of the caller's ec_matrix_list_t are
 * used (ec-types.h:549-562, embedded by value in ec_t at ec-types.h:677):
 *   lru     -> LRU ring of unreferenced cached inverses (next, prev)
 *   lock    -> pthread mutex around cache get/put (ec-method.c:206, 250)
 *   columns/rows/max/count/stripe -> same meaning as the reference
 *   gf      -> shared GF(2^8) tables          code -> engine context
 *   encode  -> encode matrix                  objects -> mask-sorted cache
 */
#define _GNU_SOURCE
#include <errno.h>
#include <pthread.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "../../include/ec_method.h"
#include "ec_cpu.h"
#include "ec_device.h"

_Static_assert(sizeof(ec_matrix_list_t) == 120, "ec_matrix_list_t must stay 120 bytes");
_Static_assert(offsetof(ec_matrix_list_t, columns) == 56, "layout of ec-types.h:549");
_Static_assert(offsetof(ec_matrix_list_t, objects) == 112, "layout of ec-types.h:561");

#define ECM_MAX_K EC_METHOD_MAX_FRAGMENTS
#define ECM_MAX_N EC_MI355X_MAX_NODES

/* ------------------------------------------------------------- logging */

static void
ecm_log(const char *fmt, ...)
{
    static int quiet = -1;
    va_list ap;

    if (quiet < 0) {
        const char *e = getenv("EC_MI355X_QUIET");
        quiet = (e && *e && *e != '0') ? 1 : 0;
    }
    if (quiet)
        return;
    va_start(ap, fmt);
    fputs("[ec-mi355x] ", stderr);
    vfprintf(stderr, fmt, ap);
    fputc('\n', stderr);
    va_end(ap);
}

/* ------------------------------------------------------------ GF(2^8) */

typedef struct {
    uint32_t log[EC_GF_SIZE];
    uint32_t exp[2 * EC_GF_SIZE]; /* exp[i] = 2^i, doubled to skip a mod */
} ecm_gf_t;

static ecm_gf_t ecm_gf;
static pthread_once_t ecm_gf_once = PTHREAD_ONCE_INIT;

/* Generator 2, modulus x^8+x^4+x^3+x^2+1 (EC_GF_MOD, ec-galois.c:59-69). */
static void
ecm_gf_build(void)
{
    uint32_t i, x = 1;

    for (i = 0; i < EC_GF_SIZE - 1; i++) {
        ecm_gf.exp[i] = x;
        ecm_gf.exp[i + EC_GF_SIZE - 1] = x;
        ecm_gf.log[x] = i;
        x <<= 1;
        if (x & EC_GF_SIZE)
            x ^= EC_GF_MOD;
    }
    ecm_gf.log[0] = EC_GF_SIZE; /* undefined; ec-galois.c:61 uses size too */
}

static const ecm_gf_t *
ecm_gf_get(void)
{
    pthread_once(&ecm_gf_once, ecm_gf_build);
    return &ecm_gf;
}

/* ec-galois.c:135-147 semantics (operands >= 256 yield 256). */
uint32_t
ec_method_gf_mul(uint32_t a, uint32_t b)
{
    const ecm_gf_t *gf = ecm_gf_get();

    if (a >= EC_GF_SIZE || b >= EC_GF_SIZE)
        return EC_GF_SIZE;
    if (a == 0 || b == 0)
        return 0;
    return gf->exp[gf->log[a] + gf->log[b]];
}

/* ec-galois.c:149-164 semantics (division by 0 yields 256). */
uint32_t
ec_method_gf_div(uint32_t a, uint32_t b)
{
    const ecm_gf_t *gf = ecm_gf_get();

    if (a >= EC_GF_SIZE || b >= EC_GF_SIZE || b == 0)
        return EC_GF_SIZE;
    if (a == 0)
        return 0;
    return gf->exp[gf->log[a] + EC_GF_SIZE - 1 - gf->log[b]];
}

static uint32_t
ecm_gf_pow(uint32_t a, uint32_t e)
{
    uint32_t r = 1;

    while (e--)
        r = ec_method_gf_mul(r, a);
    return r;
}

/* ----------------------------------------------------------- matrices */

/* Encode row i (brick i) evaluates the data polynomial at v = i + 1 with
 * the coefficients in reversed order: E[i][j] = v^(k-1-j)
 * (ec-method.c:22-36 with values[i] = i + 1 from ec-method.c:284-286). */
int32_t
ec_method_encode_matrix(uint32_t k, uint32_t n, uint32_t *m)
{
    uint32_t i, j;

    if (k < 1 || k > ECM_MAX_K || n < k || n > ECM_MAX_N || !m)
        return -EINVAL;
    for (i = 0; i < n; i++)
        for (j = 0; j < k; j++)
            m[i * k + j] = ecm_gf_pow(i + 1, k - 1 - j);
    return 0;
}

/* Inverse of the k x k reversed-Vandermonde submatrix for the evaluation
 * points x_p = rows[p] (ec-method.c:38-72 computes the same unique matrix).
 * Lagrange form: column p holds the coefficients of
 *   L_p(x) = prod_{q != p} (x + x_q) / prod_{q != p} (x_p + x_q),
 * highest degree first, so that data_j = sum_p inv[j][p] * fragment_p. */
int32_t
ec_method_inverse_matrix(uint32_t k, const uint32_t *rows, uint32_t *inv)
{
    uint32_t master[ECM_MAX_K + 1], num[ECM_MAX_K];
    uint32_t i, j, p, q, den, dinv;

    if (k < 1 || k > ECM_MAX_K || !rows || !inv)
        return -EINVAL;
    for (p = 0; p < k; p++) {
        if (rows[p] == 0 || rows[p] >= EC_GF_SIZE)
            return -EINVAL;
        for (q = 0; q < p; q++)
            if (rows[q] == rows[p])
                return -EINVAL;
    }
    /* master(x) = prod_q (x + x_q); master[d] = coefficient of x^d */
    memset(master, 0, sizeof(master));
    master[0] = 1;
    for (q = 0; q < k; q++) {
        for (i = q + 1; i > 0; i--)
            master[i] = master[i - 1] ^ ec_method_gf_mul(master[i], rows[q]);
        master[0] = ec_method_gf_mul(master[0], rows[q]);
    }
    for (p = 0; p < k; p++) {
        /* num(x) = master(x) / (x + x_p), synthetic division from the top */
        num[k - 1] = master[k];
        for (i = k - 1; i > 0; i--)
            num[i - 1] = master[i] ^ ec_method_gf_mul(num[i], rows[p]);
        den = 1;
        for (q = 0; q < k; q++)
            if (q != p)
                den = ec_method_gf_mul(den, rows[p] ^ rows[q]);
        dinv = ec_method_gf_div(1, den);
        for (j = 0; j < k; j++)
            inv[j * k + p] = ec_method_gf_mul(num[k - 1 - j], dinv);
    }
    return 0;
}

/* ------------------------------------------------------ engine context */

typedef struct ecm_matrix {
    struct ecm_matrix *next, *prev; /* LRU links while unreferenced */
    uint32_t refs;
    int cached;
    uintptr_t mask;
    uint32_t k;
    uint32_t rows[ECM_MAX_K];
    uint32_t inv[ECM_MAX_K * ECM_MAX_K];
} ecm_matrix_t;

enum { ECM_ENGINE_GPU = 0, ECM_ENGINE_CPU = 1 };

typedef struct {
    uint32_t k, n;
    uint32_t enc[ECM_MAX_N * ECM_MAX_K];
    uint8_t enc_pat[ECM_MAX_K + ECM_MAX_N * ECM_MAX_K]; /* src[k] + n x k */
    char gen[16];
    int engine; /* ECM_ENGINE_GPU: gfx950 + CPU crossover / fallback */
    int isa;    /* CPU engine ISA level (ec_cpu.h)                   */
    char engine_name[48];
    uint64_t serial; /* unique per ec_method_init: keys the decode memo */
    /* host calls of fewer user bytes than this (per op) go to the CPU
     * engine without routing: see small_cpu_below */
    uint64_t cpu_small[2];
} ecm_ctx_t;

/* Per-thread memo of the last packed decode patterns (the inverse of a
 * mask is fixed for a volume), so a repeated single-mask decode -- every
 * read of a degraded volume -- skips the two locked trips through the
 * shared matrix cache (ec-method.c:206,250 lock them too): with 16 client
 * threads the list lock made a 128 KiB 4+2 decode wait ~15 us for ~3 us of
 * coding.  Keyed by the context's serial, so a volume re-created at the
 * same address never sees another's entry. */
#define ECM_MEMO 4
static __thread struct {
    uint64_t serial;
    uintptr_t mask;
    uint8_t pat[ECM_MAX_K + ECM_MAX_K * ECM_MAX_K];
} ecm_memo[ECM_MEMO];
static __thread unsigned ecm_memo_next;
static uint64_t ecm_serial;

/* ------------------------------------------------------ engine counters */

/* Sharded by thread, one cache line per shard: a single shared counter
 * line written by every call of 16 client threads, next to the read-mostly
 * crossover constants, cost the CPU path ~2 us per 128 KiB call (false
 * sharing; tools/kbench/ab_auto_cpu.sh). */
enum { ECM_STAT_GPU = 0, ECM_STAT_CPU = 1, ECM_STAT_FALLBACK = 2 };
#define ECM_STAT_SHARDS 64
static struct {
    uint64_t c[3];
} __attribute__((aligned(64))) ecm_stats[ECM_STAT_SHARDS];
static __thread int ecm_stat_slot = -1;

static void
stat_add(int which)
{
    static unsigned next;

    if (ecm_stat_slot < 0)
        ecm_stat_slot = (int)(__atomic_fetch_add(&next, 1, __ATOMIC_RELAXED) % ECM_STAT_SHARDS);
    __atomic_fetch_add(&ecm_stats[ecm_stat_slot].c[which], 1, __ATOMIC_RELAXED);
}

static uint64_t
stat_sum(int which)
{
    uint64_t v = 0;
    int i;

    for (i = 0; i < ECM_STAT_SHARDS; i++)
        v += __atomic_load_n(&ecm_stats[i].c[which], __ATOMIC_RELAXED);
    return v;
}

void
ec_method_get_stats(ec_method_stats_t *st)
{
    if (!st)
        return;
    st->gpu_calls = stat_sum(ECM_STAT_GPU);
    st->cpu_calls = stat_sum(ECM_STAT_CPU);
    st->cpu_fallbacks = stat_sum(ECM_STAT_FALLBACK);
}

void
ec_method_inject_device_faults(uint32_t count)
{
    ecd_inject_faults(count);
}

/* Host-buffer crossover.  GlusterFS codes one fop per
 * call -- 128 KiB FUSE writes (fuse-bridge.c:5179) up to 4 MiB heal blocks
 * (ec-heal.c:2063-2068) -- on several threads at once, and each call can run
 * on its own thread (the CPU engine) or be shipped to a GPU over PCIe.  The
 * library estimates both completion times and takes the shorter:
 *
 *   CPU: user bytes / rate, rate = EC_CPU_ENC_GBPS_K2 (260) / (k + 2) for
 *        encodes and EC_CPU_DEC_GBPS_K (200) / k for decode-type calls
 *        (decode, mixed, heal): 43 / 26 / 14 and 50 / 25 / 12.5 GB/s per
 *        thread for k = 4 / 8 / 16 with AVX-512 on the MI355X hosts' EPYC
 *        9575F (tools/kbench/xover_cells.sh, profiles/xover_r02k_*.log,
 *        xover_r02x_dec_*.log); x0.7 with AVX2, x0.4 base x86-64; calls
 *        moving 32 MiB or more (past a CCD's L3) stream from DRAM:
 *        min(rate, 24);
 *   GPU: latency + (bytes in flight on the least-loaded host GPU + this
 *        call) / rate, per call: 30 us and 26 GB/s of user data for pinned,
 *        device-mapped buffers (zero copy); 40 us and 14 GB/s for pageable
 *        ones (staging copies), 21 GB/s from 8 MiB of user data on (the copy
 *        pool splits a call into 2 MiB pieces, so larger calls copy on more
 *        threads); EC_GPU_{PINNED,PAGEABLE}_{US,GBPS}, EC_GPU_PAGEABLE_GBPS_L;
 *        a call with some buffers mapped and some not is costed in between,
 *        by the fraction of its bytes that must be staged (r04).
 *
 * So FUSE-sized calls and light codes stay on the calling thread, wide-code
 * decodes and large pinned calls go to the GPU, and concurrent callers queue
 * on a GPU only while the queue is shorter than their own CPU time.
 * EC_CPU_BELOW_KB forces calls below it to the CPU; EC_GPU_ALWAYS=1 sends
 * every host call to the GPU (tests of the host kernels). */
static uint64_t
env_u64(const char *name, uint64_t dflt)
{
    const char *e = getenv(name);
    char *end = NULL;
    unsigned long long v;

    if (!e || !*e)
        return dflt;
    v = strtoull(e, &end, 10);
    return (end && *end == 0) ? (uint64_t)v : dflt;
}

static struct {
    uint64_t cpu_below, enc_k2, dec_k, pin_us, pin_gbps, page_us, page_gbps, page_gbps_l, always;
    uint64_t adapt, hybrid, hybrid_share, copy_gbps, learn;
} __attribute__((aligned(64))) ecm_x;
static pthread_once_t ecm_xover_once __attribute__((aligned(64))) = PTHREAD_ONCE_INIT;

static void
xover_init(void)
{
    ecm_x.cpu_below = env_u64("EC_CPU_BELOW_KB", 0) << 10;
    ecm_x.enc_k2 = env_u64("EC_CPU_ENC_GBPS_K2", 260);
    ecm_x.dec_k = env_u64("EC_CPU_DEC_GBPS_K", 200);
    ecm_x.pin_us = env_u64("EC_GPU_PINNED_US", 30);
    ecm_x.pin_gbps = env_u64("EC_GPU_PINNED_GBPS", 26);
    ecm_x.page_us = env_u64("EC_GPU_PAGEABLE_US", 40);
    ecm_x.page_gbps = env_u64("EC_GPU_PAGEABLE_GBPS", 14);
    ecm_x.page_gbps_l = env_u64("EC_GPU_PAGEABLE_GBPS_L", 21);
    ecm_x.always = env_u64("EC_GPU_ALWAYS", 0);
    ecm_x.adapt = env_u64("EC_XOVER_ADAPT", 1);
    ecm_x.hybrid = env_u64("EC_HYBRID", 1);
    ecm_x.hybrid_share = env_u64("EC_HYBRID_SHARE", 0); /* tests: a fixed GPU share, 1..999 per mille */
    if (ecm_x.hybrid_share >= 1000)
        ecm_x.hybrid_share = 0;
    /* one CPU thread's copy rate between pageable and pinned memory (the
     * staging copies of a GPU call with pageable buffers); 0: no busy rule */
    ecm_x.copy_gbps = env_u64("EC_STAGE_COPY_GBPS", 10);
    ecm_x.learn = env_u64("EC_SPLIT_LEARN", 1);   /* 0: the model's split shares (A/B) */
}

enum { ECM_ENCODE = 0, ECM_DECODE = 1 };

/* Observed rates (r03, size-bucketed in r04).  The constants above are
 * calibrated on calls that re-code cache-resident buffers; a self-heal sweep
 * streams through a file (ec-heal.c:2048-2107), and there the CPU engine ran
 * at a fraction of its modelled rate while the GPU with registered buffers
 * ran 1.9x faster (bench.py heal_sweep, profiles/r03*_bench.log).  So every
 * host call of >= 256 KiB of user data records the user-byte rate it achieved
 * as an exponential average (weight 1/4), per engine (CPU; GPU with every
 * buffer mapped; GPU with every buffer staged; GPU with some of each),
 * direction, code width and call size (log4 buckets from 256 KiB: a rate
 * learned on cache-resident 256 KiB calls, or one that includes a small
 * call's fixed latency, is never applied to a multi-GiB call).  Once a slot
 * has samples its observed rate replaces the model for calls of that size;
 * the CPU's keeps the DRAM cap for calls moving >= 32 MiB.  An engine the
 * router keeps losing to is re-sampled by one call of >= 1 MiB in 8 until it
 * has 4 samples, then in 64 (exploration), so a change in load or residency
 * is noticed.  EC_XOVER_ADAPT=0 keeps the static model. */
enum { ECM_OBS_CPU = 0, ECM_OBS_GPU_MAPPED = 1, ECM_OBS_GPU_PAGEABLE = 2, ECM_OBS_GPU_MIXED = 3 };
#define ECM_OBS_ENGINES 4
#define ECM_OBS_SIZES 5
#define ECM_OBS_MIN (256u << 10)
#define ECM_OBS_EXPLORE (1u << 20)
#define ECM_STAGED_UNKNOWN UINT64_MAX

typedef struct {
    uint64_t kbps;   /* user KB per second, EWMA; 0: no sample yet */
    uint32_t lost;   /* calls routed away from this engine since its last sample */
    uint32_t n;      /* samples taken (the first, a cold start, is dropped) */
    uint32_t pad[12];
} __attribute__((aligned(64))) ecm_obs_t;

static ecm_obs_t ecm_obs[ECM_OBS_ENGINES][2][3][ECM_OBS_SIZES];

static int
kbucket(uint32_t k)
{
    return k <= 4 ? 0 : k <= 8 ? 1 : 2;
}

/* [256 KiB, 1 MiB), [1, 4), [4, 16), [16, 64), >= 64 MiB of user data */
static int
sbucket(uint64_t user)
{
    int b = 0;

    for (user >>= 20; user && b < ECM_OBS_SIZES - 1; user >>= 2)
        b++;
    return b;
}

static ecm_obs_t *
obs_slot(int eng, int op, uint32_t k, uint64_t user)
{
    return &ecm_obs[eng][op][kbucket(k)][sbucket(user)];
}

/* the GPU observation slot of a call with `staged` of `moved` bytes staged */
static int
gpu_obs_engine(uint64_t staged, uint64_t moved)
{
    return staged == 0 ? ECM_OBS_GPU_MAPPED
                       : staged >= moved ? ECM_OBS_GPU_PAGEABLE : ECM_OBS_GPU_MIXED;
}

static uint64_t
now_ns(void)
{
    struct timespec ts;

    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}

/* One sample: `user` bytes coded in `ns` by engine `eng`, into the slot of
 * calls of `call_user` bytes (a split call's share, r05, is a sample of the
 * rate its engine reaches inside calls of the whole call's size). */
static void
obs_record_part(int eng, int op, uint32_t k, uint64_t call_user, uint64_t user, uint64_t ns)
{
    ecm_obs_t *o = obs_slot(eng, op, k, call_user);
    uint64_t old, upd, sample;

    if (call_user < ECM_OBS_MIN || user == 0 || ns == 0 || !ecm_x.adapt)
        return;
    __atomic_store_n(&o->lost, 0, __ATOMIC_RELAXED);
    /* the first call of an engine pays its cold start (page faults on fresh
     * outputs, lazy set-up): a sample of it would bar the engine for long */
    if (__atomic_fetch_add(&o->n, 1, __ATOMIC_RELAXED) == 0)
        return;
    sample = user * 1000000ull / ns;                   /* KB/s = B/ns * 1e6 / 1e3 */
    old = __atomic_load_n(&o->kbps, __ATOMIC_RELAXED);
    do
        upd = old ? old + ((int64_t)sample - (int64_t)old) / 4 : sample;
    while (!__atomic_compare_exchange_n(&o->kbps, &old, upd, 1, __ATOMIC_RELAXED,
                                        __ATOMIC_RELAXED));
}

static void
obs_record(int eng, int op, uint32_t k, uint64_t user, uint64_t ns)
{
    obs_record_part(eng, op, k, user, user, ns);
}

/* The GPU's fixed cost of a host call, microseconds: the model's latency,
 * interpolated between pinned (zero-copy) and staged buffers by the fraction
 * of its bytes that are staged. */
static double
gpu_lat_us(uint64_t staged, uint64_t moved)
{
    const double f = moved ? (double)(staged < moved ? staged : moved) / (double)moved : 0.0;

    return (double)ecm_x.pin_us + f * ((double)ecm_x.page_us - (double)ecm_x.pin_us);
}

/* A split call's GPU share (r06): `part` of the call's `user`
 * bytes took `ns`, which hold the GPU's fixed latency L once.  The slot of
 * calls of `user` bytes prices a whole call as user / rate, with L inside the
 * rate, so the share is recorded as the time the whole call would have
 * taken, L + (ns - L) * user / part.  Recording part / ns (r05) charged L
 * 1 / f times over: at f = 0.35 the whole-call estimate came out ~3x L too
 * high, the next share came out smaller, and each smaller share inflated the
 * next estimate further (tests/test_xover.py::test_split_samples_keep_routing). */
static void
obs_record_gpu_part(int eng, int op, uint32_t k, uint64_t user, uint64_t part, uint64_t ns,
                    uint64_t staged, uint64_t moved)
{
    const double lat = gpu_lat_us(staged, moved) * 1e3, sc = part ? (double)user / (double)part : 0;
    double whole;

    if (part == 0 || part > user || ns == 0)
        return;
    whole = (double)ns > lat ? lat + ((double)ns - lat) * sc : (double)ns * sc;
    obs_record(eng, op, k, user, (uint64_t)whole);
}

static double
obs_gbps(int eng, int op, uint32_t k, uint64_t user)
{
    if (user < ECM_OBS_MIN)
        return 0;
    return (double)__atomic_load_n(&obs_slot(eng, op, k, user)->kbps, __ATOMIC_RELAXED) / 1e6;
}

/* 1: send this call to the engine the router did not pick, to re-sample it
 * (every 8th such call while the slot has fewer than 4 samples, then every
 * 64th, or every 512th when that engine is estimated at over 4x the time of
 * the one picked: a cache-resident 1 MiB call codes in ~20 us on the CPU,
 * and one in 64 of them sent to a GPU 5x slower cost a tight loop of such
 * calls ~25 %, tools/kbench/xover_cells.sh, profiles/r05/r05ai_xover_*.log) */
static int
obs_explore(int eng, int op, uint32_t k, uint64_t user, int far)
{
    ecm_obs_t *o = obs_slot(eng, op, k, user);
    const uint32_t every = __atomic_load_n(&o->n, __ATOMIC_RELAXED) < 4 ? 8 : far ? 512 : 64;

    if (!ecm_x.adapt || user < ECM_OBS_EXPLORE)
        return 0;
    return __atomic_add_fetch(&o->lost, 1, __ATOMIC_RELAXED) % every == 0;
}

/* 1: code this host-buffer call on the CPU engine.  `user`: user bytes of the
 * call; `moved`: bytes read + written; `op`: ECM_ENCODE / ECM_DECODE;
 * `staged`: bytes of its buffers that are not pinned, device-mapped host
 * memory (0: the zero-copy path for every buffer; `moved`: staging copies for
 * every buffer; in between, a call whose fragments are registered iobufs but
 * whose output is not, or the reverse -- the device layer reads the mapped
 * buffers in place and stages only the others, ec_device.hip
 * run_decode_dev); `infl`: bytes queued on the least-loaded host GPU.  The
 * model's GPU cost is interpolated between the two pure cases by the staged
 * fraction. */
/* The two estimates of a host call, in microseconds: `cpu` on the calling
 * thread, `gpu` on the least-loaded host GPU with `infl` bytes queued ahead
 * of it, `lat` the GPU's fixed part; returns 1 when `gpu` comes from an
 * observed rate (which includes the call's latency). */
static int
xover_costs(uint32_t k, int isa, uint64_t user, uint64_t moved, int op, uint64_t staged,
            uint64_t infl, double *cpu, double *gpu, double *lat)
{
    static const double isa_f[] = {0.4, 0.7, 1.0};
    double cpu_gbps, q, obs, f, page_gbps;

    cpu_gbps = (op == ECM_ENCODE ? (double)ecm_x.enc_k2 / (k + 2) : (double)ecm_x.dec_k / k) *
               isa_f[isa < 0 ? 0 : isa > 2 ? 2 : isa];
    if ((obs = obs_gbps(ECM_OBS_CPU, op, k, user)) > 0)
        cpu_gbps = obs;
    if (moved >= (32u << 20))
        cpu_gbps = cpu_gbps < 24.0 ? cpu_gbps : 24.0;
    *cpu = (double)user / (cpu_gbps * 1e3);
    q = (double)infl * ((double)user / (double)moved); /* queued user bytes */
    if (staged > moved)
        staged = moved;
    f = (double)staged / (double)moved;
    *lat = gpu_lat_us(staged, moved);
    obs = obs_gbps(gpu_obs_engine(staged, moved), op, k, user);
    if (obs > 0) {
        *gpu = (q + user) / (obs * 1e3);
        return 1;
    }
    page_gbps = (double)(user >= (8u << 20) ? ecm_x.page_gbps_l : ecm_x.page_gbps);
    *gpu = *lat + (q + user) * ((1.0 - f) / (double)ecm_x.pin_gbps + f / page_gbps) / 1e3;
    return 0;
}

/* 0: the GPU; 1: the CPU engine; ECM_ROUTE_CPU_BUSY: the CPU engine because
 * the call stages buffers while `others` large host calls are in flight (no
 * exploration of the GPU for it).  The staging copies of a GPU call run on
 * the library's CPU threads; while other callers keep the cores busy, a call
 * whose copies take at least as much CPU time as coding it on the calling
 * thread would (8+4 heal windows on pageable buffers: copying 2-2.5x the user
 * bytes against a ~7-13 GB/s coder) frees no CPU for them and only adds the
 * trip to the GPU.  8 threads of 4 MiB heal windows on pageable buffers ran
 * 40.6 GB/s auto against 47.7 CPU-only (profiles/r05/r05t_concur.log); most
 * of that was the buffer-mapping queries (now cached, ec_device.hip
 * mapped()), and with this rule too the GPU takes ~20 of such calls a second
 * instead of ~390, within 3 % of the CPU engine alone; pool buffers, which
 * stage nothing, keep their +12-30 % (profiles/r05/r05w_busyab_*.log). */
#define ECM_ROUTE_CPU_BUSY 2

static int
route_cpu_q(uint32_t k, int isa, uint64_t user, uint64_t moved, int op, uint64_t staged,
            uint64_t infl, uint32_t others)
{
    double cpu_us, gpu_us, lat;

    pthread_once(&ecm_xover_once, xover_init);
    if (ecm_x.always)
        return 0;
    if (moved < ecm_x.cpu_below || infl == UINT64_MAX)
        return 1;
    /* a near tie on observed rates stays on the caller's CPU */
    if (xover_costs(k, isa, user, moved, op, staged, infl, &cpu_us, &gpu_us, &lat))
        gpu_us *= 1.1;
    if (others && staged && ecm_x.copy_gbps &&
        (double)(staged < moved ? staged : moved) / ((double)ecm_x.copy_gbps * 1e3) >= cpu_us)
        return ECM_ROUTE_CPU_BUSY;
    return cpu_us <= gpu_us;
}

/* Split calls (r05).  A host call the two engines would code in comparable
 * times runs on both: the GPU takes the first f of its stripes (submitted
 * from a helper thread, as the device layer's host path blocks) while the
 * calling thread codes the rest on the CPU engine.  With C and G the whole
 * call's CPU and GPU estimates (the GPU's queue included) and L the GPU's
 * fixed latency, the share f finishes in max(L + f (G - L), (1 - f) C),
 * balanced at f = (C - L) / (C + G - L).  Calls below 1 MiB of user data,
 * or a share under 15 % either way, stay whole (the hand-off costs ~10 us).
 * Calls that stage a buffer split only when no other large call is in
 * flight (below).
 * Returns f in thousandths, or -1 for no split.  EC_HYBRID=0 turns splits
 * off; EC_HYBRID_SHARE fixes f for any call (tests). */
#define ECM_HYBRID_MIN (1u << 20)

/* Host calls of >= 1 MiB in flight in the process (own cache line: every
 * such call writes it twice). */
static struct {
    uint32_t n;
} __attribute__((aligned(64))) ecm_big_calls;

static void
big_call(uint64_t user, int d)
{
    if (user >= ECM_HYBRID_MIN)
        __atomic_add_fetch(&ecm_big_calls.n, (uint32_t)d, __ATOMIC_RELAXED);
}

/* Learned split shares (r05).  The model's share comes from whole-call
 * estimates; inside a split call the two engines share the host's memory
 * and the GPU share's latency is the model's constant, so the balance can sit
 * elsewhere: a single stream of 4 MiB 8+4 heal windows ran 8.1-8.3 GB/s on
 * pageable buffers at the model's share and 9.6-10.3 at a fixed 35 %, the
 * fused heal 36.0-37.4 against 39.1-39.7 (profiles/r05/r05aa_sharesweep.log).
 * So every split call reports how long each share took, from the hand-off to
 * each engine's end; with C the CPU's time scaled to the whole call, G1 the
 * GPU's beyond the model's latency L scaled likewise, the share that would
 * have balanced them is f* = (C - L) / (C + G1), and an exponential average
 * (weight 1/4; the first sample, a cold start, dropped) of f* per call class
 * (encode, k-row decode, fewer-row combination), code width, call size and
 * buffer provenance replaces the model's share once it has a sample.  Its
 * fixed point is the share at which both engines finish together, whatever
 * L is.  The model still decides WHETHER to split; the queue ahead on the
 * GPU moves the learned share as it moves the model's.  EC_XOVER_ADAPT=0
 * or EC_SPLIT_LEARN=0 keeps the model's share. */
enum { ECM_CLS_ENCODE = 0, ECM_CLS_DECODE = 1, ECM_CLS_PART = 2 };
typedef struct {
    uint32_t f;      /* share in thousandths, EWMA; 0: no sample yet */
    uint32_t n;      /* samples seen (the first dropped) */
    uint32_t pad[14];
} __attribute__((aligned(64))) ecm_share_t;

static ecm_share_t ecm_share[3][3][ECM_OBS_SIZES][3];

static ecm_share_t *
share_slot(int cls, uint32_t k, uint64_t user, uint64_t staged, uint64_t moved)
{
    return &ecm_share[cls][kbucket(k)][sbucket(user)][gpu_obs_engine(staged, moved) - 1];
}

/* one split call: `sg` of `n` stripes on the GPU took gpu_ns from the
 * hand-off, the rest cpu_ns on the calling thread */
static void
share_learn(int cls, int op, uint32_t k, int isa, uint64_t user, uint64_t moved,
            uint64_t staged, uint64_t n, uint64_t sg, uint64_t gpu_ns, uint64_t cpu_ns)
{
    ecm_share_t *sl;
    double c, g, lat, C, G1, f;
    uint32_t old, upd, fm;

    pthread_once(&ecm_xover_once, xover_init);
    if (!ecm_x.adapt || !ecm_x.learn || sg == 0 || sg >= n || gpu_ns == 0 || cpu_ns == 0 ||
        user < ECM_HYBRID_MIN || staged == ECM_STAGED_UNKNOWN)
        return;
    sl = share_slot(cls, k, user, staged, moved);
    if (__atomic_fetch_add(&sl->n, 1, __ATOMIC_RELAXED) == 0)
        return;
    xover_costs(k, isa, user, moved, op, staged, 0, &c, &g, &lat);
    lat *= 1e3;                                             /* ns */
    C = (double)cpu_ns * (double)n / (double)(n - sg);
    G1 = ((double)gpu_ns - lat) * (double)n / (double)sg;
    if (G1 < 0)
        G1 = 0;
    f = (C - lat) / (C + G1);
    f = f < 0.05 ? 0.05 : f > 0.95 ? 0.95 : f;
    fm = (uint32_t)(f * 1000.0);
    old = __atomic_load_n(&sl->f, __ATOMIC_RELAXED);
    do
        upd = old ? (uint32_t)((int32_t)old + ((int32_t)fm - (int32_t)old) / 4) : fm;
    while (!__atomic_compare_exchange_n(&sl->f, &old, upd, 1, __ATOMIC_RELAXED,
                                        __ATOMIC_RELAXED));
}

/* `alone`: no other large host call is in flight, so a staged GPU share's
 * copies do not compete with other callers' CPU work; `cls`: ECM_CLS_* */
static int
hybrid_share_q(uint32_t k, int isa, uint64_t user, uint64_t moved, int op, uint64_t staged,
               uint64_t infl, int alone, int cls)
{
    double c, g, lat, f, f0;
    uint32_t learned;

    pthread_once(&ecm_xover_once, xover_init);
    if (!ecm_x.hybrid || ecm_x.always || user < ECM_HYBRID_MIN || moved < ecm_x.cpu_below ||
        infl == UINT64_MAX || staged == ECM_STAGED_UNKNOWN)
        return -1;
    if (ecm_x.hybrid_share)
        return (int)ecm_x.hybrid_share;
    /* a staged GPU share is copied by the library's CPU threads, so beside
     * the CPU share it competes for the same cores: 8 client threads of
     * 4 MiB 8+4 heal windows on pageable buffers fell from 41.2 to 26.6 GB/s
     * split (tools/kbench/concur, profiles/r05/r05o_concur_hybrid.log).  So
     * calls that stage split only while no other large call is in flight
     * (one stream: 6.5 -> 10.1 GB/s on pageable windows, r05o) */
    if (staged != 0 && !alone)
        return -1;
    xover_costs(k, isa, user, moved, op, staged, infl, &c, &g, &lat);
    if (g <= lat || c <= lat)
        return -1;
    f = (c - lat) / (c + g - lat);
    if (f < 0.15 || f > 0.85)
        return -1;
    learned = ecm_x.adapt ? __atomic_load_n(&share_slot(cls, k, user, staged, moved)->f,
                                            __ATOMIC_RELAXED)
                          : 0;
    if (learned) {
        f0 = f;
        if (infl) {             /* the queue's effect, as the model sees it */
            xover_costs(k, isa, user, moved, op, staged, 0, &c, &g, &lat);
            f0 = g > lat && c > lat ? (c - lat) / (c + g - lat) : f;
        }
        f = (double)learned / 1000.0 + (f - f0);
        f = f < 0.05 ? 0.05 : f > 0.95 ? 0.95 : f;
    }
    return (int)(f * 1000.0);
}

/* Host calls the router cannot send anywhere but the CPU engine (r06,
 * VERDICT r05 #3).  Below ECM_OBS_MIN (256 KiB) a call keeps no observed
 * rate, is never split (ECM_HYBRID_MIN) nor explored (ECM_OBS_EXPLORE), so
 * route_cpu_q compares the static model only: user / C against the idle,
 * all-mapped GPU's L + user / P (a queue or a staged buffer only add to
 * the GPU's side).  That is monotone in user: the CPU wins every call up to
 * U* = L / (1 / C - 1 / P), or every call when C >= P.  Such a call skips
 * the routing (queue and split probes, in-flight counters, two clock reads),
 * which cost ~0.1-0.3 us per call -- 3-6 % of a 128 KiB FUSE write coded in
 * ~4 us by one AVX-512 thread, measured as auto 431 against 461 GB/s for the
 * CPU engine alone in the round-5 driver bench (16 threads, 0 GPU calls). */
static uint64_t
small_cpu_below(uint32_t k, int isa, int op)
{
    static const double isa_f[] = {0.4, 0.7, 1.0};
    const double c = (op == ECM_ENCODE ? (double)ecm_x.enc_k2 / (k + 2) : (double)ecm_x.dec_k / k) *
                     isa_f[isa < 0 ? 0 : isa > 2 ? 2 : isa];
    const double p = (double)ecm_x.pin_gbps;
    double u;

    if (c <= 0)
        return 0;
    if (p <= 0 || c >= p)
        return ECM_OBS_MIN;
    u = (double)ecm_x.pin_us * 1e3 / (1.0 / c - 1.0 / p);   /* bytes */
    return u >= ECM_OBS_MIN ? ECM_OBS_MIN : (uint64_t)u;
}

static int
small_cpu(const ecm_ctx_t *ctx, uint64_t user, int op)
{
    return user < ctx->cpu_small[op] && !ecm_x.always;
}

static int
hybrid_share(const ecm_ctx_t *ctx, uint64_t user, uint64_t moved, int op, uint64_t staged,
             int cls)
{
    if (ctx->engine == ECM_ENGINE_CPU)
        return -1;
    return hybrid_share_q(ctx->k, ctx->isa, user, moved, op, staged, ecd_host_inflight(),
                          __atomic_load_n(&ecm_big_calls.n, __ATOMIC_RELAXED) <= 1, cls);
}

/* The split share of a call, querying where its buffers live only when an
 * all-mapped call of its size would be split (the queries serialise in the
 * HIP runtime); *staged is filled in when it was queried. */
static int
split_share(const ecm_ctx_t *ctx, uint64_t user, uint64_t moved, int op, int cls,
            uint64_t (*staged_of)(const void *), const void *arg, uint64_t *staged)
{
    if (hybrid_share(ctx, user, moved, op, 0, cls) <= 0)
        return -1;
    if (*staged == ECM_STAGED_UNKNOWN)
        *staged = staged_of(arg);
    return hybrid_share(ctx, user, moved, op, *staged, cls);
}

/* Helper threads that run the GPU share of split calls (at most 8; a call
 * finding none free is not split). */
typedef struct ecm_task {
    int (*fn)(void *);
    void *arg;
    int rc, done;
    uint64_t ns;                 /* the share's duration */
    uint64_t t_sub, wall;        /* hand-off time; done - hand-off */
    char err[256];               /* its error text when it failed */
    struct ecm_task *next;
} ecm_task_t;

#define ECM_HELPERS_MAX 8
static pthread_mutex_t ecm_pool_mu = PTHREAD_MUTEX_INITIALIZER;
static pthread_cond_t ecm_pool_cv = PTHREAD_COND_INITIALIZER;
static pthread_cond_t ecm_done_cv = PTHREAD_COND_INITIALIZER;
static ecm_task_t *ecm_q_head, **ecm_q_tail = &ecm_q_head;
static int ecm_helpers, ecm_helpers_idle, ecm_q_len;

static void *
helper_main(void *unused)
{
    ecm_task_t *t;
    uint64_t seq, t0;
    int rc;

    (void)unused;
    pthread_once(&ecm_xover_once, xover_init);
    pthread_mutex_lock(&ecm_pool_mu);
    for (;;) {
        while (!ecm_q_head) {
            /* (helpers that poll 50 or 200 us before sleeping measured
             * within run-to-run noise, profiles/r05/r05ab_spinab.log) */
            ecm_helpers_idle++;
            pthread_cond_wait(&ecm_pool_cv, &ecm_pool_mu);
            ecm_helpers_idle--;
        }
        t = ecm_q_head;
        ecm_q_head = t->next;
        if (!ecm_q_head)
            ecm_q_tail = &ecm_q_head;
        __atomic_sub_fetch(&ecm_q_len, 1, __ATOMIC_RELAXED);
        pthread_mutex_unlock(&ecm_pool_mu);
        seq = ecd_error_seq();
        t0 = now_ns();
        rc = t->fn(t->arg);
        t->ns = now_ns() - t0;
        t->wall = t0 + t->ns - t->t_sub;
        t->err[0] = 0;
        if (rc && ecd_error_seq() != seq)
            snprintf(t->err, sizeof t->err, "%s", ecd_last_error());
        pthread_mutex_lock(&ecm_pool_mu);
        t->rc = rc;
        t->done = 1;
        pthread_cond_broadcast(&ecm_done_cv);
    }
    return NULL;
}

/* fork() copies the pool's counters but none of its threads: a child that
 * split a call would queue it for helpers that do not exist and wait forever
 * (ADVICE r05).  The pool lock is held across fork, and the child starts with
 * an empty pool (its first split call starts its own helpers). */
static void
pool_atfork_prepare(void)
{
    pthread_mutex_lock(&ecm_pool_mu);
}

static void
pool_atfork_parent(void)
{
    pthread_mutex_unlock(&ecm_pool_mu);
}

static void
pool_atfork_child(void)
{
    pthread_mutex_init(&ecm_pool_mu, NULL);
    pthread_cond_init(&ecm_pool_cv, NULL);
    pthread_cond_init(&ecm_done_cv, NULL);
    ecm_q_head = NULL;
    ecm_q_tail = &ecm_q_head;
    ecm_helpers = ecm_helpers_idle = ecm_q_len = 0;
}

static pthread_once_t ecm_pool_once = PTHREAD_ONCE_INIT;

static void
pool_once(void)
{
    (void)pthread_atfork(pool_atfork_prepare, pool_atfork_parent, pool_atfork_child);
}

/* 0: queued for a free helper; -1: none free (the caller does not split) */
static int
helper_submit(ecm_task_t *t)
{
    pthread_attr_t at;
    pthread_t th;
    int ok = 1;

    pthread_once(&ecm_pool_once, pool_once);
    t->done = 0;
    t->next = NULL;
    t->t_sub = now_ns();
    pthread_mutex_lock(&ecm_pool_mu);
    if (ecm_helpers_idle <= ecm_q_len) {
        ok = ecm_helpers < ECM_HELPERS_MAX && pthread_attr_init(&at) == 0;
        if (ok) {
            pthread_attr_setdetachstate(&at, PTHREAD_CREATE_DETACHED);
            ok = pthread_create(&th, &at, helper_main, NULL) == 0;
            pthread_attr_destroy(&at);
        }
        if (ok)
            ecm_helpers++;
    }
    if (ok) {
        *ecm_q_tail = t;
        ecm_q_tail = &t->next;
        __atomic_add_fetch(&ecm_q_len, 1, __ATOMIC_RELAXED);
        pthread_cond_signal(&ecm_pool_cv);
    }
    pthread_mutex_unlock(&ecm_pool_mu);
    return ok ? 0 : -1;
}

static void
helper_wait(ecm_task_t *t)
{
    pthread_mutex_lock(&ecm_pool_mu);
    while (!t->done)
        pthread_cond_wait(&ecm_done_cv, &ecm_pool_mu);
    pthread_mutex_unlock(&ecm_pool_mu);
}

/* Stripes of a split call's GPU share: `share` thousandths of nstripes, a
 * multiple of `unit` (pattern groups), leaving each engine at least one
 * unit; 0 when the call is too short to split. */
static uint64_t
split_stripes(uint64_t nstripes, int share, uint64_t unit)
{
    const uint64_t sg = nstripes * (uint64_t)share / 1000u / unit * unit;

    return sg >= unit && sg + unit <= nstripes ? sg : 0;
}

/* other large host calls in flight beside the caller's own (which counts
 * itself when it is one) */
static uint32_t
big_others(uint64_t user)
{
    const uint32_t n = __atomic_load_n(&ecm_big_calls.n, __ATOMIC_RELAXED);
    const uint32_t self = user >= ECM_HYBRID_MIN;

    return n > self ? n - self : 0;
}

static int
route_cpu(const ecm_ctx_t *ctx, uint64_t user, uint64_t moved, int op, uint64_t staged)
{
    if (ctx->engine == ECM_ENGINE_CPU)
        return 1;
    return route_cpu_q(ctx->k, ctx->isa, user, moved, op, staged, ecd_host_inflight(),
                       big_others(user));
}

/* The engine for a host call: 1 = GPU.  `*staged` (in: ECM_STAGED_UNKNOWN)
 * is filled in when the placement of the buffers had to be queried. */
static int
route_gpu(const ecm_ctx_t *ctx, uint64_t user, uint64_t moved, int op,
          uint64_t (*staged_of)(const void *), const void *arg, uint64_t *staged)
{
    int gpu = 0, r = 1;

    /* the all-mapped GPU estimate is the optimistic one: a call that the CPU
     * wins against it skips the pointer queries (which serialise in the HIP
     * runtime: ~11 us each with 16 calling threads, tools/kbench/ptrq) */
    if (!route_cpu(ctx, user, moved, op, 0)) {
        *staged = staged_of(arg);
        r = route_cpu(ctx, user, moved, op, *staged);
        gpu = !r;
    }
    if (ctx->engine == ECM_ENGINE_CPU || ecm_x.always || moved < ecm_x.cpu_below ||
        r == ECM_ROUTE_CPU_BUSY)
        return gpu;
    if (user < ECM_OBS_EXPLORE)
        return gpu;
    if (*staged == ECM_STAGED_UNKNOWN)
        *staged = staged_of(arg);
    {
        double c, g, lat;

        xover_costs(ctx->k, ctx->isa, user, moved, op, *staged, ecd_host_inflight(), &c, &g,
                    &lat);
        if (gpu) {
            if (obs_explore(ECM_OBS_CPU, op, ctx->k, user, c > 4.0 * g))
                gpu = 0;
        } else if (route_cpu(ctx, user, moved, op, *staged) != ECM_ROUTE_CPU_BUSY &&
                   obs_explore(gpu_obs_engine(*staged, moved), op, ctx->k, user, g > 4.0 * c)) {
            /* (not while other callers keep the CPU busy and the call's
             * staging copies would cost more CPU than coding it) */
            gpu = 1;
        }
    }
    return gpu;
}

/* Crossover probes for tests (include/ec_method.h): the router of a GPU
 * volume, with the queue given, needs no device. */
int32_t
ec_method_xover_route(uint32_t k, int32_t op, uint64_t user, uint64_t moved, uint64_t staged,
                      uint64_t inflight)
{
    if (k < 1 || k > ECM_MAX_K || moved == 0 || (op != ECM_ENCODE && op != ECM_DECODE))
        return -EINVAL;
    return route_cpu_q(k, ecc_isa_max(), user, moved, op, staged, inflight, 0) != 0;
}

int32_t
ec_method_xover_plan(uint32_t k, int32_t op, uint64_t user, uint64_t moved, uint64_t staged,
                     uint64_t inflight, uint32_t others, int32_t *share)
{
    int r;

    if (k < 1 || k > ECM_MAX_K || moved == 0 || (op != ECM_ENCODE && op != ECM_DECODE))
        return -EINVAL;
    r = route_cpu_q(k, ecc_isa_max(), user, moved, op, staged, inflight, others);
    if (share)
        *share = hybrid_share_q(k, ecc_isa_max(), user, moved, op, staged, inflight,
                                others == 0, op);
    return r;
}

int32_t
ec_method_xover_observe_split(int32_t op, uint32_t k, uint64_t user, uint64_t moved,
                              uint64_t staged, uint32_t gpu_share, uint64_t gpu_ns,
                              uint64_t cpu_ns)
{
    const uint64_t n = 1000;

    if (k < 1 || k > ECM_MAX_K || moved == 0 || (op != ECM_ENCODE && op != ECM_DECODE) ||
        gpu_share == 0 || gpu_share >= 1000)
        return -EINVAL;
    share_learn(op, op, k, ecc_isa_max(), user, moved, staged, n, gpu_share, gpu_ns, cpu_ns);
    return 0;
}

int32_t
ec_method_xover_observe_part(int32_t engine, int32_t op, uint32_t k, uint64_t user, uint64_t part,
                             uint64_t ns, uint64_t staged, uint64_t moved)
{
    if (engine < 0 || engine >= ECM_OBS_ENGINES || (op != ECM_ENCODE && op != ECM_DECODE) ||
        k < 1 || k > ECM_MAX_K || part == 0 || part > user || moved == 0)
        return -EINVAL;
    pthread_once(&ecm_xover_once, xover_init);
    if (engine == ECM_OBS_CPU)
        obs_record_part(engine, op, k, user, part, ns);
    else
        obs_record_gpu_part(engine, op, k, user, part, ns, staged, moved);
    return 0;
}

int32_t
ec_method_xover_split(uint32_t k, int32_t op, uint64_t user, uint64_t moved, uint64_t staged,
                      uint64_t inflight)
{
    if (k < 1 || k > ECM_MAX_K || moved == 0 || (op != ECM_ENCODE && op != ECM_DECODE))
        return -EINVAL;
    return hybrid_share_q(k, ecc_isa_max(), user, moved, op, staged, inflight, 0, op);
}

int32_t
ec_method_xover_observe(int32_t engine, int32_t op, uint32_t k, uint64_t user, uint64_t ns)
{
    if (engine < 0 || engine >= ECM_OBS_ENGINES || (op != ECM_ENCODE && op != ECM_DECODE) ||
        k < 1 || k > ECM_MAX_K)
        return -EINVAL;
    pthread_once(&ecm_xover_once, xover_init);
    obs_record(engine, op, k, user, ns);
    return 0;
}

/* Field by field with atomic stores: obs_record / obs_explore update the
 * same fields atomically from coding threads, so a reset during traffic is
 * not a data race (a memset was, under TSan).  A call in flight may still
 * add its sample after the reset. */
void
ec_method_xover_reset(void)
{
    ecm_obs_t *o = &ecm_obs[0][0][0][0];
    ecm_share_t *sh = &ecm_share[0][0][0][0];
    size_t i;

    for (i = 0; i < sizeof(ecm_obs) / sizeof(ecm_obs[0][0][0][0]); i++) {
        __atomic_store_n(&o[i].kbps, 0, __ATOMIC_RELAXED);
        __atomic_store_n(&o[i].lost, 0, __ATOMIC_RELAXED);
        __atomic_store_n(&o[i].n, 0, __ATOMIC_RELAXED);
    }
    for (i = 0; i < sizeof(ecm_share) / sizeof(ecm_share[0][0][0][0]); i++) {
        __atomic_store_n(&sh[i].f, 0, __ATOMIC_RELAXED);
        __atomic_store_n(&sh[i].n, 0, __ATOMIC_RELAXED);
    }
}

/* bytes of the n buffers b[0..n) (len bytes each; NULL entries skipped) that
 * are not pinned, device-mapped host memory */
static uint64_t
staged_bytes(const void *const *b, uint32_t n, uint64_t len)
{
    uint64_t s = 0;
    uint32_t i;

    for (i = 0; i < n; i++)
        if (b[i] && !ecd_host_mapped(b[i], len))
            s += len;
    return s;
}

/* A failed device submission for host buffers: log once, count, and let
 * the caller redo the call on the CPU engine (-EINVAL is an argument error
 * the CPU would reject as well, and is returned). */
static int
gpu_failed(int rc)
{
    static int logged;

    if (rc == 0 || rc == -EINVAL || rc == -E2BIG)
        return 0;
    stat_add(ECM_STAT_FALLBACK);
    if (!__atomic_exchange_n(&logged, 1, __ATOMIC_RELAXED))
        ecm_log("device submission failed (%d: %s); coding on the CPU engine", rc,
                ecd_last_error());
    return 1;
}

static int32_t ecm_ret(const char *fn, uint64_t seq, int32_t rc);

#define CTX(list) ((ecm_ctx_t *)(list)->code)
#define LRU_HEAD(list) ((ecm_matrix_t *)(void *)(list)->lru)

static void
lru_init(ec_matrix_list_t *list)
{
    list->lru[0] = list->lru;
    list->lru[1] = list->lru;
}

/* The list head is the two-pointer lru field; matrices link through their
 * leading next/prev pointers, so the head can be treated as a node. */
static void
lru_unlink(ecm_matrix_t *m)
{
    m->prev->next = m->next;
    m->next->prev = m->prev;
    m->next = m->prev = m;
}

static void
lru_push_tail(ec_matrix_list_t *list, ecm_matrix_t *m)
{
    ecm_matrix_t *head = LRU_HEAD(list);

    m->next = head;
    m->prev = head->prev;
    head->prev->next = m;
    head->prev = m;
}

static ecm_matrix_t *
lru_first(ec_matrix_list_t *list)
{
    ecm_matrix_t *head = LRU_HEAD(list);

    return head->next == head ? NULL : head->next;
}

/* Binary search of the mask-sorted cache (ec-method.c:145-169). */
static ecm_matrix_t *
cache_lookup(ec_matrix_list_t *list, uintptr_t mask, uint32_t *pos)
{
    ecm_matrix_t **obj = (ecm_matrix_t **)list->objects;
    uint32_t lo = 0, hi = list->count, mid;

    while (lo < hi) {
        mid = (lo + hi) >> 1;
        if (obj[mid]->mask == mask) {
            *pos = mid;
            return obj[mid];
        }
        if (obj[mid]->mask < mask)
            lo = mid + 1;
        else
            hi = mid;
    }
    *pos = lo;
    return NULL;
}

static void
cache_remove(ec_matrix_list_t *list, ecm_matrix_t *m)
{
    ecm_matrix_t **obj = (ecm_matrix_t **)list->objects;
    uint32_t pos;

    if (cache_lookup(list, m->mask, &pos) == m) {
        list->count--;
        memmove(obj + pos, obj + pos + 1, sizeof(*obj) * (list->count - pos));
    }
    m->cached = 0;
}

static void
cache_insert(ec_matrix_list_t *list, ecm_matrix_t *m)
{
    ecm_matrix_t **obj = (ecm_matrix_t **)list->objects;
    uint32_t pos;

    (void)cache_lookup(list, m->mask, &pos);
    memmove(obj + pos + 1, obj + pos, sizeof(*obj) * (list->count - pos));
    obj[pos] = m;
    list->count++;
    m->cached = 1;
}

static int
mask_rows_ok(const ec_matrix_list_t *list, uintptr_t mask, const uint32_t *rows)
{
    uint32_t p, bits = 0;
    uintptr_t seen = 0;

    for (p = 0; p < list->rows && p < sizeof(uintptr_t) * 8; p++)
        bits += (mask >> p) & 1;
    if (bits != list->columns || (mask >> list->rows) != 0)
        return 0;
    for (p = 0; p < list->columns; p++) {
        if (rows[p] < 1 || rows[p] > list->rows)
            return 0;
        if (p && rows[p] <= rows[p - 1])
            return 0;
        seen |= (uintptr_t)1 << (rows[p] - 1);
    }
    return seen == mask;
}

static void
rows_from_mask(uintptr_t mask, uint32_t *rows)
{
    uint32_t i, p = 0;

    for (i = 0; i < sizeof(uintptr_t) * 8; i++)
        if ((mask >> i) & 1)
            rows[p++] = i + 1;
}

/* ec-method.c:200-245: cached inverse for `mask`, refcount held. */
static ecm_matrix_t *
matrix_get(ec_matrix_list_t *list, uintptr_t mask, const uint32_t *rows)
{
    ecm_matrix_t *m;
    uint32_t pos;

    pthread_mutex_lock(&list->lock);
    m = cache_lookup(list, mask, &pos);
    if (m) {
        if (m->refs++ == 0)
            lru_unlink(m);
        pthread_mutex_unlock(&list->lock);
        return m;
    }
    if (list->count >= list->max && (m = lru_first(list)) != NULL) {
        lru_unlink(m);
        cache_remove(list, m);
    } else {
        m = (ecm_matrix_t *)calloc(1, sizeof(*m));
        if (!m) {
            pthread_mutex_unlock(&list->lock);
            return NULL;
        }
    }
    m->next = m->prev = m;
    m->refs = 1;
    m->mask = mask;
    m->k = list->columns;
    memcpy(m->rows, rows, sizeof(uint32_t) * list->columns);
    ec_method_inverse_matrix(list->columns, rows, m->inv);
    if (list->count < list->max)
        cache_insert(list, m);
    pthread_mutex_unlock(&list->lock);
    return m;
}

/* ec-method.c:247-255 / :133-143 */
static void
matrix_put(ec_matrix_list_t *list, ecm_matrix_t *m)
{
    pthread_mutex_lock(&list->lock);
    if (--m->refs == 0) {
        if (m->cached)
            lru_push_tail(list, m);
        else
            free(m);
    }
    pthread_mutex_unlock(&list->lock);
}

/* Pack {src[k], coef[rows][k]} for the combine kernel. */
static uint32_t
pack_pattern(uint8_t *dst, uint32_t k, const uint8_t *src, uint32_t rows,
             const uint32_t *coef)
{
    uint32_t i;

    memcpy(dst, src, k);
    for (i = 0; i < rows * k; i++)
        dst[k + i] = (uint8_t)coef[i];
    return k + rows * k;
}

/* --------------------------------------------------- on-disk config guard */

#define ECM_CONFIG_VERSION 0   /* EC_CONFIG_VERSION, ec-common.h:22   */
#define ECM_CONFIG_ALGORITHM 0 /* EC_CONFIG_ALGORITHM, ec-common.h:24 */

void
ec_method_config_fill(uint32_t bricks, uint32_t redundancy, ec_config_t *c)
{
    c->version = ECM_CONFIG_VERSION;
    c->algorithm = ECM_CONFIG_ALGORITHM;
    c->gf_word_size = EC_GF_BITS;
    c->bricks = (uint8_t)bricks;
    c->redundancy = (uint8_t)redundancy;
    c->chunk_size = EC_METHOD_CHUNK_SIZE;
}

int32_t
ec_method_config_pack(const ec_config_t *c, uint8_t value[8])
{
    uint64_t data;
    int i;

    if (!c || !value || c->version > ECM_CONFIG_VERSION)
        return -EINVAL;
    data = (uint64_t)c->version << 56 | (uint64_t)c->algorithm << 48 |
           (uint64_t)c->gf_word_size << 40 | (uint64_t)c->bricks << 32 |
           (uint64_t)c->redundancy << 24 | (uint64_t)(c->chunk_size & 0xFFFFFF);
    for (i = 0; i < 8; i++) /* big-endian, as htobe64 */
        value[i] = (uint8_t)(data >> (56 - 8 * i));
    return 0;
}

int32_t
ec_method_config_unpack(const void *value, size_t len, ec_config_t *c)
{
    const uint8_t *v = (const uint8_t *)value;
    uint64_t data = 0;
    int i;

    if (!value || !c || len != 8)
        return -EINVAL;
    for (i = 0; i < 8; i++)
        data = data << 8 | v[i];
    if (data == 0)
        return -ENODATA; /* a zero config is a missing xattr (ec-helpers.c:359) */
    c->version = (uint32_t)(data >> 56) & 0xFF;
    if (c->version > ECM_CONFIG_VERSION)
        return -EINVAL;
    c->algorithm = (uint8_t)(data >> 48);
    c->gf_word_size = (uint8_t)(data >> 40);
    c->bricks = (uint8_t)(data >> 32);
    c->redundancy = (uint8_t)(data >> 24);
    c->chunk_size = (uint32_t)(data & 0xFFFFFF);
    return 0;
}

int32_t
ec_method_config_check(uint32_t bricks, uint32_t redundancy, const ec_config_t *c)
{
    uint32_t data_bricks;

    if (!c)
        return -EINVAL;
    if (c->version == ECM_CONFIG_VERSION && c->algorithm == ECM_CONFIG_ALGORITHM &&
        c->gf_word_size == EC_GF_BITS && c->bricks == bricks &&
        c->redundancy == redundancy && c->chunk_size == EC_METHOD_CHUNK_SIZE)
        return 0;
    /* the corruption test of ec-common.c:1162-1180 (data_bricks is computed
     * in unsigned arithmetic there too; bricks <= redundancy is caught by
     * the 2 * redundancy >= bricks test before it can matter) */
    data_bricks = (uint32_t)c->bricks - c->redundancy;
    if (c->redundancy < 1 || c->redundancy * 2 >= c->bricks || c->gf_word_size == 0 ||
        (c->gf_word_size & (c->gf_word_size - 1)) != 0 ||
        (uint32_t)(c->chunk_size * 8u) % (c->gf_word_size * data_bricks) != 0)
        return -EINVAL;
    return -ENOTSUP;
}

/* ------------------------------------------------------------ the API */

int32_t
ec_method_device_count(void)
{
    return ecd_device_count();
}

int32_t
ec_method_device_numa_node(int32_t device)
{
    return ecd_device_numa_node(device);
}

int32_t
ec_method_copy_threads(void)
{
    return ecd_copy_threads();
}

const char *
ec_method_last_error(void)
{
    return ecd_last_error();
}

void *
ec_method_host_alloc(size_t bytes)
{
    return ecd_host_alloc(bytes);
}

void
ec_method_host_free(void *p)
{
    ecd_host_free(p);
}

static int32_t
ecm_host_register_impl(void *p, size_t bytes)
{
    return ecd_host_register(p, bytes);
}

static int32_t
ecm_host_unregister_impl(void *p)
{
    return ecd_host_unregister(p);
}

static int32_t
ecm_host_register_async_impl(void *p, size_t bytes)
{
    return ecd_host_register_async(p, bytes);
}

void
ec_method_host_register_flush(void)
{
    ecd_host_register_flush();
}

void *
ec_method_buffer_get(size_t bytes)
{
    return ecd_buffer_get(bytes);
}

int32_t
ec_method_buffer_put(void *p)
{
    return ecd_buffer_put(p);
}

void
ec_method_pool_stats(ec_method_pool_stats_t *st)
{
    ecd_pool_stats_t s;

    if (!st)
        return;
    ecd_pool_stats(&s);
    st->pool_bytes = s.pool_bytes;
    st->in_use_bytes = s.in_use_bytes;
    st->gets = s.gets;
    st->misses = s.misses;
    st->slabs = s.slabs;
    st->slab_register_us = s.slab_register_us;
    st->deferred_registers = s.deferred_registers;
    st->deferred_register_us = s.deferred_register_us;
    st->deferred_register_failures = s.deferred_register_failures;
    st->unregisters = s.unregisters;
    st->unregister_us = s.unregister_us;
}

void
ec_method_jit_stats(ec_method_jit_stats_t *st)
{
    ecd_jit_stats_t s;

    if (!st)
        return;
    ecd_jit_stats(&s);
    st->compiled = s.compiled;
    st->failed = s.failed;
    st->launches = s.launches;
    st->compile_us = s.compile_us;
    st->lookups = s.lookups;
    st->entries = s.entries;
}

int32_t
ec_method_jit_prepare(uint32_t k, uint32_t rows, const uint8_t *coef)
{
    return ecd_jit_prepare(k, rows, coef);
}

int32_t
ec_method_jit_compile_check(uint32_t k, uint32_t rows, const uint8_t *coef, uint32_t *ops)
{
    char log[512];

    return ecd_jit_compile_check(k, rows, coef, ops, log, sizeof log);
}

/* disperse.cpu-extensions (ec.c:1786-1794) -> engine.  The reference maps
 * none to portable C and x64 / sse / avx to its JIT back ends, auto to the
 * best of them (ec-code.c:59-69, 977-1060).  Here auto (and hip) select the
 * gfx950 engine when a device is visible -- with the CPU engine beside it
 * for small calls and as the fallback -- and the CPU engine otherwise; none,
 * x64 and sse select the CPU engine at the base x86-64 level, avx the best
 * AVX level of this CPU (library extensions, not in ec.c's option table:
 * avx2 / avx512 pin that level, for tests and tuning).  Unknown values warn
 * and act as auto, as the reference's fall back to C with a warning
 * (ec-code.c:1007-1013). */
static void
pick_engine(ecm_ctx_t *ctx, const char *gen)
{
    int isa_best = ecc_isa_max(), want_gpu = 1;

    ctx->isa = isa_best;
    if (gen && (!strcmp(gen, "none") || !strcmp(gen, "x64") || !strcmp(gen, "sse"))) {
        want_gpu = 0;
        ctx->isa = ECC_ISA_BASE;
    } else if (gen && !strcmp(gen, "avx")) {
        want_gpu = 0;
    } else if (gen && !strcmp(gen, "avx2")) {
        want_gpu = 0;
        ctx->isa = isa_best < ECC_ISA_AVX2 ? isa_best : ECC_ISA_AVX2;
    } else if (gen && !strcmp(gen, "avx512")) {
        want_gpu = 0;
    } else if (gen && strcmp(gen, "auto") && strcmp(gen, "hip")) {
        ecm_log("unknown cpu-extensions value '%s', using 'auto'", gen);
    }
    if (want_gpu && ecd_device_count() == 0) {
        ecm_log("no MI355X (gfx950) device visible (%s): CPU engine", ecd_last_error());
        want_gpu = 0;
    }
    ctx->engine = want_gpu ? ECM_ENGINE_GPU : ECM_ENGINE_CPU;
    pthread_once(&ecm_xover_once, xover_init);
    ctx->cpu_small[ECM_ENCODE] = want_gpu ? small_cpu_below(ctx->k, ctx->isa, ECM_ENCODE) : 0;
    ctx->cpu_small[ECM_DECODE] = want_gpu ? small_cpu_below(ctx->k, ctx->isa, ECM_DECODE) : 0;
    if (want_gpu)
        snprintf(ctx->engine_name, sizeof(ctx->engine_name), "gfx950 x%d + cpu/%s",
                 ecd_device_count(), ecc_isa_name(ctx->isa));
    else
        snprintf(ctx->engine_name, sizeof(ctx->engine_name), "cpu/%s", ecc_isa_name(ctx->isa));
}

static int32_t
ecm_init_impl(xlator_t *xl, ec_matrix_list_t *list, uint32_t columns, uint32_t rows,
             uint32_t max, const char *gen)
{
    ecm_ctx_t *ctx;
    uint32_t i;

    (void)xl;
    if (!list)
        return -EINVAL;
    memset(list, 0, sizeof(*list));
    if (columns < 1 || columns > ECM_MAX_K || rows < columns || rows > ECM_MAX_N)
        return -EINVAL;

    ctx = (ecm_ctx_t *)calloc(1, sizeof(*ctx));
    list->objects = (void **)calloc(max ? max : 1, sizeof(void *));
    if (!ctx || !list->objects) {
        free(ctx);
        free(list->objects);
        list->objects = NULL;
        return -ENOMEM;
    }
    ctx->k = columns;
    ctx->n = rows;
    ctx->serial = __atomic_add_fetch(&ecm_serial, 1, __ATOMIC_RELAXED);
    snprintf(ctx->gen, sizeof(ctx->gen), "%s", gen ? gen : "auto");
    pick_engine(ctx, gen);
    ec_method_encode_matrix(columns, rows, ctx->enc);
    {
        uint8_t src[ECM_MAX_K];
        for (i = 0; i < columns; i++)
            src[i] = (uint8_t)i;
        pack_pattern(ctx->enc_pat, columns, src, rows, ctx->enc);
    }

    list->columns = columns;
    list->rows = rows;
    list->max = max;
    list->count = 0;
    list->stripe = EC_METHOD_CHUNK_SIZE * columns;
    list->gf = (void *)ecm_gf_get();
    list->code = ctx;
    list->encode = ctx->enc;
    lru_init(list);
    pthread_mutex_init(&list->lock, NULL);
    ecm_log("disperse %u+%u: %s engine (cpu-extensions=%s%s)", columns, rows - columns,
            ctx->engine_name, ctx->gen,
            ctx->engine == ECM_ENGINE_GPU
                ? (ecd_has_vander(columns, rows) ? ", specialised encoder" : ", generic encoder")
                : "");
    return 0;
}

const char *
ec_method_engine(const ec_matrix_list_t *list)
{
    const ecm_ctx_t *ctx = list ? (const ecm_ctx_t *)list->code : NULL;

    return ctx ? ctx->engine_name : "";
}

void
ec_method_fini(ec_matrix_list_t *list)
{
    ecm_matrix_t *m;

    if (!list || !list->code)
        return;
    while ((m = lru_first(list)) != NULL) {
        lru_unlink(m);
        cache_remove(list, m);
        free(m);
    }
    /* referenced matrices cannot exist here: callers hold refs only inside
     * a decode call (ec-method.c:369 asserts the same) */
    pthread_mutex_destroy(&list->lock);
    free(list->objects);
    free(list->code);
    memset(list, 0, sizeof(*list));
}

static int32_t
ecm_update_impl(xlator_t *xl, ec_matrix_list_t *list, const char *gen)
{
    (void)xl;
    (void)list;
    (void)gen;
    return 0;
}

/* 1 when every non-NULL buffer of b[0..n) is on `dev` (-1: host memory).
 * Host and device buffers cannot be mixed in one call: the kernels would
 * read host addresses as device ones, the staging copies device addresses
 * as host ones. */
static int
bufs_on(const void *const *b, uint32_t n, int dev)
{
    uint32_t i;

    for (i = 0; i < n; i++)
        if (b[i] && ecd_ptr_device(b[i]) != dev)
            return 0;
    return 1;
}

static uint32_t
popcount_mask(uintptr_t m)
{
    uint32_t c = 0;

    for (; m; m &= m - 1)
        c++;
    return c;
}

/* Host-buffer encode: the GPU pipeline, or the CPU engine (crossover,
 * CPU-only volumes, and the fallback when the device submission fails). */
struct enc_bufs {
    const void *in;
    void *const *out;
    uint32_t k, n;
    uint64_t fl;
};

static uint64_t
enc_staged(const void *arg)
{
    const struct enc_bufs *b = (const struct enc_bufs *)arg;

    return (ecd_host_mapped(b->in, b->fl * b->k) ? 0 : b->fl * b->k) +
           staged_bytes((const void *const *)b->out, b->n, b->fl);
}

/* the GPU share of a split encode (helper thread) */
struct enc_share {
    const ecm_ctx_t *ctx;
    uint64_t nstripes;
    const void *in;
    void *const *out;
};

static int
enc_share_gpu(void *a)
{
    const struct enc_share *e = (const struct enc_share *)a;

    return ecd_encode_host(0, e->ctx->k, e->ctx->n, e->nstripes, e->in, e->out,
                           e->ctx->enc_pat);
}

/* A split host encode: stripes [0, sg) on a GPU, the rest on the CPU engine
 * meanwhile; a failed GPU share is redone on the CPU.  -EAGAIN: not split. */
static int
encode_split(ecm_ctx_t *ctx, uint64_t nstripes, const void *in, void *const *out, int share,
             uint64_t staged)
{
    const uint64_t S = (uint64_t)ctx->k * EC_METHOD_CHUNK_SIZE, user = nstripes * S;
    const uint64_t sg = split_stripes(nstripes, share, 1);
    struct enc_share es = {ctx, sg, in, out};
    ecm_task_t t = {enc_share_gpu, &es, 0, 0, 0, 0, 0, "", NULL};
    uint8_t *o2[ECM_MAX_N];
    uint64_t t0;
    uint32_t i;

    if (!sg || helper_submit(&t) != 0)
        return -EAGAIN;
    for (i = 0; i < ctx->n; i++)
        o2[i] = (uint8_t *)out[i] + sg * EC_METHOD_CHUNK_SIZE;
    t0 = now_ns();
    ecc_encode(ctx->isa, ctx->k, ctx->n, nstripes - sg, (const uint8_t *)in + sg * S, o2);
    t0 = now_ns() - t0;
    obs_record_part(ECM_OBS_CPU, ECM_ENCODE, ctx->k, user, (nstripes - sg) * S, t0);
    stat_add(ECM_STAT_CPU);
    helper_wait(&t);
    if (t.rc == 0) {
        const uint64_t moved = nstripes * EC_METHOD_CHUNK_SIZE * (ctx->k + ctx->n);

        stat_add(ECM_STAT_GPU);
        obs_record_gpu_part(gpu_obs_engine(staged, moved), ECM_ENCODE, ctx->k, user, sg * S, t.ns,
                            staged, moved);
        share_learn(ECM_CLS_ENCODE, ECM_ENCODE, ctx->k, ctx->isa, user, moved, staged, nstripes,
                    sg, t.wall, t0);
        return 0;
    }
    if (t.err[0])
        ecd_set_error(t.err);
    if (!gpu_failed(t.rc))
        return t.rc;
    ecc_encode(ctx->isa, ctx->k, ctx->n, sg, (const uint8_t *)in, (uint8_t *const *)out);
    return 0;
}

static int
host_encode_1(ecm_ctx_t *ctx, uint64_t nstripes, const void *in, void *const *out)
{
    const uint64_t fl = nstripes * EC_METHOD_CHUNK_SIZE, user = fl * ctx->k;
    const uint64_t bytes = fl * (ctx->k + ctx->n);
    const struct enc_bufs eb = {in, out, ctx->k, ctx->n, fl};
    uint64_t t0, staged = ECM_STAGED_UNKNOWN;
    int rc, gpu, share;

    gpu = route_gpu(ctx, user, bytes, ECM_ENCODE, enc_staged, &eb, &staged);
    share = split_share(ctx, user, bytes, ECM_ENCODE, ECM_CLS_ENCODE, enc_staged, &eb, &staged);
    if (share > 0 && (rc = encode_split(ctx, nstripes, in, out, share, staged)) != -EAGAIN)
        return rc;
    if (gpu) {
        t0 = now_ns();
        rc = ecd_encode_host(0, ctx->k, ctx->n, nstripes, in, out, ctx->enc_pat);
        if (!gpu_failed(rc)) {
            if (rc == 0) {
                stat_add(ECM_STAT_GPU);
                if (staged != ECM_STAGED_UNKNOWN)
                    obs_record(gpu_obs_engine(staged, bytes), ECM_ENCODE, ctx->k, user,
                               now_ns() - t0);
            }
            return rc;
        }
    }
    t0 = now_ns();
    ecc_encode(ctx->isa, ctx->k, ctx->n, nstripes, (const uint8_t *)in, (uint8_t *const *)out);
    if (ctx->engine != ECM_ENGINE_CPU)
        obs_record(ECM_OBS_CPU, ECM_ENCODE, ctx->k, user, now_ns() - t0);
    stat_add(ECM_STAT_CPU);
    return 0;
}

/* (large calls counted in flight: the split rule for staged calls) */
static int
host_encode(ecm_ctx_t *ctx, uint64_t nstripes, const void *in, void *const *out)
{
    const uint64_t user = nstripes * EC_METHOD_CHUNK_SIZE * ctx->k;
    int rc;

    if (small_cpu(ctx, user, ECM_ENCODE)) {
        ecc_encode(ctx->isa, ctx->k, ctx->n, nstripes, (const uint8_t *)in, (uint8_t *const *)out);
        stat_add(ECM_STAT_CPU);
        return 0;
    }
    big_call(user, 1);
    rc = host_encode_1(ctx, nstripes, in, out);
    big_call(user, -1);
    return rc;
}

struct dec_bufs {
    const void *const *frags;
    uint32_t nfrags;
    void *out;
    void *const *outs;
    uint32_t rows;
    uint64_t fl;
};

static uint64_t
dec_staged(const void *arg)
{
    const struct dec_bufs *b = (const struct dec_bufs *)arg;

    return staged_bytes(b->frags, b->nfrags, b->fl) +
           (b->outs ? staged_bytes((const void *const *)b->outs, b->rows, b->fl)
                    : (ecd_host_mapped(b->out, b->fl * b->rows) ? 0 : b->fl * b->rows));
}

/* The arguments of a host combination (ecd_decode_host's). */
struct dec_call {
    uint32_t k, rows, nfrags, npat, shift;
    uint64_t nstripes;
    const void *const *frags;
    void *out;
    void *const *outs;
    const uint8_t *pats, *gp;
};

static int
dec_share_gpu(void *a)
{
    const struct dec_call *c = (const struct dec_call *)a;

    return ecd_decode_host(0, c->k, c->rows, c->nstripes, c->nfrags, c->frags, c->out, c->outs,
                           c->npat, c->pats, c->gp, c->shift);
}

/* Stripes [s0, s1) of a host combination on the CPU engine (s0: a multiple
 * of the pattern group). */
static int
cpu_decode(const ecm_ctx_t *ctx, const struct dec_call *c, uint64_t s0, uint64_t s1)
{
    ecd_combine_desc_t d;
    uint32_t f, r;

    memset(&d, 0, offsetof(ecd_combine_desc_t, pat));
    d.k = c->k;
    d.rows = c->rows;
    d.nstripes = s1 - s0;
    d.in_stride = EC_METHOD_CHUNK_SIZE;
    for (f = 0; f < c->nfrags; f++)      /* NULL: a fragment no pattern reads */
        d.in_base[f] = c->frags[f] ? (const uint8_t *)c->frags[f] + s0 * EC_METHOD_CHUNK_SIZE
                                   : NULL;
    if (c->outs) {
        d.out_stride = EC_METHOD_CHUNK_SIZE;
        for (r = 0; r < c->rows; r++)
            d.out_base[r] = (uint8_t *)c->outs[r] + s0 * EC_METHOD_CHUNK_SIZE;
    } else {
        d.out_stride = (uint64_t)c->rows * EC_METHOD_CHUNK_SIZE;
        for (r = 0; r < c->rows; r++)
            d.out_base[r] = (uint8_t *)c->out + s0 * d.out_stride + (uint64_t)r * EC_METHOD_CHUNK_SIZE;
    }
    d.npatterns = c->npat;
    d.pat_bytes = c->k + c->rows * c->k;
    d.pat_ext = c->pats;
    d.group_pattern = c->gp ? c->gp + (s0 >> c->shift) : NULL;
    d.group_shift = c->shift;
    return ecc_combine(ctx->isa, &d);
}

/* A split host combination: [0, sg) on a GPU, the rest here on the CPU
 * engine; a failed GPU share is redone on the CPU.  -EAGAIN: not split. */
static int
decode_split(ecm_ctx_t *ctx, const struct dec_call *c, int share, uint64_t staged)
{
    const uint64_t unit = c->gp ? 1ull << c->shift : 1;
    const uint64_t sg = split_stripes(c->nstripes, share, unit);
    const uint64_t per = (uint64_t)c->k * EC_METHOD_CHUNK_SIZE, user = c->nstripes * per;
    struct dec_call g = *c;
    ecm_task_t t = {dec_share_gpu, &g, 0, 0, 0, 0, 0, "", NULL};
    uint64_t t0;
    int rc;

    g.nstripes = sg;
    if (!sg || helper_submit(&t) != 0)
        return -EAGAIN;
    t0 = now_ns();
    rc = cpu_decode(ctx, c, sg, c->nstripes);
    t0 = now_ns() - t0;
    if (rc == 0) {
        obs_record_part(ECM_OBS_CPU, ECM_DECODE, c->k, user, (c->nstripes - sg) * per, t0);
        stat_add(ECM_STAT_CPU);
    }
    helper_wait(&t);
    if (t.rc == 0) {
        const uint64_t moved = c->nstripes * EC_METHOD_CHUNK_SIZE * (c->k + c->rows);

        stat_add(ECM_STAT_GPU);
        obs_record_gpu_part(gpu_obs_engine(staged, moved), ECM_DECODE, c->k, user, sg * per,
                            t.ns, staged, moved);
        if (rc == 0)
            share_learn(c->rows == c->k ? ECM_CLS_DECODE : ECM_CLS_PART, ECM_DECODE, c->k,
                        ctx->isa, user, moved, staged, c->nstripes, sg, t.wall, t0);
        return rc;
    }
    if (t.err[0])
        ecd_set_error(t.err);
    if (!gpu_failed(t.rc))
        return t.rc;
    return rc ? rc : cpu_decode(ctx, c, 0, sg);
}

/* Host-buffer combination (decode, mixed decode, heal): the GPU pipeline or
 * the CPU engine, same arguments as ecd_decode_host. */
static int
host_decode_1(ecm_ctx_t *ctx, uint32_t k, uint32_t rows, uint64_t nstripes, uint32_t nfrags,
              const void *const *frags, void *out, void *const *outs, uint32_t npat,
              const uint8_t *pats, const uint8_t *gp, uint32_t shift)
{
    const uint64_t bytes = nstripes * EC_METHOD_CHUNK_SIZE * (k + rows);
    const uint64_t fl = nstripes * EC_METHOD_CHUNK_SIZE;
    const struct dec_bufs db = {frags, nfrags, out, outs, rows, fl};
    const struct dec_call call = {k, rows, nfrags, npat, shift, nstripes, frags, out, outs, pats, gp};
    uint64_t t0, staged = ECM_STAGED_UNKNOWN;
    int rc, gpu, share;

    gpu = route_gpu(ctx, fl * k, bytes, ECM_DECODE, dec_staged, &db, &staged);
    share = split_share(ctx, fl * k, bytes, ECM_DECODE,
                        rows == k ? ECM_CLS_DECODE : ECM_CLS_PART, dec_staged, &db, &staged);
    if (share > 0 && (rc = decode_split(ctx, &call, share, staged)) != -EAGAIN)
        return rc;
    if (gpu) {
        t0 = now_ns();
        rc = ecd_decode_host(0, k, rows, nstripes, nfrags, frags, out, outs, npat, pats, gp,
                             shift);
        if (!gpu_failed(rc)) {
            if (rc == 0) {
                stat_add(ECM_STAT_GPU);
                if (staged != ECM_STAGED_UNKNOWN)
                    obs_record(gpu_obs_engine(staged, bytes), ECM_DECODE, k, fl * k,
                               now_ns() - t0);
            }
            return rc;
        }
    }
    t0 = now_ns();
    rc = cpu_decode(ctx, &call, 0, nstripes);
    if (rc == 0) {
        if (ctx->engine != ECM_ENGINE_CPU)
            obs_record(ECM_OBS_CPU, ECM_DECODE, k, fl * k, now_ns() - t0);
        stat_add(ECM_STAT_CPU);
    }
    return rc;
}

static int
host_decode(ecm_ctx_t *ctx, uint32_t k, uint32_t rows, uint64_t nstripes, uint32_t nfrags,
            const void *const *frags, void *out, void *const *outs, uint32_t npat,
            const uint8_t *pats, const uint8_t *gp, uint32_t shift)
{
    const uint64_t user = nstripes * EC_METHOD_CHUNK_SIZE * k;
    int rc;

    if (small_cpu(ctx, user, ECM_DECODE)) {
        const struct dec_call call = {k, rows, nfrags, npat, shift, nstripes, frags, out, outs,
                                      pats, gp};

        rc = cpu_decode(ctx, &call, 0, nstripes);
        if (rc == 0)
            stat_add(ECM_STAT_CPU);
        return rc;
    }
    big_call(user, 1);
    rc = host_decode_1(ctx, k, rows, nstripes, nfrags, frags, out, outs, npat, pats, gp, shift);
    big_call(user, -1);
    return rc;
}

static int
encode_any(ec_matrix_list_t *list, uint64_t nstripes, const void *in, void *const *out)
{
    ecm_ctx_t *ctx = CTX(list);
    uint32_t i;
    int dev;

    if (nstripes == 0)
        return 0;
    for (i = 0; i < ctx->n; i++)
        if (!out[i])
            return -EINVAL;
    dev = ecd_ptr_device(in);
    if (!bufs_on((const void *const *)out, ctx->n, dev))
        return -EINVAL; /* mixed host/device buffers are not supported */
    if (dev >= 0) {
        int rc = ec_method_encode_device(list, dev, NULL, nstripes, in, out);
        return rc ? rc : ecd_sync(dev, NULL);
    }
    return host_encode(ctx, nstripes, in, out);
}

void
ec_method_encode(ec_matrix_list_t *list, uint64_t size, void *in, void **out)
{
    ecm_ctx_t *ctx = CTX(list);
    uint64_t seq;
    uint32_t i;
    int rc;

    if (!ctx || size % list->stripe != 0) {
        ecm_log("ec_method_encode: size %llu is not a multiple of the stripe (%u)",
                (unsigned long long)size, list->stripe);
        abort();
    }
    /* host buffers cannot fail here (a device error is redone on the CPU
     * engine); what is left is a caller error or a fault of caller-provided
     * device memory, which no fallback can read */
    seq = ecd_error_seq();
    rc = encode_any(list, size / list->stripe, in, out);
    if (rc != 0) {
        ecm_ret("ec_method_encode", seq, rc);
        ecm_log("ec_method_encode failed (%d): %s", rc, ecd_last_error());
        abort(); /* the reference's encode cannot fail; never return bad data */
    }
    for (i = 0; i < ctx->n; i++)
        out[i] = (uint8_t *)out[i] + size / list->columns;
}

static int32_t
ecm_encode_batch_impl(ec_matrix_list_t *list, uint64_t nstripes, const void *in,
                     void *const *out)
{
    if (!list || !CTX(list) || (!in && nstripes) || (!out && nstripes))
        return -EINVAL;
    return encode_any(list, nstripes, in, out);
}

/* ------------------------------------------- encode of selected fragments */

/* The encode-matrix rows of the bricks in row_mask (ec_method_matrix_normal,
 * ec-method.c:22-36) as a k -> m combination of the stripe's data chunks;
 * outs[] = the selected out[] entries in brick order. */
static int
rows_pattern(const ecm_ctx_t *ctx, uintptr_t row_mask, void *const *out, uint8_t *pat,
             void **outs, uint32_t *m)
{
    uint32_t coef[ECM_MAX_N * ECM_MAX_K];
    uint8_t src[ECM_MAX_K];
    uint32_t i, p, t = 0;

    if (row_mask == 0 || (row_mask >> ctx->n) != 0)
        return -EINVAL;
    for (i = 0; i < ctx->n; i++) {
        if (!((row_mask >> i) & 1))
            continue;
        if (!out[i])
            return -EINVAL;
        for (p = 0; p < ctx->k; p++)
            coef[t * ctx->k + p] = ctx->enc[i * ctx->k + p];
        outs[t++] = out[i];
    }
    for (p = 0; p < ctx->k; p++)
        src[p] = (uint8_t)p;
    pack_pattern(pat, ctx->k, src, t, coef);
    *m = t;
    return 0;
}

/* Host buffers: the GPU pipeline's generic encode (the zero-copy combine with
 * the selected rows as its pattern) or the CPU engine's combination.  Routed
 * with the model and observations of a k -> m combination (a heal moves the
 * same bytes) and not recorded: its rate per user byte is neither an
 * encode's nor a full decode's, and exploration calls that never record
 * would recur forever. */
/* Stripes [s0, s1) of a row-masked encode on the CPU engine. */
static int
cpu_encode_rows(const ecm_ctx_t *ctx, uint64_t s0, uint64_t s1, const void *in, uint32_t m,
                void *const *outs, const uint8_t *pat)
{
    const uint64_t S = (uint64_t)ctx->k * EC_METHOD_CHUNK_SIZE;
    ecd_combine_desc_t d;
    uint32_t p;

    memset(&d, 0, offsetof(ecd_combine_desc_t, pat));
    d.k = ctx->k;
    d.rows = m;
    d.nstripes = s1 - s0;
    d.in_stride = S;
    d.out_stride = EC_METHOD_CHUNK_SIZE;
    for (p = 0; p < ctx->k; p++)
        d.in_base[p] = (const uint8_t *)in + s0 * S + (uint64_t)p * EC_METHOD_CHUNK_SIZE;
    for (p = 0; p < m; p++)
        d.out_base[p] = (uint8_t *)outs[p] + s0 * EC_METHOD_CHUNK_SIZE;
    d.npatterns = 1;
    d.pat_bytes = ctx->k + m * ctx->k;
    d.pat_ext = pat;
    return ecc_combine(ctx->isa, &d);
}

struct rows_share {
    const ecm_ctx_t *ctx;
    uint64_t nstripes;
    const void *in;
    uint32_t m;
    void *const *outs;
    const uint8_t *pat;
};

static int
rows_share_gpu(void *a)
{
    const struct rows_share *r = (const struct rows_share *)a;

    return ecd_encode_host_rows(0, r->ctx->k, r->m, r->nstripes, r->in, r->outs, r->pat);
}

static int
host_encode_rows_1(ecm_ctx_t *ctx, uint64_t nstripes, const void *in, uint32_t m,
                   void *const *outs, const uint8_t *pat)
{
    const uint64_t fl = nstripes * EC_METHOD_CHUNK_SIZE, user = fl * ctx->k;
    const uint64_t bytes = fl * (ctx->k + m);
    const struct enc_bufs eb = {in, outs, ctx->k, m, fl};
    uint64_t staged = ECM_STAGED_UNKNOWN, sg;
    int rc, share;

    /* a near tie: the GPU takes the first share, the CPU the rest */
    share = split_share(ctx, user, bytes, ECM_DECODE, ECM_CLS_PART, enc_staged, &eb, &staged);
    sg = share > 0 ? split_stripes(nstripes, share, 1) : 0;
    if (sg) {
        struct rows_share rs = {ctx, sg, in, m, outs, pat};
        ecm_task_t t = {rows_share_gpu, &rs, 0, 0, 0, 0, 0, "", NULL};

        if (helper_submit(&t) == 0) {
            uint64_t t0 = now_ns();

            rc = cpu_encode_rows(ctx, sg, nstripes, in, m, outs, pat);
            t0 = now_ns() - t0;
            if (rc == 0)
                stat_add(ECM_STAT_CPU);
            helper_wait(&t);
            if (t.rc == 0) {
                stat_add(ECM_STAT_GPU);
                if (rc == 0)
                    share_learn(ECM_CLS_PART, ECM_DECODE, ctx->k, ctx->isa, user, bytes, staged,
                                nstripes, sg, t.wall, t0);
                return rc;
            }
            if (t.err[0])
                ecd_set_error(t.err);
            if (!gpu_failed(t.rc))
                return t.rc;
            return rc ? rc : cpu_encode_rows(ctx, 0, sg, in, m, outs, pat);
        }
    }
    if (!route_cpu(ctx, user, bytes, ECM_DECODE, 0)) {
        if (staged == ECM_STAGED_UNKNOWN)
            staged = enc_staged(&eb);
        if (!route_cpu(ctx, user, bytes, ECM_DECODE, staged)) {
            rc = ecd_encode_host_rows(0, ctx->k, m, nstripes, in, outs, pat);
            if (!gpu_failed(rc)) {
                if (rc == 0)
                    stat_add(ECM_STAT_GPU);
                return rc;
            }
        }
    }
    rc = cpu_encode_rows(ctx, 0, nstripes, in, m, outs, pat);
    if (rc == 0)
        stat_add(ECM_STAT_CPU);
    return rc;
}

static int
host_encode_rows(ecm_ctx_t *ctx, uint64_t nstripes, const void *in, uint32_t m,
                 void *const *outs, const uint8_t *pat)
{
    const uint64_t user = nstripes * EC_METHOD_CHUNK_SIZE * ctx->k;
    int rc;

    big_call(user, 1);
    rc = host_encode_rows_1(ctx, nstripes, in, m, outs, pat);
    big_call(user, -1);
    return rc;
}

/* the k -> m combination of encode_rows on device buffers, queued on stream */
static int
device_encode_rows(ecm_ctx_t *ctx, int dev, void *stream, uint64_t nstripes, const void *in,
                   uint32_t m, void *const *outs, const uint8_t *pat)
{
    ecd_combine_desc_t d;
    uint32_t p;

    memset(&d, 0, offsetof(ecd_combine_desc_t, pat));
    d.k = ctx->k;
    d.rows = m;
    d.nstripes = nstripes;
    d.in_stride = (uint64_t)ctx->k * EC_METHOD_CHUNK_SIZE;
    d.out_stride = EC_METHOD_CHUNK_SIZE;
    for (p = 0; p < ctx->k; p++)
        d.in_base[p] = (const uint8_t *)in + (uint64_t)p * EC_METHOD_CHUNK_SIZE;
    for (p = 0; p < m; p++)
        d.out_base[p] = outs[p];
    d.npatterns = 1;
    d.pat_bytes = ctx->k + m * ctx->k;
    memcpy(d.pat, pat, d.pat_bytes);
    return ecd_combine(dev, stream, &d);
}

static int
encode_rows_any(ec_matrix_list_t *list, uint64_t nstripes, const void *in, uintptr_t row_mask,
                void *const *out)
{
    ecm_ctx_t *ctx = CTX(list);
    uint8_t pat[ECM_MAX_K + ECM_MAX_N * ECM_MAX_K];
    void *outs[ECM_MAX_N];
    uint32_t m = 0;
    int dev, rc;

    rc = rows_pattern(ctx, row_mask, out, pat, outs, &m);
    if (rc || nstripes == 0)
        return rc;
    dev = ecd_ptr_device(in);
    if (!bufs_on((const void *const *)outs, m, dev))
        return -EINVAL; /* mixed host/device buffers are not supported */
    if (dev < 0)
        return host_encode_rows(ctx, nstripes, in, m, outs, pat);
    rc = device_encode_rows(ctx, dev, NULL, nstripes, in, m, outs, pat);
    return rc ? rc : ecd_sync(dev, NULL);
}

static int32_t
ecm_encode_rows_device_impl(ec_matrix_list_t *list, int device, void *stream,
                           uint64_t nstripes, const void *in, uintptr_t row_mask,
                           void *const *out)
{
    uint8_t pat[ECM_MAX_K + ECM_MAX_N * ECM_MAX_K];
    void *outs[ECM_MAX_N];
    uint32_t m = 0;
    int rc;

    if (!list || !CTX(list) || !out || (!in && nstripes))
        return -EINVAL;
    if (row_mask == 0 || nstripes == 0)
        return (row_mask >> CTX(list)->n) ? -EINVAL : 0;
    rc = rows_pattern(CTX(list), row_mask, out, pat, outs, &m);
    if (rc)
        return rc;
    return device_encode_rows(CTX(list), device, stream, nstripes, in, m, outs, pat);
}

void
ec_method_encode_rows(ec_matrix_list_t *list, uint64_t size, void *in, uintptr_t row_mask,
                      void **out)
{
    ecm_ctx_t *ctx = CTX(list);
    uint64_t seq;
    uint32_t i;
    int rc;

    if (ctx && row_mask == ((uintptr_t)1 << ctx->n) - 1) {
        ec_method_encode(list, size, in, out);
        return;
    }
    if (!ctx || size % list->stripe != 0 || !out || (!in && size)) {
        ecm_log("ec_method_encode_rows: bad arguments (size %llu, stripe %u, in %p, out %p)",
                (unsigned long long)size, list->stripe, in, (void *)out);
        abort();
    }
    if (row_mask == 0)
        return; /* no fragment wanted */
    seq = ecd_error_seq();
    rc = encode_rows_any(list, size / list->stripe, in, row_mask, out);
    if (rc != 0) {
        ecm_ret("ec_method_encode_rows", seq, rc);
        ecm_log("ec_method_encode_rows(mask 0x%llx) failed (%d): %s",
                (unsigned long long)row_mask, rc, ecd_last_error());
        abort(); /* as ec_method_encode: never return bad data */
    }
    for (i = 0; i < ctx->n; i++)
        if ((row_mask >> i) & 1)
            out[i] = (uint8_t *)out[i] + size / list->columns;
}

static int
decode_any(ec_matrix_list_t *list, uint64_t nstripes, uintptr_t mask, const uint32_t *rows,
           const void *const *in, void *out)
{
    uint8_t pat[ECM_MAX_K + ECM_MAX_K * ECM_MAX_K];
    uint8_t src[ECM_MAX_K];
    ecm_matrix_t *m;
    ecm_ctx_t *ctx;
    uint32_t k = list->columns, p;
    int dev, rc;

    if (!mask_rows_ok(list, mask, rows))
        return -EINVAL;
    if (nstripes == 0)
        return 0;
    for (p = 0; p < k; p++)
        if (!in[p])
            return -EINVAL;
    dev = ecd_ptr_device(out);
    if (!bufs_on(in, k, dev))
        return -EINVAL;
    if (dev >= 0) {
        rc = ec_method_decode_device(list, dev, NULL, nstripes, mask, in, out);
        return rc ? rc : ecd_sync(dev, NULL);
    }
    ctx = CTX(list);
    for (p = 0; p < ECM_MEMO; p++)
        if (ecm_memo[p].serial == ctx->serial && ecm_memo[p].mask == mask)
            return host_decode(ctx, k, k, nstripes, k, in, out, NULL, 1, ecm_memo[p].pat, NULL,
                               0);
    m = matrix_get(list, mask, rows);
    if (!m)
        return -ENOMEM;
    for (p = 0; p < k; p++)
        src[p] = (uint8_t)p;
    pack_pattern(pat, k, src, k, m->inv);
    matrix_put(list, m);
    p = ecm_memo_next++ % ECM_MEMO;
    ecm_memo[p].serial = ctx->serial;
    ecm_memo[p].mask = mask;
    memcpy(ecm_memo[p].pat, pat, k + k * k);
    return host_decode(ctx, k, k, nstripes, k, in, out, NULL, 1, pat, NULL, 0);
}

static int32_t
ecm_decode_impl(ec_matrix_list_t *list, uint64_t size, uintptr_t mask, uint32_t *rows,
               void **in, void *out)
{
    if (!list || !CTX(list) || size % EC_METHOD_CHUNK_SIZE != 0 || !rows || !in ||
        (!out && size))
        return -EINVAL;
    return decode_any(list, size / EC_METHOD_CHUNK_SIZE, mask, rows,
                      (const void *const *)in, out);
}

static int32_t
ecm_decode_batch_impl(ec_matrix_list_t *list, uint64_t nstripes, uintptr_t mask,
                     const uint32_t *rows, const void *const *in, void *out)
{
    if (!list || !CTX(list) || !rows || !in || (!out && nstripes))
        return -EINVAL;
    return decode_any(list, nstripes, mask, rows, in, out);
}

/* Build the packed pattern for `mask` reading from the n-fragment array. */
static int
mask_pattern(ec_matrix_list_t *list, uintptr_t mask, uint8_t *pat)
{
    uint32_t rows[ECM_MAX_K];
    uint8_t src[ECM_MAX_K];
    ecm_matrix_t *m;
    uint32_t p, k = list->columns;

    rows_from_mask(mask, rows);
    if (!mask_rows_ok(list, mask, rows))
        return -EINVAL;
    m = matrix_get(list, mask, rows);
    if (!m)
        return -ENOMEM;
    for (p = 0; p < k; p++)
        src[p] = (uint8_t)(rows[p] - 1);
    pack_pattern(pat, k, src, k, m->inv);
    matrix_put(list, m);
    return 0;
}

/* Every brick a mask reads must have a fragment buffer (frags[] may hold
 * NULL for bricks no mask reads): a NULL here would be dereferenced by the
 * kernel and fault the device instead of failing the call. */
static int
mask_frags_ok(const ec_matrix_list_t *list, uintptr_t mask, const void *const *frags)
{
    uint32_t b;

    for (b = 0; b < list->rows; b++)
        if (((mask >> b) & 1) && !frags[b])
            return 0;
    return 1;
}

/* Per-thread memo of the packed pattern sets of the last mixed calls (r05).
 * A self-heal sweep passes the same mask set call after call, and a set
 * larger than the decode-matrix cache (2 x nodes entries, as ec.c sizes it)
 * cycles through its LRU, so every call re-inverted every mask: 64 masks of
 * 16+4 cost ~170 us of host time per call (tools/patcache_threads.py: a
 * 4 MiB device heal window took ~190 us, ~23 us with one mask).  Keyed by
 * the volume's serial and the exact mask list; the returned patterns are
 * valid until this thread's next call of pattern_set. */
#define ECM_SETMEMO 2
typedef struct {
    uint64_t serial, hash;
    uint32_t nmasks;
    uintptr_t *masks;
    uint8_t *pats;
    size_t cap_masks, cap_pats; /* entries of masks[], bytes of pats[] */
} ecm_setmemo_t;

typedef struct {
    ecm_setmemo_t e[ECM_SETMEMO];
    unsigned next;
} ecm_setmemos_t;

static pthread_key_t ecm_setmemo_key;
static pthread_once_t ecm_setmemo_once = PTHREAD_ONCE_INIT;
static int ecm_setmemo_ok;

static void
setmemo_free(void *v)
{
    ecm_setmemos_t *s = (ecm_setmemos_t *)v;
    unsigned i;

    for (i = 0; i < ECM_SETMEMO; i++) {
        free(s->e[i].masks);
        free(s->e[i].pats);
    }
    free(s);
}

static void
setmemo_init(void)
{
    ecm_setmemo_ok = pthread_key_create(&ecm_setmemo_key, setmemo_free) == 0;
}

/* The packed patterns (k + k*k bytes each, in `masks` order) of a mask set;
 * NULL with *rc set on a bad mask or no memory. */
static const uint8_t *
pattern_set(ec_matrix_list_t *list, const uintptr_t *masks, uint32_t nmasks, int *rc)
{
    ecm_ctx_t *ctx = (ecm_ctx_t *)list->code;
    const size_t pb = (size_t)list->columns * (1 + list->columns);
    ecm_setmemos_t *s;
    ecm_setmemo_t *e;
    uint64_t h = 1469598103934665603ull; /* FNV-1a */
    uint32_t u;
    unsigned i;

    for (u = 0; u < nmasks; u++)
        h = (h ^ (uint64_t)masks[u]) * 1099511628211ull;
    pthread_once(&ecm_setmemo_once, setmemo_init);
    s = ecm_setmemo_ok ? (ecm_setmemos_t *)pthread_getspecific(ecm_setmemo_key) : NULL;
    if (!s && ecm_setmemo_ok) {
        s = (ecm_setmemos_t *)calloc(1, sizeof(*s));
        if (s && pthread_setspecific(ecm_setmemo_key, s) != 0) {
            free(s);
            s = NULL;
        }
    }
    if (!s) {
        *rc = -ENOMEM;
        return NULL;
    }
    for (i = 0; i < ECM_SETMEMO; i++) {
        e = &s->e[i];
        if (e->serial == ctx->serial && e->nmasks == nmasks && e->hash == h &&
            memcmp(e->masks, masks, nmasks * sizeof(*masks)) == 0)
            return e->pats;
    }
    e = &s->e[s->next++ % ECM_SETMEMO];
    e->serial = 0;
    if (e->cap_masks < nmasks) {   /* (volumes of any k share the entries) */
        uintptr_t *m = (uintptr_t *)realloc(e->masks, nmasks * sizeof(*masks));

        if (!m) {
            *rc = -ENOMEM;
            return NULL;
        }
        e->masks = m;
        e->cap_masks = nmasks;
    }
    if (e->cap_pats < nmasks * pb) {
        uint8_t *p = (uint8_t *)realloc(e->pats, nmasks * pb);

        if (!p) {
            *rc = -ENOMEM;
            return NULL;
        }
        e->pats = p;
        e->cap_pats = nmasks * pb;
    }
    for (u = 0; u < nmasks; u++)
        if ((*rc = mask_pattern(list, masks[u], e->pats + u * pb)) != 0)
            return NULL;
    memcpy(e->masks, masks, nmasks * sizeof(*masks));
    e->nmasks = nmasks;
    e->hash = h;
    e->serial = ctx->serial;
    return e->pats;
}

static int32_t
ecm_decode_mixed_impl(ec_matrix_list_t *list, uint64_t nstripes, uint64_t group_stripes,
                     const uintptr_t *group_masks, const void *const *frags, void *out)
{
    const uint8_t *pats;
    uintptr_t uniq[ECD_MAX_PATTERNS];
    uint8_t *gp;
    uint64_t g, ngroups;
    uint32_t shift = 0, nu = 0, u, k;
    int rc;

    if (!list || !CTX(list) || !group_masks || !frags || (!out && nstripes))
        return -EINVAL;
    if (group_stripes == 0 || (group_stripes & (group_stripes - 1)))
        return -EINVAL;
    while ((1ull << shift) < group_stripes)
        shift++;
    if (nstripes == 0)
        return 0;
    k = list->columns;
    ngroups = (nstripes + group_stripes - 1) / group_stripes;
    gp = (uint8_t *)malloc(ngroups);
    if (!gp)
        return -ENOMEM;
    rc = 0;
    for (g = 0; g < ngroups && rc == 0; g++) {
        for (u = 0; u < nu; u++)
            if (uniq[u] == group_masks[g])
                break;
        if (u == nu) {
            if (nu == ECD_MAX_PATTERNS) {
                rc = -E2BIG;
                break;
            }
            if (!mask_frags_ok(list, group_masks[g], frags)) {
                rc = -EINVAL;
                break;
            }
            uniq[nu++] = group_masks[g];
        }
        gp[g] = (uint8_t)u;
    }
    pats = NULL;
    if (rc == 0)
        pats = pattern_set(list, uniq, nu, &rc);
    if (rc == 0 && (!bufs_on(frags, list->rows, -1) || ecd_ptr_device(out) >= 0))
        rc = -EINVAL; /* host entry point: device buffers go to _device */
    if (rc == 0)
        rc = host_decode(CTX(list), k, k, nstripes, list->rows, frags, out, NULL, nu, pats, gp,
                         shift);
    free(gp);
    return rc;
}

/* Heal matrix: rows of the encode matrix for the target bricks times the
 * inverse for `mask` -> m x k coefficients applied to the k fragments. */
static int
heal_pattern(ec_matrix_list_t *list, uintptr_t mask, const uint32_t *rows,
             uintptr_t target_mask, uint8_t *pat, uint32_t *ntargets)
{
    ecm_ctx_t *ctx = CTX(list);
    uint32_t coef[ECM_MAX_N * ECM_MAX_K];
    uint8_t src[ECM_MAX_K];
    ecm_matrix_t *m;
    uint32_t k = list->columns, t = 0, i, j, p, acc;

    if ((target_mask >> list->rows) != 0 || target_mask == 0)
        return -EINVAL;
    m = matrix_get(list, mask, rows);
    if (!m)
        return -ENOMEM;
    for (i = 0; i < list->rows; i++) {
        if (!((target_mask >> i) & 1))
            continue;
        for (p = 0; p < k; p++) {
            acc = 0;
            for (j = 0; j < k; j++)
                acc ^= ec_method_gf_mul(ctx->enc[i * k + j], m->inv[j * k + p]);
            coef[t * k + p] = acc;
        }
        t++;
    }
    matrix_put(list, m);
    for (p = 0; p < k; p++)
        src[p] = (uint8_t)p;
    pack_pattern(pat, k, src, t, coef);
    *ntargets = t;
    return 0;
}

static int32_t
ecm_heal_impl(ec_matrix_list_t *list, uint64_t nstripes, uintptr_t mask,
             const void *const *in, uintptr_t target_mask, void *const *out)
{
    uint8_t pat[ECM_MAX_K + ECM_MAX_N * ECM_MAX_K];
    uint32_t rows[ECM_MAX_K], nt = 0, p;
    int dev, rc;

    if (!list || !CTX(list) || !in || !out)
        return -EINVAL;
    rows_from_mask(mask, rows);
    if (!mask_rows_ok(list, mask, rows))
        return -EINVAL;
    if (nstripes == 0)
        return 0;
    if ((target_mask >> list->rows) != 0 || target_mask == 0)
        return -EINVAL;
    for (p = 0; p < list->columns; p++)
        if (!in[p])
            return -EINVAL;
    dev = ecd_ptr_device(in[0]);
    if (!bufs_on(in, list->columns, dev) ||
        !bufs_on((const void *const *)out, popcount_mask(target_mask), dev))
        return -EINVAL;
    if (dev >= 0) {
        rc = ec_method_heal_device(list, dev, NULL, nstripes, mask, in, target_mask, out);
        return rc ? rc : ecd_sync(dev, NULL);
    }
    rc = heal_pattern(list, mask, rows, target_mask, pat, &nt);
    if (rc)
        return rc;
    return host_decode(CTX(list), list->columns, nt, nstripes, list->columns, in, NULL, out, 1,
                       pat, NULL, 0);
}

/* ------------------------------------------------- partial-stripe writes */

static int32_t
ecm_writev_encode_impl(ec_matrix_list_t *list, uint64_t head, const struct iovec *iov,
                      int count, const void *old_head, const void *old_tail,
                      void *const *out)
{
    ecm_ctx_t *ctx;
    const void *segp[3 + 64];
    uint64_t segl[3 + 64], user = 0, S, b2, nst;
    const uint8_t *hs = (const uint8_t *)old_head, *ts = (const uint8_t *)old_tail;
    uint32_t ns = 0, i;
    int c, dev;

    if (!list || !(ctx = CTX(list)) || !out || count < 0 || count > 64 || (count && !iov))
        return -EINVAL;
    S = list->stripe;
    if (head >= S)
        return -EINVAL;
    for (c = 0; c < count; c++)
        user += iov[c].iov_len;
    if (user == 0)
        return 0;
    b2 = head + user;
    nst = (b2 + S - 1) / S;
    /* device buffers: the fused kernel (one contiguous user buffer) */
    dev = ecd_ptr_device(iov[0].iov_base);
    {
        const void *olds[2] = {old_head, old_tail};
        for (c = 1; c < count; c++)
            if (ecd_ptr_device(iov[c].iov_base) != dev)
                return -EINVAL;
        if (!bufs_on(olds, 2, dev) || !bufs_on((const void *const *)out, ctx->n, dev))
            return -EINVAL;
        for (i = 0; i < ctx->n; i++)
            if (!out[i])
                return -EINVAL;
    }
    if (dev >= 0) {
        if (count != 1)
            return -EINVAL;
        c = ec_method_writev_encode_device(list, dev, NULL, head, user, iov[0].iov_base,
                                           old_head, old_tail, out);
        return c ? c : ecd_sync(dev, NULL);
    }
    if (nst == 1) { /* one stripe: its old content fills both ends */
        hs = hs ? hs : ts;
        ts = hs ? hs + b2 : NULL;
    } else if (ts) {
        ts += b2 - (nst - 1) * S;
    }
    segp[ns] = hs;
    segl[ns++] = head;
    for (c = 0; c < count; c++) {
        segp[ns] = iov[c].iov_base;
        segl[ns++] = iov[c].iov_len;
    }
    segp[ns] = ts;
    segl[ns++] = nst * S - b2;
    /* the padded input is always gathered into the staging slots; the
     * fragments are staged unless they are mapped (the estimate with mapped
     * fragments first: it is the optimistic one, so a call the CPU wins
     * anyway makes no pointer query) */
    if (!route_cpu(ctx, nst * EC_METHOD_CHUNK_SIZE * ctx->k,
                   nst * EC_METHOD_CHUNK_SIZE * (ctx->k + ctx->n), ECM_ENCODE,
                   nst * EC_METHOD_CHUNK_SIZE * ctx->k) &&
        !route_cpu(ctx, nst * EC_METHOD_CHUNK_SIZE * ctx->k,
                   nst * EC_METHOD_CHUNK_SIZE * (ctx->k + ctx->n), ECM_ENCODE,
                   nst * EC_METHOD_CHUNK_SIZE * ctx->k +
                       staged_bytes((const void *const *)out, ctx->n,
                                    nst * EC_METHOD_CHUNK_SIZE))) {
        c = ecd_encode_host_gather(0, ctx->k, ctx->n, nst, ns, segp, segl, out, ctx->enc_pat);
        if (!gpu_failed(c)) {
            if (c == 0)
                stat_add(ECM_STAT_GPU);
            return c;
        }
    }
    c = ecc_encode_gather(ctx->isa, ctx->k, ctx->n, nst, ns, segp, segl, (uint8_t *const *)out);
    if (c == 0)
        stat_add(ECM_STAT_CPU);
    return c;
}

static int32_t
ecm_writev_encode_device_impl(ec_matrix_list_t *list, int device, void *stream, uint64_t head,
                             uint64_t size, const void *user, const void *old_head,
                             const void *old_tail, void *const *out)
{
    ecm_ctx_t *ctx;

    if (!list || !(ctx = CTX(list)) || !out)
        return -EINVAL;
    if (size == 0)
        return 0;
    return ecd_writev_encode_device(device, stream, ctx->k, ctx->n, head, size, user, old_head,
                                    old_tail, out, ctx->enc_pat);
}

/* ---------------------------------------------------- device-resident */

static void
desc_init(ecd_combine_desc_t *d, uint32_t k, uint32_t rows, uint64_t nstripes)
{
    memset(d, 0, offsetof(ecd_combine_desc_t, pat));
    d->k = k;
    d->rows = rows;
    d->nstripes = nstripes;
    d->npatterns = 1;
    d->pat_bytes = k + rows * k;
}

static int32_t
ecm_encode_device_impl(ec_matrix_list_t *list, int device, void *stream, uint64_t nstripes,
                      const void *in, void *const *out)
{
    ecm_ctx_t *ctx;
    ecd_combine_desc_t d;
    uint32_t p;

    if (!list || !(ctx = CTX(list)) || !in || !out)
        return -EINVAL;
    if (nstripes == 0)
        return 0;
    if (ecd_has_vander(ctx->k, ctx->n))
        return ecd_encode_vander(device, stream, ctx->k, ctx->n, nstripes, in, out);
    desc_init(&d, ctx->k, ctx->n, nstripes);
    d.in_stride = (uint64_t)ctx->k * EC_METHOD_CHUNK_SIZE;
    d.out_stride = EC_METHOD_CHUNK_SIZE;
    for (p = 0; p < ctx->k; p++)
        d.in_base[p] = (const uint8_t *)in + (uint64_t)p * EC_METHOD_CHUNK_SIZE;
    for (p = 0; p < ctx->n; p++)
        d.out_base[p] = out[p];
    memcpy(d.pat, ctx->enc_pat, d.pat_bytes);
    return ecd_combine(device, stream, &d);
}

static int32_t
ecm_decode_device_impl(ec_matrix_list_t *list, int device, void *stream, uint64_t nstripes,
                      uintptr_t mask, const void *const *in, void *out)
{
    uint32_t rows[ECM_MAX_K], k, p, r;
    uint8_t src[ECM_MAX_K];
    ecd_combine_desc_t d;
    ecm_matrix_t *m;

    if (!list || !CTX(list) || !in || !out)
        return -EINVAL;
    k = list->columns;
    rows_from_mask(mask, rows);
    if (!mask_rows_ok(list, mask, rows))
        return -EINVAL;
    if (nstripes == 0)
        return 0;
    m = matrix_get(list, mask, rows);
    if (!m)
        return -ENOMEM;
    desc_init(&d, k, k, nstripes);
    d.in_stride = EC_METHOD_CHUNK_SIZE;
    d.out_stride = (uint64_t)k * EC_METHOD_CHUNK_SIZE;
    for (p = 0; p < k; p++) {
        d.in_base[p] = in[p];
        src[p] = (uint8_t)p;
    }
    for (r = 0; r < k; r++)
        d.out_base[r] = (uint8_t *)out + (uint64_t)r * EC_METHOD_CHUNK_SIZE;
    pack_pattern(d.pat, k, src, k, m->inv);
    matrix_put(list, m);
    return ecd_combine(device, stream, &d);
}

static int32_t
ecm_decode_mixed_device_impl(ec_matrix_list_t *list, int device, void *stream,
                            uint64_t nstripes, uint64_t group_stripes,
                            const uint8_t *group_pattern, uint32_t nmasks,
                            const uintptr_t *masks, const void *const *frags, void *out)
{
    ecd_combine_desc_t d;
    uint32_t k, r, u, shift = 0;
    const uint8_t *pats;
    int rc;

    if (!list || !CTX(list) || !group_pattern || !masks || !frags || !out || nmasks == 0)
        return -EINVAL;
    if (group_stripes == 0 || (group_stripes & (group_stripes - 1)))
        return -EINVAL;
    while ((1ull << shift) < group_stripes)
        shift++;
    k = list->columns;
    if (nmasks > ECD_MAX_PATTERNS)
        return -E2BIG;
    if (nstripes == 0)
        return 0;
    desc_init(&d, k, k, nstripes);
    d.npatterns = nmasks;
    d.in_stride = EC_METHOD_CHUNK_SIZE;
    d.out_stride = (uint64_t)k * EC_METHOD_CHUNK_SIZE;
    for (u = 0; u < list->rows; u++)
        d.in_base[u] = frags[u];
    for (r = 0; r < k; r++)
        d.out_base[r] = (uint8_t *)out + (uint64_t)r * EC_METHOD_CHUNK_SIZE;
    rc = 0;
    for (u = 0; u < nmasks && rc == 0; u++)
        if (!mask_frags_ok(list, masks[u], frags))
            rc = -EINVAL;
    pats = rc == 0 ? pattern_set(list, masks, nmasks, &rc) : NULL;
    if (rc)
        return rc;
    /* more masks than the kernel-argument space holds: the launcher moves
     * them to a device table (ec_kernels.hip upload_table), reading them
     * during the call */
    if ((uint64_t)nmasks * d.pat_bytes > ECD_MAX_PAT_BYTES)
        d.pat_ext = pats;
    else
        memcpy(d.pat, pats, (size_t)nmasks * d.pat_bytes);
    d.group_pattern = group_pattern;
    d.group_shift = shift;
    return ecd_combine(device, stream, &d);
}

static int32_t
ecm_heal_device_impl(ec_matrix_list_t *list, int device, void *stream, uint64_t nstripes,
                    uintptr_t mask, const void *const *in, uintptr_t target_mask,
                    void *const *out)
{
    uint32_t rows[ECM_MAX_K], nt = 0, p;
    ecd_combine_desc_t d;
    int rc;

    if (!list || !CTX(list) || !in || !out)
        return -EINVAL;
    rows_from_mask(mask, rows);
    if (!mask_rows_ok(list, mask, rows))
        return -EINVAL;
    if (nstripes == 0)
        return 0;
    memset(&d, 0, offsetof(ecd_combine_desc_t, pat));
    rc = heal_pattern(list, mask, rows, target_mask, d.pat, &nt);
    if (rc)
        return rc;
    d.k = list->columns;
    d.rows = nt;
    d.nstripes = nstripes;
    d.npatterns = 1;
    d.pat_bytes = d.k + nt * d.k;
    d.in_stride = EC_METHOD_CHUNK_SIZE;
    d.out_stride = EC_METHOD_CHUNK_SIZE;
    for (p = 0; p < d.k; p++)
        d.in_base[p] = in[p];
    for (p = 0; p < nt; p++)
        d.out_base[p] = out[p];
    return ecd_combine(device, stream, &d);
}

static int32_t
ecm_sync_device_impl(int device, void *stream)
{
    return ecd_sync(device, stream);
}

/* ------------------------------------------- per-thread error reporting */

/* Every entry point that fails leaves the calling thread a reason in
 * ec_method_last_error(): the device layer records what failed (the HIP call
 * or kernel and its error); a failure it did not record -- an argument
 * error, a geometry the call does not take -- is recorded here as the entry
 * point and its errno, so a client's log line (ec.c / ec-heal.c callers,
 * many epoll threads) never shows another call's text. */
static int32_t
ecm_ret(const char *fn, uint64_t seq, int32_t rc)
{
    char buf[192];

    if (rc < 0 && ecd_error_seq() == seq) {
        snprintf(buf, sizeof buf, "%s: %s (%d)", fn, strerror(-rc), (int)rc);
        ecd_set_error(buf);
    }
    return rc;
}

int32_t
ec_method_init(xlator_t *xl, ec_matrix_list_t *list, uint32_t columns, uint32_t rows,
               uint32_t max, const char *gen)
{
    const uint64_t seq = ecd_error_seq();
    return ecm_ret("ec_method_init", seq,
                   ecm_init_impl(xl, list, columns, rows, max, gen));
}

int32_t
ec_method_update(xlator_t *xl, ec_matrix_list_t *list, const char *gen)
{
    const uint64_t seq = ecd_error_seq();
    return ecm_ret("ec_method_update", seq,
                   ecm_update_impl(xl, list, gen));
}

int32_t
ec_method_encode_batch(ec_matrix_list_t *list, uint64_t nstripes, const void *in,
                       void *const *out)
{
    const uint64_t seq = ecd_error_seq();
    return ecm_ret("ec_method_encode_batch", seq,
                   ecm_encode_batch_impl(list, nstripes, in, out));
}

int32_t
ec_method_encode_rows_device(ec_matrix_list_t *list, int device, void *stream, uint64_t nstripes,
                             const void *in, uintptr_t row_mask, void *const *out)
{
    const uint64_t seq = ecd_error_seq();
    return ecm_ret("ec_method_encode_rows_device", seq,
                   ecm_encode_rows_device_impl(list, device, stream, nstripes, in, row_mask,
                                               out));
}

int32_t
ec_method_decode(ec_matrix_list_t *list, uint64_t size, uintptr_t mask, uint32_t *rows,
                 void **in, void *out)
{
    const uint64_t seq = ecd_error_seq();
    return ecm_ret("ec_method_decode", seq,
                   ecm_decode_impl(list, size, mask, rows, in, out));
}

int32_t
ec_method_decode_batch(ec_matrix_list_t *list, uint64_t nstripes, uintptr_t mask,
                       const uint32_t *rows, const void *const *in, void *out)
{
    const uint64_t seq = ecd_error_seq();
    return ecm_ret("ec_method_decode_batch", seq,
                   ecm_decode_batch_impl(list, nstripes, mask, rows, in, out));
}

int32_t
ec_method_decode_mixed(ec_matrix_list_t *list, uint64_t nstripes, uint64_t group_stripes,
                       const uintptr_t *group_masks, const void *const *frags, void *out)
{
    const uint64_t seq = ecd_error_seq();
    return ecm_ret("ec_method_decode_mixed", seq,
                   ecm_decode_mixed_impl(list, nstripes, group_stripes, group_masks, frags, out));
}

int32_t
ec_method_heal(ec_matrix_list_t *list, uint64_t nstripes, uintptr_t mask, const void *const *in,
               uintptr_t target_mask, void *const *out)
{
    const uint64_t seq = ecd_error_seq();
    return ecm_ret("ec_method_heal", seq,
                   ecm_heal_impl(list, nstripes, mask, in, target_mask, out));
}

int32_t
ec_method_writev_encode(ec_matrix_list_t *list, uint64_t head, const struct iovec *iov,
                        int count, const void *old_head, const void *old_tail, void *const *out)
{
    const uint64_t seq = ecd_error_seq();
    return ecm_ret("ec_method_writev_encode", seq,
                   ecm_writev_encode_impl(list, head, iov, count, old_head, old_tail, out));
}

int32_t
ec_method_writev_encode_device(ec_matrix_list_t *list, int device, void *stream, uint64_t head,
                               uint64_t size, const void *user, const void *old_head,
                               const void *old_tail, void *const *out)
{
    const uint64_t seq = ecd_error_seq();
    return ecm_ret("ec_method_writev_encode_device", seq,
                   ecm_writev_encode_device_impl(list, device, stream, head, size, user, old_head,
                                                 old_tail, out));
}

int32_t
ec_method_encode_device(ec_matrix_list_t *list, int device, void *stream, uint64_t nstripes,
                        const void *in, void *const *out)
{
    const uint64_t seq = ecd_error_seq();
    return ecm_ret("ec_method_encode_device", seq,
                   ecm_encode_device_impl(list, device, stream, nstripes, in, out));
}

int32_t
ec_method_decode_device(ec_matrix_list_t *list, int device, void *stream, uint64_t nstripes,
                        uintptr_t mask, const void *const *in, void *out)
{
    const uint64_t seq = ecd_error_seq();
    return ecm_ret("ec_method_decode_device", seq,
                   ecm_decode_device_impl(list, device, stream, nstripes, mask, in, out));
}

int32_t
ec_method_decode_mixed_device(ec_matrix_list_t *list, int device, void *stream,
                              uint64_t nstripes, uint64_t group_stripes,
                              const uint8_t *group_pattern, uint32_t nmasks,
                              const uintptr_t *masks, const void *const *frags, void *out)
{
    const uint64_t seq = ecd_error_seq();
    return ecm_ret("ec_method_decode_mixed_device", seq,
                   ecm_decode_mixed_device_impl(list, device, stream, nstripes, group_stripes,
                                                group_pattern, nmasks, masks, frags, out));
}

int32_t
ec_method_heal_device(ec_matrix_list_t *list, int device, void *stream, uint64_t nstripes,
                      uintptr_t mask, const void *const *in, uintptr_t target_mask,
                      void *const *out)
{
    const uint64_t seq = ecd_error_seq();
    return ecm_ret("ec_method_heal_device", seq,
                   ecm_heal_device_impl(list, device, stream, nstripes, mask, in, target_mask,
                                        out));
}

int32_t
ec_method_sync_device(int device, void *stream)
{
    const uint64_t seq = ecd_error_seq();
    return ecm_ret("ec_method_sync_device", seq,
                   ecm_sync_device_impl(device, stream));
}

int32_t
ec_method_host_register(void *p, size_t bytes)
{
    const uint64_t seq = ecd_error_seq();
    return ecm_ret("ec_method_host_register", seq,
                   ecm_host_register_impl(p, bytes));
}

int32_t
ec_method_host_unregister(void *p)
{
    const uint64_t seq = ecd_error_seq();
    return ecm_ret("ec_method_host_unregister", seq,
                   ecm_host_unregister_impl(p));
}

int32_t
ec_method_host_register_async(void *p, size_t bytes)
{
    const uint64_t seq = ecd_error_seq();
    return ecm_ret("ec_method_host_register_async", seq,
                   ecm_host_register_async_impl(p, bytes));
}
