/*
 * ec_jit.hip -- per-pattern whole-matrix kernels, compiled at run time (r06).
 *
 * The reference JITs one x86 routine per matrix row when a decode matrix
 * enters its cache (ec-code.c:722-809, ec_code_build_interleaved from
 * ec_method_matrix_get, ec-method.c:201-246).  This is the gfx950
 * counterpart, for the k >= 12 combines whose compute is what keeps them
 * off the HBM roofline:
 *
 *   The shipped k = 16 combine evaluates every output row as 16 multiply-
 *   accumulates, each a searched straight-line program over one input's 8
 *   bit-planes (ec_gf8_asm.h, 12.85 v_bitop3 / v_xor per multiply), entered
 *   by a wave-uniform jump per coefficient: ~3,300 instructions per dword
 *   column of a dense 16 x 16 matrix, with a scalar dispatch per multiply.
 *   Knowing the matrix at compile time, the whole 128 x 128 GF(2) matrix
 *   (output plane (r, b) x input plane (p, j): bit b of c_rp * x^j) becomes
 *   one straight-line program that shares sub-sums across all outputs
 *   (four Russians over 4-plane groups: each group's 15 nonzero XOR
 *   combinations built once, 11 instructions; each output plane then takes
 *   one entry per group, both groups of an input in one v_bitop3).  kb3's
 *   dense 16 x 16 matrix: 2,381 instructions per column for all 16 rows,
 *   2,725 as two 8-row programs (tools/gen/gen_wm16.py).
 *
 * Kernel: one 4-stripe tile per block, staged by LDS-DMA exactly as the
 * shipped tile kernels stage it (input p, plane b, stripe s at
 * ((p * 8 + b) * 4 + s) * 64); two waves, each running the program of half
 * of the rows on its lane's dword column; the rows go back through the
 * tile's LDS and leave as 16-byte lane stores: one contiguous run per tile
 * for a full decode's stripe-major output, 512-byte runs per stripe and row
 * otherwise.  One process, 1 GiB 16+4 decode of kb3's dense matrix
 * (profiles/r06/r06c_kb3_wm.log, medians of 7 rounds): shipped 0.3733 ms,
 * this structure 0.3500 ms (0.767 of 8 TB/s); compute alone 0.1256 ms
 * against 0.1912.
 *
 * Life of a pattern: a device combine with one pattern, k >= 12 and enough
 * stripes (EC_MI355X_JIT_MIN_STRIPES, default 1024) looks its coefficient
 * matrix up here.  The first sight queues a compile (~1-2 s: the compiler
 * process ec_jitc runs hiprtc, waited for by one library thread) and the call
 * runs the shipped kernel; once the code object exists, calls of that matrix
 * load it on their device (once) and launch it.  32 matrices are kept, least
 * recently used first out.  Without ec_jitc or hiprtc (or with
 * EC_MI355X_JIT=0) nothing changes.  EC_MI355X_JIT_SYNC=1 compiles on the
 * calling thread (tests, benchmarks).
 */
#include <hip/hip_runtime.h>

#include <dlfcn.h>
#include <fcntl.h>
#include <spawn.h>
#include <sys/wait.h>
#include <unistd.h>
#include <pthread.h>
#include <errno.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "ec_device.h"
#include "ec_jit.h"

extern char **environ;

namespace {

using u32 = uint32_t;
constexpr int kMaxDev = 16;
constexpr size_t kEntries = 32;
/* entries ever created per process: an evicted entry's modules stay loaded
 * (a queued launch may still run them), so this bounds that memory: 256
 * code objects of ~50-100 KB per device */
constexpr uint64_t kMaxCreated = 256;

/* ------------------------------------------------------------ generator */

u32 gf_mul(u32 a, u32 b)
{
    u32 r = 0;
    while (b) {
        if (b & 1)
            r ^= a;
        a <<= 1;
        if (a & 0x100)
            a ^= 0x11D;   /* EC_GF_MOD, ec-method.h:18 */
        b >>= 1;
    }
    return r;
}

/* bits j of input p's planes that feed output plane b of a row whose
 * coefficient for input p is c (the 8 x 8 GF(2) matrix of c, row b) */
u32 plane_mask(u32 c, int b)
{
    u32 m = 0;
    for (int j = 0; j < 8; ++j)
        m |= ((gf_mul(c, 1u << j) >> b) & 1u) << j;
    return m;
}

struct Gen {
    std::string s;
    u32 ops = 0;

    void line(const char *fmt, ...) __attribute__((format(printf, 2, 3)))
    {
        char buf[256];
        va_list ap, aq;
        va_start(ap, fmt);
        va_copy(aq, ap);
        const int n = vsnprintf(buf, sizeof buf, fmt, ap);
        va_end(ap);
        if (n >= (int)sizeof buf) {               /* a long declaration line */
            std::string big((size_t)n + 1, '\0');
            vsnprintf(&big[0], big.size(), fmt, aq);
            big.resize((size_t)n);
            s += big;
        } else if (n > 0) {
            s += buf;
        }
        va_end(aq);
        s += '\n';
    }
};

/* The program of output rows [r0, r1) over k inputs, as function prog<w>. */
void emit_program(Gen &g, int w, u32 k, u32 T, const uint8_t *coef, u32 r0, u32 r1)
{
    const u32 ps = T * 64u;             /* plane stride of the tile */
    const u32 no = (r1 - r0) * 8;
    g.line("__device__ __forceinline__ void prog%d(u32 col, u32 *acc)", w);
    g.line("{");
    /* an opaque copy of the lane's LDS offset per program: both programs read
     * the same LDS words, and without it the compiler hoists the common loads
     * and tables above the wave's branch (201 VGPRs instead of 128).  An
     * integer offset read through an LDS pointer (LDW) keeps them ds_read_b32:
     * laundering a generic pointer turned them into flat loads, each input's
     * waited for with vmcnt(0) lgkmcnt(0) */
    g.line("    asm volatile(\"\" : \"+v\"(col));");
    std::string decl = "    u32 x0, x1, x2, x3, x4, x5, x6, x7, n0, n1, n2, n3, n4, n5, n6, n7";
    for (u32 o = 0; o < no; ++o)
        decl += ", a" + std::to_string(o);
    g.line("%s;", decl.c_str());
    for (int b = 0; b < 8; ++b)
        g.line("    n%d = LDW(col + %uu);", b, (u32)b * ps);
    std::vector<bool> started(no, false);
    for (u32 p = 0; p < k; ++p) {
        g.line("    x0 = n0; x1 = n1; x2 = n2; x3 = n3; x4 = n4; x5 = n5; x6 = n6; x7 = n7;");
        if (p + 1 < k)
            for (int b = 0; b < 8; ++b)
                g.line("    n%d = LDW(col + %uu);", b, ((p + 1) * 8 + (u32)b) * ps);
        g.line("    __builtin_amdgcn_sched_barrier(0);");
        g.line("    {");
        std::vector<u32> masks(no);
        for (u32 o = 0; o < no; ++o)
            masks[o] = plane_mask(coef[(size_t)(r0 + o / 8) * k + p], (int)(o % 8));
        for (int h = 0; h < 2; ++h) {
            bool need[16] = {};
            for (u32 o = 0; o < no; ++o)
                need[(masks[o] >> (4 * h)) & 15] = true;
            bool have[16] = {};
            for (int j = 0; j < 4; ++j) {
                g.line("        const u32 t%d_%d = x%d;", h, 1 << j, 4 * h + j);
                have[1 << j] = true;
            }
            /* pairs, then triples, then the quad ((ab) ^ c ^ d) */
            for (int pc = 2; pc <= 4; ++pc)
                for (int m = 1; m < 16; ++m) {
                    if (__builtin_popcount(m) != pc || !(need[m] || (pc == 2 && m == 3 && need[15])))
                        continue;
                    if (have[m])
                        continue;
                    int bits[4], nb = 0;
                    for (int j = 0; j < 4; ++j)
                        if (m >> j & 1)
                            bits[nb++] = 1 << j;
                    if (pc == 2)
                        g.line("        const u32 t%d_%d = t%d_%d ^ t%d_%d;", h, m, h, bits[0], h, bits[1]);
                    else if (pc == 3)
                        g.line("        const u32 t%d_%d = xr3(t%d_%d, t%d_%d, t%d_%d);", h, m, h, bits[0],
                               h, bits[1], h, bits[2]);
                    else
                        g.line("        const u32 t%d_15 = xr3(t%d_3, t%d_4, t%d_8);", h, h, h, h);
                    have[m] = true;
                    ++g.ops;
                }
        }
        for (u32 o = 0; o < no; ++o) {
            const u32 m0 = masks[o] & 15, m1 = masks[o] >> 4;
            char t0[16] = "", t1[16] = "";
            if (m0)
                snprintf(t0, sizeof t0, "t0_%u", m0);
            if (m1)
                snprintf(t1, sizeof t1, "t1_%u", m1);
            if (!m0 && !m1)
                continue;
            if (!started[o]) {
                if (m0 && m1) {
                    g.line("        a%u = %s ^ %s;", o, t0, t1);
                    ++g.ops;
                } else {
                    g.line("        a%u = %s;", o, m0 ? t0 : t1);
                }
                started[o] = true;
            } else if (m0 && m1) {
                g.line("        a%u = xr3(a%u, %s, %s);", o, o, t0, t1);
                ++g.ops;
            } else {
                g.line("        a%u ^= %s;", o, m0 ? t0 : t1);
                ++g.ops;
            }
        }
        g.line("    }");
        g.line("    __builtin_amdgcn_sched_barrier(0);");
    }
    for (u32 o = 0; o < no; ++o)
        g.line("    acc[%u] = %s;", o, started[o] ? ("a" + std::to_string(o)).c_str() : "0u");
    g.line("}");
}

const char *kPrologue = R"(
typedef unsigned int u32;
typedef unsigned long long u64;
typedef u32 v4u __attribute__((ext_vector_type(4)));
#define LDW(off) (*(const __attribute__((address_space(3))) u32 *)(off))
__device__ __forceinline__ u32 xr3(u32 a, u32 b, u32 c)
{
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
struct JitArgs {
    const unsigned char *in[16];
    unsigned char *out[16];
    u64 in_stride, out_stride, nstripes;
    u64 contig;    /* out[r] = out[0] + r * 512 and out_stride = ROWS * 512 */
};
)";

/* body<LA>: LA = the LDS-DMA cache policy (0 default, 2 non-temporal), an
 * immediate of the load instruction, hence two kernels */
const char *kBody = R"(
template <int LA>
__device__ __forceinline__ void body(const JitArgs &a)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    constexpr u32 NW = T / 2u, PER = T / 2u, NT = NW * 64u;
    const u32 tid = threadIdx.x, lane = tid & 63u;
    const u32 wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const u64 t0 = (u64)blockIdx.x * T;
    /* the shipped tile kernels' staging (ec_kernels_impl.h stage_tile): input
     * p, plane b, stripe s at ((p * 8 + b) * T + s) * 64 */
    for (u32 ins = wave; ins < K * PER; ins += NW) {
        const u32 p = ins / PER, el = (ins % PER) * 64u + lane, seg = el >> 2;
        const u64 st = t0 + seg % T;
        if (st < a.nstripes) {
            const unsigned char *gp = a.in[p] + st * a.in_stride + (seg / T) * 64u + (el & 3u) * 16u;
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)gp,
                                             (__attribute__((address_space(3))) void *)(lds + ins * 1024u),
                                             16, 0, LA);
        }
    }
    /* every wave's LDS-DMA has landed before any wave reads the tile: the
     * hiprtc build of __syncthreads() waits only for lgkmcnt (the product
     * build adds vmcnt(0) itself), so the wait is explicit */
    __builtin_amdgcn_s_waitcnt(0x0070);          /* vmcnt(0) lgkmcnt(0) */
    __syncthreads();
    /* wave w: rows half (w & 1), stripes 4 * (w >> 1) .. + 3 */
    const u32 half = wave & 1u, s = (wave >> 1) * 4u + (lane >> 4), cc = lane & 15u;
    const u32 col = (u32)(unsigned long long)(lds + s * 64u + cc * 4u);
    u32 acc[NA];
    if (half == 0)
        prog0(col, acc);
    else
        prog1(col, acc);
    __syncthreads();
    /* stripe s, row r at (s * ROWS + r) * 512: a full decode's tile is then
     * its output as it lies in memory (ec_method_decode's stripe-major out) */
    unsigned char *ob = lds + s * (ROWS * 512u) + cc * 4u;
    const u32 rb = half == 0 ? 0u : R0;
    const u32 nr = half == 0 ? R0 : ROWS - R0;
#pragma unroll
    for (u32 o = 0; o < NA; ++o)
        if (o < nr * 8u)
            *(u32 *)(ob + (rb + o / 8u) * 512u + (o % 8u) * 64u) = acc[o];
    __syncthreads();
    const u64 left = a.nstripes - t0;
    const u32 ns = (u32)(left < T ? left : T);
    if (a.contig) {
        /* one run of ns * ROWS * 512 bytes */
        unsigned char *o = a.out[0] + t0 * a.out_stride;
        for (u32 i = tid * 16u; i < ns * ROWS * 512u; i += NT * 16u)
            __builtin_nontemporal_store(*(const v4u *)(lds + i), (v4u *)(o + i));
    } else {
        /* row by row: 512-byte runs, one per stripe (fragment-major outputs) */
        for (u32 r = 0; r < ROWS; ++r) {
            const u32 ss = tid >> 5, q = tid & 31u;
            if (ss < ns)
                __builtin_nontemporal_store(*(const v4u *)(lds + (ss * ROWS + r) * 512u + q * 16u),
                                            (v4u *)(a.out[r] + (t0 + ss) * a.out_stride + q * 16u));
        }
    }
}
extern "C" __global__ __launch_bounds__(T / 2 * 64) void ec_jit_combine(JitArgs a) { body<0>(a); }
extern "C" __global__ __launch_bounds__(T / 2 * 64) void ec_jit_combine_nt(JitArgs a) { body<2>(a); }
)";

/* ----------------------------------------------------------- compiler */

/* The compiler runs as a child process (ec_jitc, next to this library:
 * hiprtc in a process of its own).  Round 6's first version called hiprtc on
 * a library thread: a client that exited while that thread compiled crashed
 * (the compiler's static destructors ran under the compile; reproduced on
 * the CPU host with ec_method_jit_prepare + exit, 3 of 3 runs), and LLVM
 * lived in every client's address space. */
struct Compiler {
    std::string path, why;
    bool ok = false;

    Compiler()
    {
        if (const char *e = getenv("EC_MI355X_JITC")) {
            path = e;
        } else {
            Dl_info di;
            if (dladdr((const void *)&ecd_jit_stats, &di) && di.dli_fname) {
                path = di.dli_fname;
                const size_t sl = path.rfind('/');
                path = (sl == std::string::npos ? std::string(".") : path.substr(0, sl)) +
                       "/ec_jitc";
            }
        }
        ok = !path.empty() && access(path.c_str(), X_OK) == 0;
        if (!ok)
            why = "compiler " + (path.empty() ? std::string("ec_jitc") : path) + " not found";
    }
};

Compiler &compiler()
{
    static Compiler *c = new Compiler;   /* never destroyed (threads may outlive exit) */
    return *c;
}

bool read_file(const std::string &p, std::vector<char> &out)
{
    FILE *f = fopen(p.c_str(), "rb");
    if (!f)
        return false;
    char buf[1 << 16];
    size_t n;
    out.clear();
    while ((n = fread(buf, 1, sizeof buf, f)) > 0)
        out.insert(out.end(), buf, buf + n);
    fclose(f);
    return true;
}

/* 0: `code` holds the code object of `src`; else the compiler's log */
int run_compiler(const std::string &src, std::vector<char> &code, std::string &log)
{
    Compiler &c = compiler();
    if (!c.ok) {
        log = c.why;
        return -ENOSYS;
    }
    const char *tmp = getenv("TMPDIR");
    std::string base = std::string(tmp && *tmp ? tmp : "/tmp") + "/ec_jit_XXXXXX";
    std::vector<char> name(base.begin(), base.end());
    name.push_back('\0');
    const int fd = mkstemp(name.data());
    if (fd < 0) {
        log = "mkstemp failed";
        return -EIO;
    }
    const std::string sp(name.data()), cp = sp + ".co", lp = sp + ".log";
    const bool wrote = write(fd, src.data(), src.size()) == (ssize_t)src.size();
    close(fd);
    int rc = -EIO;
    if (wrote) {
        posix_spawn_file_actions_t fa;
        posix_spawn_file_actions_init(&fa);
        posix_spawn_file_actions_addopen(&fa, 1, "/dev/null", O_WRONLY, 0);
        posix_spawn_file_actions_addopen(&fa, 2, lp.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0600);
        char *argv[] = {const_cast<char *>(c.path.c_str()), const_cast<char *>(sp.c_str()),
                        const_cast<char *>(cp.c_str()), nullptr};
        pid_t pid = -1;
        if (posix_spawn(&pid, c.path.c_str(), &fa, nullptr, argv, environ) == 0) {
            int st = 0;
            while (waitpid(pid, &st, 0) < 0 && errno == EINTR) {
            }
            if (WIFEXITED(st) && WEXITSTATUS(st) == 0 && read_file(cp, code) && !code.empty())
                rc = 0;
            else
                rc = WIFEXITED(st) && WEXITSTATUS(st) == 2 ? -ENOSYS : -EIO;
        } else {
            log = "posix_spawn of the compiler failed";
        }
        posix_spawn_file_actions_destroy(&fa);
        if (rc) {
            std::vector<char> l;
            if (read_file(lp, l))
                log += std::string(l.begin(), l.end());
        }
    }
    unlink(sp.c_str());
    unlink(cp.c_str());
    unlink(lp.c_str());
    return rc;
}

/* ------------------------------------------------------------- cache */

struct Key {
    u32 k = 0, rows = 0;
    uint8_t coef[ECJ_MAX * ECJ_MAX] = {};
    bool operator==(const Key &o) const
    {
        return k == o.k && rows == o.rows && !memcmp(coef, o.coef, (size_t)k * rows);
    }
};

enum { kQueued = 0, kReady = 1, kFailed = 2 };

struct Entry {
    Key key;
    std::atomic<int> state{kQueued};
    std::vector<char> code;
    hipModule_t mod[kMaxDev] = {};
    hipFunction_t fn[kMaxDev][2] = {};
    int load_failed[kMaxDev] = {};
    uint64_t last_use = 0;
};

struct Jit {
    std::mutex mu;
    std::condition_variable cv;
    std::vector<Entry *> entries;     /* owned; never freed while a launch may use them */
    std::deque<Entry *> queue;
    bool worker = false;
    uint64_t tick = 0;
    uint64_t created = 0;
    std::atomic<uint64_t> compiled{0}, failed{0}, launches{0}, compile_us{0}, lookups{0};
    std::string last_log;
};

Jit &jit()
{
    static Jit *j = new Jit;   /* never destroyed: the worker may outlive exit */
    return *j;
}

long env_long(const char *name, long dflt)
{
    const char *e = getenv(name);
    return e && *e ? strtol(e, nullptr, 10) : dflt;
}

bool jit_on()
{
    static const bool v = env_long("EC_MI355X_JIT", 1) != 0;
    return v;
}

bool jit_sync()
{
    static const bool v = env_long("EC_MI355X_JIT_SYNC", 0) != 0;
    return v;
}

/* stripes per tile: 4 (two waves, 32 KiB of LDS for k = 16; up to 5 blocks
 * per CU).  The body also takes 8 (four waves, 64 KiB, 2 blocks per CU, as
 * the shipped k = 16 combine): 1-2 % slower through bench.py
 * (profiles/r06/r06h_jitab.log), so 4. */
constexpr u32 kJitTile = 4;
u32 jit_tile()
{
    return kJitTile;
}

uint64_t jit_min_stripes()
{
    static const uint64_t v = (uint64_t)env_long("EC_MI355X_JIT_MIN_STRIPES", 1024);
    return v;
}

std::string source_of(const Key &key, u32 *ops)
{
    Gen g;
    const u32 r0 = (key.rows + 1) / 2;
    g.s += kPrologue;
    g.line("#define K %uu", key.k);
    g.line("#define ROWS %uu", key.rows);
    g.line("#define R0 %uu", r0);
    g.line("#define NA %uu", r0 * 8);
    g.line("#define T %uu", jit_tile());

    emit_program(g, 0, key.k, jit_tile(), key.coef, 0, r0);
    emit_program(g, 1, key.k, jit_tile(), key.coef, r0, key.rows);
    g.s += kBody;
    if (ops)
        *ops = g.ops;
    return g.s;
}

/* compile one entry (any thread; the result is published by `state`) */
void compile_entry(Entry *e)
{
    Jit &j = jit();
    const auto t0 = std::chrono::steady_clock::now();
    u32 ops = 0;
    const std::string src = source_of(e->key, &ops);
    std::string log;
    const int st = run_compiler(src, e->code, log) == 0 ? kReady : kFailed;
    j.compile_us += (uint64_t)std::chrono::duration_cast<std::chrono::microseconds>(
                        std::chrono::steady_clock::now() - t0).count();
    (st == kReady ? j.compiled : j.failed)++;
    if (st != kReady) {
        std::lock_guard<std::mutex> g(j.mu);
        j.last_log = log.substr(0, 2000);
    }
    e->state.store(st, std::memory_order_release);
}

/* The compile thread: it waits for the compiler process of each queued
 * matrix.  It is neither stopped nor joined at exit (a compile then finishes
 * in its own process, or is orphaned; nothing in this process is torn down
 * under it: the cache and the compiler record are never destroyed). */
std::thread *g_worker;
bool g_stop;

void worker_main()
{
    Jit &j = jit();
    for (;;) {
        Entry *e;
        {
            std::unique_lock<std::mutex> g(j.mu);
            j.cv.wait(g, [&] { return g_stop || !j.queue.empty(); });
            if (g_stop)
                return;
            e = j.queue.front();
            j.queue.pop_front();
        }
        compile_entry(e);
    }
}

/* A child forked after the worker started has no worker (and maybe a held
 * lock): it starts empty-queued, and its first queued matrix starts its own
 * thread.  Entries the parent had queued stay "queued" in the child and
 * keep running the shipped kernel. */
void fork_prepare()
{
    jit().mu.lock();
}

void fork_parent()
{
    jit().mu.unlock();
}

void fork_child()
{
    Jit &j = jit();
    new (&j.mu) std::mutex();
    new (&j.cv) std::condition_variable();
    j.queue.clear();
    j.worker = false;
    g_worker = nullptr;       /* the parent's thread object is not ours */
}

/* the entry of `key`, inserted (and queued or compiled) on first sight;
 * nullptr when the cache is full of entries still queued */
Entry *lookup(const Key &key)
{
    Jit &j = jit();
    Entry *fresh = nullptr;
    {
        std::lock_guard<std::mutex> g(j.mu);
        for (Entry *e : j.entries)
            if (e->key == key) {
                e->last_use = ++j.tick;
                return e;
            }
        if (j.entries.size() >= kEntries) {
            /* replace the least recently used finished entry; its modules
             * stay loaded (a stream may still run them) -- a bounded leak of
             * one code object per replacement is the price of no waits */
            size_t lru = j.entries.size();
            for (size_t i = 0; i < j.entries.size(); ++i)
                if (j.entries[i]->state.load() != kQueued &&
                    (lru == j.entries.size() || j.entries[i]->last_use < j.entries[lru]->last_use))
                    lru = i;
            if (lru == j.entries.size())
                return nullptr;
            j.entries.erase(j.entries.begin() + (long)lru);
        }
        if (j.created >= kMaxCreated)
            return nullptr;
        ++j.created;
        fresh = new Entry;
        fresh->key = key;
        fresh->last_use = ++j.tick;
        j.entries.push_back(fresh);
        if (!jit_sync()) {
            j.queue.push_back(fresh);
            if (!j.worker) {
                static std::once_flag once;
                std::call_once(once, [] { pthread_atfork(fork_prepare, fork_parent, fork_child); });
                g_worker = new std::thread(worker_main);
                j.worker = true;
            }
            j.cv.notify_one();
        }
    }
    if (jit_sync())
        compile_entry(fresh);
    return fresh;
}

/* the entry's kernel on the calling thread's current device */
hipFunction_t function_of(Entry *e, bool nt)
{
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDev) {
        (void)hipGetLastError();
        return nullptr;
    }
    Jit &j = jit();
    std::lock_guard<std::mutex> g(j.mu);
    if (e->load_failed[dev])
        return nullptr;
    if (!e->mod[dev]) {
        hipModule_t m = nullptr;
        hipFunction_t f0 = nullptr, f1 = nullptr;
        if (hipModuleLoadData(&m, e->code.data()) != hipSuccess ||
            hipModuleGetFunction(&f0, m, "ec_jit_combine") != hipSuccess ||
            hipModuleGetFunction(&f1, m, "ec_jit_combine_nt") != hipSuccess) {
            (void)hipGetLastError();
            e->load_failed[dev] = 1;
            return nullptr;
        }
        e->mod[dev] = m;
        e->fn[dev][0] = f0;
        e->fn[dev][1] = f1;
    }
    return e->fn[dev][nt ? 1 : 0];
}

struct JitArgs {
    const uint8_t *in[16];
    uint8_t *out[16];
    uint64_t in_stride, out_stride, nstripes;
    uint64_t contig;
};

} // namespace

/* development hook (tools/kbench/kb3.hip): extra LDS per block, to trade
 * blocks per CU against the tile in A/B runs; 0 in the library */
extern "C" int ecj_lds_pad_kb = 0;

extern "C" int ecj_eligible(const ecd_combine_desc_t *d)
{
    if (!jit_on() || d->npatterns != 1 || d->group_pattern || d->k < 12 || d->k > ECJ_MAX ||
        d->rows < 12 || d->rows > ECJ_MAX || d->nstripes < jit_min_stripes() ||
        d->nstripes / 4 + 1 > 0x7fffffffull)
        return 0;
    /* 16-byte stores of 512-byte runs */
    if (d->out_stride % 16)
        return 0;
    for (uint32_t r = 0; r < d->rows; ++r)
        if (!d->out_base[r] || ((uintptr_t)d->out_base[r] & 15))
            return 0;
    return 1;
}

extern "C" int ecj_launch(hipStream_t s, const ecd_combine_desc_t *d, int nt)
{
    if (!ecj_eligible(d) || !compiler().ok)
        return -EAGAIN;
    const uint8_t *pat = d->pat_ext ? d->pat_ext : d->pat;
    Key key;
    key.k = d->k;
    key.rows = d->rows;
    memcpy(key.coef, pat + d->k, (size_t)d->rows * d->k);
    jit().lookups++;
    Entry *e = lookup(key);
    if (!e || e->state.load(std::memory_order_acquire) != kReady)
        return -EAGAIN;
    hipFunction_t f = function_of(e, nt != 0);
    if (!f)
        return -EAGAIN;
    JitArgs a;
    memset(&a, 0, sizeof a);
    for (uint32_t p = 0; p < d->k; ++p) {
        a.in[p] = static_cast<const uint8_t *>(d->in_base[pat[p]]);
        if (!a.in[p])
            return -EAGAIN;
    }
    for (uint32_t r = 0; r < d->rows; ++r)
        a.out[r] = static_cast<uint8_t *>(d->out_base[r]);
    a.in_stride = d->in_stride;
    a.out_stride = d->out_stride;
    a.nstripes = d->nstripes;
    a.contig = d->out_stride == (uint64_t)d->rows * 512;
    for (uint32_t r = 1; r < d->rows && a.contig; ++r)
        a.contig = a.out[r] == a.out[0] + (size_t)r * 512;
    const u32 T = jit_tile();
    const size_t lds = (size_t)(d->k > d->rows ? d->k : d->rows) * T * 512 +
                       (size_t)ecj_lds_pad_kb * 1024;
    if (lds > (64u << 10))
        return -EAGAIN;         /* the default dynamic LDS limit of a launch */
    void *params[] = {&a};
    const hipError_t rc = hipModuleLaunchKernel(f, (u32)((d->nstripes + T - 1) / T), 1, 1, T / 2 * 64,
                                                1, 1, (u32)lds, s, params, nullptr);
    if (rc != hipSuccess) {
        (void)hipGetLastError();
        return -EAGAIN;       /* the shipped kernel codes the call */
    }
    jit().launches++;
    return 0;
}

extern "C" void ecd_jit_stats(ecd_jit_stats_t *st)
{
    Jit &j = jit();
    st->compiled = j.compiled.load();
    st->failed = j.failed.load();
    st->launches = j.launches.load();
    st->compile_us = j.compile_us.load();
    st->lookups = j.lookups.load();
    std::lock_guard<std::mutex> g(j.mu);
    st->entries = j.entries.size();
}

extern "C" int ecd_jit_prepare(uint32_t k, uint32_t rows, const uint8_t *coef)
{
    if (k < 1 || k > ECJ_MAX || rows < 2 || rows > ECJ_MAX || !coef)
        return -EINVAL;
    if (!jit_on())
        return -EPERM;
    if (!compiler().ok)
        return -ENOSYS;
    Key key;
    key.k = k;
    key.rows = rows;
    memcpy(key.coef, coef, (size_t)k * rows);
    return lookup(key) ? 0 : -ENOSPC;
}

extern "C" int ecd_jit_compile_check(uint32_t k, uint32_t rows, const uint8_t *coef, uint32_t *ops,
                                 char *log, size_t log_len)
{
    if (k < 1 || k > ECJ_MAX || rows < 2 || rows > ECJ_MAX || !coef)
        return -EINVAL;
    if (!compiler().ok) {
        if (log && log_len)
            snprintf(log, log_len, "%s", compiler().why.c_str());
        return -ENOSYS;
    }
    Entry e;
    e.key.k = k;
    e.key.rows = rows;
    memcpy(e.key.coef, coef, (size_t)k * rows);
    const std::string src = source_of(e.key, ops);
    compile_entry(&e);
    /* EC_MI355X_JIT_DUMP=prefix: the source and code object, for inspection */
    if (const char *d = getenv("EC_MI355X_JIT_DUMP")) {
        if (FILE *f = fopen((std::string(d) + ".hip").c_str(), "w")) {
            fwrite(src.data(), 1, src.size(), f);
            fclose(f);
        }
        if (!e.code.empty())
            if (FILE *f = fopen((std::string(d) + ".co").c_str(), "wb")) {
                fwrite(e.code.data(), 1, e.code.size(), f);
                fclose(f);
            }
    }
    if (e.state.load() != kReady && log && log_len) {
        std::lock_guard<std::mutex> g(jit().mu);
        snprintf(log, log_len, "%s", jit().last_log.c_str());
    }
    return e.state.load() == kReady ? (int)e.code.size() : -EIO;
}
