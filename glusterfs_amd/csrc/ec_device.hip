/*
 * ec_device.hip -- HIP runtime side of the MI355X disperse coder.
 *
 * Owns everything the reference never needed because its coder ran inline on
 * the calling CPU thread (ec-method.c:394-433): device discovery, per-call
 * streams, device/pinned staging buffers, the PCIe pipeline for callers that
 * hand over host memory, and the stripe-range partition across all visible
 * MI355X devices (stripes are independent, no collective).
 *
 * Host buffers (the reference codes iobufs in place) are coded
 * by kernels that read and write pinned host memory directly over PCIe; no
 * SDMA copies, no device staging.  Pageable buffers bounce through two pinned
 * slots copied by a CPU thread pool, overlapped with the GPU coding the other
 * slot.  See "host-buffer pipeline" below for the measurements behind this.
 */
#include <hip/hip_runtime.h>

#include <ctype.h>
#include <errno.h>
#include <sched.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <shared_mutex>
#include <string>
#include <thread>
#include <vector>

#include "ec_device.h"
#include "ec_kernels.h"

static uint64_t hostpage_ttl_ns();   /* the host-page caches' lifetime (below) */
static uint64_t coarse_ns();

namespace {

constexpr int kMaxDev = 16;
/* Stripes per pipeline batch are sized to this many input bytes; the
 * EC_PIPE_BATCH_MB / EC_COPY_THREADS environment overrides exist for tuning
 * (tools/kbench/e2e.c). */
uint64_t pipe_batch_bytes()
{
    static const uint64_t v = [] {
        const char *e = getenv("EC_PIPE_BATCH_MB");
        const long mb = e ? atol(e) : 0;
        return (uint64_t)(mb > 0 && mb <= 1024 ? mb : 32) << 20;
    }();
    return v;
}

/* CPUs this process may use: its affinity, capped by the cgroup CPU quota
 * (the GPU pool grants 16 CPUs of a 256-thread host; ranks of one job share
 * it, so bench.py also sets EC_COPY_THREADS to its share per rank). */
int usable_cpus()
{
    cpu_set_t cs;
    int n = sched_getaffinity(0, sizeof(cs), &cs) == 0 ? CPU_COUNT(&cs) : 1;
    if (FILE *f = fopen("/sys/fs/cgroup/cpu.max", "r")) {
        char q[32] = "";
        long per = 0;
        if (fscanf(f, "%31s %ld", q, &per) == 2 && strcmp(q, "max") != 0 && per > 0)
            n = std::min<long>(n, std::max<long>(1, atol(q) / per));
        fclose(f);
    }
    return std::max(n, 1);
}

int copy_threads()
{
    static const int v = [] {
        const char *e = getenv("EC_COPY_THREADS");
        const int t = e ? atoi(e) : std::min(8, usable_cpus());
        return std::min(std::max(t, 0), 64);
    }();
    return v;
}

/* Error text of the last failure, per calling thread (ec_method_last_error):
 * a GlusterFS client codes on several epoll threads and the heal syncenv, so
 * a process-wide slot handed one thread's failure to another's log line (r04:
 * a combine's -EIO reported a much earlier test's hipHostUnregister text).
 * t_err_seq counts the failures this thread recorded, so ec_method.c can tell
 * whether a failing call already said why. */
thread_local std::string t_err;
thread_local uint64_t t_err_seq = 0;
/* set once by discover(): the reason a node has no usable device */
std::string g_discover_err;

void set_err_text(std::string s)
{
    t_err = std::move(s);
    ++t_err_seq;
}

/* Records a failed HIP call's error as this thread's and consumes the HIP
 * runtime's sticky copy of it: a failure the library reports by its return
 * code must not surface again at the caller's next HIP or torch call
 * (test_register_errors' refused unregister, left pending, failed the next
 * test's torch copy with hipErrorHostMemoryNotRegistered). */
void set_err(const char *what, hipError_t e)
{
    (void)hipGetLastError();
    set_err_text(std::string(what) + ": " + hipGetErrorString(e) + " (" +
                 std::to_string((int)e) + ")");
}

/* A HIP error the thread left pending before this call (the caller's own
 * unchecked call, or one the runtime records without failing the call) is
 * not this call's: drop it, so the launch checks below -- hipGetLastError
 * after each launch -- see only the launch. */
inline void clear_stale_error()
{
    (void)hipGetLastError();
}

#define HIPCHK(call)                                                           \
    do {                                                                       \
        hipError_t e_ = (call);                                                \
        if (e_ != hipSuccess) {                                                \
            set_err(#call, e_);                                                \
            return -EIO;                                                       \
        }                                                                      \
    } while (0)

std::once_flag g_dev_once;
int g_ndev = 0;
int g_dev_ids[kMaxDev];
/* Devices the host-buffer entry points spread their stripes over (indices
 * into g_dev_ids): all of them, or the comma list in EC_MI355X_HOST_DEVICES,
 * e.g. to keep a client on its NUMA-local GPUs or one rank per GPU. */
int g_nhost = 0;
int g_host_devs[kMaxDev];

void host_devices_from_env()
{
    const char *e = getenv("EC_MI355X_HOST_DEVICES");
    /* EC_MI355X_TEST_SPLIT=1 keeps repeated entries ("0,0"), so the
     * in-library stripe split runs its multi-device code on one GPU (tests) */
    const char *ts = getenv("EC_MI355X_TEST_SPLIT");
    const bool dup = ts && *ts == '1';
    bool seen[kMaxDev] = {};
    while (e && *e && g_nhost < kMaxDev) {
        char *end = nullptr;
        const long v = strtol(e, &end, 10);
        if (end == e)
            break;
        if (v >= 0 && v < g_ndev && (dup || !seen[v])) {
            seen[v] = true;
            g_host_devs[g_nhost++] = (int)v;
        }
        e = *end == ',' ? end + 1 : end;
    }
    if (g_nhost == 0)
        for (int i = 0; i < g_ndev; ++i)
            g_host_devs[g_nhost++] = i;
}

/* EC_MI355X_DEBUG=1: count the HIP pointer queries of the host-call checks
 * and print them at exit (development probe for the routing cost). */
std::atomic<uint64_t> g_ptr_queries{0}, g_map_queries{0};
/* Generation of the library's own host-memory frees: invalidates the
 * per-thread host-page cache of ecd_ptr_device (below). */
std::atomic<uint32_t> g_host_gen{0};
/* Generation of the library's host-memory registrations (every successful
 * hipHostRegister and pinned allocation): invalidates the per-thread cache of
 * ranges found unmapped (mapped(), below). */
std::atomic<uint32_t> g_map_gen{0};

void print_query_counts()
{
    fprintf(stderr, "[ec-mi355x] pointer queries: %llu attribute, %llu mapping\n",
            (unsigned long long)g_ptr_queries.load(), (unsigned long long)g_map_queries.load());
}

void discover()
{
    if (getenv("EC_MI355X_DEBUG") && atoi(getenv("EC_MI355X_DEBUG")))
        atexit(print_query_counts);
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) {
        (void)hipGetLastError();
        n = 0;
    }
    for (int i = 0; i < n && g_ndev < kMaxDev; ++i) {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, i) != hipSuccess) {
            (void)hipGetLastError();
            continue;
        }
        if (strncmp(prop.gcnArchName, "gfx950", 6) != 0)
            continue; /* kernels are built for gfx950 only */
        g_dev_ids[g_ndev++] = i;
    }
    host_devices_from_env();
    if (g_ndev == 0)
        g_discover_err = "no gfx950 (MI355X) device visible";
}

hipStream_t pick_stream(void *stream)
{
    return stream ? static_cast<hipStream_t>(stream) : hipStreamPerThread;
}

/* Every entry point that selects a device restores the calling thread's
 * current device on return: the library shares the HIP runtime with its
 * caller (torch, or a GlusterFS client that uses HIP itself), whose later
 * allocations and launches must not move to another GPU. */
class DeviceGuard {
  public:
    DeviceGuard()
    {
        if (hipGetDevice(&prev_) != hipSuccess) {
            (void)hipGetLastError();
            prev_ = -1;
        }
    }
    ~DeviceGuard()
    {
        int cur = -1;
        if (prev_ >= 0 && (hipGetDevice(&cur) != hipSuccess ||
                           (cur != prev_ && hipSetDevice(prev_) != hipSuccess)))
            (void)hipGetLastError();
    }
    DeviceGuard(const DeviceGuard &) = delete;
    DeviceGuard &operator=(const DeviceGuard &) = delete;

  private:
    int prev_ = -1;
};

/* ------------------------------------------------- host-buffer pipeline */

/* Host buffers never go through SDMA copies here: the coding kernels read
 * and write pinned host memory directly over PCIe.  Measured on MI355X with
 * tools/kbench/zerocopy.hip, CU-issued accesses move ~56 GB/s host->device,
 * ~55 GB/s device->host and ~45 GB/s EACH WAY when a kernel does both at once
 * (~90 GB/s bidirectional), while SDMA copies chained behind kernels through
 * cross-stream events reached only 45-65 GB/s in total and stalled the
 * enqueueing thread (tools/kbench/e2e.c, EC_PIPE_TRACE).  So:
 *   - pinned (page-locked, device-mapped) caller buffers are coded in place:
 *     one kernel per batch, no copies at all;
 *   - pageable caller buffers are staged through two pinned slots by a pool
 *     of CPU threads: batch b's input copy and batch b-1's output copy run
 *     on the CPU while the GPU codes batch b from the other slot. */

/* Pool of CPU threads for staging copies (shared by all devices/callers). */
class CopyPool {
  public:
    struct Piece {
        uint8_t *dst;
        const uint8_t *src;
        size_t n;
    };

    void run(const std::vector<Piece> &pieces)
    {
        if (pieces.empty())
            return;
        start();
        Job j;
        j.p = &pieces;
        if (!th_.empty() && pieces.size() > 1) {
            std::lock_guard<std::mutex> g(mu_);
            q_.push_back(&j);
            cv_.notify_all();
        }
        work(j);
        std::unique_lock<std::mutex> g(mu_);
        done_cv_.wait(g, [&] { return j.done.load() == pieces.size() && j.active == 0; });
        for (auto it = q_.begin(); it != q_.end(); ++it)
            if (*it == &j) {
                q_.erase(it);
                break;
            }
    }

    ~CopyPool()
    {
        {
            std::lock_guard<std::mutex> g(mu_);
            stop_ = true;
            cv_.notify_all();
        }
        for (auto &t : th_)
            t.join();
    }

  private:
    struct Job {
        const std::vector<Piece> *p;
        std::atomic<size_t> next{0}, done{0};
        int active = 0; /* workers inside work(); guarded by mu_ */
    };

    void start()
    {
        std::call_once(once_, [this] {
            for (int i = 0; i < copy_threads(); ++i)
                th_.emplace_back([this] { loop(); });
        });
    }

    void work(Job &j)
    {
        const std::vector<Piece> &p = *j.p;
        for (size_t i; (i = j.next.fetch_add(1)) < p.size();) {
            if (p[i].src)
                memcpy(p[i].dst, p[i].src, p[i].n);
            else
                memset(p[i].dst, 0, p[i].n); /* gathered zero fill */
            j.done.fetch_add(1);
        }
    }

    /* A job stays at the front of the queue until all of its pieces are
     * claimed, so every idle worker joins it (popping it on first sight
     * left one helper per copy, whatever EC_COPY_THREADS said).  The owner
     * erases it in run() once it is done; a worker that finds it fully
     * claimed pops it. */
    void loop()
    {
        std::unique_lock<std::mutex> g(mu_);
        for (;;) {
            cv_.wait(g, [&] { return stop_ || !q_.empty(); });
            if (stop_)
                return;
            Job *j = q_.front();
            if (j->next.load() >= j->p->size()) {
                q_.pop_front();
                continue;
            }
            ++j->active;
            g.unlock();
            work(*j);
            g.lock();
            --j->active;
            if (!q_.empty() && q_.front() == j)
                q_.pop_front();
            done_cv_.notify_all();
        }
    }

    std::once_flag once_;
    std::mutex mu_;
    std::condition_variable cv_, done_cv_;
    std::deque<Job *> q_;
    std::vector<std::thread> th_;
    bool stop_ = false;
};

CopyPool g_copy_pool;

/* Split [dst, src, n) copies into pieces for the pool: n / copy threads,
 * between 256 KiB and 2 MiB (64 KiB multiples).  Fixed 2 MiB pieces left a
 * 4 MiB heal-window output on two of the eight threads (r04: a registered-
 * fragment decode into a pageable output took 323 us against 185 us with
 * every buffer mapped, bench.py heal_sweep ec_provenance_calloc). */
void add_copy(std::vector<CopyPool::Piece> &v, uint8_t *dst, const uint8_t *src, size_t n)
{
    const size_t t = (size_t)std::max(1, copy_threads());
    const size_t piece =
        std::min<size_t>(2u << 20, std::max<size_t>(256u << 10, (n / t + 0xFFFF) & ~(size_t)0xFFFF));
    for (size_t o = 0; o < n; o += piece)
        v.push_back({dst + o, src ? src + o : nullptr, std::min(piece, n - o)});
}

/* Stripes per pipeline batch of a call that stages some of its buffers:
 * `full` (the batch sized by pipe_batch_bytes), but a call of a single such
 * batch is cut into up to 4 batches of >= 1 MiB of input, so the copies of
 * one batch overlap the kernel of the next (a 4 MiB heal window was one
 * batch: copy in, kernel, copy out, strictly in turn).  `in_stripe` = input
 * bytes per stripe, `unit` = stripes the batches must be a multiple of. */
uint64_t staged_batch(uint64_t full, uint64_t cnt_all, uint64_t in_stripe, uint64_t unit)
{
    static const int split = [] {              /* EC_PIPE_SPLIT=1: one batch (A/B) */
        const char *e = getenv("EC_PIPE_SPLIT");
        return e ? atoi(e) : 4;
    }();
    if (split <= 1 || cnt_all > full)
        return full;
    const uint64_t min_st = std::max<uint64_t>(1, (1u << 20) / in_stripe);
    uint64_t nb = std::min<uint64_t>((uint64_t)split, cnt_all / min_st);
    if (nb <= 1)
        return full;
    uint64_t b = (cnt_all + nb - 1) / nb;
    b = (b + unit - 1) / unit * unit;
    return std::max<uint64_t>(b, unit);
}

/* A virtual input made of consecutive segments (nullptr = zeros): the
 * padded write buffer of a partial-stripe write (ec_method_writev_encode). */
struct Seg {
    const uint8_t *p;
    size_t n;
};

/* Copy bytes [voff, voff + n) of the virtual input `segs` to dst. */
void add_gather(std::vector<CopyPool::Piece> &v, uint8_t *dst, const std::vector<Seg> &segs,
                uint64_t voff, size_t n)
{
    uint64_t base = 0;
    for (const Seg &sg : segs) {
        const uint64_t lo = std::max<uint64_t>(base, voff);
        const uint64_t hi = std::min<uint64_t>(base + sg.n, voff + n);
        if (lo < hi)
            add_copy(v, dst + (lo - voff), sg.p ? sg.p + (lo - base) : nullptr, hi - lo);
        base += sg.n;
    }
}

/* Device-visible address of [p, p+n) when it lies in pinned, device-mapped
 * host memory (hipHostMalloc / ec_method_host_alloc / hipHostRegister),
 * else nullptr.  16-byte alignment is required for the kernels' vector
 * accesses. */
bool pool_owns(const void *p, size_t n);

bool user_range_live(const void *p, size_t n);
bool numa_alloc_live(const void *p, size_t n);

/* Ranges found NOT mapped, per thread (direct-mapped on the start page).
 * The two hipHostGetDevicePointer queries of a range serialise in the HIP
 * runtime like the attribute queries (ecd_ptr_device, below): a pageable
 * 8+4 heal window asks for 22 ranges, and 8 client threads asking on every
 * call ran 8 % below the CPU engine alone with almost every call on the CPU
 * (profiles/r05/r05u_busyab.log).  Only the negative verdict is cached, for
 * EC_HOSTPAGE_MS and until the library registers or pins more memory
 * (g_map_gen): a stale one stages a buffer that has become mapped -- the
 * same bytes, coded a little slower -- while a stale positive one would let a
 * kernel read memory that is no longer mapped, so those are never cached. */
struct Unmapped {
    uintptr_t p;
    size_t n;
    uint64_t until_ns;
    uint32_t gen;
};
thread_local Unmapped t_unmapped[256];

uint8_t *mapped(const void *p, size_t n)
{
    if (!p || ((uintptr_t)p & 15))
        return nullptr;
    /* the library's own mappings -- a pool buffer, a range registered
     * through ec_method_host_register[_async], ec_method_host_alloc memory --
     * are known without asking the HIP runtime, whose queries serialise
     * across threads (~11 us each with 16 callers, tools/kbench/ptrq) and
     * cannot be cached for mapped memory (above): registered at the same
     * address, live until their owner unregisters or frees them */
    if (pool_owns(p, n) || user_range_live(p, n) || numa_alloc_live(p, n))
        return static_cast<uint8_t *>(const_cast<void *>(p));
    const uint64_t ttl = hostpage_ttl_ns();
    const uintptr_t pg = (uintptr_t)p >> 12;
    Unmapped &u = t_unmapped[(uint64_t)(pg * 0x9E3779B97F4A7C15ull) >> 56];
    const uint32_t gen = g_map_gen.load(std::memory_order_acquire);
    const uint64_t now = ttl ? coarse_ns() : 0;
    if (ttl && u.p == (uintptr_t)p && u.n == n && u.gen == gen && now < u.until_ns)
        return nullptr;
    void *d0 = nullptr, *d1 = nullptr;
    g_map_queries.fetch_add(1, std::memory_order_relaxed);
    if (hipHostGetDevicePointer(&d0, const_cast<void *>(p), 0) != hipSuccess ||
        (n > 1 && hipHostGetDevicePointer(&d1, (uint8_t *)p + n - 1, 0) != hipSuccess) ||
        /* one contiguous mapping, at the same address on both sides (ROCm
         * maps pinned host memory at its host virtual address) */
        d0 != p || (n > 1 && (uint8_t *)d1 != (uint8_t *)d0 + n - 1)) {
        (void)hipGetLastError();
        if (ttl)
            u = Unmapped{(uintptr_t)p, n, now + ttl, gen};
        return nullptr;
    }
    return static_cast<uint8_t *>(d0);
}

/* ---------------------------------------------- NUMA-local pinned memory */

/* NUMA node of device index `dev` (sysfs numa_node of its PCI function),
 * -1 when unknown or on a single-node host. */
int g_numa[kMaxDev];
std::once_flag g_numa_once;

int count_numa_nodes()
{
    int n = 0;
    for (int i = 0; i < 1024; ++i) {
        char path[64];
        snprintf(path, sizeof path, "/sys/devices/system/node/node%d", i);
        if (access(path, F_OK) != 0)
            break;
        ++n;
    }
    return n;
}

void discover_numa()
{
    const bool multi = count_numa_nodes() > 1;
    for (int d = 0; d < kMaxDev; ++d)
        g_numa[d] = -1;
    for (int d = 0; d < g_ndev; ++d) {
        char bus[64] = "", path[128];
        if (hipDeviceGetPCIBusId(bus, sizeof bus, g_dev_ids[d]) != hipSuccess) {
            (void)hipGetLastError();
            continue;
        }
        for (char *c = bus; *c; ++c)
            *c = (char)tolower((unsigned char)*c);
        snprintf(path, sizeof path, "/sys/bus/pci/devices/%s/numa_node", bus);
        if (FILE *f = fopen(path, "r")) {
            int node = -1;
            if (fscanf(f, "%d", &node) == 1 && node >= 0)
                g_numa[d] = multi || getenv("EC_NUMA_FORCE") ? node : -1;
            fclose(f);
        }
    }
}

int device_numa(int dev)
{
    std::call_once(g_numa_once, discover_numa);
    return dev >= 0 && dev < g_ndev ? g_numa[dev] : -1;
}

/* Pinned, device-mapped host memory whose pages sit on NUMA node `node`:
 * an anonymous mapping bound (preferred) to the node, faulted in there,
 * then registered with the HIP runtime.  hipHostMalloc places pages by the
 * calling thread's first touch, i.e. wherever the caller happens to run --
 * on a 2-socket host half the ranks would stage across the socket link.
 * Node < 0, or any step failing: hipHostMalloc. */
std::shared_mutex g_numa_mu;        /* shared: the lookups of every host call */
std::map<void *, size_t> g_numa_allocs;

bool numa_alloc_live(const void *p, size_t n)
{
    std::shared_lock<std::shared_mutex> g(g_numa_mu);
    auto it = g_numa_allocs.upper_bound(const_cast<void *>(p));
    if (it == g_numa_allocs.begin())
        return false;
    --it;
    const uintptr_t b = (uintptr_t)it->first, a = (uintptr_t)p;
    return a >= b && a + n <= b + it->second;
}

void *pinned_alloc(size_t bytes, int node)
{
    bytes = bytes ? bytes : 1;
    if (node >= 0 && node < 1024 && !getenv("EC_NUMA_OFF")) {
        const size_t pg = 4096, len = (bytes + pg - 1) / pg * pg;
        void *p = mmap(nullptr, len, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
        if (p != MAP_FAILED) {
            unsigned long mask[1024 / (8 * sizeof(unsigned long))] = {};
            mask[node / (8 * sizeof(unsigned long))] |= 1ul << (node % (8 * sizeof(unsigned long)));
            /* MPOL_PREFERRED (1): the node if it has room, else anywhere */
            (void)syscall(SYS_mbind, p, len, 1, mask, (unsigned long)1024, 0u);
            memset(p, 0, len);                       /* fault in on the node */
            if (hipHostRegister(p, len, hipHostRegisterMapped) == hipSuccess) {
                g_map_gen.fetch_add(1, std::memory_order_release);
                std::unique_lock<std::shared_mutex> g(g_numa_mu);
                g_numa_allocs[p] = len;
                return p;
            }
            (void)hipGetLastError();
            munmap(p, len);
        }
    }
    void *p = nullptr;
    if (hipHostMalloc(&p, bytes, hipHostMallocDefault) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    g_map_gen.fetch_add(1, std::memory_order_release);
    return p;
}

void pinned_free(void *p)
{
    if (!p)
        return;
    size_t len = 0;
    {
        std::unique_lock<std::shared_mutex> g(g_numa_mu);
        auto it = g_numa_allocs.find(p);
        if (it != g_numa_allocs.end()) {
            len = it->second;
            g_numa_allocs.erase(it);
        }
    }
    if (len) {
        (void)hipHostUnregister(p);
        munmap(p, len);
    } else {
        (void)hipHostFree(p);
    }
    g_host_gen.fetch_add(1, std::memory_order_release);
}

uint64_t mono_us()
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (uint64_t)ts.tv_sec * 1000000ull + (uint64_t)ts.tv_nsec / 1000;
}

/* ------------------------------------------------ pinned buffer pool (r04) */

/* Pinned, device-mapped buffers recycled by size, for a client's own I/O
 * buffers (ec_method_buffer_get / _put).  The integration patch hands
 * GlusterFS's non-arena iobufs to it -- iobuf_get_from_small (<= 128 KiB,
 * GF_MALLOC) and iobuf_get_from_stdalloc (> 1 MiB, GF_CALLOC),
 * iobuf.c:439-510 -- which is where ec_buffer_alloc (ec-helpers.c:134-165)
 * puts a heal window's decode output (4 MiB + 64, ec-inode-read.c:1191) and
 * re-encode output (n/k x 4 MiB, ec-inode-write.c:1871), and where the RPC
 * layer puts small fragment replies; the coder then reads and writes them in
 * place over PCIe.  hipHostRegister runs once per slab, when the pool grows,
 * never per buffer.
 *   - one reserved virtual range (EC_POOL_MB, default 2048 MiB) in 2 MiB
 *     granules, so ownership and size class of an address are O(1) (and a
 *     pool buffer is known to be mapped without a HIP pointer query);
 *   - classes 4 KiB .. 1 MiB (powers of two) share one-granule slabs; larger
 *     buffers are runs of g granules (g <= 64, 128 MiB), one free list per g;
 *   - slab pages are bound (preferred) to the NUMA node of the first
 *     host-buffer GPU and faulted in before registration;
 *   - nothing is returned to the system before exit; when the range is used
 *     up, get() returns NULL and the caller allocates as before.
 * Contents are not cleared (GF_MALLOC'd iobufs are not either). */
class BufPool {
  public:
    static constexpr size_t kGran = 2u << 20;
    static constexpr int kMinShift = 12, kMaxSmallShift = 20;
    static constexpr int kNSmall = kMaxSmallShift - kMinShift + 1;
    static constexpr int kMaxRun = 64;
    static constexpr int kNClass = kNSmall + kMaxRun;
    static constexpr uint8_t kFree = 0, kBody = 0xFF;

    void *get(size_t bytes)
    {
        if (!ready())
            return nullptr;
        gets_.fetch_add(1, std::memory_order_relaxed);
        if (bytes == 0 || bytes > (size_t)kMaxRun * kGran) {
            misses_.fetch_add(1, std::memory_order_relaxed);
            return nullptr;
        }
        const int c = cls(bytes);
        for (;;) {
            {
                std::lock_guard<std::mutex> g(mu_[c]);
                if (!free_[c].empty()) {
                    void *p = free_[c].back();
                    free_[c].pop_back();
                    in_use_.fetch_add(csize(c), std::memory_order_relaxed);
                    return p;
                }
            }
            if (!grow(c)) {    /* (another thread may take the new slab: retry) */
                misses_.fetch_add(1, std::memory_order_relaxed);
                return nullptr;
            }
        }
    }

    /* true when p is a buffer of the pool (now free again) */
    bool put(void *p)
    {
        int c;
        if (!chunk_of(p, &c))
            return false;
        in_use_.fetch_sub(csize(c), std::memory_order_relaxed);
        std::lock_guard<std::mutex> g(mu_[c]);
        free_[c].push_back(p);
        return true;
    }

    /* [p, p + n) inside one buffer of the pool: pinned and mapped */
    bool owns(const void *p, size_t n) const
    {
        const uint8_t *b = base_.load(std::memory_order_acquire);
        const uint8_t *q = static_cast<const uint8_t *>(p);
        if (!b || q < b || q >= b + span_)
            return false;
        const size_t gi = (size_t)(q - b) / kGran;
        uint8_t m = meta_[gi].load(std::memory_order_acquire);
        size_t gh = gi;
        while (m == kBody && gh > 0)            /* inside a run: find its head */
            m = meta_[--gh].load(std::memory_order_acquire);
        if (m == kFree || m == kBody)
            return false;
        const int c = m - 1;
        const size_t cs = csize(c);
        const size_t off = (size_t)(q - (b + gh * kGran));
        return off % cs + n <= cs;
    }

    /* [p, p + n) touches the pool's reserved range (registered or not) */
    bool overlaps(const void *p, size_t n) const
    {
        const uint8_t *b = base_.load(std::memory_order_acquire);
        const uintptr_t q = (uintptr_t)p;
        return b && q < (uintptr_t)b + span_ && q + n > (uintptr_t)b;
    }

    void stats(ecd_pool_stats_t *s) const
    {
        s->pool_bytes = grown_.load() * kGran;
        s->in_use_bytes = in_use_.load();
        s->gets = gets_.load();
        s->misses = misses_.load();
        s->slabs = slabs_.load();
        s->slab_register_us = slab_us_.load();
    }

  private:
    static int cls(size_t bytes)
    {
        if (bytes <= ((size_t)1 << kMaxSmallShift)) {
            int s = kMinShift;
            while (((size_t)1 << s) < bytes)
                ++s;
            return s - kMinShift;
        }
        return kNSmall + (int)((bytes + kGran - 1) / kGran) - 1;
    }
    static size_t csize(int c)
    {
        return c < kNSmall ? (size_t)1 << (c + kMinShift) : (size_t)(c - kNSmall + 1) * kGran;
    }

    bool chunk_of(const void *p, int *c) const
    {
        const uint8_t *b = base_.load(std::memory_order_acquire);
        const uint8_t *q = static_cast<const uint8_t *>(p);
        if (!b || q < b || q >= b + span_)
            return false;
        const size_t gi = (size_t)(q - b) / kGran;
        const uint8_t m = meta_[gi].load(std::memory_order_acquire);
        if (m == kFree || m == kBody)
            return false;
        *c = m - 1;
        return (size_t)(q - (b + gi * kGran)) % csize(*c) == 0;
    }

    bool ready()
    {
        std::call_once(once_, [this] {
            if (g_ndev == 0)
                return;
            const char *e = getenv("EC_POOL_MB");
            const long mb = e ? atol(e) : 2048;
            if (mb <= 0)
                return;
            ngran_ = ((size_t)mb << 20) / kGran;
            if (ngran_ == 0)
                return;
            const size_t len = ngran_ * kGran + kGran;
            void *r = mmap(nullptr, len, PROT_NONE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE,
                           -1, 0);
            if (r == MAP_FAILED)
                return;
            uint8_t *b = (uint8_t *)(((uintptr_t)r + kGran - 1) & ~(uintptr_t)(kGran - 1));
            meta_.reset(new std::atomic<uint8_t>[ngran_]);
            for (size_t i = 0; i < ngran_; ++i)
                meta_[i].store(kFree, std::memory_order_relaxed);
            span_ = ngran_ * kGran;
            base_.store(b, std::memory_order_release);
        });
        return base_.load(std::memory_order_acquire) != nullptr;
    }

    /* new slab for class c: g granules, mapped, bound, faulted in, registered */
    bool grow(int c)
    {
        std::lock_guard<std::mutex> g(grow_mu_);
        {
            std::lock_guard<std::mutex> f(mu_[c]);   /* another thread grew it */
            if (!free_[c].empty())
                return true;
        }
        const size_t ng = c < kNSmall ? 1 : (size_t)(c - kNSmall + 1);
        if (next_ + ng > ngran_)
            return false;
        uint8_t *b = base_.load(std::memory_order_relaxed) + next_ * kGran;
        const size_t len = ng * kGran;
        const uint64_t t0 = mono_us();
        if (mprotect(b, len, PROT_READ | PROT_WRITE) != 0)
            return false;
        const int node = device_numa(g_host_devs[0]);
        if (node >= 0 && node < 1024 && !getenv("EC_NUMA_OFF")) {
            unsigned long mask[1024 / (8 * sizeof(unsigned long))] = {};
            mask[node / (8 * sizeof(unsigned long))] |= 1ul << (node % (8 * sizeof(unsigned long)));
            (void)syscall(SYS_mbind, b, len, 1, mask, (unsigned long)1024, 0u);
        }
        memset(b, 0, len);
        void *dp = nullptr;
        if (hipHostRegister(b, len, hipHostRegisterMapped) != hipSuccess ||
            hipHostGetDevicePointer(&dp, b, 0) != hipSuccess || dp != b) {
            (void)hipGetLastError();
            (void)hipHostUnregister(b);
            (void)hipGetLastError();
            madvise(b, len, MADV_DONTNEED);
            (void)mprotect(b, len, PROT_NONE);
            return false;
        }
        slab_us_.fetch_add(mono_us() - t0, std::memory_order_relaxed);
        meta_[next_].store((uint8_t)(c + 1), std::memory_order_release);
        for (size_t i = 1; i < ng; ++i)
            meta_[next_ + i].store(kBody, std::memory_order_release);
        next_ += ng;
        grown_.fetch_add(ng);
        slabs_.fetch_add(1);
        std::lock_guard<std::mutex> f(mu_[c]);
        const size_t cs = csize(c);
        for (size_t o = len; o >= cs; o -= cs)     /* lowest address handed out first */
            free_[c].push_back(b + o - cs);
        return true;
    }

    std::once_flag once_;
    std::atomic<uint8_t *> base_{nullptr};
    size_t span_ = 0, ngran_ = 0, next_ = 0;
    std::unique_ptr<std::atomic<uint8_t>[]> meta_;
    std::mutex grow_mu_;
    std::mutex mu_[kNClass];
    std::vector<void *> free_[kNClass];
    std::atomic<uint64_t> gets_{0}, misses_{0}, in_use_{0}, grown_{0}, slabs_{0}, slab_us_{0};
};

/* never destroyed: its memory stays registered until the process exits */
BufPool &buf_pool()
{
    static BufPool *p = new BufPool;
    return *p;
}

/* ---------------------------------------- deferred host registration (r04) */

/* Ranges registered through ec_method_host_register[_async], page-rounded.
 * The runtime pins and maps whole pages, so two registrations that share a
 * page would share its GPU mapping, and unregistering one would unmap a page
 * the other's kernels still use (tools/fuzz_api.py registered neighbouring
 * heap arrays this way: a mismatch in r04x, a GPU memory fault in r04z2).
 * A registration overlapping a live one is refused with -EEXIST instead (the
 * range stays pageable to the coder, which stages it); GlusterFS's arenas
 * are page-aligned mmaps and never overlap. */
class RangeSet {
  public:
    /* reserve [p, p + n) rounded out to pages; false if it overlaps */
    bool reserve(const void *p, size_t n)
    {
        const uintptr_t s = (uintptr_t)p & ~kPageMask;
        const uintptr_t e = ((uintptr_t)p + n + kPageMask) & ~kPageMask;
        std::unique_lock<std::shared_mutex> g(mu_);
        auto it = by_start_.lower_bound(s);
        if (it != by_start_.end() && it->first < e)
            return false;
        if (it != by_start_.begin() && std::prev(it)->second.e > s)
            return false;
        by_start_[s] = Range{e, (uintptr_t)p, (uintptr_t)p + n, false};
        start_of_[(uintptr_t)p] = s;
        return true;
    }

    /* p's registration succeeded: its range is mapped from now on */
    void mark_ready(const void *p)
    {
        std::unique_lock<std::shared_mutex> g(mu_);
        const auto it = start_of_.find((uintptr_t)p);
        if (it != start_of_.end())
            by_start_[it->second].ready = true;
    }

    /* [q, q + n) lies inside one range whose registration has succeeded and
     * that its owner has not unregistered: mapped, at the same address */
    bool live(const void *q, size_t n)
    {
        const uintptr_t a = (uintptr_t)q;
        std::shared_lock<std::shared_mutex> g(mu_);
        auto it = by_start_.upper_bound(a);
        if (it == by_start_.begin())
            return false;
        const Range &r = std::prev(it)->second;
        return r.ready && a >= r.p && a + n <= r.end;
    }

    /* Drop the reservation of p.  Returns false when p's registration had
     * failed (mark_failed): the owner's unregister must then not call
     * hipHostUnregister, which could unmap another caller's registration
     * at the same start address. */
    bool release(const void *p)
    {
        std::unique_lock<std::shared_mutex> g(mu_);
        const auto it = start_of_.find((uintptr_t)p);
        if (it == start_of_.end())
            return true;
        by_start_.erase(it->second);
        start_of_.erase(it);
        return failed_.erase((uintptr_t)p) == 0;
    }

    /* A deferred registration of p failed: the range stays reserved (so no
     * other registration can take its pages) until its owner unregisters. */
    void mark_failed(const void *p)
    {
        std::unique_lock<std::shared_mutex> g(mu_);
        if (start_of_.count((uintptr_t)p))
            failed_.insert((uintptr_t)p);
    }

  private:
    static constexpr uintptr_t kPageMask = 4095;
    struct Range {
        uintptr_t e;      /* page-rounded end */
        uintptr_t p, end; /* the registered bytes */
        bool ready;       /* registered (a deferred one: done) */
    };
    std::shared_mutex mu_;
    std::map<uintptr_t, Range> by_start_;                            /* s -> range */
    std::map<uintptr_t, uintptr_t> start_of_;                        /* p -> s */
    std::set<uintptr_t> failed_;                                     /* p       */
};

RangeSet &user_ranges()
{
    static RangeSet *r = new RangeSet;
    return *r;
}

bool user_range_live(const void *p, size_t n)
{
    return user_ranges().live(p, n);
}

/* ec_method_host_register_async: GlusterFS calls the arena hook from
 * __iobuf_pool_add_arena with iobuf_pool->mutex held (iobuf.c:157), so a
 * hipHostRegister there (hundreds of us for a 2-4 MiB arena, and arenas of
 * 1 MiB pages hold only two) would stall every iobuf allocation of the client.
 * The hook only queues the range; one library thread registers it.  Until it
 * has, buffers in the range are pageable to the coder (staged, or coded on the
 * CPU).  Unregistering a range still in the queue drops it; one being
 * registered is waited for first, so the memory is never unmapped while the
 * runtime holds it. */
class RegQueue {
  public:
    int submit(void *p, size_t n)
    {
        if (!user_ranges().reserve(p, n))
            return -EEXIST;
        std::lock_guard<std::mutex> g(mu_);
        if (!started_) {
            std::thread([this] { loop(); }).detach();
            started_ = true;
        }
        q_.push_back({p, n});
        cv_.notify_one();
        return 0;
    }

    /* the unregister half: drop, or wait, then hipHostUnregister */
    int unregister(void *p)
    {
        {
            std::unique_lock<std::mutex> g(mu_);
            for (auto it = q_.begin(); it != q_.end(); ++it)
                if (it->first == p) {
                    q_.erase(it);
                    user_ranges().release(p);
                    return 0;
                }
            done_cv_.wait(g, [&] { return busy_ != p; });
        }
        if (!user_ranges().release(p))
            return 0;      /* its deferred registration failed: nothing mapped */
        const uint64_t t0 = mono_us();
        const hipError_t e = hipHostUnregister(p);
        unreg_us_.fetch_add(mono_us() - t0, std::memory_order_relaxed);
        unregs_.fetch_add(1, std::memory_order_relaxed);
        g_host_gen.fetch_add(1, std::memory_order_release);
        if (e != hipSuccess) {
            set_err("hipHostUnregister", e);
            return -EINVAL;
        }
        return 0;
    }

    void flush()
    {
        std::unique_lock<std::mutex> g(mu_);
        done_cv_.wait(g, [&] { return q_.empty() && busy_ == nullptr; });
    }

    void stats(ecd_pool_stats_t *s) const
    {
        s->deferred_registers = regs_.load();
        s->deferred_register_us = reg_us_.load();
        s->deferred_register_failures = fails_.load();
        s->unregisters = unregs_.load();
        s->unregister_us = unreg_us_.load();
    }

  private:
    void loop()
    {
        std::unique_lock<std::mutex> g(mu_);
        for (;;) {
            cv_.wait(g, [&] { return !q_.empty(); });
            const auto r = q_.front();
            q_.pop_front();
            busy_ = r.first;
            g.unlock();
            const uint64_t t0 = mono_us();
            const hipError_t e = hipHostRegister(r.first, r.second, hipHostRegisterMapped);
            const uint64_t dt = mono_us() - t0;
            if (e != hipSuccess) {
                (void)hipGetLastError();
                user_ranges().mark_failed(r.first);
                if (fails_.fetch_add(1) == 0)
                    fprintf(stderr, "[ec-mi355x] deferred hipHostRegister(%p, %zu) failed: %s; "
                                    "buffers there stay pageable\n",
                            r.first, r.second, hipGetErrorString(e));
            } else {
                user_ranges().mark_ready(r.first);
                g_map_gen.fetch_add(1, std::memory_order_release);
                regs_.fetch_add(1, std::memory_order_relaxed);
                reg_us_.fetch_add(dt, std::memory_order_relaxed);
            }
            g.lock();
            busy_ = nullptr;
            done_cv_.notify_all();
        }
    }

    std::mutex mu_;
    std::condition_variable cv_, done_cv_;
    std::deque<std::pair<void *, size_t>> q_;
    void *busy_ = nullptr;
    bool started_ = false;
    std::atomic<uint64_t> regs_{0}, reg_us_{0}, fails_{0}, unregs_{0}, unreg_us_{0};
};

RegQueue &reg_queue()
{
    static RegQueue *q = new RegQueue;
    return *q;
}

bool pool_owns(const void *p, size_t n)
{
    return buf_pool().owns(p, n);
}

/* a caller registration that would overlap the pool's range: refused (the
 * pool's slabs are registered already, and the rest of its range is
 * reserved for them) */
bool pool_overlaps(const void *p, size_t n)
{
    return buf_pool().overlaps(p, n);
}

/* Per-device pipeline resources (pooled). */
constexpr int kSlots = 2;

/* Events are created with hipEventBlockingSync: a host call that waits for
 * its batch sleeps instead of spinning a core (the client's CPU is shared
 * with the CPU engine and the network stack). */
struct Stage {
    int dev = -1;
    hipStream_t stream = nullptr;
    hipEvent_t done[kSlots] = {};
    uint8_t *pin_in[kSlots] = {}, *pin_out[kSlots] = {}, *pin_grp[kSlots] = {};
    size_t cap_in = 0, cap_out = 0, cap_grp = 0;
};

std::mutex g_pool_mu;
std::vector<Stage *> g_pool[kMaxDev];

/* Staging slots hold at most one batch of the call (never more than its
 * data), so their size follows the call.  They grow to the next power of two:
 * a split call's GPU share (ec_method.c) varies from call to call, and slots
 * sized to each new largest share were freed and re-pinned every time the
 * share set a new high -- unregistering, mapping, faulting in and
 * registering MiBs of memory inside the call (a single stream of pageable
 * 4 MiB heal windows ran 4.2-10.8 GB/s from run to run). */
int grow(uint8_t *(&slot)[kSlots], size_t &cap, size_t want, int dev)
{
    if (want <= cap)
        return 0;
    if (want < ((size_t)1 << 62))
        want = (size_t)1 << (64 - __builtin_clzll((unsigned long long)want - 1));
    for (auto &p : slot)
        if (p) {
            pinned_free(p);
            p = nullptr;
        }
    cap = 0;
    for (auto &p : slot) {
        p = static_cast<uint8_t *>(pinned_alloc(want, device_numa(dev)));
        if (!p) {
            set_err_text("pinned staging allocation of " + std::to_string(want) + " bytes failed");
            return -ENOMEM;
        }
    }
    cap = want;
    return 0;
}

Stage *acquire(int dev)
{
    {
        std::lock_guard<std::mutex> g(g_pool_mu);
        if (!g_pool[dev].empty()) {
            Stage *s = g_pool[dev].back();
            g_pool[dev].pop_back();
            return s;
        }
    }
    Stage *s = new Stage;
    s->dev = dev;
    DeviceGuard dg;
    bool ok = hipSetDevice(g_dev_ids[dev]) == hipSuccess &&
              hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking) == hipSuccess;
    for (int i = 0; ok && i < kSlots; ++i)
        ok = hipEventCreateWithFlags(&s->done[i], hipEventDisableTiming | hipEventBlockingSync) ==
             hipSuccess;
    if (!ok) {
        set_err("staging stream / event creation", hipGetLastError());
        delete s;
        return nullptr;
    }
    return s;
}

void release(Stage *s)
{
    std::lock_guard<std::mutex> g(g_pool_mu);
    g_pool[s->dev].push_back(s);
}

/* One caller buffer region of a batch.  `kptr` is what the kernel uses:
 * the caller's own (mapped) memory, or `pin_off` inside the slot's pinned
 * staging buffer when the caller's memory is pageable. */
struct Region {
    uint8_t *host;
    size_t n;
    bool staged;
    size_t pin_off;
    const std::vector<Seg> *gather = nullptr; /* input: bytes [voff, voff+n) */
    uint64_t voff = 0;                        /* of a virtual input          */
};

struct Batch {
    std::vector<Region> in, out;
    std::function<int(hipStream_t)> launch;
};

/* Run `nbatches` batches: make(b, slot, batch) describes batch b's regions
 * and its launch (which reads kernel addresses from the regions' slots). */
int run_pipeline(Stage *s, uint64_t nbatches,
                 const std::function<int(uint64_t, int, Batch &)> &make)
{
    int rc = 0;
    Batch prev;
    int prev_slot = -1;
    auto ok = [&](hipError_t e) {
        if (e != hipSuccess && rc == 0) {
            set_err("pipeline", e);
            rc = -EIO;
        }
        return rc == 0;
    };
    auto drain = [&]() {
        /* wait for the previous batch and copy its staged outputs back */
        if (prev_slot < 0)
            return;
        if (ok(hipEventSynchronize(s->done[prev_slot]))) {
            std::vector<CopyPool::Piece> pc;
            for (const Region &r : prev.out)
                if (r.staged)
                    add_copy(pc, r.host, s->pin_out[prev_slot] + r.pin_off, r.n);
            g_copy_pool.run(pc);
        }
        prev_slot = -1;
    };
    for (uint64_t b = 0; rc == 0 && b < nbatches; ++b) {
        const int slot = (int)(b % kSlots); /* free: batch b-2 was drained */
        Batch bt;
        if ((rc = make(b, slot, bt)) != 0)
            break;
        std::vector<CopyPool::Piece> pc;
        for (const Region &r : bt.in)
            if (r.gather)
                add_gather(pc, s->pin_in[slot] + r.pin_off, *r.gather, r.voff, r.n);
            else if (r.staged)
                add_copy(pc, s->pin_in[slot] + r.pin_off, r.host, r.n);
        g_copy_pool.run(pc);
        if ((rc = bt.launch(s->stream)) != 0 || !ok(hipEventRecord(s->done[slot], s->stream)))
            break;
        drain();
        prev = std::move(bt);
        prev_slot = slot;
    }
    drain();
    /* wait by a blocking event, not a stream spin: the calling thread then
     * sleeps while the GPU codes, and a GlusterFS client's other threads (or
     * CPU-engine calls beside this one) keep the core */
    if (rc == 0 && ok(hipEventRecord(s->done[0], s->stream)))
        ok(hipEventSynchronize(s->done[0]));
    else
        (void)hipStreamSynchronize(s->stream);
    return rc;
}

/* Kernel address of a region of the current batch. */
inline uint8_t *kaddr(const Stage *s, int slot, const Region &r, bool out)
{
    if (!r.staged)
        return r.host; /* mapped: device address == host address (checked) */
    return (out ? s->pin_out[slot] : s->pin_in[slot]) + r.pin_off;
}

/* ---------------------------------------------------------------- encode */

struct EncodeJob {
    uint32_t k, n;
    const uint8_t *in;      /* whole user input                           */
    const std::vector<Seg> *gather; /* or a virtual input (in == nullptr) */
    uint8_t *const *out;    /* n whole fragment buffers                   */
    const uint8_t *enc_pat; /* generic coefficients (k + n*k bytes)       */
    uint64_t s0, s1;        /* stripe range of this device                */
    bool generic;           /* rows of enc_pat, not the k+n Vandermonde   */
};

/* A 16+4 host-buffer encode launch of 2048 to 8191 stripes (16 to 64 MiB of
 * input) runs as a combine with the encode matrix as its pattern (r06): the
 * double-buffered zero-copy combine stages its inputs in 512-byte pieces
 * through LDS (1 KiB per wave instruction), where the register-resident
 * ec_encode_vander_zc<16, 20> reads 64-byte plane segments.  Pinned calls,
 * same box, alternating (tools/zc_sizes.py, profiles/r06/r06w_zcsizes.log):
 * 16 MiB 739 -> 596-600 us (+23 %), 64 MiB a tie, 256 / 512 MiB 4 % slower
 * (the register encoder's 36.4-36.9 GB/s there is the link's write side),
 * hence the upper bound.  EC_MI355X_ZCENC16=0 keeps the register encoder. */
constexpr uint64_t kZcEnc16MinStripes = 2048, kZcEnc16MaxStripes = 8192;
static bool zcenc16_combine()
{
    static const bool v = [] {
        const char *e = getenv("EC_MI355X_ZCENC16");
        return !(e && *e == '0');
    }();
    return v;
}

int launch_encode(hipStream_t st, const EncodeJob &j, const uint8_t *din, uint8_t *const *outs,
                  uint64_t cnt)
{
    const bool as_combine = j.generic || !ecdk_has_vander(j.k, j.n) ||
                            (j.k > 8 && cnt >= kZcEnc16MinStripes && cnt < kZcEnc16MaxStripes &&
                             j.enc_pat && zcenc16_combine());
    if (!as_combine)                           /* host buffers: the zero-copy kernel */
        return ecdk_encode_vander(st, j.k, j.n, cnt, din, (void *const *)outs, true);
    ecd_combine_desc_t d;
    memset(&d, 0, offsetof(ecd_combine_desc_t, pat));
    d.k = j.k;
    d.rows = j.n;
    d.nstripes = cnt;
    d.in_stride = (uint64_t)j.k * ECD_CHUNK;
    d.out_stride = ECD_CHUNK;
    for (uint32_t p = 0; p < j.k; ++p)
        d.in_base[p] = din + (uint64_t)p * ECD_CHUNK;
    for (uint32_t i = 0; i < j.n; ++i)
        d.out_base[i] = outs[i];
    d.npatterns = 1;
    d.pat_bytes = j.k + j.n * j.k;
    memcpy(d.pat, j.enc_pat, d.pat_bytes);
    return ecdk_combine_host(st, &d);
}

int run_encode_dev(int dev, const EncodeJob &j)
{
    if (j.s1 <= j.s0)
        return 0;
    DeviceGuard dg;
    clear_stale_error();
    HIPCHK(hipSetDevice(g_dev_ids[dev]));
    const uint64_t stripe_in = (uint64_t)j.k * ECD_CHUNK, cnt_all = j.s1 - j.s0;
    const bool in_direct =
        !j.gather && mapped(j.in + j.s0 * stripe_in, cnt_all * stripe_in) != nullptr;
    bool out_direct[ECD_MAX_ROWS], all_direct = in_direct;
    for (uint32_t i = 0; i < j.n; ++i) {
        out_direct[i] = mapped(j.out[i] + j.s0 * ECD_CHUNK, cnt_all * ECD_CHUNK) != nullptr;
        all_direct &= out_direct[i];
    }
    /* fully mapped jobs still run in batches so one launch stays short */
    uint64_t B = std::min<uint64_t>(
        cnt_all, std::max<uint64_t>(1, (all_direct ? 8 : 1) * pipe_batch_bytes() / stripe_in));
    if (!all_direct)
        B = std::min<uint64_t>(cnt_all, staged_batch(B, cnt_all, stripe_in, 1));
    Stage *s = acquire(dev);
    if (!s)
        return -EIO;
    int rc = grow(s->pin_in, s->cap_in, in_direct ? 0 : B * stripe_in, dev);
    if (rc == 0)
        rc = grow(s->pin_out, s->cap_out, all_direct ? 0 : B * j.n * ECD_CHUNK, dev);
    const uint64_t nb = (cnt_all + B - 1) / B;
    if (rc == 0)
        rc = run_pipeline(s, nb, [&](uint64_t b, int slot, Batch &bt) {
            const uint64_t a = j.s0 + b * B, cnt = std::min(B, j.s1 - a);
            if (j.gather)
                bt.in.push_back({nullptr, cnt * stripe_in, true, 0, j.gather, a * stripe_in});
            else
                bt.in.push_back({const_cast<uint8_t *>(j.in) + a * stripe_in, cnt * stripe_in,
                                 !in_direct, 0});
            for (uint32_t i = 0; i < j.n; ++i)
                bt.out.push_back({j.out[i] + a * ECD_CHUNK, cnt * ECD_CHUNK, !out_direct[i],
                                  (size_t)i * B * ECD_CHUNK});
            const uint8_t *din = kaddr(s, slot, bt.in[0], false);
            std::vector<uint8_t *> outs(j.n);
            for (uint32_t i = 0; i < j.n; ++i)
                outs[i] = kaddr(s, slot, bt.out[i], true);
            bt.launch = [&j, din, outs, cnt](hipStream_t st) {
                return launch_encode(st, j, din, outs.data(), cnt);
            };
            return 0;
        });
    release(s);
    return rc;
}

/* ---------------------------------------------------------------- decode */

struct DecodeJob {
    uint32_t k, rows, nfrags, npatterns, group_shift;
    const uint8_t *const *frags;
    uint8_t *out;
    uint8_t *const *outs;
    const uint8_t *pats;
    const uint8_t *group_pattern;
    uint64_t s0, s1;
};

int run_decode_dev(int dev, const DecodeJob &j)
{
    if (j.s1 <= j.s0)
        return 0;
    DeviceGuard dg;
    clear_stale_error();
    HIPCHK(hipSetDevice(g_dev_ids[dev]));
    const uint64_t out_stripe = (uint64_t)j.rows * ECD_CHUNK, cnt_all = j.s1 - j.s0;
    bool in_direct[ECD_MAX_ROWS] = {}, out_direct[ECD_MAX_ROWS] = {}, all_direct = true;
    bool any_in_staged = false;
    for (uint32_t f = 0; f < j.nfrags; ++f)
        if (j.frags[f]) {
            in_direct[f] = mapped(j.frags[f] + j.s0 * ECD_CHUNK, cnt_all * ECD_CHUNK) != nullptr;
            all_direct &= in_direct[f];
            any_in_staged |= !in_direct[f];
        }
    if (j.outs) {
        for (uint32_t r = 0; r < j.rows; ++r) {
            out_direct[r] = mapped(j.outs[r] + j.s0 * ECD_CHUNK, cnt_all * ECD_CHUNK) != nullptr;
            all_direct &= out_direct[r];
        }
    } else {
        out_direct[0] = mapped(j.out + j.s0 * out_stripe, cnt_all * out_stripe) != nullptr;
        all_direct &= out_direct[0];
    }
    uint64_t B = std::max<uint64_t>(
        1, (all_direct ? 8 : 1) * pipe_batch_bytes() / ((uint64_t)j.nfrags * ECD_CHUNK));
    const uint64_t grp = j.group_pattern ? (1ull << j.group_shift) : 1;
    if (!all_direct)
        B = staged_batch(B, cnt_all, (uint64_t)j.nfrags * ECD_CHUNK, 1);
    if (j.group_pattern)
        B = std::max<uint64_t>(grp, B / grp * grp);
    /* batches start at multiples of B (whole groups), but the staging slots
     * never hold more than the data: Bs = stripes per slot */
    const uint64_t Bs = std::min<uint64_t>(B, cnt_all);
    Stage *s = acquire(dev);
    if (!s)
        return -EIO;
    int rc = grow(s->pin_in, s->cap_in, any_in_staged ? Bs * j.nfrags * ECD_CHUNK : 0, dev);
    if (rc == 0)
        rc = grow(s->pin_out, s->cap_out, all_direct ? 0 : Bs * out_stripe, dev);
    if (rc == 0)
        rc = grow(s->pin_grp, s->cap_grp, j.group_pattern ? (Bs + grp - 1) / grp + 1 : 0, dev);
    const uint64_t nb = (cnt_all + B - 1) / B;
    if (rc == 0)
        rc = run_pipeline(s, nb, [&](uint64_t b, int slot, Batch &bt) {
            const uint64_t a = j.s0 + b * B, cnt = std::min(B, j.s1 - a);
            auto d = std::make_shared<ecd_combine_desc_t>();
            memset(d.get(), 0, offsetof(ecd_combine_desc_t, pat));
            d->k = j.k;
            d->rows = j.rows;
            d->nstripes = cnt;
            d->in_stride = ECD_CHUNK;
            for (uint32_t f = 0; f < j.nfrags; ++f) {
                if (!j.frags[f])
                    continue;
                bt.in.push_back({const_cast<uint8_t *>(j.frags[f]) + a * ECD_CHUNK,
                                 cnt * ECD_CHUNK, !in_direct[f], (size_t)f * Bs * ECD_CHUNK});
                d->in_base[f] = kaddr(s, slot, bt.in.back(), false);
            }
            if (j.outs) {
                d->out_stride = ECD_CHUNK;
                for (uint32_t r = 0; r < j.rows; ++r) {
                    bt.out.push_back({j.outs[r] + a * ECD_CHUNK, cnt * ECD_CHUNK,
                                      !out_direct[r], (size_t)r * Bs * ECD_CHUNK});
                    d->out_base[r] = kaddr(s, slot, bt.out.back(), true);
                }
            } else {
                d->out_stride = out_stripe;
                bt.out.push_back({j.out + a * out_stripe, cnt * out_stripe, !out_direct[0], 0});
                uint8_t *o = kaddr(s, slot, bt.out.back(), true);
                for (uint32_t r = 0; r < j.rows; ++r)
                    d->out_base[r] = o + (uint64_t)r * ECD_CHUNK;
            }
            d->npatterns = j.npatterns;
            d->pat_bytes = j.k + j.rows * j.k;
            if ((size_t)j.npatterns * d->pat_bytes <= ECD_MAX_PAT_BYTES)
                memcpy(d->pat, j.pats, (size_t)j.npatterns * d->pat_bytes);
            else
                d->pat_ext = j.pats;   /* read at launch, inside this call */
            if (j.group_pattern) {
                /* a is a multiple of the group size (B is, and s0 is aligned);
                 * the kernel reads the group-map slice from the slot's pinned
                 * buffer (free: its previous batch has been drained) */
                const uint64_t g0 = a >> j.group_shift;
                const uint64_t gn = (cnt + grp - 1) >> j.group_shift;
                memcpy(s->pin_grp[slot], j.group_pattern + g0, gn);
                d->group_pattern = s->pin_grp[slot];
                d->group_shift = j.group_shift;
            }
            bt.launch = [d](hipStream_t st) { return ecdk_combine_host(st, d.get()); };
            return 0;
        });
    release(s);
    return rc;
}

/* ------------------------------------------------ device placement */

/* GlusterFS codes one fop per call on many client threads: 128 KiB
 * FUSE / write-behind writes (fuse-bridge.c:5179, write-behind.c:3198) up
 * to 4 MiB self-heal blocks.  Splitting such a call
 * across all GPUs of the node multiplies its fixed cost (a launch and a
 * synchronisation per device, ~20 us) for PCIe time it does not save, so a
 * call below split_min_bytes() runs whole on the device with the fewest
 * bytes in flight; concurrent calls spread over the devices and overlap on
 * per-call streams.  (Coalescing concurrent calls into one segmented launch
 * was measured slower on MI355X -- see DESIGN.md, profiles/smallcalls_r01_*.) */
uint64_t split_min_bytes()
{
    static const uint64_t v = [] {
        const char *e = getenv("EC_SPLIT_MIN_MB");
        const long mb = e ? atol(e) : 64;
        return (uint64_t)(mb >= 0 && mb <= 65536 ? mb : 64) << 20;
    }();
    return v;
}

std::atomic<uint64_t> g_inflight[kMaxDev];

/* Device for a whole call: fewest bytes in flight, rotating on ties. */
int pick_device(uint64_t bytes)
{
    static std::atomic<unsigned> rr{0};
    const unsigned start = rr.fetch_add(1);
    int best = g_host_devs[start % g_nhost];
    uint64_t lo = g_inflight[best].load();
    for (int i = 1; i < g_nhost; ++i) {
        const int d = g_host_devs[(start + i) % g_nhost];
        const uint64_t v = g_inflight[d].load();
        if (v < lo) {
            lo = v;
            best = d;
        }
    }
    g_inflight[best].fetch_add(bytes);
    return best;
}

/* Test hook (ec_method_inject_device_faults): the next N host-buffer
 * submissions fail with -EIO before touching a device. */
std::atomic<uint32_t> g_inject_faults{0};

bool take_injected_fault()
{
    uint32_t v = g_inject_faults.load();
    while (v > 0 && !g_inject_faults.compare_exchange_weak(v, v - 1))
        ;
    if (v > 0) {
        set_err_text("injected device fault (ec_method_inject_device_faults)");
        return true;
    }
    return false;
}

/* Run fn(dev, s0, s1) over a stripe-range partition; `align` keeps every
 * range boundary a multiple of it (pattern groups).  Bytes in flight are
 * tracked per device for placement and for the CPU crossover
 * (ecd_host_inflight). */
template <typename F>
int partition(int ndev, uint64_t nstripes, uint64_t align, uint64_t bytes, F fn)
{
    if (g_ndev == 0)
        return -ENODEV;
    if (take_injected_fault())
        return -EIO;
    if (ndev <= 0 || ndev > g_nhost)
        ndev = g_nhost;
    if (ndev == 1 || bytes < split_min_bytes()) {
        const int d = ndev == 1 ? g_host_devs[0] : pick_device(bytes);
        if (ndev == 1)
            g_inflight[d].fetch_add(bytes);
        const int rc = fn(d, 0, nstripes);
        g_inflight[d].fetch_sub(bytes);
        return rc;
    }
    const uint64_t units = (nstripes + align - 1) / align;
    if ((uint64_t)ndev > units)
        ndev = (int)std::max<uint64_t>(1, units);
    std::vector<int> rcs(ndev, 0);
    std::vector<std::string> errs(ndev);   /* a worker's failure, for the caller */
    std::vector<uint64_t> share(ndev, 0);
    std::vector<std::thread> th;
    for (int d = 0; d < ndev; ++d) {
        const uint64_t s0 = std::min(nstripes, units * d / ndev * align);
        const uint64_t s1 = std::min(nstripes, units * (d + 1) / ndev * align);
        const int dev = g_host_devs[d];
        share[d] = nstripes ? bytes / nstripes * (s1 - s0) : 0;
        g_inflight[dev].fetch_add(share[d]);
        if (d == ndev - 1)
            rcs[d] = fn(dev, s0, s1);
        else
            th.emplace_back([&, d, dev, s0, s1] {
                const uint64_t seq = t_err_seq;
                rcs[d] = fn(dev, s0, s1);
                if (rcs[d] && t_err_seq != seq)
                    errs[d] = t_err;
            });
    }
    for (auto &t : th)
        t.join();
    for (int d = 0; d < ndev; ++d)
        g_inflight[g_host_devs[d]].fetch_sub(share[d]);
    for (int d = 0; d < ndev; ++d)
        if (rcs[d]) {
            if (!errs[d].empty())
                set_err_text("device " + std::to_string(g_host_devs[d]) + ": " + errs[d]);
            return rcs[d];
        }
    return 0;
}

} // namespace

extern "C" {

int ecd_device_count(void)
{
    std::call_once(g_dev_once, discover);
    return g_ndev;
}

const char *ecd_last_error(void)
{
    if (t_err.empty() && g_ndev == 0)
        return g_discover_err.c_str();   /* written once, before any call returns */
    return t_err.c_str();
}

uint64_t ecd_error_seq(void)
{
    return t_err_seq;
}

void ecd_set_error(const char *text)
{
    set_err_text(text ? text : "");
}

int ecd_hip_fail(const char *what, int hip_error)
{
    set_err(what, (hipError_t)hip_error);
    return -EIO;
}

int ecd_has_vander(uint32_t k, uint32_t n)
{
    return ecdk_has_vander(k, n);
}

int ecd_encode_vander(int device, void *stream, uint32_t k, uint32_t n, uint64_t nstripes,
                      const void *in, void *const *out)
{
    if (ecd_device_count() <= device || device < 0)
        return -ENODEV;
    DeviceGuard dg;
    clear_stale_error();
    HIPCHK(hipSetDevice(g_dev_ids[device]));
    return ecdk_encode_vander(pick_stream(stream), k, n, nstripes, in, out);
}

int ecd_combine(int device, void *stream, const ecd_combine_desc_t *d)
{
    if (ecd_device_count() <= device || device < 0)
        return -ENODEV;
    DeviceGuard dg;
    clear_stale_error();
    HIPCHK(hipSetDevice(g_dev_ids[device]));
    return ecdk_combine(pick_stream(stream), d);
}

int ecd_sync(int device, void *stream)
{
    if (ecd_device_count() <= device || device < 0)
        return -ENODEV;
    DeviceGuard dg;
    HIPCHK(hipSetDevice(g_dev_ids[device]));
    HIPCHK(hipStreamSynchronize(pick_stream(stream)));
    return 0;
}

static int encode_host(int ndev, uint32_t k, uint32_t n, uint64_t nstripes, const void *in,
                       const std::vector<Seg> *gather, void *const *out, const uint8_t *enc_pat,
                       bool generic = false)
{
    if (ecd_device_count() == 0)
        return -ENODEV;
    EncodeJob base;
    base.generic = generic;
    base.k = k;
    base.n = n;
    base.in = static_cast<const uint8_t *>(in);
    base.gather = gather;
    base.out = reinterpret_cast<uint8_t *const *>(out);
    base.enc_pat = enc_pat;
    return partition(ndev, nstripes, 1, nstripes * ECD_CHUNK * (k + n),
                     [&](int d, uint64_t s0, uint64_t s1) {
        EncodeJob j = base;
        j.s0 = s0;
        j.s1 = s1;
        return run_encode_dev(d, j);
    });
}

int ecd_encode_host(int ndev, uint32_t k, uint32_t n, uint64_t nstripes, const void *in,
                    void *const *out, const uint8_t *enc_pat)
{
    return encode_host(ndev, k, n, nstripes, in, nullptr, out, enc_pat);
}

int ecd_encode_host_rows(int ndev, uint32_t k, uint32_t rows, uint64_t nstripes, const void *in,
                         void *const *out, const uint8_t *pat)
{
    if (!pat || rows == 0 || rows > ECD_MAX_ROWS || k == 0 || k > ECD_MAX_K)
        return -EINVAL;
    return encode_host(ndev, k, rows, nstripes, in, nullptr, out, pat, true);
}

int ecd_encode_host_gather(int ndev, uint32_t k, uint32_t n, uint64_t nstripes, uint32_t nsegs,
                           const void *const *seg_ptr, const uint64_t *seg_len,
                           void *const *out, const uint8_t *enc_pat)
{
    std::vector<Seg> segs;
    uint64_t total = 0;
    for (uint32_t i = 0; i < nsegs; ++i) {
        segs.push_back({static_cast<const uint8_t *>(seg_ptr[i]), seg_len[i]});
        total += seg_len[i];
    }
    if (total != nstripes * k * ECD_CHUNK)
        return -EINVAL;
    return encode_host(ndev, k, n, nstripes, nullptr, &segs, out, enc_pat);
}

int ecd_writev_encode_device(int device, void *stream, uint32_t k, uint32_t n, uint64_t head,
                             uint64_t user_size, const void *user, const void *old_head,
                             const void *old_tail, void *const *out, const uint8_t *enc_pat)
{
    if (ecd_device_count() <= device || device < 0)
        return -ENODEV;
    const uint64_t S = (uint64_t)k * ECD_CHUNK;
    if (head >= S || user_size == 0 || !user)
        return -EINVAL;
    const uint64_t b1 = head, b2 = head + user_size, nst = (b2 + S - 1) / S;
    const uint8_t *u = static_cast<const uint8_t *>(user);
    const uint8_t *hs = static_cast<const uint8_t *>(old_head);
    const uint8_t *ts = static_cast<const uint8_t *>(old_tail);
    /* one stripe: its old content (either pointer) fills both ends, as
     * ec_merge_stripe_head_locked does (ec-inode-write.c:1886-1895) */
    if (nst == 1) {
        hs = hs ? hs : ts;
        ts = hs ? hs + b2 : nullptr;
    } else if (ts) {
        ts += b2 - (nst - 1) * S; /* ec_merge_stripe_tail_locked, :1898-1908 */
    }
    DeviceGuard dg;
    clear_stale_error();
    HIPCHK(hipSetDevice(g_dev_ids[device]));
    hipStream_t st = pick_stream(stream);
    const bool fused = ecdk_has_vander(k, n);
    const uint64_t scratch = fused ? (nst == 1 ? 1 : 2) * S : nst * S;
    uint8_t *buf = nullptr;
    HIPCHK(hipMallocAsync(reinterpret_cast<void **>(&buf), scratch, st));
    int rc;
    if (fused) {
        rc = ecdk_rmw_gather(st, hs, u, ts, b1, b2, 0, S, buf);
        if (rc == 0 && nst > 1)
            rc = ecdk_rmw_gather(st, hs, u, ts, b1, b2, (nst - 1) * S, S, buf + S);
        if (rc == 0)
            rc = ecdk_encode_vander_rmw(st, k, n, nst, buf, u - head, out);
    } else {
        rc = ecdk_rmw_gather(st, hs, u, ts, b1, b2, 0, nst * S, buf);
        if (rc == 0) {
            EncodeJob j{};
            j.k = k;
            j.n = n;
            j.enc_pat = enc_pat;
            rc = launch_encode(st, j, buf, reinterpret_cast<uint8_t *const *>(out), nst);
        }
    }
    const hipError_t fe = hipFreeAsync(buf, st);
    if (rc == 0 && fe != hipSuccess) {
        set_err("hipFreeAsync", fe);
        rc = -EIO;
    }
    return rc;
}

int ecd_decode_host(int ndev, uint32_t k, uint32_t rows, uint64_t nstripes, uint32_t nfrags,
                    const void *const *frags, void *out, void *const *outs, uint32_t npatterns,
                    const uint8_t *pats, const uint8_t *group_pattern, uint32_t group_shift)
{
    if (ecd_device_count() == 0)
        return -ENODEV;
    if (nfrags == 0 || nfrags > ECD_MAX_ROWS || k == 0 || k > ECD_MAX_K || rows == 0 ||
        rows > ECD_MAX_ROWS || npatterns == 0 ||
        npatterns > ECD_MAX_PATTERNS)
        return -EINVAL;
    if (group_pattern && group_shift > 40)
        return -EINVAL;
    DecodeJob base;
    base.k = k;
    base.rows = rows;
    base.nfrags = nfrags;
    base.npatterns = npatterns;
    base.group_shift = group_shift;
    base.frags = reinterpret_cast<const uint8_t *const *>(frags);
    base.out = static_cast<uint8_t *>(out);
    base.outs = reinterpret_cast<uint8_t *const *>(outs);
    base.pats = pats;
    base.group_pattern = group_pattern;
    const uint64_t align = group_pattern ? (1ull << group_shift) : 1;
    return partition(ndev, nstripes, align, nstripes * ECD_CHUNK * (nfrags + rows),
                     [&](int d, uint64_t s0, uint64_t s1) {
        DecodeJob j = base;
        j.s0 = s0;
        j.s1 = s1;
        return run_decode_dev(d, j);
    });
}

uint64_t ecd_host_inflight(void)
{
    if (ecd_device_count() == 0)
        return UINT64_MAX;
    uint64_t lo = UINT64_MAX;
    for (int i = 0; i < g_nhost; ++i)
        lo = std::min<uint64_t>(lo, g_inflight[g_host_devs[i]].load());
    return lo;
}

int ecd_host_mapped(const void *p, size_t n)
{
    return ecd_device_count() > 0 && mapped(p, n) != nullptr;
}

void ecd_inject_faults(uint32_t n)
{
    g_inject_faults.store(n);
}

/* Pages already found to be plain host memory, per thread (direct-mapped).
 * hipPointerGetAttributes serialises in the HIP runtime -- 0.07 us from one
 * thread, ~11 us per call with 16 threads on pageable memory
 * (tools/kbench/ptrq.hip) -- and a host call checks every buffer, so
 * GlusterFS's recycled iobufs are looked up here first.  Only pages the
 * runtime does not know at all (pageable malloc / mmap memory: the query
 * reports hipMemoryTypeUnregistered, or fails) are cached.  Memory the
 * runtime allocated -- device buffers, and pinned host buffers, which come
 * from the same GPU virtual range -- is queried every time: once freed, its
 * addresses are handed out again, and a pinned page cached as "host" came
 * back as a torch device tensor in the GPU tests (-EINVAL on a
 * device-resident encode).
 * An entry also expires: a pageable buffer can be unmapped and its range
 * handed to a later device allocation (the thunk maps GPU virtual memory
 * with mmap too), and a stale "host" verdict would send device memory down
 * the CPU path.  So every entry carries the time it was made (coarse
 * monotonic clock, vDSO: ~20 ns) and the generation of the library's own
 * frees (ecd_host_free / unregister / staging growth bump g_host_gen); it
 * is trusted for EC_HOSTPAGE_MS (default 20 ms) -- at most ~50 queries per
 * second per page and thread, against one per call without the cache. */
struct HostPage {
    uintptr_t pg;        /* page number + 1; 0 = empty */
    uint64_t until_ns;
    uint32_t gen;
};
static thread_local HostPage t_host_page[256];

static uint64_t hostpage_ttl_ns()
{
    static const uint64_t v = [] {
        const char *e = getenv("EC_HOSTPAGE_MS");
        const long ms = e ? atol(e) : 20;
        return (uint64_t)(ms >= 0 && ms <= 10000 ? ms : 20) * 1000000ull;
    }();
    return v;
}

static uint64_t coarse_ns()
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC_COARSE, &ts);
    return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}

int ecd_ptr_device(const void *p)
{
    if (!p || ecd_device_count() == 0 || buf_pool().owns(p, 1))
        return -1;
    const uintptr_t pg = (uintptr_t)p >> 12;
    /* Fibonacci hashing: iobufs sit at regular page strides (65 pages for
     * 256 KiB mmap'ed buffers), which a xor-fold of the page number mapped
     * onto a few slots (~4 misses per decode call, 16 threads) */
    HostPage &slot = t_host_page[(uint64_t)(pg * 0x9E3779B97F4A7C15ull) >> 56];
    const uint32_t gen = g_host_gen.load(std::memory_order_acquire);
    const uint64_t now = hostpage_ttl_ns() ? coarse_ns() : 0;
    if (slot.pg == pg + 1 && slot.gen == gen && now < slot.until_ns)
        return -1;
    hipPointerAttribute_t a;
    g_ptr_queries.fetch_add(1, std::memory_order_relaxed);
    const HostPage fresh = {pg + 1, now + hostpage_ttl_ns(), gen};
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        slot = fresh;
        return -1;
    }
    if (a.type != hipMemoryTypeDevice) {
        if (a.type == hipMemoryTypeUnregistered)
            slot = fresh;
        return -1;
    }
    for (int i = 0; i < g_ndev; ++i)
        if (g_dev_ids[i] == a.device)
            return i;
    return -1;
}

/* On the NUMA node of the first host-buffer device (EC_MI355X_HOST_DEVICES:
 * one rank per GPU gets its own GPU's node). */
void *ecd_host_alloc(size_t bytes)
{
    if (ecd_device_count() == 0)
        return nullptr;
    return pinned_alloc(bytes, device_numa(g_host_devs[0]));
}

void ecd_host_free(void *p)
{
    pinned_free(p);
}

int ecd_device_numa_node(int device)
{
    if (ecd_device_count() <= device || device < 0)
        return -ENODEV;
    return device_numa(device);
}

int ecd_copy_threads(void)
{
    return copy_threads();
}

int ecd_host_register(void *p, size_t bytes)
{
    if (ecd_device_count() == 0)
        return -ENODEV;
    if (!p || bytes == 0)
        return -EINVAL;
    if (pool_overlaps(p, bytes) || !user_ranges().reserve(p, bytes)) {
        set_err("hipHostRegister", hipErrorHostMemoryAlreadyRegistered);
        return -EEXIST;
    }
    const hipError_t e = hipHostRegister(p, bytes, hipHostRegisterMapped);
    if (e != hipSuccess) {
        user_ranges().release(p);
        set_err("hipHostRegister", e);
        return e == hipErrorHostMemoryAlreadyRegistered ? -EEXIST : -ENOMEM;
    }
    user_ranges().mark_ready(p);
    g_map_gen.fetch_add(1, std::memory_order_release);
    return 0;
}

int ecd_host_unregister(void *p)
{
    if (ecd_device_count() == 0)
        return -ENODEV;
    if (!p)
        return -EINVAL;
    return reg_queue().unregister(p);
}

int ecd_host_register_async(void *p, size_t bytes)
{
    if (ecd_device_count() == 0)
        return -ENODEV;
    if (!p || bytes == 0)
        return -EINVAL;
    if (pool_overlaps(p, bytes)) {
        set_err("hipHostRegister (deferred)", hipErrorHostMemoryAlreadyRegistered);
        return -EEXIST;
    }
    return reg_queue().submit(p, bytes);
}

void ecd_host_register_flush(void)
{
    if (ecd_device_count() > 0)
        reg_queue().flush();
}

void *ecd_buffer_get(size_t bytes)
{
    if (ecd_device_count() == 0)
        return nullptr;
    return buf_pool().get(bytes);
}

int ecd_buffer_put(void *p)
{
    return p && buf_pool().put(p) ? 1 : 0;
}

void ecd_pool_stats(ecd_pool_stats_t *s)
{
    memset(s, 0, sizeof(*s));
    buf_pool().stats(s);
    reg_queue().stats(s);
}

} /* extern "C" */
