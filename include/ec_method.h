/*
 * ec_method.h -- drop-in C ABI of the MI355X (gfx950) disperse coder.
 *
 * This library (glusterfs_amd/lib/libec_mi355x.so) replaces the coding layer
 * of GlusterFS's disperse translator: ec-method.c, ec-code*.c, ec-galois.c and
 * ec-gf8.c in xlators/cluster/ec/src.  The five ec_method_* prototypes below
 * are exactly those of ec-method.h:31-46, with the same argument meaning,
 * return conventions (0 / negative errno) and data layout (512-byte chunks of
 * 8 bit-planes x 64 bytes, EC_METHOD_CHUNK_SIZE), so ec.c, ec-inode-write.c,
 * ec-inode-read.c and ec-heal.c link against it unchanged.
 *
 * Data buffers may be host memory (pageable or pinned) or MI355X device
 * memory; host data crosses PCIe inside the call, or is coded on the calling
 * thread by the library's CPU engine: on nodes without a gfx950 device, for
 * cpu-extensions = none / x64 / sse / avx, for host calls below the
 * CPU/GPU crossover or while every GPU is saturated, and as the fallback
 * when a device submission fails (the reference coder never fails).
 */
#ifndef EC_MI355X_EC_METHOD_H
#define EC_MI355X_EC_METHOD_H

#include <pthread.h>
#include <stddef.h>
#include <stdint.h>
#include <sys/uio.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Constants of ec-method.h:17-29. */
#define EC_GF_BITS 8
#define EC_GF_MOD 0x11D
#define EC_GF_SIZE (1 << EC_GF_BITS)
#define EC_METHOD_MAX_FRAGMENTS 16
#define EC_METHOD_MAX_NODES (EC_GF_SIZE - 1)
#define EC_METHOD_WORD_SIZE 64
#define EC_METHOD_CHUNK_SIZE (EC_METHOD_WORD_SIZE * EC_GF_BITS)

/* Largest brick count the library accepts (EC_MAX_NODES, ec.h:27-32). */
#define EC_MI355X_MAX_NODES 31

#ifndef __EC_TYPES_H__
/* On-disk coding parameters stored in each fragment file's
 * trusted.ec.config xattr (ec-types.h:145-152). */
typedef struct _ec_config ec_config_t;
struct _ec_config {
    uint32_t version;
    uint8_t algorithm;
    uint8_t gf_word_size;
    uint8_t bricks;
    uint8_t redundancy;
    uint32_t chunk_size;
};

/* Standalone declarations.  Inside GlusterFS, ec-types.h (included first)
 * provides the real definitions; the layout below is byte-compatible with
 * ec-types.h:549-562 (sizeof == 120 on LP64, same field offsets), which is
 * the only storage the library uses: the caller embeds the list by value in
 * ec_t (ec-types.h:677). */
typedef struct _xlator xlator_t;
typedef struct _ec_matrix_list ec_matrix_list_t;

struct _ec_matrix_list {
    void *lru[2];           /* struct list_head lru           @0   */
    pthread_mutex_t lock;   /* gf_lock_t lock                 @16  */
    uint32_t columns;       /* k                              @56  */
    uint32_t rows;          /* n                              @60  */
    uint32_t max;           /* decode-matrix cache capacity   @64  */
    uint32_t count;         /* cached decode matrices         @68  */
    uint32_t stripe;        /* EC_METHOD_CHUNK_SIZE * k       @72  */
    void *pool;             /* struct mem_pool *pool          @80  */
    void *gf;               /* ec_gf_t *gf                    @88  */
    void *code;             /* ec_code_t *code                @96  */
    void *encode;           /* ec_matrix_t *encode            @104 */
    void **objects;         /* ec_matrix_t **objects          @112 */
};
#endif

/* ------------------------------------------------------------------------
 * Drop-in entry points (ec-method.h:31-46).
 * --------------------------------------------------------------------- */

/* Replaces ec-method.c:299-353, called from ec.c:837.  columns = k data
 * fragments, rows = n bricks, max = decode matrix cache size (2n in ec.c),
 * gen = the disperse.cpu-extensions value (ec.c:1786-1794) or "hip":
 *   auto, hip        gfx950 engine when a device is visible (with the CPU
 *                    engine for small calls and as the fallback), else CPU
 *   none, x64, sse   CPU engine, base x86-64 code
 *   avx              CPU engine, best AVX level of the host (AVX2/AVX-512)
 * Unknown values warn and act as auto (ec-code.c:1007-1013).  Returns 0,
 * -EINVAL (bad geometry) or -ENOMEM. */
int32_t ec_method_init(xlator_t *xl, ec_matrix_list_t *list, uint32_t columns,
                       uint32_t rows, uint32_t max, const char *gen);

/* Replaces ec-method.c:355-383 (ec.c:198).  Safe on a list whose init failed. */
void ec_method_fini(ec_matrix_list_t *list);

/* Replaces ec-method.c:385-391 (ec.c:293): a no-op returning 0, as in the
 * reference (changing the engine needs a remount there too). */
int32_t ec_method_update(xlator_t *xl, ec_matrix_list_t *list, const char *gen);

/* Replaces ec-method.c:393-408 (ec-inode-write.c:2136).  size: user bytes,
 * a multiple of EC_METHOD_CHUNK_SIZE * k.  out[i] receives size/k bytes of
 * fragment i and, as in the reference, each out[i] is advanced by size/k.
 * Like the reference it cannot fail on host buffers: a device error is redone
 * by the CPU engine.  Invalid arguments, or a fault with caller-provided
 * device buffers, abort with a diagnostic (ec_method_encode_batch returns an
 * error code instead). */
void ec_method_encode(ec_matrix_list_t *list, uint64_t size, void *in, void **out);

/* Replaces ec-method.c:410-433 (ec-inode-read.c:1196).  size: bytes per
 * fragment (multiple of EC_METHOD_CHUNK_SIZE).  mask: the k bricks used;
 * rows[p] = brick index + 1 of in[p], ascending.  out: size * k bytes.
 * Returns 0, -EINVAL, -ENOMEM or -EIO. */
int32_t ec_method_decode(ec_matrix_list_t *list, uint64_t size, uintptr_t mask,
                         uint32_t *rows, void **in, void *out);

/* ------------------------------------------------------------------------
 * Batched / device-resident entry points (new).
 * --------------------------------------------------------------------- */

/* Encode nstripes stripes; in = nstripes*k*512 bytes, out[i] = nstripes*512
 * bytes.  Host buffers are split by stripe range across all visible MI355X
 * devices with overlapped PCIe transfers; device buffers run on device 0.
 * Does not modify out[].  Returns 0 or -errno. */
int32_t ec_method_encode_batch(ec_matrix_list_t *list, uint64_t nstripes,
                               const void *in, void *const *out);

/* Decode nstripes stripes with one mask (as ec_method_decode, sizes in
 * stripes).  Returns 0 or -errno. */
int32_t ec_method_decode_batch(ec_matrix_list_t *list, uint64_t nstripes,
                               uintptr_t mask, const uint32_t *rows,
                               const void *const *in, void *out);

/* Self-heal style reconstruction with mixed erasure patterns: frags[0..n)
 * are all n fragment buffers (nstripes*512 bytes each; entries of bricks no
 * group reads may be NULL), group g = stripes [g*group_stripes,
 * (g+1)*group_stripes) is decoded from the k bricks in group_masks[g].
 * group_stripes is a power of two (groups of 1, 2 or 4 stripes are sorted
 * by pattern into 8-stripe tiles on the device first).
 * out = nstripes*k*512 bytes.
 * Up to 256 distinct masks per call (-E2BIG beyond). */
int32_t ec_method_decode_mixed(ec_matrix_list_t *list, uint64_t nstripes,
                               uint64_t group_stripes, const uintptr_t *group_masks,
                               const void *const *frags, void *out);

/* Encode of selected fragments: ec_method_encode restricted to the fragments
 * whose bit i is set in row_mask (bit i = brick i, the numbering of decode
 * masks).  A heal write goes to the bad bricks only (ec-heal.c:327-329:
 * ec_writev with heal->bad) and a degraded write skips the bricks that are
 * down, yet ec_writev_encode (ec-inode-write.c:2125-2138) computes all n
 * fragments; this computes |row_mask| of them, i.e. writes m*size/k instead
 * of n*size/k bytes and does m/n of the arithmetic.  out[] is indexed by
 * brick as in ec_method_encode: out[i] is read and advanced by size/k only for
 * the bits of row_mask (the others may be NULL and are left alone).  A full
 * row_mask is ec_method_encode, an empty one a no-op.  Cannot fail on host buffers; invalid
 * arguments abort with a diagnostic, as ec_method_encode. */
void ec_method_encode_rows(ec_matrix_list_t *list, uint64_t size, void *in,
                           uintptr_t row_mask, void **out);

/* Fused heal: regenerate the fragments of the bricks
 * in `target_mask` straight from the k fragments in `mask`, without
 * materialising the decoded data: out[j] (nstripes*512 bytes) is the fragment
 * of the j-th set bit of target_mask.  Returns 0 or -errno. */
int32_t ec_method_heal(ec_matrix_list_t *list, uint64_t nstripes, uintptr_t mask,
                       const void *const *in, uintptr_t target_mask,
                       void *const *out);

/* Partial-stripe write: the read-modify-write of
 * ec_writev_start (ec-inode-write.c:1987-2085) fused with ec_writev_encode.
 * The write's user data is the iovec list iov[0..count) (as the writev fop
 * carries it) and starts `head` bytes into its first stripe (fop->head =
 * offset % stripe, ec-inode-write.c:1833).  The encoded range is the
 * padded buffer of ec_writev_prepare_buffers (:1825-1848):
 *   bytes [0, head)                 old_head[0, head)      (head merge, :1883)
 *   bytes [head, head + user bytes) the user data
 *   the rest of the last stripe     the same bytes of old_tail (tail merge,
 *                                   :1898-1908)
 * old_head / old_tail are the current (decoded) contents of the first / last
 * stripe -- from the stripe cache or a read -- or NULL beyond end of file
 * (zeros, :2007-2008).  When the write lies in one stripe its old content
 * fills both ends (old_head, or old_tail when old_head is NULL).  out[i]
 * receives ceil((head + user bytes) / (512k)) chunks of fragment i.  The
 * merge happens in the staging copy for host buffers and inside the
 * kernel for device buffers (count must be 1 there); the interior of the
 * write is never copied separately.  Returns 0 or -errno. */
int32_t ec_method_writev_encode(ec_matrix_list_t *list, uint64_t head, const struct iovec *iov,
                                int count, const void *old_head, const void *old_tail,
                                void *const *out);

/* Device-resident, asynchronous variants for callers that keep stripes in
 * MI355X memory: all buffers are device pointers on `device` (index among
 * the visible gfx950 devices), work is queued on `stream` (a hipStream_t;
 * NULL = the calling thread's per-thread default stream) and the call returns
 * without waiting.  The decode matrix travels in the kernel arguments, so no
 * host state outlives the call. */
int32_t ec_method_encode_device(ec_matrix_list_t *list, int device, void *stream,
                                uint64_t nstripes, const void *in, void *const *out);
int32_t ec_method_decode_device(ec_matrix_list_t *list, int device, void *stream,
                                uint64_t nstripes, uintptr_t mask,
                                const void *const *in, void *out);
/* group_pattern: device array of nstripes/group_stripes bytes indexing
 * masks[0..nmasks), nmasks <= 256 (ids >= nmasks are clamped to the last
 * mask).  Decode matrices that fit the 2 KiB kernel-argument segment travel
 * there; more go to a per-call device table, asynchronously on `stream`. */
int32_t ec_method_decode_mixed_device(ec_matrix_list_t *list, int device,
                                      void *stream, uint64_t nstripes,
                                      uint64_t group_stripes,
                                      const uint8_t *group_pattern,
                                      uint32_t nmasks, const uintptr_t *masks,
                                      const void *const *frags, void *out);
int32_t ec_method_heal_device(ec_matrix_list_t *list, int device, void *stream,
                              uint64_t nstripes, uintptr_t mask,
                              const void *const *in, uintptr_t target_mask,
                              void *const *out);
/* ec_method_encode_rows on device buffers: out[i] (indexed by brick) is
 * written for the bits of row_mask only; out[] is not modified. */
int32_t ec_method_encode_rows_device(ec_matrix_list_t *list, int device, void *stream,
                                     uint64_t nstripes, const void *in, uintptr_t row_mask,
                                     void *const *out);
int32_t ec_method_writev_encode_device(ec_matrix_list_t *list, int device, void *stream,
                                       uint64_t head, uint64_t size, const void *user,
                                       const void *old_head, const void *old_tail,
                                       void *const *out);
int32_t ec_method_sync_device(int device, void *stream);

/* ------------------------------------------------------------------------
 * On-disk format guard (trusted.ec.config).
 *
 * The fragments this library writes are the reference's on-disk format bit
 * for bit: config version 0 (EC_CONFIG_VERSION, ec-common.h:22), algorithm 0
 * (the non-systematic Vandermonde code, ec-common.h:24), 8-bit GF words and
 * 512-byte chunks.  These helpers produce and check the xattr exactly as the
 * xlator does, so a volume coded on MI355X stays readable by CPU clients and
 * a brick written with any other layout is refused before it is decoded.
 * They need no GPU.
 * --------------------------------------------------------------------- */

/* The config a write stores for a volume of `bricks` = n bricks with
 * `redundancy` = n - k (ec-dir-write.c:144-151, ec-heal.c:1268-1275). */
void ec_method_config_fill(uint32_t bricks, uint32_t redundancy, ec_config_t *config);
/* Serialise to the 8-byte big-endian xattr value (ec_dict_set_config,
 * ec-helpers.c:298-330).  Returns 0, or -EINVAL for a version newer than 0. */
int32_t ec_method_config_pack(const ec_config_t *config, uint8_t value[8]);
/* Parse an xattr value (ec_dict_del_config, ec-helpers.c:333-380).  Returns 0,
 * -EINVAL (length != 8 or unsupported version) or -ENODATA (all zeros: the
 * xattr is absent, as the reference treats it). */
int32_t ec_method_config_unpack(const void *value, size_t len, ec_config_t *config);
/* ec_config_check (ec-common.c:1151-1195) for a volume of `bricks` bricks
 * with `redundancy` redundancy: 0 when the fragment layout is the one this
 * coder reads and writes, -EINVAL when the config is invalid or corrupted
 * (redundancy < 1, 2*redundancy >= bricks, gf_word_size not a power of two,
 * chunk bits not a multiple of word size x data bricks), -ENOTSUP when it is
 * well formed but describes another layout or geometry. */
int32_t ec_method_config_check(uint32_t bricks, uint32_t redundancy,
                               const ec_config_t *config);

/* ------------------------------------------------------------------------
 * Utilities.
 * --------------------------------------------------------------------- */

/* Number of visible gfx950 devices (0 = CPU engine only). */
int32_t ec_method_device_count(void);
/* NUMA node of gfx950 device `device` (-1: unknown or a one-node host,
 * -ENODEV: no such device): where a client should run the threads that
 * fill its buffers, and where ec_method_host_alloc places its pages. */
int32_t ec_method_device_numa_node(int32_t device);
/* CPU threads the library uses to stage pageable buffers: EC_COPY_THREADS,
 * else min(8, CPUs usable by the process -- affinity and cgroup quota). */
int32_t ec_method_copy_threads(void);
/* The engine a volume's coder runs ("gfx950 x8 + cpu/avx512", "cpu/avx2"...),
 * as logged by ec_method_init (cf. ec-code.c:1048-1053). */
const char *ec_method_engine(const ec_matrix_list_t *list);

/* Process-wide engine counters: host-buffer calls coded on a GPU, calls
 * coded by the CPU engine, and, among the latter, fallbacks after a failed
 * device submission.  A split call (r05: a GPU codes the first share of its
 * stripes, the calling thread's CPU engine the rest) adds 1 to both
 * gpu_calls and cpu_calls, so gpu_calls + cpu_calls counts engine runs, not
 * API calls; when its GPU share fails and is redone on the CPU engine,
 * cpu_fallbacks goes up and cpu_calls stays as the split left it. */
typedef struct {
    uint64_t gpu_calls;
    uint64_t cpu_calls;
    uint64_t cpu_fallbacks;
} ec_method_stats_t;
void ec_method_get_stats(ec_method_stats_t *stats);
/* Fault injection for tests (cf. debug/error-gen): the next `count`
 * host-buffer device submissions fail with -EIO before touching a device,
 * so the CPU fallback runs. */
void ec_method_inject_device_faults(uint32_t count);
/* HIP errors and the caller: every device entry point first clears any
 * non-sticky HIP error left pending on the calling thread
 * (hipGetLastError), so that its own launch checks see only its own
 * launches.  A caller that shares the thread's HIP runtime (torch, a
 * client's own kernels) must read its own pending error before calling in:
 * the library consumes it, and records it nowhere.
 *
 * Why the calling thread's last failing call failed (diagnostics): the
 * device layer's record (the HIP call or kernel and its error), or the
 * entry point and errno of a failure it did not record (an argument error).
 * Per thread: a client's epoll threads each read their own.  The text stays
 * until the thread's next failure ("" if it never failed; on a node without
 * a device, why none was used).  The pointer is valid until that thread's
 * next call into the library. */
const char *ec_method_last_error(void);
/* Pinned, device-mapped host memory.  Host buffers in such memory (16-byte
 * aligned) are coded in place by the GPU over PCIe with no staging copy;
 * pageable buffers are staged through pinned slots by CPU threads.  The
 * pages are placed on the NUMA node of the first host-buffer GPU
 * (EC_MI355X_HOST_DEVICES), as are the staging slots of each GPU. */
void *ec_method_host_alloc(size_t bytes);
void ec_method_host_free(void *p);
/* Pin and map an existing host range (e.g. a GlusterFS iobuf arena, see
 * INTEGRATION.md) so buffers inside it take the zero-copy path.  Returns 0
 * or -errno; -EEXIST for a range sharing a page with a live registration
 * (or inside the pinned pool): pages are mapped whole, and unregistering one
 * of two registrations of a page would unmap it under the other.  Unregister
 * before freeing the memory. */
int32_t ec_method_host_register(void *p, size_t bytes);
/* Unregister a range registered by either call below or above (a range still
 * waiting in the deferred queue is dropped; one being registered is waited
 * for).  Returns 0 or -errno. */
int32_t ec_method_host_unregister(void *p);
/* Deferred registration: queue the range for a library thread and return at
 * once (0 or -errno, -EEXIST as above, checked at once).  For callers holding a lock, such as GlusterFS's arena
 * hook, which runs under iobuf_pool->mutex (iobuf.c:157): until the thread has
 * registered the range, buffers in it are coded as pageable memory. */
int32_t ec_method_host_register_async(void *p, size_t bytes);
/* Wait until every queued registration has been done (tests, benchmarks). */
void ec_method_host_register_flush(void);

/* Pinned buffer pool for a client's own I/O buffers (the integration patch's
 * iobuf data allocator): pinned, device-mapped buffers of
 * any size up to 128 MiB, recycled by size class (4 KiB .. 1 MiB powers of
 * two, then 2 MiB steps), so hipHostRegister runs once per 2 MiB slab as the
 * pool grows and never per buffer.  At least 4 KiB aligned, contents not
 * cleared.  Returns NULL without a gfx950 device, for larger requests, or once
 * the pool's range (EC_POOL_MB, default 2048 MiB) is used up -- the caller
 * then allocates as it would without the pool. */
void *ec_method_buffer_get(size_t bytes);
/* Release a buffer: returns 1 when p came from ec_method_buffer_get (it is
 * back in the pool), 0 when it did not (the caller frees it). */
int32_t ec_method_buffer_put(void *p);

/* Host-call crossover probes (tests and tuning; no device needed).
 * ec_method_xover_route: would a host call of a volume with k data bricks go
 * to the CPU engine (1) or a GPU (0)?  op 0 = encode, 1 = decode-type; user
 * = user bytes, moved = bytes read + written, staged = bytes of its buffers
 * that are not pinned and mapped, inflight = bytes queued on the GPU.
 * ec_method_xover_observe feeds the router one completed call (engine 0 =
 * CPU, 1 = GPU with every buffer mapped, 2 = every buffer staged, 3 = some of
 * each; ns = its duration), as the library does after calls of >= 256 KiB;
 * ec_method_xover_reset forgets every observation.  -EINVAL on bad args. */
int32_t ec_method_xover_route(uint32_t k, int32_t op, uint64_t user, uint64_t moved,
                              uint64_t staged, uint64_t inflight);
/* Split calls (r05): the share of such a call's stripes, in thousandths, that
 * a GPU codes while the calling thread codes the rest on the CPU engine, or
 * -1 when the call stays whole (below 1 MiB of user data, one engine would
 * take under 15 %, or -- costed as if other large calls were in flight -- a
 * buffer that is not pinned and mapped: a real call with staged buffers
 * splits only while it is the only large host call).  Same arguments as
 * ec_method_xover_route. */
int32_t ec_method_xover_split(uint32_t k, int32_t op, uint64_t user, uint64_t moved,
                              uint64_t staged, uint64_t inflight);
/* Both decisions for a call with `others` large (>= 1 MiB) host calls in
 * flight beside it (r05): returns 0 (a GPU) or nonzero (the CPU engine; 2
 * when the call stages buffers and its staging copies would take at least the
 * CPU time coding it on the calling thread takes -- with other callers busy
 * the GPU route then frees no CPU; EC_STAGE_COPY_GBPS, default 10, is the
 * copy rate assumed, 0 turns the rule off), and, when `share` is not NULL,
 * the split share as ec_method_xover_split gives it (staged calls split only
 * when `others` is 0).  -EINVAL on bad args. */
int32_t ec_method_xover_plan(uint32_t k, int32_t op, uint64_t user, uint64_t moved,
                             uint64_t staged, uint64_t inflight, uint32_t others,
                             int32_t *share);
/* A split call as the library records one (r05, tests): `gpu_share` per
 * mille of the call's stripes took `gpu_ns` on a GPU from the hand-off, the
 * rest `cpu_ns` on the CPU engine.  The share later calls of this class,
 * width, size and provenance get moves toward the one that would have
 * balanced the two (ec_method.c share_learn; the first sample of a slot is
 * a cold start and dropped; ec_method_xover_reset forgets them).  -EINVAL on
 * bad args. */
int32_t ec_method_xover_observe_split(int32_t op, uint32_t k, uint64_t user, uint64_t moved,
                                      uint64_t staged, uint32_t gpu_share, uint64_t gpu_ns,
                                      uint64_t cpu_ns);
/* One engine's share of a split call as the library records it (r06, tests):
 * `part` of the call's `user` bytes took `ns` on `engine` (as in
 * ec_method_xover_observe).  The CPU's share is a sample of its rate inside
 * calls of `user` bytes; a GPU share, whose time holds the GPU's fixed latency
 * once, is recorded as the time the whole call would have taken (latency
 * from `staged` / `moved` as the router models it).  -EINVAL on bad args. */
int32_t ec_method_xover_observe_part(int32_t engine, int32_t op, uint32_t k, uint64_t user,
                                     uint64_t part, uint64_t ns, uint64_t staged,
                                     uint64_t moved);
int32_t ec_method_xover_observe(int32_t engine, int32_t op, uint32_t k, uint64_t user,
                                uint64_t ns);
void ec_method_xover_reset(void);

/* Pool and deferred-registration counters (times in microseconds). */
typedef struct {
    uint64_t pool_bytes;           /* pinned bytes the pool has grown to      */
    uint64_t in_use_bytes;         /* of which handed out now (class sizes)   */
    uint64_t gets;                 /* ec_method_buffer_get calls              */
    uint64_t misses;               /* of which returned NULL                  */
    uint64_t slabs;                /* slabs registered                        */
    uint64_t slab_register_us;     /* time to map, fault in and register them */
    uint64_t deferred_registers;   /* ranges registered by the library thread */
    uint64_t deferred_register_us; /* hipHostRegister time of those           */
    uint64_t deferred_register_failures;
    uint64_t unregisters;          /* ec_method_host_unregister calls done    */
    uint64_t unregister_us;        /* hipHostUnregister time of those         */
} ec_method_pool_stats_t;
void ec_method_pool_stats(ec_method_pool_stats_t *stats);

/* Per-pattern kernels compiled at run time (r06; the counterpart of the
 * reference's per-row JIT, ec-code.c:722-809).  A device-buffer combine with
 * one erasure pattern of a wide code (k >= 12 data and >= 12 output rows,
 * e.g. a 16+4 decode; >= EC_MI355X_JIT_MIN_STRIPES stripes, default 1024)
 * queues its coefficient matrix for compilation (hiprtc, opened with dlopen;
 * one library thread, ~1-2 s) as one straight-line XOR program over the
 * whole matrix, and runs the shipped kernel until that code exists; later
 * calls of the matrix run it.  Results are identical either way.
 * EC_MI355X_JIT=0 turns this off, EC_MI355X_JIT_SYNC=1 compiles on the
 * calling thread.  Counters: */
typedef struct {
    uint64_t compiled;    /* matrices compiled                          */
    uint64_t failed;      /* compilations that failed (shipped kernel)  */
    uint64_t launches;    /* calls that ran a compiled kernel           */
    uint64_t compile_us;  /* time spent compiling                       */
    uint64_t lookups;     /* eligible calls                             */
    uint64_t entries;     /* matrices in the cache now (<= 32)          */
} ec_method_jit_stats_t;
void ec_method_jit_stats(ec_method_jit_stats_t *stats);
/* Queue the kernel of a rows x k coefficient matrix for compilation before
 * its first call (e.g. a heal daemon that knows the bricks it will read):
 * 0, -EPERM (EC_MI355X_JIT=0), -ENOSYS (no hiprtc), -ENOSPC (the per-process
 * compile budget is spent), -EINVAL.  Needs no device. */
int32_t ec_method_jit_prepare(uint32_t k, uint32_t rows, const uint8_t *coef);
/* Generate and compile (without loading) the kernel of a rows x k matrix of
 * GF(2^8) coefficients (row-major): returns its code size in bytes, or
 * -errno (-ENOSYS without hiprtc, -EIO when the compiler failed); *ops, when
 * not NULL, gets the program's XOR instructions per dword column.  Needs no
 * device (tests). */
int32_t ec_method_jit_compile_check(uint32_t k, uint32_t rows, const uint8_t *coef,
                                    uint32_t *ops);

/* Host-side matrix helpers, exported for tests and tools: the n x k encode
 * matrix (ec-method.c:22-36) and the k x k inverse for ascending rows
 * (ec-method.c:38-72), as uint32 values in [0, 255].  Return 0 or -EINVAL. */
int32_t ec_method_encode_matrix(uint32_t columns, uint32_t rows, uint32_t *matrix);
int32_t ec_method_inverse_matrix(uint32_t columns, const uint32_t *rows,
                                 uint32_t *matrix);
uint32_t ec_method_gf_mul(uint32_t a, uint32_t b);
uint32_t ec_method_gf_div(uint32_t a, uint32_t b);

#ifdef __cplusplus
}
#endif

#endif /* EC_MI355X_EC_METHOD_H */
