/*
 * ec_device.h -- internal boundary between the C host layer (ec_method.c) and
 * the HIP device layer (ec_device.hip, ec_kernels.hip).  C-compatible; no HIP
 * types leak into the C side (streams are opaque void pointers).
 */
#ifndef EC_MI355X_DEVICE_H
#define EC_MI355X_DEVICE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ECD_CHUNK 512u      /* EC_METHOD_CHUNK_SIZE (ec-method.h:29) */
#define ECD_MAX_K 16u       /* EC_METHOD_MAX_FRAGMENTS (ec-method.h:23) */
#define ECD_MAX_ROWS 32u    /* >= EC_MAX_NODES (31, ec.h:27-32) */
#define ECD_MAX_PAT_BYTES 2048u
#define ECD_MAX_PATTERNS 256u /* pattern ids are bytes */

/* One launch of the generic GF(2^8) combination kernel:
 *   for every stripe t < nstripes and row r < rows:
 *     out_base[r] + t*out_stride = XOR_p coef[r][p] * (in_base[src[p]] + t*in_stride)
 * on 512-byte bit-sliced chunks.  A "pattern" is the packed byte string
 * {src[k], coef[rows][k]}; with group_pattern != NULL, stripe t uses pattern
 * group_pattern[t >> group_shift] (mixed per-stripe-range erasure patterns),
 * otherwise pattern 0; ids >= npatterns are clamped to the last pattern. */
typedef struct ecd_combine_desc {
    uint32_t k;             /* inputs per stripe (kernel template parameter) */
    uint32_t rows;          /* output rows per stripe                        */
    uint64_t nstripes;
    uint64_t in_stride;     /* bytes between consecutive stripes of an input */
    uint64_t out_stride;    /* bytes between consecutive stripes of a row    */
    const void *in_base[ECD_MAX_ROWS];
    void *out_base[ECD_MAX_ROWS];
    const uint8_t *group_pattern; /* device array, or NULL                   */
    uint32_t group_shift;         /* log2(stripes per pattern group)         */
    uint32_t npatterns;
    uint32_t pat_bytes;           /* bytes per packed pattern = k + rows*k   */
    uint32_t pad;
    /* when non-NULL, the npatterns (<= ECD_MAX_PATTERNS) packed patterns are
     * read from here instead of pat[] (host memory, read during the call);
     * patterns beyond the kernel-argument space go to a device table */
    const uint8_t *pat_ext;
    uint8_t pat[ECD_MAX_PAT_BYTES];
} ecd_combine_desc_t;

/* Number of usable gfx950 devices (0 when none: the host layer then codes
 * with its CPU engine, ec_cpu.h). */
int ecd_device_count(void);
/* The calling thread's last failure ("" if none; on a node without a device,
 * why).  ecd_error_seq counts the failures the thread has recorded, so a
 * caller can tell whether a failing call said why; ecd_set_error records a
 * failure of the host layer (argument errors and the like). */
const char *ecd_last_error(void);
uint64_t ecd_error_seq(void);
void ecd_set_error(const char *text);

/* ---- device-pointer entry points: asynchronous on `stream` (NULL = the
 * calling thread's per-thread default stream of `device`); 0 or -errno. */

/* Compile-time specialised Vandermonde encode (k+r in the shipped table). */
int ecd_has_vander(uint32_t k, uint32_t n);
int ecd_encode_vander(int device, void *stream, uint32_t k, uint32_t n,
                      uint64_t nstripes, const void *in, void *const *out);
/* Generic combination (decode, mixed decode, generic encode, heal). */
int ecd_combine(int device, void *stream, const ecd_combine_desc_t *d);
int ecd_sync(int device, void *stream);

/* ---- host-memory entry points: stripes are partitioned across `ndev`
 * devices (0 = all visible), each device moves its range over PCIe with
 * pinned staging and overlapped H2D / compute / D2H, and the call blocks.
 * Buffers may be pageable or pinned host memory. */

/* Encode: in = nstripes*k*512 bytes, out[i] = nstripes*512 bytes.  enc_pat
 * (k + n*k bytes, direct coefficients) is used when no specialised encoder
 * exists for k+n. */
int ecd_encode_host(int ndev, uint32_t k, uint32_t n, uint64_t nstripes,
                    const void *in, void *const *out, const uint8_t *enc_pat);
/* The same for `rows` arbitrary encode-matrix rows (ec_method_encode_rows):
 * always the generic combination with `pat` (k + rows*k bytes), never the
 * specialised encoders -- rows == 20 of a 16+8 volume are not the 16+4
 * Vandermonde rows. */
int ecd_encode_host_rows(int ndev, uint32_t k, uint32_t rows, uint64_t nstripes,
                         const void *in, void *const *out, const uint8_t *pat);

/* Encode of a virtual input: the concatenation of nsegs segments
 * (seg_ptr[i] == NULL: seg_len[i] zero bytes), nstripes*k*512 bytes in
 * total, gathered into the pinned staging slots by the copy threads --
 * the padded buffer of a partial-stripe write without a separate copy. */
int ecd_encode_host_gather(int ndev, uint32_t k, uint32_t n, uint64_t nstripes, uint32_t nsegs,
                           const void *const *seg_ptr, const uint64_t *seg_len,
                           void *const *out, const uint8_t *enc_pat);

/* Partial-stripe write on device memory (asynchronous on `stream`): encode
 * the padded buffer {old_head[0:head) | user[0:user_size) | old tail bytes}
 * (NULL old stripes = zeros; one-stripe writes take both ends from old_head,
 * or old_tail when old_head is NULL) into out[0..n), ceil((head +
 * user_size) / (512k)) chunks each.  user may have any alignment. */
int ecd_writev_encode_device(int device, void *stream, uint32_t k, uint32_t n, uint64_t head,
                             uint64_t user_size, const void *user, const void *old_head,
                             const void *old_tail, void *const *out, const uint8_t *enc_pat);

/* Decode / reconstruct: frags[0..nfrags) are fragment buffers of
 * nstripes*512 bytes (NULL for fragments no pattern reads).  Output: when
 * outs is NULL, out = nstripes*rows*512 bytes, stripe-major (decoded data);
 * otherwise outs[r] = nstripes*512 bytes per row (regenerated fragments).  pats
 * holds npatterns packed patterns of k + rows*k bytes whose src[] index
 * frags[]; group_pattern (host, nstripes >> group_shift entries) selects a
 * pattern per stripe group, or NULL for pattern 0 everywhere. */
int ecd_decode_host(int ndev, uint32_t k, uint32_t rows, uint64_t nstripes,
                    uint32_t nfrags, const void *const *frags, void *out,
                    void *const *outs, uint32_t npatterns, const uint8_t *pats,
                    const uint8_t *group_pattern, uint32_t group_shift);

/* Bytes of host-buffer work in flight on the least-loaded host device
 * (UINT64_MAX without a device): the queue a new call would wait behind. */
uint64_t ecd_host_inflight(void);

/* 1 when [p, p + n) lies in pinned, device-mapped host memory (the
 * zero-copy path), 0 for pageable memory or without a device. */
int ecd_host_mapped(const void *p, size_t n);

/* Test hook: the next n host-buffer submissions fail with -EIO before
 * touching a device (exercises the CPU fallback). */
void ecd_inject_faults(uint32_t n);

/* Pointer classification: index of the (gfx950) device owning device
 * memory `p`, or -1 for host memory (pageable or pinned). */
int ecd_ptr_device(const void *p);

/* Pinned host allocation helpers (zero-copy PCIe transfers); allocations
 * are placed on the NUMA node of the first host-buffer device. */
void *ecd_host_alloc(size_t bytes);
/* NUMA node of device index `device` (-1: unknown / single node). */
int ecd_device_numa_node(int device);
/* Staging copy threads this process uses (EC_COPY_THREADS, else at most 8
 * and at most the usable CPUs). */
int ecd_copy_threads(void);
void ecd_host_free(void *p);
int ecd_host_register(void *p, size_t bytes);
/* unregisters a registered range, or drops it from the deferred queue */
int ecd_host_unregister(void *p);
/* queue [p, p + bytes) for registration by the library's thread */
int ecd_host_register_async(void *p, size_t bytes);
/* wait until every queued registration has run */
void ecd_host_register_flush(void);

/* Pinned buffer pool (ec_device.hip BufPool): NULL when no device, too
 * large, or the pool's range is used up; put returns 1 for pool buffers. */
void *ecd_buffer_get(size_t bytes);
int ecd_buffer_put(void *p);

typedef struct ecd_pool_stats {
    uint64_t pool_bytes, in_use_bytes, gets, misses, slabs, slab_register_us;
    uint64_t deferred_registers, deferred_register_us, deferred_register_failures;
    uint64_t unregisters, unregister_us;
} ecd_pool_stats_t;
void ecd_pool_stats(ecd_pool_stats_t *s);

/* Per-pattern whole-matrix kernels compiled at run time (ec_jit.hip, r06). */
typedef struct ecd_jit_stats {
    uint64_t compiled, failed, launches, compile_us, lookups, entries;
} ecd_jit_stats_t;
void ecd_jit_stats(ecd_jit_stats_t *s);
/* Generate and compile the kernel of one coefficient matrix (rows x k bytes)
 * without loading it: its code size, or -errno (-ENOSYS without hiprtc);
 * *ops = v_xor / v_bitop3 instructions per dword column; log = compiler
 * output on failure. */
int ecd_jit_compile_check(uint32_t k, uint32_t rows, const uint8_t *coef, uint32_t *ops,
                          char *log, size_t log_len);
/* queue (or, EC_MI355X_JIT_SYNC=1, compile now) the kernel of a matrix */
int ecd_jit_prepare(uint32_t k, uint32_t rows, const uint8_t *coef);

#ifdef __cplusplus
}
#endif

#endif
