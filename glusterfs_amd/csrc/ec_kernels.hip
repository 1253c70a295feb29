/*
 * ec_kernels.hip -- launchers of the gfx950 kernels in ec_kernels_impl.h
 * (see that header for the kernels and the reference functions they replace).
 *
 * Shipped configuration (r03; one-process A/Bs in tools/kbench/kb3.hip,
 * profiles/kb3_r03*.log, and round 1-2's tools/kbench/kbench.hip):
 *   encode   4+2, 8+4: narrow-tile encoders (ec_encode_tile_t, 4-stripe
 *            tiles, per-wave 2 KiB row runs); 16+4: the row-group encoder
 *            (ec_encode_tile_rb, 2 rows per wave), at any input alignment
 *            (LDS-DMA); 2+1 and pinned-host (zero-copy) calls: the
 *            register-resident ec_encode_vander
 *   combine  k <= 8 (decode, heal, mixed, sorted slots, device pattern
 *            table): the narrow-tile ec_combine_n, 4 or 8 waves; k > 8: the
 *            8-stripe ec_combine, 16 waves (two blocks fill a CU's 32 wave
 *            slots); both stage by LDS-DMA into a plane-major tile and
 *            multiply by a jump into the searched XOR programs
 *   stores   non-temporal on every device-path kernel except the 2+1 / 4+2
 *            register encoders (profiles/kbench_r01_nts.log)
 *   staging  LDS-DMA loads non-temporal for calls whose input exceeds the
 *            MALL (256 MiB), default policy up to it (nt_staging)
 *   host     pinned buffers: the zero-copy kernels (ec_combine_zc,
 *            ec_encode_vander_zc), 1 KiB requests over PCIe
 */
#include <hip/hip_runtime.h>

#include <errno.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <memory>
#include <mutex>
#include <vector>

#include <cstddef>
#include <cstring>

#include "ec_kernels.h"
#include "ec_kernels_impl.h"
#include "ec_jit.h"

using namespace ecdev;

/* LDS-DMA staging policy override for A/B runs: -1 = by size (shipped),
 * 0 = default policy always, 2 = non-temporal always.  EC_MI355X_LDSNT=0/1
 * sets it at load; tools/kbench/kb3.hip sets it directly. */
int ecdk_ldsnt_override = [] {
    const char *e = getenv("EC_MI355X_LDSNT");
    return e && *e ? (*e == '0' ? kLdsDmaDefault : kLdsDmaNT) : -1;
}();

namespace {

/* Status of the launch just issued on this thread: the entry points clear
 * any stale error first (ec_device.hip clear_stale_error), so a failure here
 * is the launch's, and it is recorded under the kernel's name. */
int launch_ok(const char *what)
{
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : ecd_hip_fail(what, e);
}

/* Check a HIP call whose failure fails the call: recorded, -EIO. */
int hip_ok(hipError_t e, const char *what)
{
    if (e == hipSuccess)
        return 0;
    (void)hipGetLastError();
    return ecd_hip_fail(what, e);
}

/* Non-temporal staging loads for a call that reads more than 256 MiB, the
 * MALL's capacity: none of its input can still be cached when the same data
 * comes round again, and default-policy allocation only costs.  Below that,
 * input a previous call (or producer) left in the MALL is hit.  Same process,
 * shipped / default / nt interleaved (tools/kbench/kb3.hip group ldsnt,
 * profiles/r03/kb3_r03y_ldsnt.log, kb3_r03z_ldsnt_sizes.log), ms:
 *   1 GiB    decode 4+2 0.355 -> 0.327, 8+4 0.356 -> 0.334, 16+4 0.388 ->
 *            0.376; encoders within 0.5 %
 *   320 MiB  decode 4+2 0.109 -> 0.105, 16+4 0.138 -> 0.129; encoders tie
 *   256 MiB  default wins: decode 4+2 0.077 vs 0.086, encode 4+2 0.093 vs
 *            0.107 (a 64K-stripe 8+4 batch is 256 MiB: configs[2])
 *   <= 128 MiB default wins or ties, except small 4+2 decodes */
constexpr uint64_t kNtStagingBytes = 256ull << 20;

/* every input base (and the stride) 16-byte aligned: no staging piece
 * straddles a cache line (see encode_tiles) */
bool inputs_aligned(const CombineArgs &a)
{
    uintptr_t o = (uintptr_t)a.in_stride;
    for (u32 p = 0; p < ECD_MAX_ROWS; ++p)   /* unused entries are null */
        o |= (uintptr_t)a.in_base[p];
    return (o & 15u) == 0;
}

bool nt_staging(uint64_t in_bytes)
{
    if (ecdk_ldsnt_override >= 0)
        return ecdk_ldsnt_override == kLdsDmaNT;
    return in_bytes > kNtStagingBytes;
}

/* Tile order of the tile encoders: block b codes tile b, except for 16+4
 * encodes of >= 4 GiB of input, where each XCD walks its own contiguous run
 * of tiles (blocks go round-robin to the 8 XCDs; ec_kernels_impl.h
 * enc_tile<true>).  A 16+4 encode depends on where its 20 fragments sit (up
 * to +-12 %); at 4-8 GiB the XCD runs were faster for seven
 * placements of eight (4 % on average, the worst placement 7 %), at 2 GiB
 * slower for five of six (3 % on average).  Medians of three rounds after
 * 150 ms of load, ms per call, tile b / XCD runs (profiles/r05/
 * r05at_permab.log, r05au_permab.log, r05av_permab.log):
 *   8 GiB, 6 placements  3.194-3.559 / 3.170-3.296 (mean 3.352 / 3.208)
 *   4 GiB, 2 placements  1.667, 1.604 / 1.627, 1.585
 *   2 GiB, 6 placements  0.801-0.913 / 0.812-0.944 (mean 0.834 / 0.859)
 * For 4+2 and 8+4 at 8 GiB the sign depends on the placement (+-7 %), so
 * they keep tile b.  (Measured and retired in r05/r06: golden-ratio order,
 * 20-28 % slower everywhere, r05as_permab.log; launches cut into 512 MiB /
 * 1 GiB pieces, a third of the 8 GiB 16+4 loss back but every other call
 * slower, r05ao_chunkab.log, r05ap_chunkab.log.) */
constexpr uint64_t kXcdTilesBytes = 4ull << 30;

/* hipFuncAttributeMaxDynamicSharedMemorySize is per device: set it once per
 * (kernel, device), for the device current on the launching thread (a
 * process-wide once-flag left every GPU but the first unconfigured). */
int ensure_lds_limit(const void *kern, int bytes)
{
    static std::mutex mu;
    static std::vector<std::pair<const void *, int>> done;
    int dev = 0;
    if (int rc = hip_ok(hipGetDevice(&dev), "hipGetDevice"))
        return rc;
    std::lock_guard<std::mutex> g(mu);
    for (const auto &e : done)
        if (e.first == kern && e.second == dev)
            return 0;
    if (int rc = hip_ok(hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, bytes),
                        "hipFuncSetAttribute(MaxDynamicSharedMemorySize)"))
        return rc;
    done.emplace_back(kern, dev);
    return 0;
}

template <int K, int N, int W, bool NTS = false>
int launch_vander(hipStream_t s, uint64_t nstripes, const void *in, void *const *out, bool zc)
{
    FragPtrs f;
    for (int i = 0; i < N; ++i)
        f.p[i] = static_cast<uint8_t *>(out[i]);
    if (zc && vander_use_zc<W>(nstripes)) {
        hipLaunchKernelGGL((ec_encode_vander_zc<K, N, W>), dim3((u32)kZcBlocks), dim3(kBlock), 0,
                           s, static_cast<const uint8_t *>(in), f, nstripes);
        return launch_ok("launch_vander");
    }
    const uint64_t g = vander_grid<W>(nstripes);
    if (g == 0)
        return 0;
    if (g > 0x7fffffffull)
        return -EINVAL;
    hipLaunchKernelGGL((ec_encode_vander<K, N, W, NTS>), dim3((u32)g), dim3(kBlock), 0, s,
                       static_cast<const uint8_t *>(in), f, nstripes);
    return launch_ok("launch_vander");
}

/* The 8-stripe ec_combine (k > 8): single pattern, mixed patterns (kernel
 * arguments or, PG, the device table), or sorted slots (SL). */
template <int K, int NW, bool NTS, bool SL = false, int LA = kLdsDmaDefault>
int launch_combine(hipStream_t s, const CombineArgs &a)
{
    /* sorted slots: every pattern's run may carry up to 7 padding slots */
    const uint64_t g = SL ? (a.nstripes + 8ull * a.npatterns) / 8 + 1 : combine_grid<1>(a.nstripes);
    if (g == 0)
        return 0;
    if (g > 0x7fffffffull)
        return -EINVAL;
    const size_t lds = combine_lds<1>(a.k);
    if (a.patg) {
        hipLaunchKernelGGL((ec_combine<K, 1, NW, true, NTS, 2, true, true, 1, SL, 1, LA>), dim3((u32)g),
                           dim3(NW * 64), lds, s, a);
    } else if (a.group_pattern) {
        hipLaunchKernelGGL((ec_combine<K, 1, NW, true, NTS, 2, false, true, 1, SL, 1, LA>), dim3((u32)g),
                           dim3(NW * 64), lds, s, a);
    } else {
        hipLaunchKernelGGL((ec_combine<K, 1, NW, false, NTS, 2, false, true, 1, false, 1, LA>), dim3((u32)g),
                           dim3(NW * 64), lds, s, a);
    }
    return launch_ok("launch_combine");
}

} // namespace

int ecdk_has_vander(uint32_t k, uint32_t n)
{
    return (k == 2 && n == 3) || (k == 4 && n == 6) || (k == 8 && n == 12) ||
           (k == 16 && n == 20);
}

/* EC_MI355X_ENC=0 keeps the register-resident encoder for every geometry
 * (A/B runs); unset = the tile encoders. */
static bool enc_tiles()
{
    static const bool v = [] {
        const char *e = getenv("EC_MI355X_ENC");
        return !(e && *e == '0');
    }();
    return v;
}

namespace {

/* Narrow-tile encoder (ec_encode_tile_t): 4-stripe tiles, NW waves, each
 * fragment row's 4 chunks stored as one 2 KiB run (tools/kbench/kb3.hip,
 * profiles/kb3_r03*.log).  SM: staging mode (ec_kernels_impl.h
 * stage_encode_tile; 1 = partial-stripe write). */
template <int K, int N, int NW, bool DIRECT, int SM, int LA>
int launch_encode_narrow(hipStream_t s, uint64_t nstripes, EncSrc src, void *const *out)
{
    FragPtrs f;
    for (int i = 0; i < N; ++i)
        f.p[i] = static_cast<uint8_t *>(out[i]);
    const uint64_t g = (nstripes + 3) / 4;
    if (g == 0)
        return 0;
    if (g > 0x7fffffffull)
        return -EINVAL;
    hipLaunchKernelGGL((ec_encode_tile_t<K, N, 4, NW, true, DIRECT, true, SM, LA>), dim3((u32)g),
                       dim3(NW * 64), (encode_tile_t_lds<4, NW, true>(K)), s, src, f, nstripes);
    return launch_ok("launch_encode_narrow");
}

/* Row-group encoder (ec_encode_tile_rb): 4-stripe tiles, RB rows per wave,
 * so the tile is read from LDS N / RB times instead of N times.  XR: XCD
 * tile runs (kXcdTilesBytes). */
template <int K, int N, int RB, int SM, int LA, bool XR = false>
int launch_encode_rb(hipStream_t s, uint64_t nstripes, EncSrc src, void *const *out)
{
    FragPtrs f;
    for (int i = 0; i < N; ++i)
        f.p[i] = static_cast<uint8_t *>(out[i]);
    const uint64_t g = (nstripes + 3) / 4;
    if (g == 0)
        return 0;
    if (g > 0x7fffffffull)
        return -EINVAL;
    hipLaunchKernelGGL((ec_encode_tile_rb<K, N, 4, RB, true, true, SM, LA, XR>), dim3((u32)g),
                       dim3((N / RB) * 64), (encode_tile_rb_lds<N, 4, RB, true>(K)), s, src, f,
                       nstripes);
    return launch_ok("launch_encode_rb");
}

/* The shipped tile encoder of a geometry (4+2, 8+4, 16+4), -ENOTSUP else. */
template <int SM, int LA>
int encode_tiles_la(hipStream_t s, uint32_t k, uint32_t n, uint64_t nstripes, EncSrc src,
                    void *const *out)
{
    if (k == 4 && n == 6)
        return launch_encode_narrow<4, 6, 6, true, SM, LA>(s, nstripes, src, out);
    if (k == 8 && n == 12)
        return launch_encode_narrow<8, 12, 12, false, SM, LA>(s, nstripes, src, out);
    if (k == 16 && n == 20) {
        if constexpr (SM == 0 && LA == kLdsDmaNT)
            if (nstripes * 16 * ECD_CHUNK >= kXcdTilesBytes)
                return launch_encode_rb<16, 20, 2, SM, LA, true>(s, nstripes, src, out);
        return launch_encode_rb<16, 20, 2, SM, LA>(s, nstripes, src, out);
    }
    return -ENOTSUP;
}

/* Partial-stripe writes (SM = 1) keep the default policy: their interior is
 * read at the caller's byte alignment, so neighbouring 16-byte pieces share
 * cache lines, and the non-temporal loads lost there (kb3 ldsnt,
 * profiles/r03/kb3_r03ac_ldsnt_rmw.log, 1 GiB at +3 bytes: 4+2 0.450 ->
 * 0.464 ms, 16+4 0.441 -> 0.447); so do misaligned device inputs. */
template <int SM>
int encode_tiles(hipStream_t s, uint32_t k, uint32_t n, uint64_t nstripes, EncSrc src,
                 void *const *out)
{
    const bool aligned = ((uintptr_t)src.in & 15u) == 0;
    if constexpr (SM == 0)
        if (aligned && nt_staging(nstripes * k * ECD_CHUNK))
            return encode_tiles_la<SM, kLdsDmaNT>(s, k, n, nstripes, src, out);
    /* a byte-misaligned input (a partial write's interior, or a device
     * buffer at an odd offset): dword-aligned loads shifted through
     * registers (SM = 3, ec_kernels_impl.h stage_tile_shift) instead of
     * LDS-DMA at the caller's byte address, whose loads do not coalesce.
     * One process, 1 GiB partial writes, interior 3 bytes off, LDS-DMA ->
     * shift staging (profiles/r05/kb3_r05i_rmw.log; aligned encode beside):
     * 4+2 0.455 -> 0.431 ms (0.429), 8+4 0.513 -> 0.447 (0.419), 16+4 0.440
     * -> 0.424 (0.403).  (With ds_bpermute for the neighbour's dword instead
     * of DPP, 16+4 lost: 0.445 -> 0.455, kb3_r05h_rmw.log -- its row-group
     * encoder is short of LDS cycles.) */
    if (((uintptr_t)src.in & 3u) != 0)
        return encode_tiles_la<3, kLdsDmaDefault>(s, k, n, nstripes, src, out);
    return encode_tiles_la<SM, kLdsDmaDefault>(s, k, n, nstripes, src, out);
}

} // namespace

int ecdk_encode_vander(hipStream_t s, uint32_t k, uint32_t n, uint64_t nstripes,
                       const void *in, void *const *out, bool zc)
{
    /* narrow-tile encoders, kb3 A/B against round 2's encoders (ms per GiB
     * unless noted, profiles/kb3_r03d.log): 4+2 0.438 -> 0.423 (6 waves,
     * direct products), 8+4 0.443 -> 0.411 and 64K-stripe batches 0.126 ->
     * 0.095 ms (12 waves, Horner: one row per wave; the 2 KiB row runs also
     * remove the 64-B segment writes of the register encoder, PMC 1.10x);
     * 16+4: row groups, 2 rows per wave, 10 waves (profiles/r03/
     * kb3_r03j_rowgroups_ct.log: 1 GiB 0.492 -> 0.401 ms, 32K stripes 0.103
     * -> 0.092 against the 8-stripe one-row tile encoder).  They stage by
     * LDS-DMA, which takes any source alignment (a tensor slice at an odd
     * offset; tools/kbench/ldsdma_align.hip). */
    if (!zc && enc_tiles() && ecdk_has_vander(k, n) && k != 2)
        return encode_tiles<0>(s, k, n, nstripes, EncSrc{static_cast<const uint8_t *>(in), nullptr},
                               out);
    if (k == 2 && n == 3)
        return launch_vander<2, 3, 4>(s, nstripes, in, out, zc);
    if (k == 4 && n == 6)
        return launch_vander<4, 6, 2>(s, nstripes, in, out, zc);
    if (k == 8 && n == 12)
        return launch_vander<8, 12, 1, true>(s, nstripes, in, out, zc);
    if (k == 16 && n == 20)
        return launch_vander<16, 20, 1, true>(s, nstripes, in, out, zc);
    return -ENOTSUP;
}

int ecdk_rmw_gather(hipStream_t s, const uint8_t *head, const uint8_t *user, const uint8_t *tail,
                    uint64_t b1, uint64_t b2, uint64_t o0, uint64_t n, uint8_t *dst)
{
    if (n % 16 || ((uintptr_t)dst & 15))
        return -EINVAL;
    const uint64_t g = (n / 16 + kBlock - 1) / kBlock;
    if (g == 0)
        return 0;
    if (g > 0x7fffffffull)
        return -EINVAL;
    RmwSrc v{head, user, tail, b1, b2};
    hipLaunchKernelGGL(ec_rmw_gather, dim3((u32)g), dim3(kBlock), 0, s, v, o0, n, dst);
    return launch_ok("ecdk_rmw_gather");
}

template <int K, int N, int W, int LM>
int launch_vander_rmw(hipStream_t s, uint64_t nstripes, const uint8_t *edge,
                      const uint8_t *user_shift, void *const *out)
{
    FragPtrs f;
    for (int i = 0; i < N; ++i)
        f.p[i] = static_cast<uint8_t *>(out[i]);
    const uint64_t g = vander_grid<W>(nstripes);
    if (g == 0)
        return 0;
    if (g > 0x7fffffffull)
        return -EINVAL;
    hipLaunchKernelGGL((ec_encode_vander_rmw<K, N, W, LM>), dim3((u32)g), dim3(kBlock), 0, s, edge,
                       user_shift, f, nstripes);
    return launch_ok("launch_vander_rmw");
}

/* LM = 1: dword-aligned loads + v_alignbyte for the interior stripes.
 * Same box, against byte-address loads (profiles/kbench_r02m.log,
 * kbench_r02o.log): 4+2 0.556 -> 0.516 ms per GiB (aligned encoder 0.494),
 * 8+4 0.560 -> 0.548, 16+4 0.535 -> 0.474. */
int ecdk_encode_vander_rmw(hipStream_t s, uint32_t k, uint32_t n, uint64_t nstripes,
                           const uint8_t *edge, const uint8_t *user_shift, void *const *out)
{
    /* the tile encoders (r03): the edges from `edge`, the interior in place
     * at any alignment, both by LDS-DMA.  One process, 1 GiB, interior 3
     * bytes off (profiles/r03/kb3_r03q_ldsdma_unaligned.log): 4+2 0.515 ->
     * 0.453 ms, 8+4 0.545 -> 0.512, 16+4 0.475 -> 0.440 against the
     * register kernel, which 2+1 keeps */
    if (enc_tiles() && k != 2 && ecdk_has_vander(k, n))
        return encode_tiles<1>(s, k, n, nstripes, EncSrc{user_shift, edge}, out);
    if (k == 2 && n == 3)
        return launch_vander_rmw<2, 3, 4, 1>(s, nstripes, edge, user_shift, out);
    if (k == 4 && n == 6)
        return launch_vander_rmw<4, 6, 2, 1>(s, nstripes, edge, user_shift, out);
    if (k == 8 && n == 12)
        return launch_vander_rmw<8, 12, 1, 1>(s, nstripes, edge, user_shift, out);
    if (k == 16 && n == 20)
        return launch_vander_rmw<16, 20, 1, 1>(s, nstripes, edge, user_shift, out);
    return -ENOTSUP;
}

namespace {

const uint8_t *desc_pats(const ecd_combine_desc_t *d)
{
    return d->pat_ext ? d->pat_ext : d->pat;
}

/* Re-lay the packed byte patterns {src[k], coef[rows][k]} out in words:
 * src[] then one word-aligned row per output, pwords words per pattern. */
void pack_words(const ecd_combine_desc_t *d, u32 kw, u32 pwords, u32 *words)
{
    uint8_t *pb = reinterpret_cast<uint8_t *>(words);
    const uint8_t *pats = desc_pats(d);
    for (u32 q = 0; q < d->npatterns; ++q) {
        const uint8_t *src = pats + (size_t)q * d->pat_bytes;
        uint8_t *dst = pb + (size_t)q * pwords * 4;
        memcpy(dst, src, d->k);
        for (u32 r = 0; r < d->rows; ++r)
            memcpy(dst + (size_t)(1 + r) * kw * 4, src + d->k + (size_t)r * d->k, d->k);
    }
}

/* One upload of up to kPatWords pattern words into the device table, the
 * words travelling in the kernel-argument segment (copied at launch, so the
 * host buffer may go away; stream-ordered before the combine that reads it). */
struct PatChunk {
    u32 *dst;
    u32 n;
    u32 w[kPatWords];
};

__global__ __launch_bounds__(256) void ec_pat_upload(const PatChunk c)
{
    for (u32 i = threadIdx.x; i < c.n; i += 256u)
        c.dst[i] = c.w[i];
}

/* Enqueue the upload of `w` into the device table `tab` on `s`. */
int enqueue_upload(hipStream_t s, const std::vector<u32> &w, u32 *tab)
{
    PatChunk c;
    for (size_t o = 0; o < w.size(); o += kPatWords) {
        c.dst = tab + o;
        c.n = (u32)std::min<size_t>(kPatWords, w.size() - o);
        memcpy(c.w, w.data() + o, (size_t)c.n * 4);
        hipLaunchKernelGGL(ec_pat_upload, dim3(1), dim3(256), 0, s, c);
    }
    return launch_ok("enqueue_upload");
}

/* Mixed calls whose patterns exceed the 2 KiB argument space read their
 * decode matrices from a device table.  A self-heal sweep passes the same
 * mask set call after call, so the tables of recent calls stay on the
 * device (per device, LRU): a repeated call skips the allocation and the
 * upload launches (one per 2 KiB: ~9 for 64 masks of 16+4, ~50 us of
 * stream time per call).  An entry is reused only for identical words, and
 * evicted (LRU) only when no call holds it.
 *
 * Ordering is all on the device; no call waits on the host (r05):
 *   - a table is uploaded on the stream of the call that missed, which
 *     records the entry's `ready` event; a call that hits makes its stream
 *     wait for `ready`;
 *   - every stream that read the table records its own reader event at
 *     release(); a reader is a (stream, thread) pair, because
 *     hipStreamPerThread is one handle for a different stream in every
 *     thread, and re-recording a reader's event for its next call is exact
 *     (one in-order stream);
 *   - eviction makes the evicting call's stream wait for every reader event,
 *     then frees the old table and allocates the new one stream-ordered
 *     (hipFreeAsync / hipMallocAsync) on that stream, so the memory is reused
 *     only after every read of it;
 *   - the reader list stays bounded without a wait: entries whose event has
 *     completed are dropped, and past kMaxReaders live readers the oldest is
 *     folded into the releasing stream (it waits for that event, so the
 *     event it records next covers both).
 * r04 waited on the host instead (hipEventSynchronize + hipFree with the
 * lock dropped at eviction, hipEventSynchronize under the lock at the fold)
 * and ignored those calls' errors; one of them failed under the 4-thread
 * evict/hit/upload test on a fresh box and surfaced as a launch -EIO. */
class PatTableCache {
  public:
    struct Ref {
        int slot = -1;
        u32 *ptr = nullptr;
    };

    /* A table holding `w` on the current device, ordered before work that
     * `s` runs after this call; release() it once that work is enqueued. */
    int acquire(hipStream_t s, const std::vector<u32> &w, Ref &ref)
    {
        static const bool off = [] {   /* EC_MI355X_PATCACHE=0: per-call tables (A/B) */
            const char *e = getenv("EC_MI355X_PATCACHE");
            return e && *e == '0';
        }();
        if (off)
            return -EBUSY;
        int dev = 0;
        if (int rc = hip_ok(hipGetDevice(&dev), "hipGetDevice"))
            return rc;
        uint64_t h = 1469598103934665603ull;     /* FNV-1a over the words */
        for (u32 x : w)
            h = (h ^ x) * 1099511628211ull;
        std::lock_guard<std::mutex> g(mu_);
        int victim = -1;
        for (int i = 0; i < kEntries; ++i) {
            Entry &e = e_[i];
            if (e.ptr && e.dev == dev && e.hash == h && e.words == w) {
                if (int rc = hip_ok(hipStreamWaitEvent(s, e.ready, 0),
                                    "hipStreamWaitEvent(pattern table ready)"))
                    return rc;
                ++e.inflight;
                e.tick = ++tick_;
                ref.slot = i;
                ref.ptr = e.ptr;
                return 0;
            }
            if (e.inflight == 0 && (e.dev == dev || !e.ptr) &&
                (victim < 0 || !e.ptr || (e_[victim].ptr && e.tick < e_[victim].tick)))
                victim = i;
        }
        if (victim < 0)
            return -EBUSY;                    /* every entry in use: per call */
        Entry &e = e_[victim];
        if (e.ptr) {
            /* evict: s waits for every reader, then frees the old table */
            for (const Reader &r : e.readers)
                if (int rc = hip_ok(hipStreamWaitEvent(s, r.ev, 0),
                                    "hipStreamWaitEvent(pattern table reader)"))
                    return rc;                /* entry left as it was */
            if (int rc = hip_ok(hipFreeAsync(e.ptr, s), "hipFreeAsync(pattern table)"))
                return rc;
            e.ptr = nullptr;
            e.hash = 0;
            e.words.clear();
            drop_readers(e);                  /* their reads are waited for by s */
        }
        if (e.dev != dev) {                   /* an empty entry moves device */
            drop_readers(e);
            if (e.ready)
                (void)hipEventDestroy(e.ready);
            (void)hipGetLastError();
            e.ready = nullptr;
            e.dev = -1;
            if (int rc = hip_ok(hipEventCreateWithFlags(&e.ready, hipEventDisableTiming),
                                "hipEventCreate(pattern table)")) {
                e.ready = nullptr;
                return rc;
            }
            e.dev = dev;
        }
        u32 *p = nullptr;
        if (hipMallocAsync(reinterpret_cast<void **>(&p), w.size() * 4, s) != hipSuccess) {
            (void)hipGetLastError();
            return -EBUSY;                    /* the per-call table says why */
        }
        int rc = enqueue_upload(s, w, p);
        if (rc == 0)
            rc = hip_ok(hipEventRecord(e.ready, s), "hipEventRecord(pattern table ready)");
        if (rc) {
            (void)hipFreeAsync(p, s);
            (void)hipGetLastError();
            return rc;
        }
        e.ptr = p;
        e.hash = h;
        e.words = w;
        e.tick = ++tick_;
        e.inflight = 1;
        ref.slot = victim;
        ref.ptr = p;
        return 0;
    }

    /* The work that reads the table has been enqueued on `s`.  0, or the
     * error that made release() drain `s` instead of tracking it. */
    int release(const Ref &ref, hipStream_t s)
    {
        const uint64_t tok = s == hipStreamPerThread ? thread_token() : 0;
        int rc = 0;
        {
            std::lock_guard<std::mutex> g(mu_);
            Entry &e = e_[ref.slot];
            hipEvent_t ev = nullptr;
            for (const Reader &r : e.readers)
                if (r.s == s && r.tok == tok)
                    ev = r.ev;
            if (!ev) {
                prune_readers(e, s);
                rc = hip_ok(hipEventCreateWithFlags(&ev, hipEventDisableTiming),
                            "hipEventCreate(pattern table reader)");
                if (rc == 0)
                    e.readers.push_back({s, tok, ev});
                else
                    ev = nullptr;
            }
            if (ev)
                rc = hip_ok(hipEventRecord(ev, s), "hipEventRecord(pattern table reader)");
            --e.inflight;
        }
        if (rc)                                /* untracked: drain the stream */
            (void)hip_ok(hipStreamSynchronize(s), "hipStreamSynchronize");
        return rc;
    }

  private:
    struct Reader {
        hipStream_t s;
        uint64_t tok;        /* thread token for hipStreamPerThread, else 0 */
        hipEvent_t ev;
    };
    struct Entry {
        int dev = -1;
        uint64_t hash = 0, tick = 0;
        std::vector<u32> words;
        u32 *ptr = nullptr;
        hipEvent_t ready = nullptr;           /* the upload has landed */
        std::vector<Reader> readers;
        int inflight = 0;
    };

    /* a token per thread, never reused (a thread id can be) */
    static uint64_t thread_token()
    {
        static std::atomic<uint64_t> next{1};
        static thread_local const uint64_t tok = next.fetch_add(1);
        return tok;
    }

    /* events may be destroyed with work pending on them: the runtime frees
     * them once the work completes, and waits already enqueued still hold */
    static void drop_readers(Entry &e)
    {
        for (const Reader &r : e.readers)
            (void)hipEventDestroy(r.ev);
        e.readers.clear();
        (void)hipGetLastError();
    }

    /* Make room for a new reader without a host wait: drop readers whose
     * reads have completed; if kMaxReaders are still live, `s` waits for the
     * oldest, whose reads the event `s` records next then covers. */
    void prune_readers(Entry &e, hipStream_t s)
    {
        if (e.readers.size() < kMaxReaders)
            return;
        size_t o = 0;
        for (size_t i = 0; i < e.readers.size(); ++i) {
            const hipError_t q = hipEventQuery(e.readers[i].ev);
            if (q == hipSuccess)
                (void)hipEventDestroy(e.readers[i].ev);
            else
                e.readers[o++] = e.readers[i];
        }
        e.readers.resize(o);
        (void)hipGetLastError();              /* hipErrorNotReady is no error */
        if (e.readers.size() >= kMaxReaders &&
            hipStreamWaitEvent(s, e.readers.front().ev, 0) == hipSuccess) {
            (void)hipEventDestroy(e.readers.front().ev);
            e.readers.erase(e.readers.begin());
        }
        (void)hipGetLastError();
    }

    static constexpr int kEntries = 16;
    static constexpr size_t kMaxReaders = 16;
    std::mutex mu_;
    Entry e_[kEntries];
    uint64_t tick_ = 0;
};

/* never destroyed: tables and events would be freed after the runtime */
PatTableCache &pat_tables()
{
    static PatTableCache *c = new PatTableCache;
    return *c;
}

/* The device table of a mixed call: from the cache, or (all entries busy)
 * a per-call table (stream-ordered allocation, freed after the combine). */
int upload_table(hipStream_t s, const ecd_combine_desc_t *d, CombineArgs &a, u32 **tab,
                 PatTableCache::Ref &ref)
{
    const size_t nw = (size_t)a.pwords * a.npatterns;
    std::vector<u32> w(nw, 0u);
    pack_words(d, a.kw, a.pwords, w.data());
    const int rc = pat_tables().acquire(s, w, ref);
    if (rc == 0) {
        a.patg = ref.ptr;
        return 0;
    }
    if (rc != -EBUSY)
        return rc;
    if (const hipError_t e = hipMallocAsync(reinterpret_cast<void **>(tab), nw * 4, s)) {
        *tab = nullptr;
        (void)hip_ok(e, "hipMallocAsync(per-call pattern table)");
        return -ENOMEM;
    }
    a.patg = *tab;
    return enqueue_upload(s, w, *tab);
}

/* Pattern groups below one tile: sort the stripes by pattern into slot
 * runs padded to 8 (ec_slots_*), then tiles(stream, args-with-slots). */
template <bool NTS, typename F>
int sorted_slots(hipStream_t s, const CombineArgs &a0, F tiles)
{
    if (a0.nstripes == 0)
        return 0;
    if (a0.nstripes + 8ull * a0.npatterns >= 0xFFFFFFFFull)
        return -EINVAL;                 /* slots hold 32-bit stripe numbers */
    const uint64_t nslots_max = a0.nstripes + 8ull * a0.npatterns;
    u32 *ws = nullptr;
    const size_t bytes = (size_t)(512 + 1 + nslots_max) * 4;
    if (const hipError_t e = hipMallocAsync(reinterpret_cast<void **>(&ws), bytes, s)) {
        (void)hip_ok(e, "hipMallocAsync(slot workspace)");
        return -ENOMEM;
    }
    u32 *counts = ws, *cursors = ws + 256, *total = ws + 512, *slots = ws + 513;
    CombineArgs a = a0;
    a.slot_stripe = slots;
    a.slot_count = total;
    const uint64_t nb = (a.nstripes + kSlotBlock * kSlotPerThread - 1) / (kSlotBlock * kSlotPerThread);
    int rc = 0;
    rc = hip_ok(hipMemsetAsync(counts, 0, 256 * 4, s), "hipMemsetAsync(slot counts)");
    if (rc == 0)
        rc = hip_ok(hipMemsetAsync(slots, 0xFF, nslots_max * 4, s), "hipMemsetAsync(slots)");
    if (rc == 0) {
        hipLaunchKernelGGL(ec_slots_count, dim3((u32)nb), dim3(kSlotBlock), 0, s, a, counts);
        hipLaunchKernelGGL(ec_slots_scan, dim3(1), dim3(256), 0, s, counts, cursors, total);
        hipLaunchKernelGGL(ec_slots_scatter, dim3((u32)nb), dim3(kSlotBlock), 0, s, a, cursors,
                           slots);
        rc = launch_ok("sorted_slots");
    }
    if (rc == 0)
        rc = tiles(s, a);
    const int frc = hip_ok(hipFreeAsync(ws, s), "hipFreeAsync(slot workspace)");
    return rc ? rc : frc;
}

/* ------------------------------------------------ narrow tiles (r03) */

template <int K, int NW, bool MIXED, bool NTS, int WOT, bool PG, bool SL, int LA>
int launch_n1(hipStream_t s, const CombineArgs &a, uint64_t g)
{
    if (g == 0)
        return 0;
    if (g > 0x7fffffffull)
        return -EINVAL;
    const size_t lds = combine_n_lds<NW, WOT>((int)a.k);
    hipLaunchKernelGGL((ec_combine_n<K, NW, MIXED, NTS, WOT, PG, SL, 1, LA>), dim3((u32)g),
                       dim3(NW * 64), lds, s, a);
    return launch_ok("launch_n1");
}

/* one k-bucket: single pattern, mixed, device pattern table, sorted slots */
template <int K, int NW, int WOT, bool NTS, int LA>
int launch_narrow_k(hipStream_t s, const CombineArgs &a)
{
    if (!a.group_pattern)
        return launch_n1<K, NW, false, NTS, WOT, false, false, LA>(s, a, (a.nstripes + 3) / 4);
    if (a.group_shift >= 2)          /* groups of >= 4 stripes: a tile is one pattern's */
        return a.patg ? launch_n1<K, NW, true, NTS, WOT, true, false, LA>(s, a, (a.nstripes + 3) / 4)
                      : launch_n1<K, NW, true, NTS, WOT, false, false, LA>(s, a, (a.nstripes + 3) / 4);
    return sorted_slots<NTS>(s, a, [](hipStream_t st, const CombineArgs &b) {
        /* runs padded to multiples of 8 slots: worst case 7 per pattern */
        const uint64_t g = (b.nstripes + 8ull * b.npatterns) / 4 + 1;
        return b.patg ? launch_n1<K, NW, true, NTS, WOT, true, true, LA>(st, b, g)
                      : launch_n1<K, NW, true, NTS, WOT, false, true, LA>(st, b, g);
    });
}

/* The device combine for k <= 8: narrow tiles with per-wave output staging
 * (tools/kbench/kb3.hip, one process, 7 interleaved rounds against the
 * round-2 dispatch, profiles/kb3_r03d.log, ms per GiB unless noted):
 *   4+2 decode (dense)      0.366 -> 0.350   4 waves
 *   8+4 decode              0.371 -> 0.350   4 waves
 *   8+4 decode, 64K stripes 0.096 -> 0.083   8 waves (small batches)
 *   8+4 heal (4 rows)       0.316 -> 0.263   4 waves
 *   8+4 mixed, 16 masks     0.395 -> 0.375   4 waves
 * k = 16 keeps the 8-stripe ec_combine with 16 waves: 16+4 decode 0.406
 * against 0.421 at best narrow (8 waves, register stores), mixed 0.395
 * against 0.442.  Groups below a tile (8 stripes for ec_combine, 4 for the
 * narrow tiles) are sorted into slots first. */
template <bool NTS, int LA>
int launch_combine_k(hipStream_t s, const CombineArgs &a)
{
    if (a.k <= 4)
        return launch_narrow_k<4, 4, 1, NTS, LA>(s, a);
    if (a.k <= 8)
        return a.nstripes <= (1u << 17) ? launch_narrow_k<8, 8, 1, NTS, LA>(s, a)
                                        : launch_narrow_k<8, 4, 1, NTS, LA>(s, a);
    if (a.group_pattern && a.group_shift < 3)
        return sorted_slots<NTS>(s, a, [](hipStream_t st, const CombineArgs &b) {
            return launch_combine<16, 16, NTS, true, LA>(st, b);
        });
    return launch_combine<16, 16, NTS, false, LA>(s, a);
}

/* pack, then launch; -E2BIG from the packer means "use a device table" */
template <bool NTS>
int combine_any(hipStream_t s, const ecd_combine_desc_t *d)
{
    CombineArgs a;
    int rc = ecdk_pack_args(d, &a);
    u32 *tab = nullptr;
    PatTableCache::Ref ref;
    if (rc == -E2BIG && d->group_pattern)
        rc = upload_table(s, d, a, &tab, ref);
    /* staging policy by the call's input bytes; the host-buffer fallback
     * (NTS = false: pinned memory over PCIe) keeps the default policy */
    if (rc == 0) {
        if constexpr (NTS) {
            const bool nt = nt_staging(a.nstripes * a.k * ECD_CHUNK) && inputs_aligned(a);
            rc = nt ? launch_combine_k<NTS, kLdsDmaNT>(s, a)
                    : launch_combine_k<NTS, kLdsDmaDefault>(s, a);
        } else {
            rc = launch_combine_k<NTS, kLdsDmaDefault>(s, a);
        }
    }
    if (ref.slot >= 0)
        (void)pat_tables().release(ref, s);   /* a failure drained s: the call stands */
    if (tab) {
        const int frc = hip_ok(hipFreeAsync(tab, s), "hipFreeAsync(per-call pattern table)");
        rc = rc ? rc : frc;
    }
    return rc;
}

} // namespace

/* Validate and fill the kernel arguments.  Returns -E2BIG (header filled,
 * patterns not packed) when the patterns exceed the argument space. */
int ecdk_pack_args(const ecd_combine_desc_t *d, CombineArgs *a)
{
    if (d->k == 0 || d->k > ECD_MAX_K || d->rows == 0 || d->rows > ECD_MAX_ROWS)
        return -EINVAL;
    if (d->group_pattern && d->group_shift > 40)
        return -EINVAL; /* groups below 8 stripes run through sorted slots */
    if (d->npatterns == 0 || d->npatterns > ECD_MAX_PATTERNS ||
        (!d->pat_ext && (uint64_t)d->npatterns * d->pat_bytes > ECD_MAX_PAT_BYTES) ||
        d->pat_bytes < d->k + d->rows * d->k)
        return -EINVAL;
    memcpy(a->in_base, d->in_base, sizeof(a->in_base));
    memcpy(a->out_base, d->out_base, sizeof(a->out_base));
    a->in_stride = d->in_stride;
    a->out_stride = d->out_stride;
    a->nstripes = d->nstripes;
    a->group_pattern = d->group_pattern;
    a->patg = nullptr;
    a->slot_stripe = nullptr;
    a->slot_count = nullptr;
    a->k = d->k;
    a->kw = (d->k + 3) / 4;
    a->rows = d->rows;
    a->group_shift = d->group_shift;
    a->pwords = a->kw * (1 + d->rows);
    a->npatterns = d->npatterns;
    if (a->pwords > kMaxPatWords)
        return -EINVAL;
    if ((uint64_t)a->pwords * d->npatterns > kPatWords)
        return -E2BIG;
    memset(a->pat, 0, sizeof(a->pat));
    pack_words(d, a->kw, a->pwords, a->pat);
    return 0;
}

/* Every combine stages its inputs by LDS-DMA (global_load_lds_dwordx4), which
 * takes any source alignment (tools/kbench/ldsdma_align.hip,
 * profiles/r03/ldsdma_align.log): fragments at odd offsets (torch slices)
 * are read in place.  (Round 2 copied them to aligned scratch first.) */
/* A single-pattern combine of a wide code whose coefficient matrix has a
 * compiled whole-matrix kernel (ec_jit.hip, r06) runs that; every other
 * call, and the calls of a matrix whose code is still being compiled, run
 * the shipped kernels. */
int ecdk_combine(hipStream_t s, const ecd_combine_desc_t *d)
{
    if (ecj_eligible(d)) {
        uintptr_t o = (uintptr_t)d->in_stride;
        const uint8_t *pat = d->pat_ext ? d->pat_ext : d->pat;
        for (u32 p = 0; p < d->k; ++p)
            o |= (uintptr_t)d->in_base[pat[p]];
        const bool nt = nt_staging(d->nstripes * d->k * ECD_CHUNK) && (o & 15u) == 0;
        if (ecj_launch(s, d, nt) == 0)
            return 0;
    }
    return combine_any<true>(s, d);
}

/* Host-buffer combines with k <= 8 run the persistent double-buffered
 * ec_combine_zc_db (default since r04; EC_MI355X_ZCDB=0 keeps one tile per
 * block, ec_combine_zc, for A/B runs).  Pinned 8+4 / 4+2 decodes, same
 * process alternating (tools/zc_sizes.py, profiles/r03/r03af_zcsizes.log), us
 * per call one tile per block -> double-buffered: 4 MiB 177-197 -> 174 / 174
 * -> 162, 16 MiB 572 -> 518-526 / 554-568 -> 530, 64 MiB 1765-1790 -> 1757 /
 * 1760 -> 1674-1683, 256 MiB 6350 -> 6245 / 6390 -> 6178; never slower,
 * bit-exact in the knob test (ZCDB=0 and =1: decode, heal and mixed host
 * calls) and at every size probed. */
static bool zc_double_buffered()
{
    static const bool v = [] {
        const char *e = getenv("EC_MI355X_ZCDB");
        return !(e && *e == '0');
    }();
    return v;
}

/* LDS of one gfx950 CU (MI355X_MICROARCH.md): the largest block LDS */
constexpr size_t kLdsPerCu = 160u << 10;

/* A/B knobs of the persistent zero-copy combine's grid (read once):
 * EC_ZC_TPB = fixed tiles per block (r03's rule was 4), EC_ZC_INFLIGHT_KB =
 * the input bytes one round of tiles keeps in flight (default 2048). */
static uint64_t zc_env(const char *name, long lo, long hi, long dflt)
{
    const char *e = getenv(name);
    const long v = e ? atol(e) : dflt;
    return (uint64_t)(v >= lo && v <= hi ? v : dflt);
}

static uint64_t zc_fixed_tpb()
{
    static const uint64_t v = zc_env("EC_ZC_TPB", 1, 1024, 0);
    return v;
}

static uint64_t zc_inflight_bytes()
{
    static const uint64_t v = zc_env("EC_ZC_INFLIGHT_KB", 64, 1 << 20, 2048) << 10;
    return v;
}

/* CUs of the current device, queried once per device */
static int cu_count()
{
    static std::atomic<int> cus[64];
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0)
        return 256;
    if (dev < 64 && (n = cus[dev].load(std::memory_order_relaxed)) > 0)
        return n;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
        return 256;
    if (dev < 64)
        cus[dev].store(n, std::memory_order_relaxed);
    return n;
}

/* k > 8 with >= 2048 stripes (16 MiB of a 16+4 call): the 4-stripe tiles of
 * ec_combine_zc_db, two input tiles and the output tile in LDS */
static bool zc_db4_fits(const ecd_combine_desc_t *d)
{
    const size_t lds_db4 = (size_t)(2 * d->k + d->rows) * 4 * ECD_CHUNK + 8 * ECD_MAX_ROWS;
    return d->k > 8 && d->nstripes >= 2048 && lds_db4 <= (128u << 10) + 8 * ECD_MAX_ROWS;
}

/* Host-buffer path: every buffer is pinned host memory read / written over
 * PCIe (ec_device.hip run_pipeline), so the zero-copy combine with whole
 * 1 KiB request runs; default (not non-temporal) stores there, which cost
 * 12 % on the link (profiles/kbench_r01_zc.log). */
int ecdk_combine_host(hipStream_t s, const ecd_combine_desc_t *d)
{
    CombineArgs a;
    int rc = ecdk_pack_args(d, &a);
    /* more than 32 inputs + rows fit only the 4-stripe double-buffered tile
     * below (a 16+4 encode as a combine: 16 inputs, 20 rows, r06) */
    const bool wide = d->k + d->rows > 32 && !(zc_double_buffered() && zc_db4_fits(d));
    if (rc == -E2BIG || (rc == 0 && (wide || (d->group_pattern && d->group_shift < 3))))
        return combine_any<false>(s, d);   /* device pattern table / LDS limit / small groups */
    if (rc)
        return rc;
    const uint64_t g = (a.nstripes + 7) / 8;
    if (g == 0)
        return 0;
    if (g > 0x7fffffffull)
        return -EINVAL;
    const size_t lds = (size_t)(d->k + d->rows) * 8 * ECD_CHUNK;
    constexpr int NW = 8;
    const size_t lds_db = (size_t)(2 * d->k + d->rows) * 8 * ECD_CHUNK + 8 * ECD_MAX_ROWS;
    const bool db16 = d->k > 8 && lds_db <= kLdsPerCu;   /* 16+4 heal / row-masked encode */
    /* the 16-row decode of a 16+4 volume: 4-stripe tiles (half the LDS).
     * Pinned 16+4 decodes (profiles/r04/r04s_zcheal.log, one tile per block
     * -> this): 16 MiB 570-576 -> 525 us, 64 MiB 1793-1797 -> 1639; at 4 MiB
     * 172 -> 177, so calls below 2048 stripes (16 MiB) keep ec_combine_zc */
    const size_t lds_db4 = (size_t)(2 * d->k + d->rows) * 4 * ECD_CHUNK + 8 * ECD_MAX_ROWS;
    const bool db16t4 = !db16 && zc_db4_fits(d);
    if (zc_double_buffered() && db16t4) {
        const uint64_t g4 = (a.nstripes + 3) / 4;
        const uint64_t tpb = zc_fixed_tpb();
        const uint64_t want = tpb ? g4 / tpb
                                  : std::min<uint64_t>(g4 / 2, zc_inflight_bytes() /
                                                                   ((uint64_t)d->k * 4 * ECD_CHUNK));
        const uint64_t gdb = std::min<uint64_t>(std::max<uint64_t>(want, 1), (uint64_t)cu_count());
        const void *kern = a.group_pattern ? (const void *)ec_combine_zc_db<16, NW, true, 4>
                                           : (const void *)ec_combine_zc_db<16, NW, false, 4>;
        if (lds_db4 > (64u << 10) &&
            ensure_lds_limit(kern, (int)((128u << 10) + 8 * ECD_MAX_ROWS)) != 0)
            return -EIO;
        void *args[] = {&a};
        return hip_ok(hipLaunchKernel(kern, dim3((u32)gdb), dim3(NW * 64), args, lds_db4, s),
                      "hipLaunchKernel(ec_combine_zc_db)");
    }
    if (zc_double_buffered() &&
        ((d->k <= 8 && lds_db <= (128u << 10) + 8 * ECD_MAX_ROWS) || db16)) {
        /* persistent, at most one block per CU, >= 2 tiles per block so its
         * reads of tile i + 1 and writes of tile i overlap, and as many
         * blocks as keep ~2 MiB of input in flight: more only queue on the
         * link, fewer leave it idle while each block's first tile lands.
         * Pinned 8+4 / 4+2 calls, us (decode; profiles/r04/r04m_zctpb.log,
         * r03's 4 tiles per block -> this): 8+4 1 MiB 81 -> 69, 4 MiB 173
         * -> 164, 16 MiB 516 -> 505; 4+2 16 MiB 533 -> 489. */
        const uint64_t tpb = zc_fixed_tpb();
        const uint64_t want =
            tpb ? g / tpb : std::min<uint64_t>(g / 2, zc_inflight_bytes() / ((uint64_t)d->k * 8 * ECD_CHUNK));
        const uint64_t gdb = std::min<uint64_t>(std::max<uint64_t>(want, 1), (uint64_t)cu_count());
        const void *kern =
            db16 ? (a.group_pattern ? (const void *)ec_combine_zc_db<16, NW, true>
                                    : (const void *)ec_combine_zc_db<16, NW, false>)
            : d->k <= 4 ? (a.group_pattern ? (const void *)ec_combine_zc_db<4, NW, true>
                                           : (const void *)ec_combine_zc_db<4, NW, false>)
                        : (a.group_pattern ? (const void *)ec_combine_zc_db<8, NW, true>
                                           : (const void *)ec_combine_zc_db<8, NW, false>);
        if (lds_db > (64u << 10) &&
            ensure_lds_limit(kern, db16 ? (int)kLdsPerCu : (int)((128u << 10) + 8 * ECD_MAX_ROWS)) != 0)
            return -EIO;
        void *args[] = {&a};
        return hip_ok(hipLaunchKernel(kern, dim3((u32)gdb), dim3(NW * 64), args, lds_db, s),
                      "hipLaunchKernel(ec_combine_zc_db)");
    }
    if (d->k <= 4) {
        if (a.group_pattern)
            hipLaunchKernelGGL((ec_combine_zc<4, NW, true>), dim3((u32)g), dim3(NW * 64), lds, s, a);
        else
            hipLaunchKernelGGL((ec_combine_zc<4, NW, false>), dim3((u32)g), dim3(NW * 64), lds, s, a);
    } else if (d->k <= 8) {
        if (a.group_pattern)
            hipLaunchKernelGGL((ec_combine_zc<8, NW, true>), dim3((u32)g), dim3(NW * 64), lds, s, a);
        else
            hipLaunchKernelGGL((ec_combine_zc<8, NW, false>), dim3((u32)g), dim3(NW * 64), lds, s, a);
    } else {
        /* up to (16 + 16) * 4 KiB = 128 KiB of the CU's 160 KiB */
        if (lds > (64u << 10) &&
            ensure_lds_limit(a.group_pattern ? (const void *)ec_combine_zc<16, NW, true>
                                             : (const void *)ec_combine_zc<16, NW, false>,
                             128 << 10) != 0)
            return -EIO;
        if (a.group_pattern)
            hipLaunchKernelGGL((ec_combine_zc<16, NW, true>), dim3((u32)g), dim3(NW * 64), lds, s, a);
        else
            hipLaunchKernelGGL((ec_combine_zc<16, NW, false>), dim3((u32)g), dim3(NW * 64), lds, s, a);
    }
    return launch_ok("ecdk_combine_host");
}
