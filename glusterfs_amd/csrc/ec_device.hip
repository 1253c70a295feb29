/*
 * ec_device.hip -- HIP runtime side of the MI355X disperse coder.
 *
 * Owns everything the reference never needed because its coder ran inline on
 * the calling CPU thread (ec-method.c:394-433): device discovery, per-call
 * streams, device/pinned staging buffers, the PCIe pipeline for callers that
 * hand over host memory, and the stripe-range partition across all visible
 * MI355X devices (stripes are independent, no collective).
 *
 * Host-memory pipeline per device (two slots, each on its own stream):
 *   slot s:  [pageable only: memcpy user -> pinned]  H2D  kernel  D2H
 *            [pageable only: memcpy pinned -> user after the slot's sync]
 * While one slot's kernel runs, the other slot's copies are in flight (PCIe is
 * full duplex), and the CPU copies of one slot overlap the GPU work of the
 * other.  Pinned user buffers are DMA'd directly with no CPU copy.
 */
#include <hip/hip_runtime.h>

#include <errno.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "ec_device.h"
#include "ec_kernels.h"

namespace {

constexpr int kMaxDev = 16;
constexpr uint64_t kBatchBytes = 32ull << 20; /* input bytes per pipeline batch */

std::mutex g_err_mu;
std::string g_err;

void set_err(const char *what, hipError_t e)
{
    std::lock_guard<std::mutex> g(g_err_mu);
    g_err = std::string(what) + ": " + hipGetErrorString(e);
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

void discover()
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess)
        n = 0;
    for (int i = 0; i < n && g_ndev < kMaxDev; ++i) {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, i) != hipSuccess)
            continue;
        if (strncmp(prop.gcnArchName, "gfx950", 6) != 0)
            continue; /* kernels are built for gfx950 only */
        g_dev_ids[g_ndev++] = i;
    }
    if (g_ndev == 0) {
        std::lock_guard<std::mutex> g(g_err_mu);
        g_err = "no gfx950 (MI355X) device visible";
    }
}

hipStream_t pick_stream(void *stream)
{
    return stream ? static_cast<hipStream_t>(stream) : hipStreamPerThread;
}

/* Device-resident staging for one pipeline slot pair; pooled per device. */
struct Stage {
    int dev = -1;
    hipStream_t st[2] = {nullptr, nullptr};
    uint8_t *din[2] = {nullptr, nullptr};
    uint8_t *dout[2] = {nullptr, nullptr};
    uint8_t *dgrp[2] = {nullptr, nullptr};
    uint8_t *pin_in[2] = {nullptr, nullptr};
    uint8_t *pin_out[2] = {nullptr, nullptr};
    uint8_t *pin_grp[2] = {nullptr, nullptr};
    size_t cap_in = 0, cap_out = 0, cap_grp = 0;
    bool pinned_staging = false;
};

std::mutex g_pool_mu;
std::vector<Stage *> g_pool[kMaxDev];

void free_bufs(Stage *s)
{
    for (int i = 0; i < 2; ++i) {
        if (s->din[i])
            (void)hipFree(s->din[i]);
        if (s->dout[i])
            (void)hipFree(s->dout[i]);
        if (s->dgrp[i])
            (void)hipFree(s->dgrp[i]);
        if (s->pin_in[i])
            (void)hipHostFree(s->pin_in[i]);
        if (s->pin_out[i])
            (void)hipHostFree(s->pin_out[i]);
        if (s->pin_grp[i])
            (void)hipHostFree(s->pin_grp[i]);
        s->din[i] = s->dout[i] = s->dgrp[i] = nullptr;
        s->pin_in[i] = s->pin_out[i] = s->pin_grp[i] = nullptr;
    }
    s->cap_in = s->cap_out = s->cap_grp = 0;
    s->pinned_staging = false;
}

int ensure(Stage *s, size_t in, size_t out, size_t grp, bool need_pinned)
{
    if (in <= s->cap_in && out <= s->cap_out && grp <= s->cap_grp &&
        (!need_pinned || s->pinned_staging))
        return 0;
    HIPCHK(hipStreamSynchronize(s->st[0]));
    HIPCHK(hipStreamSynchronize(s->st[1]));
    in = std::max(in, s->cap_in);
    out = std::max(out, s->cap_out);
    grp = std::max<size_t>(std::max(grp, s->cap_grp), 64);
    need_pinned = need_pinned || s->pinned_staging;
    free_bufs(s);
    for (int i = 0; i < 2; ++i) {
        HIPCHK(hipMalloc(&s->din[i], in));
        HIPCHK(hipMalloc(&s->dout[i], out));
        HIPCHK(hipMalloc(&s->dgrp[i], grp));
        HIPCHK(hipHostMalloc(&s->pin_grp[i], grp, hipHostMallocDefault));
        if (need_pinned) {
            HIPCHK(hipHostMalloc(&s->pin_in[i], in, hipHostMallocDefault));
            HIPCHK(hipHostMalloc(&s->pin_out[i], out, hipHostMallocDefault));
        }
    }
    s->cap_in = in;
    s->cap_out = out;
    s->cap_grp = grp;
    s->pinned_staging = need_pinned;
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
    if (hipSetDevice(g_dev_ids[dev]) != hipSuccess ||
        hipStreamCreateWithFlags(&s->st[0], hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&s->st[1], hipStreamNonBlocking) != hipSuccess) {
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

bool is_pinned_host(const void *p)
{
    if (!p)
        return false;
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return a.type == hipMemoryTypeHost;
}

/* Copy helper that tolerates our own pinned staging or a pinned user buffer. */
void copy_bytes(void *dst, const void *src, size_t n)
{
    if (n)
        memcpy(dst, src, n);
}

/* ---------------------------------------------------------------- encode */

struct EncodeJob {
    uint32_t k, n;
    const uint8_t *in;      /* whole user input                           */
    uint8_t *const *out;    /* n whole fragment buffers                   */
    const uint8_t *enc_pat; /* generic coefficients (k + n*k bytes)       */
    uint64_t s0, s1;        /* stripe range of this device                */
};

int launch_encode(hipStream_t st, const EncodeJob &j, const uint8_t *din, uint8_t *dout,
                  uint64_t cnt, uint64_t batch_stripes)
{
    void *outs[ECD_MAX_ROWS];
    for (uint32_t i = 0; i < j.n; ++i)
        outs[i] = dout + (uint64_t)i * batch_stripes * ECD_CHUNK;
    if (ecdk_has_vander(j.k, j.n))
        return ecdk_encode_vander(st, j.k, j.n, cnt, din, outs);
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
    return ecdk_combine(st, &d);
}

int run_encode_dev(int dev, const EncodeJob &j)
{
    if (j.s1 <= j.s0)
        return 0;
    HIPCHK(hipSetDevice(g_dev_ids[dev]));
    const uint64_t stripe_in = (uint64_t)j.k * ECD_CHUNK;
    const uint64_t B = std::max<uint64_t>(1, kBatchBytes / stripe_in);
    const bool pin_in = is_pinned_host(j.in);
    bool pin_out = true;
    for (uint32_t i = 0; i < j.n && pin_out; ++i)
        pin_out = is_pinned_host(j.out[i]);
    const bool staged = !(pin_in && pin_out);

    Stage *s = acquire(dev);
    if (!s)
        return -EIO;
    int rc = ensure(s, B * stripe_in, B * j.n * ECD_CHUNK, 0, staged);
    uint64_t pend_start[2] = {0, 0}, pend_cnt[2] = {0, 0};
    int it = 0;
    for (uint64_t a = j.s0; rc == 0 && a < j.s1; a += B, ++it) {
        const int sl = it & 1;
        const uint64_t cnt = std::min(B, j.s1 - a);
        hipStream_t st = s->st[sl];
        if (staged) {
            if (hipStreamSynchronize(st) != hipSuccess) {
                rc = -EIO;
                break;
            }
            if (pend_cnt[sl] && !pin_out) {
                for (uint32_t i = 0; i < j.n; ++i)
                    copy_bytes(j.out[i] + pend_start[sl] * ECD_CHUNK,
                               s->pin_out[sl] + (uint64_t)i * B * ECD_CHUNK,
                               pend_cnt[sl] * ECD_CHUNK);
            }
            pend_cnt[sl] = 0;
        }
        const uint8_t *src = j.in + a * stripe_in;
        if (!pin_in) {
            copy_bytes(s->pin_in[sl], src, cnt * stripe_in);
            src = s->pin_in[sl];
        }
        if (hipMemcpyAsync(s->din[sl], src, cnt * stripe_in, hipMemcpyHostToDevice, st) !=
            hipSuccess) {
            rc = -EIO;
            break;
        }
        rc = launch_encode(st, j, s->din[sl], s->dout[sl], cnt, B);
        if (rc)
            break;
        for (uint32_t i = 0; i < j.n; ++i) {
            uint8_t *dst = pin_out ? j.out[i] + a * ECD_CHUNK
                                   : s->pin_out[sl] + (uint64_t)i * B * ECD_CHUNK;
            if (hipMemcpyAsync(dst, s->dout[sl] + (uint64_t)i * B * ECD_CHUNK,
                               cnt * ECD_CHUNK, hipMemcpyDeviceToHost, st) != hipSuccess) {
                rc = -EIO;
                break;
            }
        }
        pend_start[sl] = a;
        pend_cnt[sl] = cnt;
    }
    for (int sl = 0; sl < 2; ++sl) {
        if (hipStreamSynchronize(s->st[sl]) != hipSuccess)
            rc = rc ? rc : -EIO;
        if (rc == 0 && pend_cnt[sl] && !pin_out)
            for (uint32_t i = 0; i < j.n; ++i)
                copy_bytes(j.out[i] + pend_start[sl] * ECD_CHUNK,
                           s->pin_out[sl] + (uint64_t)i * B * ECD_CHUNK,
                           pend_cnt[sl] * ECD_CHUNK);
    }
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

/* Device output layout of one batch: stripe-major data (outs == NULL) or
 * one B-stripe region per row (outs != NULL). */
void flush_decode(const DecodeJob &j, const uint8_t *pin, uint64_t a, uint64_t cnt, uint64_t B)
{
    if (j.outs) {
        for (uint32_t r = 0; r < j.rows; ++r)
            copy_bytes(j.outs[r] + a * ECD_CHUNK, pin + (uint64_t)r * B * ECD_CHUNK,
                       cnt * ECD_CHUNK);
    } else {
        copy_bytes(j.out + a * (uint64_t)j.rows * ECD_CHUNK, pin,
                   cnt * (uint64_t)j.rows * ECD_CHUNK);
    }
}

int run_decode_dev(int dev, const DecodeJob &j)
{
    if (j.s1 <= j.s0)
        return 0;
    HIPCHK(hipSetDevice(g_dev_ids[dev]));
    const uint64_t out_stripe = (uint64_t)j.rows * ECD_CHUNK;
    uint64_t B = std::max<uint64_t>(1, kBatchBytes / ((uint64_t)j.nfrags * ECD_CHUNK));
    const uint64_t grp = j.group_pattern ? (1ull << j.group_shift) : 1;
    if (j.group_pattern)
        B = std::max<uint64_t>(grp, B / grp * grp);
    const uint64_t ngrp_max = j.group_pattern ? B / grp + 1 : 0;
    bool pin_in = true;
    for (uint32_t f = 0; f < j.nfrags && pin_in; ++f)
        pin_in = is_pinned_host(j.frags[f]);
    bool pin_out = true;
    if (j.outs) {
        for (uint32_t r = 0; r < j.rows && pin_out; ++r)
            pin_out = is_pinned_host(j.outs[r]);
    } else {
        pin_out = is_pinned_host(j.out);
    }
    const bool staged = !(pin_in && pin_out);

    Stage *s = acquire(dev);
    if (!s)
        return -EIO;
    int rc = ensure(s, B * j.nfrags * ECD_CHUNK, B * out_stripe, ngrp_max, staged);
    uint64_t pend_start[2] = {0, 0}, pend_cnt[2] = {0, 0};
    int it = 0;
    for (uint64_t a = j.s0; rc == 0 && a < j.s1; a += B, ++it) {
        const int sl = it & 1;
        const uint64_t cnt = std::min(B, j.s1 - a);
        hipStream_t st = s->st[sl];
        if (hipStreamSynchronize(st) != hipSuccess) {
            rc = -EIO;
            break;
        }
        if (pend_cnt[sl] && !pin_out)
            flush_decode(j, s->pin_out[sl], pend_start[sl], pend_cnt[sl], B);
        pend_cnt[sl] = 0;

        for (uint32_t f = 0; f < j.nfrags && rc == 0; ++f) {
            if (!j.frags[f])
                continue;
            const uint8_t *src = j.frags[f] + a * ECD_CHUNK;
            uint8_t *dst = s->din[sl] + (uint64_t)f * B * ECD_CHUNK;
            if (!pin_in) {
                uint8_t *pin = s->pin_in[sl] + (uint64_t)f * B * ECD_CHUNK;
                copy_bytes(pin, src, cnt * ECD_CHUNK);
                src = pin;
            }
            if (hipMemcpyAsync(dst, src, cnt * ECD_CHUNK, hipMemcpyHostToDevice, st) !=
                hipSuccess)
                rc = -EIO;
        }
        if (rc)
            break;

        ecd_combine_desc_t d;
        memset(&d, 0, offsetof(ecd_combine_desc_t, pat));
        d.k = j.k;
        d.rows = j.rows;
        d.nstripes = cnt;
        d.in_stride = ECD_CHUNK;
        for (uint32_t f = 0; f < j.nfrags; ++f)
            d.in_base[f] = s->din[sl] + (uint64_t)f * B * ECD_CHUNK;
        if (j.outs) {
            d.out_stride = ECD_CHUNK;
            for (uint32_t r = 0; r < j.rows; ++r)
                d.out_base[r] = s->dout[sl] + (uint64_t)r * B * ECD_CHUNK;
        } else {
            d.out_stride = out_stripe;
            for (uint32_t r = 0; r < j.rows; ++r)
                d.out_base[r] = s->dout[sl] + (uint64_t)r * ECD_CHUNK;
        }
        d.npatterns = j.npatterns;
        d.pat_bytes = j.k + j.rows * j.k;
        memcpy(d.pat, j.pats, (size_t)j.npatterns * d.pat_bytes);
        if (j.group_pattern) {
            /* a is a multiple of the group size (B is, and s0 is aligned) */
            const uint64_t g0 = a >> j.group_shift;
            const uint64_t gn = (cnt + grp - 1) >> j.group_shift;
            memcpy(s->pin_grp[sl], j.group_pattern + g0, gn);
            if (hipMemcpyAsync(s->dgrp[sl], s->pin_grp[sl], gn, hipMemcpyHostToDevice, st) !=
                hipSuccess) {
                rc = -EIO;
                break;
            }
            d.group_pattern = s->dgrp[sl];
            d.group_shift = j.group_shift;
        }
        rc = ecdk_combine(st, &d);
        if (rc)
            break;
        if (j.outs) {
            for (uint32_t r = 0; r < j.rows && rc == 0; ++r) {
                uint8_t *dst = pin_out ? j.outs[r] + a * ECD_CHUNK
                                       : s->pin_out[sl] + (uint64_t)r * B * ECD_CHUNK;
                if (hipMemcpyAsync(dst, s->dout[sl] + (uint64_t)r * B * ECD_CHUNK,
                                   cnt * ECD_CHUNK, hipMemcpyDeviceToHost, st) != hipSuccess)
                    rc = -EIO;
            }
        } else {
            uint8_t *dst = pin_out ? j.out + a * out_stripe : s->pin_out[sl];
            if (hipMemcpyAsync(dst, s->dout[sl], cnt * out_stripe, hipMemcpyDeviceToHost,
                               st) != hipSuccess)
                rc = -EIO;
        }
        if (rc)
            break;
        pend_start[sl] = a;
        pend_cnt[sl] = cnt;
    }
    for (int sl = 0; sl < 2; ++sl) {
        if (hipStreamSynchronize(s->st[sl]) != hipSuccess)
            rc = rc ? rc : -EIO;
        if (rc == 0 && pend_cnt[sl] && !pin_out)
            flush_decode(j, s->pin_out[sl], pend_start[sl], pend_cnt[sl], B);
    }
    release(s);
    return rc;
}

/* Run fn(dev, s0, s1) over a stripe-range partition; `align` keeps every
 * range boundary a multiple of it (pattern groups). */
template <typename F>
int partition(int ndev, uint64_t nstripes, uint64_t align, F fn)
{
    if (g_ndev == 0)
        return -ENODEV;
    if (ndev <= 0 || ndev > g_ndev)
        ndev = g_ndev;
    const uint64_t units = (nstripes + align - 1) / align;
    if ((uint64_t)ndev > units)
        ndev = (int)std::max<uint64_t>(1, units);
    std::vector<int> rcs(ndev, 0);
    std::vector<std::thread> th;
    for (int d = 0; d < ndev; ++d) {
        const uint64_t s0 = std::min(nstripes, units * d / ndev * align);
        const uint64_t s1 = std::min(nstripes, units * (d + 1) / ndev * align);
        if (d == ndev - 1)
            rcs[d] = fn(d, s0, s1);
        else
            th.emplace_back([&, d, s0, s1] { rcs[d] = fn(d, s0, s1); });
    }
    for (auto &t : th)
        t.join();
    for (int rc : rcs)
        if (rc)
            return rc;
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
    static thread_local std::string copy;
    std::lock_guard<std::mutex> g(g_err_mu);
    copy = g_err;
    return copy.c_str();
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
    HIPCHK(hipSetDevice(g_dev_ids[device]));
    return ecdk_encode_vander(pick_stream(stream), k, n, nstripes, in, out);
}

int ecd_combine(int device, void *stream, const ecd_combine_desc_t *d)
{
    if (ecd_device_count() <= device || device < 0)
        return -ENODEV;
    HIPCHK(hipSetDevice(g_dev_ids[device]));
    return ecdk_combine(pick_stream(stream), d);
}

int ecd_sync(int device, void *stream)
{
    if (ecd_device_count() <= device || device < 0)
        return -ENODEV;
    HIPCHK(hipSetDevice(g_dev_ids[device]));
    HIPCHK(hipStreamSynchronize(pick_stream(stream)));
    return 0;
}

int ecd_encode_host(int ndev, uint32_t k, uint32_t n, uint64_t nstripes, const void *in,
                    void *const *out, const uint8_t *enc_pat)
{
    if (ecd_device_count() == 0)
        return -ENODEV;
    EncodeJob base;
    base.k = k;
    base.n = n;
    base.in = static_cast<const uint8_t *>(in);
    base.out = reinterpret_cast<uint8_t *const *>(out);
    base.enc_pat = enc_pat;
    return partition(ndev, nstripes, 1, [&](int d, uint64_t s0, uint64_t s1) {
        EncodeJob j = base;
        j.s0 = s0;
        j.s1 = s1;
        return run_encode_dev(d, j);
    });
}

int ecd_decode_host(int ndev, uint32_t k, uint32_t rows, uint64_t nstripes, uint32_t nfrags,
                    const void *const *frags, void *out, void *const *outs, uint32_t npatterns,
                    const uint8_t *pats, const uint8_t *group_pattern, uint32_t group_shift)
{
    if (ecd_device_count() == 0)
        return -ENODEV;
    if (nfrags == 0 || nfrags > ECD_MAX_ROWS || k == 0 || k > ECD_MAX_K || rows == 0 ||
        rows > ECD_MAX_ROWS || npatterns == 0 ||
        (uint64_t)npatterns * (k + rows * k) > ECD_MAX_PAT_BYTES)
        return -EINVAL;
    if (group_pattern && (group_shift < 3 || group_shift > 40))
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
    return partition(ndev, nstripes, align, [&](int d, uint64_t s0, uint64_t s1) {
        DecodeJob j = base;
        j.s0 = s0;
        j.s1 = s1;
        return run_decode_dev(d, j);
    });
}

int ecd_ptr_device(const void *p)
{
    if (!p || ecd_device_count() == 0)
        return -1;
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return -1;
    }
    if (a.type != hipMemoryTypeDevice)
        return -1;
    for (int i = 0; i < g_ndev; ++i)
        if (g_dev_ids[i] == a.device)
            return i;
    return -1;
}

void *ecd_host_alloc(size_t bytes)
{
    if (ecd_device_count() == 0)
        return nullptr;
    void *p = nullptr;
    if (hipHostMalloc(&p, bytes ? bytes : 1, hipHostMallocDefault) != hipSuccess)
        return nullptr;
    return p;
}

void ecd_host_free(void *p)
{
    if (p)
        (void)hipHostFree(p);
}

} /* extern "C" */
