/* ec_kernels.h -- launch wrappers exported by ec_kernels.hip (C++ only). */
#ifndef EC_MI355X_KERNELS_H
#define EC_MI355X_KERNELS_H

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ec_device.h"

/* Record `what` failed with HIP error `hip_error` as the calling thread's
 * last error (ec_device.hip); returns -EIO. */
extern "C" int ecd_hip_fail(const char *what, int hip_error);

int ecdk_has_vander(uint32_t k, uint32_t n);
/* zc: buffers are pinned host memory coded over PCIe (ec_encode_vander_zc) */
int ecdk_encode_vander(hipStream_t s, uint32_t k, uint32_t n, uint64_t nstripes,
                       const void *in, void *const *out, bool zc = false);
int ecdk_combine(hipStream_t s, const ecd_combine_desc_t *d);
/* the same on pinned host memory (host-buffer path, zero-copy over PCIe) */
int ecdk_combine_host(hipStream_t s, const ecd_combine_desc_t *d);
/* Partial-stripe writes: materialise bytes [o0, o0+n) (n % 16 == 0) of the
 * virtual input {head[0:b1) | user[0:b2-b1) | tail[...]} into dst, and the
 * fused Vandermonde encode that reads interior stripes from user directly. */
int ecdk_rmw_gather(hipStream_t s, const uint8_t *head, const uint8_t *user, const uint8_t *tail,
                    uint64_t b1, uint64_t b2, uint64_t o0, uint64_t n, uint8_t *dst);
int ecdk_encode_vander_rmw(hipStream_t s, uint32_t k, uint32_t n, uint64_t nstripes,
                           const uint8_t *edge, const uint8_t *user_shift, void *const *out);

namespace ecdev {
struct CombineArgs;
}
int ecdk_pack_args(const ecd_combine_desc_t *d, ecdev::CombineArgs *a);

#endif
