/* ec_kernels.h -- launch wrappers exported by ec_kernels.hip (C++ only). */
#ifndef EC_MI355X_KERNELS_H
#define EC_MI355X_KERNELS_H

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ec_device.h"

int ecdk_has_vander(uint32_t k, uint32_t n);
/* zc: buffers are pinned host memory coded over PCIe (ec_encode_vander_zc) */
int ecdk_encode_vander(hipStream_t s, uint32_t k, uint32_t n, uint64_t nstripes,
                       const void *in, void *const *out, bool zc = false);
int ecdk_combine(hipStream_t s, const ecd_combine_desc_t *d);

namespace ecdev {
struct CombineArgs;
}
int ecdk_pack_args(const ecd_combine_desc_t *d, ecdev::CombineArgs *a);

#endif
