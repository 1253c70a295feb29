/* ec_jit.h -- per-pattern whole-matrix kernels compiled at run time (r06,
 * ec_jit.hip).  Device-layer internal interface. */
#ifndef EC_MI355X_JIT_H
#define EC_MI355X_JIT_H

#include <hip/hip_runtime.h>

#include "ec_device.h"

#define ECJ_MAX 16

#ifdef __cplusplus
extern "C" {
#endif

/* 1: a combine this module would run with a compiled whole-matrix kernel
 * once its pattern's code exists (one pattern, k >= 12 and rows >= 12,
 * enough stripes, 16-byte aligned outputs, EC_MI355X_JIT not 0) */
int ecj_eligible(const ecd_combine_desc_t *d);
/* Launch the pattern's kernel on s: 0, or -EAGAIN when its code is not
 * there (yet) or failed -- the caller then runs the shipped kernel.  nt:
 * non-temporal staging loads. */
int ecj_launch(hipStream_t s, const ecd_combine_desc_t *d, int nt);

#ifdef __cplusplus
}
#endif

#endif
