/*
 * ec_cpu.h -- the library's CPU coding engine (internal; C).
 *
 * The reference coder is pure CPU C and never fails (ec-method.c:393-433;
 * an unknown or unsupported engine falls back to portable C,
 * ec-code.c:1007-1013, 1030-1034).  This engine keeps that contract for the
 * MI355X library:
 *   - the coder of a volume mounted on a node without gfx950 GPU, or with
 *     cpu-extensions = none / x64 / sse / avx (ec.c:1786-1794);
 *   - the fallback when a device submission fails for host buffers, so
 *     ec_method_encode (void) never aborts on a GPU fault;
 *   - the small-call side of the CPU/GPU crossover:
 *     128 KiB FUSE writes cost less on the calling thread than a PCIe round
 *     trip, and calls that find the GPUs saturated run here.
 *
 * It works on the same bit-sliced chunks as the kernels (512-byte chunks of
 * 8 planes x 64 bytes, ec-method.h:27-29): one plane is one 64-byte vector
 * (one zmm with AVX-512, two ymm with AVX2, four xmm otherwise), and a
 * multiply by a constant is the searched straight-line program of
 * ec_gf8_prog.h, the same one the gfx950 kernels run.  It is the product's
 * own implementation: it does not use or link oracle/ (the test checker).
 * All work runs on the calling thread, as the reference's does.
 */
#ifndef EC_MI355X_CPU_H
#define EC_MI355X_CPU_H

#include <stddef.h>
#include <stdint.h>

#include "ec_device.h"

#ifdef __cplusplus
extern "C" {
#endif

enum { ECC_ISA_BASE = 0, ECC_ISA_AVX2 = 1, ECC_ISA_AVX512 = 2 };

/* Highest ISA level this CPU supports (and this build contains). */
int ecc_isa_max(void);
const char *ecc_isa_name(int isa);

/* Vandermonde encode (ec-method.c:394-408 with ec_code_c_linear's Horner
 * rows, ec-code-c.c:11647-11657): out[i] + t*512 = Horner over the k data
 * chunks of stripe t with v = i + 1.  in: nstripes*k*512 bytes. */
void ecc_encode(int isa, uint32_t k, uint32_t n, uint64_t nstripes, const uint8_t *in,
                uint8_t *const *out);

/* Encode of a virtual input (segments, NULL = zeros), nstripes*k*512 bytes:
 * stripes inside one segment are read in place, the others gathered into a
 * stripe buffer.  Returns 0 or -EINVAL (segment lengths do not add up). */
int ecc_encode_gather(int isa, uint32_t k, uint32_t n, uint64_t nstripes, uint32_t nsegs,
                      const void *const *seg_ptr, const uint64_t *seg_len, uint8_t *const *out);

/* The generic combination of ecd_combine_desc_t (decode, mixed-pattern
 * decode, heal, generic encode) on host memory: every pointer in *d is a host
 * pointer and group_pattern, when set, is a host array.  Returns 0 or
 * -EINVAL. */
int ecc_combine(int isa, const ecd_combine_desc_t *d);

/* ---- per-ISA kernels (ec_cpu_kern.c, compiled once per level) ---- */
#define ECC_DECLARE(sfx)                                                              \
    void ecc_encode_##sfx(uint32_t k, uint32_t n, uint64_t nstripes, const uint8_t *in,  \
                          uint64_t in_stride, uint8_t *const *out, uint64_t out_off);   \
    void ecc_combine_##sfx(const ecd_combine_desc_t *d, const uint8_t *pats, uint64_t s0, \
                           uint64_t s1);
ECC_DECLARE(base)
#if defined(__x86_64__)
ECC_DECLARE(avx2)
ECC_DECLARE(avx512)
#endif
#undef ECC_DECLARE

#ifdef __cplusplus
}
#endif

#endif
