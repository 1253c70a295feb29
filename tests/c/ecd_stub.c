/* Device layer stand-in for the host-only sanitizer build
 * (tests/test_sanitizers.py): no GPU, so ec_method.c takes its CPU engine
 * paths.  Every entry point of glusterfs_amd/csrc/ec_device.h. */
#include <stdio.h>
#include <stdlib.h>
#include <errno.h>
#include <stddef.h>
#include <string.h>

#include "../../glusterfs_amd/csrc/ec_cpu.h"
#include "../../glusterfs_amd/csrc/ec_device.h"

/* ECD_STUB_GPU=1: pretend one device whose host entry points code on the
 * CPU engine, so the split-call path (a helper thread codes the "GPU" share
 * while the caller codes the rest) runs under the sanitizers. */
static int stub_gpu(void)
{
    static int v = -1;
    if (v < 0) {
        const char *e = getenv("ECD_STUB_GPU");
        v = e && *e == '1';
    }
    return v;
}
int ecd_device_count(void) { return stub_gpu(); }
/* per-thread error record, as ec_device.hip keeps it */
static __thread char t_err[256];
static __thread uint64_t t_seq;
const char *ecd_last_error(void) { return t_err[0] ? t_err : "no device (sanitizer build)"; }
uint64_t ecd_error_seq(void) { return t_seq; }
void ecd_set_error(const char *text)
{
    snprintf(t_err, sizeof t_err, "%s", text ? text : "");
    t_seq++;
}
int ecd_has_vander(uint32_t k, uint32_t n) { (void)k; (void)n; return 0; }
int ecd_encode_vander(int d, void *s, uint32_t k, uint32_t n, uint64_t ns, const void *in,
                      void *const *out)
{ (void)d; (void)s; (void)k; (void)n; (void)ns; (void)in; (void)out; return -ENODEV; }
int ecd_combine(int d, void *s, const ecd_combine_desc_t *x) { (void)d; (void)s; (void)x; return -ENODEV; }
int ecd_sync(int d, void *s) { (void)d; (void)s; return -ENODEV; }
int ecd_encode_host(int nd, uint32_t k, uint32_t n, uint64_t ns, const void *in, void *const *out,
                    const uint8_t *p)
{
    (void)nd; (void)p;
    if (!stub_gpu())
        return -ENODEV;
    ecc_encode(ecc_isa_max(), k, n, ns, (const uint8_t *)in, (uint8_t *const *)out);
    return 0;
}
int ecd_encode_host_rows(int nd, uint32_t k, uint32_t r, uint64_t ns, const void *in,
                         void *const *out, const uint8_t *p)
{
    ecd_combine_desc_t d;
    (void)nd;
    if (!stub_gpu())
        return -ENODEV;
    memset(&d, 0, offsetof(ecd_combine_desc_t, pat));
    d.k = k;
    d.rows = r;
    d.nstripes = ns;
    d.in_stride = (uint64_t)k * 512;
    d.out_stride = 512;
    for (uint32_t i = 0; i < k; i++)
        d.in_base[i] = (const uint8_t *)in + i * 512;
    for (uint32_t i = 0; i < r; i++)
        d.out_base[i] = out[i];
    d.npatterns = 1;
    d.pat_bytes = k + r * k;
    d.pat_ext = p;
    return ecc_combine(ecc_isa_max(), &d);
}
int ecd_encode_host_gather(int nd, uint32_t k, uint32_t n, uint64_t ns, uint32_t sg,
                           const void *const *sp, const uint64_t *sl, void *const *out,
                           const uint8_t *p)
{ (void)nd; (void)k; (void)n; (void)ns; (void)sg; (void)sp; (void)sl; (void)out; (void)p; return -ENODEV; }
int ecd_writev_encode_device(int d, void *s, uint32_t k, uint32_t n, uint64_t h, uint64_t us,
                             const void *u, const void *oh, const void *ot, void *const *out,
                             const uint8_t *p)
{ (void)d; (void)s; (void)k; (void)n; (void)h; (void)us; (void)u; (void)oh; (void)ot; (void)out; (void)p; return -ENODEV; }
int ecd_decode_host(int nd, uint32_t k, uint32_t rows, uint64_t ns, uint32_t nf,
                    const void *const *f, void *out, void *const *outs, uint32_t np,
                    const uint8_t *p, const uint8_t *gp, uint32_t gs)
{
    ecd_combine_desc_t d;
    (void)nd;
    if (!stub_gpu())
        return -ENODEV;
    memset(&d, 0, offsetof(ecd_combine_desc_t, pat));
    d.k = k;
    d.rows = rows;
    d.nstripes = ns;
    d.in_stride = 512;
    for (uint32_t i = 0; i < nf; i++)
        d.in_base[i] = f[i];
    d.out_stride = outs ? 512 : (uint64_t)rows * 512;
    for (uint32_t r = 0; r < rows; r++)
        d.out_base[r] = outs ? outs[r] : (uint8_t *)out + r * 512;
    d.npatterns = np;
    d.pat_bytes = k + rows * k;
    d.pat_ext = p;
    d.group_pattern = gp;
    d.group_shift = gs;
    return ecc_combine(ecc_isa_max(), &d);
}
int ecd_ptr_device(const void *p) { (void)p; return -1; }
void *ecd_host_alloc(size_t b) { (void)b; return NULL; }
void ecd_host_free(void *p) { (void)p; }
int ecd_host_register(void *p, size_t b) { (void)p; (void)b; return -ENODEV; }
int ecd_host_unregister(void *p) { (void)p; return -ENODEV; }
int ecd_host_register_async(void *p, size_t b) { (void)p; (void)b; return -ENODEV; }
void ecd_host_register_flush(void) {}
void *ecd_buffer_get(size_t b) { (void)b; return NULL; }
int ecd_buffer_put(void *p) { (void)p; return 0; }
void ecd_pool_stats(ecd_pool_stats_t *s) { memset(s, 0, sizeof(*s)); }
uint64_t ecd_host_inflight(void) { return stub_gpu() ? 0 : UINT64_MAX; }
void ecd_inject_faults(uint32_t n) { (void)n; }
int ecd_host_mapped(const void *p, size_t n) { (void)p; (void)n; return stub_gpu(); }
int ecd_device_numa_node(int d) { (void)d; return -ENODEV; }
int ecd_copy_threads(void) { return 0; }
void ecd_jit_stats(ecd_jit_stats_t *s) { memset(s, 0, sizeof(*s)); }
int ecd_jit_compile_check(uint32_t k, uint32_t r, const uint8_t *c, uint32_t *o, char *l, size_t n)
{ (void)k; (void)r; (void)c; (void)o; (void)l; (void)n; return -ENOSYS; }
int ecd_jit_prepare(uint32_t k, uint32_t r, const uint8_t *c)
{ (void)k; (void)r; (void)c; return -ENOSYS; }
