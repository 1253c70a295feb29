/*
 * valu.hip -- development probe (not product): VALU issue rate of the
 * instructions the XOR-tree kernels are made of, so the 16+4 decode's VALU
 * budget is measured instead of assumed.  Each lane runs 16 independent
 * chains of inline-asm v_bitop3_b32 / v_xor_b32 (asm volatile: nothing
 * folds), with `waves` waves per CU.  Prints wave-instructions per CU per ns
 * and, at the nominal 2.4 GHz, cycles per wave-instruction per SIMD.
 *
 *   hipcc -O3 --offload-arch=gfx950 tools/kbench/valu.hip -o tools/kbench/valu
 */
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    printf("HIP error %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

template <int OP>
__global__ __launch_bounds__(256) void k_valu(unsigned *sink, int iters)
{
    unsigned a[16];
#pragma unroll
    for (int i = 0; i < 16; ++i)
        a[i] = threadIdx.x * (i + 3) + blockIdx.x;
    unsigned b = threadIdx.x ^ 0x5a5a5a5au, c = threadIdx.x * 77u;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            if constexpr (OP == 0)
                asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(a[i]) : "v"(b), "v"(c));
            else if constexpr (OP == 1)
                asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
            else
                asm volatile("v_mov_b32 %0, %1" : "=v"(a[i]) : "v"(a[(i + 1) & 15]));
        }
    }
    unsigned x = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i)
        x ^= a[i];
    if (x == 0x1234567u)
        sink[0] = x;
}

template <int OP>
void run(const char *name, int waves_per_cu, int ncu)
{
    unsigned *sink;
    CHK(hipMalloc(&sink, 4));
    const int iters = 4096;
    const int blocks = ncu * waves_per_cu / 4;   /* 256-thread blocks = 4 waves */
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    hipLaunchKernelGGL(k_valu<OP>, dim3(blocks), dim3(256), 0, 0, sink, iters);
    CHK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
        CHK(hipEventRecord(e0));
        hipLaunchKernelGGL(k_valu<OP>, dim3(blocks), dim3(256), 0, 0, sink, iters);
        CHK(hipEventRecord(e1));
        CHK(hipEventSynchronize(e1));
        float ms;
        CHK(hipEventElapsedTime(&ms, e0, e1));
        best = ms < best ? ms : best;
    }
    const double winstr = (double)blocks * 4 * iters * 16;           /* wave-instructions */
    const double per_cu_ns = winstr / ncu / (best * 1e6);
    const double cyc_per_simd = 4.0 * 2.4 / per_cu_ns;              /* at 2.4 GHz */
    printf("%-8s waves/CU=%2d  %.3f ms  %.3f wave-instr/ns/CU  %.2f cyc/instr/SIMD@2.4GHz  "
           "%.1f T lane-ops/s\n", name, waves_per_cu, best, per_cu_ns, cyc_per_simd,
           winstr * 64 / (best * 1e-3) / 1e12);
    CHK(hipFree(sink));
}

int main()
{
    hipDeviceProp_t p;
    CHK(hipGetDeviceProperties(&p, 0));
    const int ncu = p.multiProcessorCount;
    printf("%s, %d CUs\n", p.gcnArchName, ncu);
    for (int w : {4, 8, 16, 32}) {
        run<0>("bitop3", w, ncu);
        run<1>("xor", w, ncu);
        run<2>("mov", w, ncu);
    }
    return 0;
}
