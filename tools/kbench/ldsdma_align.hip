/*
 * ldsdma_align.hip -- does global_load_lds_dwordx4 (LDS-DMA, 16 B per lane)
 * honour a source address that is not 16-byte aligned?  One block, 64
 * lanes, every access in bounds; for each byte offset the LDS image is
 * copied out and compared with the expected bytes on the host.
 *   hipcc -O3 --offload-arch=gfx950 tools/kbench/ldsdma_align.hip -o tools/kbench/ldsdma_align
 */
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <vector>

__global__ __launch_bounds__(64) void probe(const uint8_t *src, uint32_t off, uint8_t *out)
{
    __shared__ __attribute__((aligned(16))) uint8_t lds[1024];
    const uint32_t lane = threadIdx.x;
    __builtin_amdgcn_global_load_lds(
        (const __attribute__((address_space(1))) void *)(src + off + lane * 16u),
        (__attribute__((address_space(3))) void *)lds, 16, 0, 0);
    __syncthreads();
    for (uint32_t i = lane; i < 256; i += 64)
        reinterpret_cast<uint32_t *>(out)[i] = reinterpret_cast<const uint32_t *>(lds)[i];
}

int main()
{
    const size_t n = 4096;
    std::vector<uint8_t> h(n);
    for (size_t i = 0; i < n; ++i)
        h[i] = (uint8_t)(i * 7 + 3);
    uint8_t *src, *out;
    if (hipMalloc(&src, n) != hipSuccess || hipMalloc(&out, 1024) != hipSuccess)
        return 1;
    hipMemcpy(src, h.data(), n, hipMemcpyHostToDevice);
    int bad = 0;
    for (uint32_t off : {0u, 1u, 2u, 3u, 4u, 5u, 8u, 12u, 15u, 16u, 33u}) {
        hipMemset(out, 0, 1024);
        hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, src, off, out);
        if (hipDeviceSynchronize() != hipSuccess) {
            printf("off %u: launch error\n", off);
            return 2;
        }
        std::vector<uint8_t> g(1024);
        hipMemcpy(g.data(), out, 1024, hipMemcpyDeviceToHost);
        const int ok = !memcmp(g.data(), h.data() + off, 1024);
        int down = -1;   /* does it match the 16-B-aligned-down source? */
        if (!ok)
            down = !memcmp(g.data(), h.data() + (off & ~15u), 1024);
        printf("off %2u: %s%s\n", off, ok ? "exact" : "MISMATCH",
               down == 1 ? " (= aligned-down source)" : "");
        bad += !ok;
    }
    printf("%s\n", bad ? "LDS-DMA needs 16-byte-aligned sources" : "LDS-DMA honours any byte address");
    return 0;
}
