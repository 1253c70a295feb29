// gpridx.hip -- does GPR indexing (s_set_gpr_idx_on, DST|SRC0) apply to VOP3
// v_bitop3_b32 on gfx950 with SRC1/SRC2 left unindexed?  (r06 feasibility
// probe for a run-time four-Russians combine; development only)
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k(unsigned *out, int idx)
{
    unsigned r[6];
    const unsigned lane = threadIdx.x;
    unsigned a0 = 0x1000u + lane, a1 = 0x2000u + lane, a2 = 0x3000u + lane;
    const unsigned t1 = 0x00F0u, t2 = 0x0F00u;
    // v[a0 + idx] = bitop3(v[a0 + idx], t1, t2) with the three a's pinned
    // contiguously (v40, v41, v42) and the tables at v50, v51
    asm volatile(
        "v_mov_b32 v40, %[a0]\n"
        "v_mov_b32 v41, %[a1]\n"
        "v_mov_b32 v42, %[a2]\n"
        "v_mov_b32 v50, %[t1]\n"
        "v_mov_b32 v51, %[t2]\n"
        "s_set_gpr_idx_on %[idx], gpr_idx(SRC0,DST)\n"
        "v_bitop3_b32 v40, v40, v50, v51 bitop3:0x96\n"
        "v_xor_b32 v40, v40, v50\n"
        "s_set_gpr_idx_off\n"
        "v_mov_b32 %[r0], v40\n"
        "v_mov_b32 %[r1], v41\n"
        "v_mov_b32 %[r2], v42\n"
        : [r0] "=v"(r[0]), [r1] "=v"(r[1]), [r2] "=v"(r[2])
        : [a0] "v"(a0), [a1] "v"(a1), [a2] "v"(a2), [t1] "v"(t1), [t2] "v"(t2), [idx] "s"(idx)
        : "v40", "v41", "v42", "v50", "v51", "m0");
    out[lane * 3 + 0] = r[0];
    out[lane * 3 + 1] = r[1];
    out[lane * 3 + 2] = r[2];
}

int main()
{
    unsigned *d, h[64 * 3];
    int bad = 0;
    if (hipMalloc(&d, sizeof h) != hipSuccess)
        return 2;
    for (int idx = 0; idx < 3; ++idx) {
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, idx);
        if (hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost) != hipSuccess)
            return 3;
        for (unsigned l = 0; l < 64; ++l)
            for (int j = 0; j < 3; ++j) {
                unsigned want = (0x1000u * (j + 1)) + l;
                if (j == idx)
                    want = want ^ 0x00F0u ^ 0x0F00u ^ 0x00F0u;   // bitop3 then xor
                if (h[l * 3 + j] != want) {
                    if (bad < 8)
                        printf("idx %d lane %u a%d: got %x want %x\n", idx, l, j, h[l * 3 + j], want);
                    bad++;
                }
            }
    }
    printf("gpridx: %s (%d mismatches)\n", bad ? "FAIL" : "ok", bad);
    return bad != 0;
}
