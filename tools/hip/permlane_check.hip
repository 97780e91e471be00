// Check (GPU) of the wave-wide broadcast from a compile-time lane built from
// DPP row_newbcast + v_permlane32_swap + v_permlane16_swap (gfx950), as
// csrc/mk_group.h wbc64 uses it: every lane must read lane k's value.
//   hipcc --offload-arch=gfx950 -O3 -o permlane_check permlane_check.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

__device__ __forceinline__ int pl_bcast(int v, int k) {
    int t = 0;
    switch (k & 15) {
#define PCK_BC(K) case K: t = __builtin_amdgcn_update_dpp(0, v, 0x150 + K, 0xf, 0xf, false); break;
        PCK_BC(0) PCK_BC(1) PCK_BC(2) PCK_BC(3) PCK_BC(4) PCK_BC(5) PCK_BC(6) PCK_BC(7)
        PCK_BC(8) PCK_BC(9) PCK_BC(10) PCK_BC(11) PCK_BC(12) PCK_BC(13) PCK_BC(14) PCK_BC(15)
#undef PCK_BC
    }
    const int r = k >> 4;
    const auto s32 = __builtin_amdgcn_permlane32_swap(t, t, false, false);
    const int u = (r < 2) ? (int)s32[0] : (int)s32[1];
    const auto s16 = __builtin_amdgcn_permlane16_swap(u, u, false, false);
    return (r & 1) ? (int)s16[1] : (int)s16[0];
}

__global__ void __launch_bounds__(64) k_check(int* bad) {
    const int lane = threadIdx.x;
    int nbad = 0;
#pragma unroll
    for (int k = 0; k < 64; ++k) {
        const int got = pl_bcast(1000 + 7 * lane, k);
        if (got != 1000 + 7 * k) ++nbad;
    }
    bad[lane] = nbad;
}

int main() {
    int* d = nullptr;
    int h[64];
    if (hipMalloc(&d, sizeof(h)) != hipSuccess) return 2;
    hipLaunchKernelGGL(k_check, dim3(1), dim3(64), 0, 0, d);
    if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 2;
    int tot = 0;
    for (int i = 0; i < 64; ++i) tot += h[i];
    printf("permlane broadcast: %d mismatches over 64 lanes x 64 sources\n", tot);
    hipFree(d);
    return tot ? 1 : 0;
}
