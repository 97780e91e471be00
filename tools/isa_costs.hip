// Issue cost of the fp64 VALU instructions the lane solver is made of
// (gfx950), measured with the shader clock (diagnostic; built and run by hand:
//   hipcc --offload-arch=gfx950 -O3 -o tools/isa_costs tools/isa_costs.hip
//   ./tools/isa_costs > isa_costs.jsonl           (on the GPU box)
// Each wavefront runs REPS x an unrolled block of 8 independent chains x 16
// instructions written in inline asm (so the encoding is the one named), and
// records its elapsed shader-clock cycles.  W waves per SIMD (grid = 1024 W
// one-wave blocks, all co-resident at this register use): cycles per
// instruction per SIMD = elapsed / (W x instructions per wave).
//   fmac_e32   v_fmac_f64_e32  (4-byte VOP2)
//   fma_vop3   v_fma_f64       (8-byte VOP3, three VGPR sources)
//   mul_vop3   v_mul_f64       (8-byte VOP3)
//   add_vop3   v_add_f64       (8-byte VOP3)
//   mul_fmac   v_mul_f64 and v_fmac_f64_e32 alternating
//   cnd_e32    v_cndmask_b32_e32 (VOP2, 32-bit)
//   rcp        v_rcp_f64       (transcendental)
//   lat_fma    one dependent chain of v_fmac_f64_e32 (latency)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define REPS 1024
static double g_wall_ns_per_inst = 0.0;

#define X8(S) S(0) S(1) S(2) S(3) S(4) S(5) S(6) S(7)

template <int OP>
__global__ void __launch_bounds__(64) k_cost(double* out, long long* cyc, double seed) {
    double v0 = seed + threadIdx.x, v1 = v0 + 1, v2 = v0 + 2, v3 = v0 + 3, v4 = v0 + 4, v5 = v0 + 5, v6 = v0 + 6,
           v7 = v0 + 7;
    double b = 1.0000001 + seed * 1e-9, c = 1e-30 * seed;
    unsigned m0 = threadIdx.x, m1 = threadIdx.x * 3u;
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_sched_barrier(0);
    const long long t0 = __builtin_readcyclecounter();
    __builtin_amdgcn_sched_barrier(0);
    for (int r = 0; r < REPS; ++r) {
#pragma unroll
        for (int k = 0; k < 16; ++k) {
#define V(i) v##i
            if constexpr (OP == 0) {
#define S(i) asm volatile("v_fmac_f64_e32 %0, %1, %2" : "+v"(V(i)) : "v"(b), "v"(c));
                X8(S)
#undef S
            } else if constexpr (OP == 1) {
#define S(i) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(V(i)) : "v"(b), "v"(c));
                X8(S)
#undef S
            } else if constexpr (OP == 2) {
#define S(i) asm volatile("v_mul_f64 %0, %0, %1" : "+v"(V(i)) : "v"(b));
                X8(S)
#undef S
            } else if constexpr (OP == 3) {
#define S(i) asm volatile("v_add_f64 %0, %0, %1" : "+v"(V(i)) : "v"(c));
                X8(S)
#undef S
            } else if constexpr (OP == 4) {
#define S(i) if ((i) & 1) asm volatile("v_fmac_f64_e32 %0, %1, %2" : "+v"(V(i)) : "v"(b), "v"(c)); \
             else asm volatile("v_mul_f64 %0, %0, %1" : "+v"(V(i)) : "v"(b));
                X8(S)
#undef S
            } else if constexpr (OP == 5) {
#define S(i) asm volatile("v_cndmask_b32_e32 %0, %0, %1, vcc" : "+v"(m0) : "v"(m1) : "vcc");
                X8(S)
#undef S
            } else if constexpr (OP == 6) {
#define S(i) asm volatile("v_rcp_f64 %0, %0" : "+v"(V(i)));
                X8(S)
#undef S
            } else {
                asm volatile("v_fmac_f64_e32 %0, %1, %2" : "+v"(v0) : "v"(b), "v"(c));
            }
#undef V
        }
    }
    __builtin_amdgcn_sched_barrier(0);
    const long long t1 = __builtin_readcyclecounter();
    __builtin_amdgcn_sched_barrier(0);
    out[blockIdx.x * 64 + threadIdx.x] = v0 + v1 + v2 + v3 + v4 + v5 + v6 + v7 + m0;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int OP>
static double run(int w, double* d_out, long long* d_cyc) {
    const int blocks = 1024 * w;
    const double per_wave = (OP == 7) ? 16.0 * REPS : 8.0 * 16.0 * REPS;
    double best = 1e30;
    static long long h[1024 * 16];
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int rep = 0; rep < 3; ++rep) {
        hipEventRecord(e0, 0);
        hipLaunchKernelGGL((k_cost<OP>), dim3(blocks), dim3(64), 0, 0, d_out, d_cyc, 1.5);
        hipEventRecord(e1, 0);
        if (hipDeviceSynchronize() != hipSuccess) { std::printf("launch failed\n"); std::exit(1); }
        float ms = 0.f;
        hipEventElapsedTime(&ms, e0, e1);
        // wall rate: wave-instructions per SIMD per ns (x 1/GHz = cycles per instruction)
        g_wall_ns_per_inst = 1e6 * ms / (per_wave * w);
        if (hipMemcpy(h, d_cyc, sizeof(long long) * blocks, hipMemcpyDeviceToHost) != hipSuccess) std::exit(1);
        double m = 0;
        for (int b = 0; b < blocks; ++b) m += (double)h[b];
        m /= blocks;
        if (m < best) best = m;
    }
    std::fprintf(stderr, "op %d w %d: %.3f ns per wave-instruction per SIMD (wall)\n", OP, w, g_wall_ns_per_inst);
    return best / (per_wave * w);
}

int main() {
    double* d_out;
    long long* d_cyc;
    if (hipMalloc(&d_out, sizeof(double) * 64 * 1024 * 16) != hipSuccess) return 1;
    if (hipMalloc(&d_cyc, sizeof(long long) * 1024 * 16) != hipSuccess) return 1;
    for (int w : {1, 2, 3, 4}) {
        std::printf("{\"waves_per_simd\": %d, \"fmac_e32\": %.2f, \"fma_vop3\": %.2f, \"mul_vop3\": %.2f, "
                    "\"add_vop3\": %.2f, \"mul_fmac\": %.2f, \"cnd_e32\": %.2f, \"rcp\": %.2f, \"lat_fma\": %.2f}\n",
                    w, run<0>(w, d_out, d_cyc), run<1>(w, d_out, d_cyc), run<2>(w, d_out, d_cyc),
                    run<3>(w, d_out, d_cyc), run<4>(w, d_out, d_cyc), run<5>(w, d_out, d_cyc),
                    run<6>(w, d_out, d_cyc), run<7>(w, d_out, d_cyc) * w);
    }
    return 0;
}
