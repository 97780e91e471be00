// Accuracy of the gfx950 v_rcp_f64 estimate and of one / two Newton steps
// on it (diagnostic: which reciprocals of the lane solver can drop a step).
//   hipcc --offload-arch=gfx950 -O3 -w -o tools/rcp_accuracy tools/rcp_accuracy.hip
// Prints the largest relative error of each against the correctly rounded
// 1/x, over 2^24 inputs spread over [1e-300, 1e300] (both signs).
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>

__global__ void k_rcp(const double* x, double* r0, double* r1, double* r2, double* ex, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double v = x[i];
    double r = __builtin_amdgcn_rcp(v);
    r0[i] = r;
    double s = __builtin_fma(__builtin_fma(-v, r, 1.0), r, r);
    r1[i] = s;
    r2[i] = __builtin_fma(__builtin_fma(-v, s, 1.0), s, s);
    ex[i] = 1.0 / v;
}

int main() {
    const int n = 1 << 24;
    double* h = (double*)std::malloc(sizeof(double) * n * 5);
    srand(7);
    for (int i = 0; i < n; ++i) {
        const double e = -300.0 + 600.0 * (double)rand() / RAND_MAX;
        const double m = 1.0 + (double)rand() / RAND_MAX;
        h[i] = ((i & 1) ? -1.0 : 1.0) * m * std::pow(10.0, e);
    }
    double *dx, *d0, *d1, *d2, *de;
    if (hipMalloc(&dx, sizeof(double) * n) || hipMalloc(&d0, sizeof(double) * n) || hipMalloc(&d1, sizeof(double) * n) ||
        hipMalloc(&d2, sizeof(double) * n) || hipMalloc(&de, sizeof(double) * n))
        return 1;
    if (hipMemcpy(dx, h, sizeof(double) * n, hipMemcpyHostToDevice)) return 1;
    hipLaunchKernelGGL(k_rcp, dim3(n / 256), dim3(256), 0, 0, dx, d0, d1, d2, de, n);
    if (hipDeviceSynchronize()) return 1;
    double* r[4] = {h + n, h + 2 * n, h + 3 * n, h + 4 * n};
    if (hipMemcpy(r[0], d0, sizeof(double) * n, hipMemcpyDeviceToHost) ||
        hipMemcpy(r[1], d1, sizeof(double) * n, hipMemcpyDeviceToHost) ||
        hipMemcpy(r[2], d2, sizeof(double) * n, hipMemcpyDeviceToHost) ||
        hipMemcpy(r[3], de, sizeof(double) * n, hipMemcpyDeviceToHost))
        return 1;
    double mx[3] = {0, 0, 0};
    long exact[3] = {0, 0, 0};
    for (int i = 0; i < n; ++i) {
        const double t = 1.0 / h[i];   // host IEEE division (correctly rounded)
        if (t != r[3][i]) { std::printf("device 1/x differs at %d\n", i); }
        for (int k = 0; k < 3; ++k) {
            const double e = std::fabs((r[k][i] - t) / t);
            if (e > mx[k]) mx[k] = e;
            exact[k] += (r[k][i] == t);
        }
    }
    std::printf("{\"n\": %d, \"rcp_max_rel\": %.3e, \"nr1_max_rel\": %.3e, \"nr2_max_rel\": %.3e, "
                "\"rcp_exact\": %.4f, \"nr1_exact\": %.4f, \"nr2_exact\": %.4f}\n",
                n, mx[0], mx[1], mx[2], exact[0] / (double)n, exact[1] / (double)n, exact[2] / (double)n);
    return 0;
}
