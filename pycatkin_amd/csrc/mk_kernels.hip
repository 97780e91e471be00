// HIP kernels + C-ABI entry points of pycatkin_amd (gfx950 / MI355X).
//
//   k_rate_constants   kernel (1): thermochemistry -> energy program -> kf/kr,
//                      one lane per condition (reaction.py:94, state.py:556)
//   k_species_rates    kernel (2): mass-action rates over the plan (old_system.py:227)
//   k_jacobian         kernel (2'): analytic Jacobian (old_system.py:293)
//   k_solve<NS>        kernel (3): Rosenbrock W-method to t_end + Newton steady-state
//                      polish, all state in VGPRs, k_eff in LDS (old_system.py:315,385)
//                      with kernel (4) fused in: TOF / activity, and in DRC mode the
//                      degree-of-rate-control combine across the lanes of one
//                      condition by wavefront shuffles (old_system.py:470-529)
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <string.h>
#include <new>
#include "mk_device.h"

using namespace pck;

struct pck_network {
    NetView nv;
    int32_t* d_ip = nullptr;
    double* d_dp = nullptr;
    double* scratch = nullptr;      // feature scratch [nfeat][cap]
    int64_t scratch_cap = 0;
    double* kbuf = nullptr;         // kf/kr scratch for pck_solve/pck_drc
    int64_t kbuf_cap = 0;
};

static thread_local char g_err[512] = "";
static int fail(int code, const char* fmt, const char* a = "", long long b = 0) {
    snprintf(g_err, sizeof(g_err), fmt, a, b);
    return code;
}
#define HIPCHK(x)                                                                  \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) return fail(PCK_E_HIP, "HIP error: %s (%lld)", hipGetErrorString(e_), (long long)e_); \
    } while (0)

static inline CondView cview(const pck_conditions* c) {
    CondView v;
    v.n = c->n;
    v.T = c->T; v.sT = c->sT;
    v.p = c->p; v.sp = c->sp;
    v.desc = c->desc; v.ld_desc = c->ld_desc; v.s_desc = c->s_desc;
    v.fixc = c->fixc; v.ld_fix = c->ld_fix; v.s_fix = c->s_fix;
    v.y0 = c->y0; v.ld_y0 = c->ld_y0; v.s_y0 = c->s_y0;
    v.inflow = c->inflow; v.ld_in = c->ld_in; v.s_in = c->s_in;
    return v;
}

// ----------------------------------------------------------------------------
// kernel (1)
// ----------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_rate_constants(NetView nv, CondView cv, double* feat, int64_t fs,
                                                        double* kf, double* kr, int64_t ld_k) {
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= cv.n) return;
    const double T = cv.T[c * cv.sT];
    const double p = cv.p[c * cv.sp];
    double* f = feat + c;
    thermo_features(nv, T, p, cv.desc + c * cv.s_desc, cv.ld_desc, f, fs);
    for (int j = 0; j < nv.NRXN; ++j) {
        double a, b;
        rate_constants_from_feat(nv, T, f, fs, j, a, b);
        kf[j * ld_k + c] = a;
        kr[j * ld_k + c] = b;
    }
}

// energy-program registers only (free / reaction energies in eV)
__global__ void __launch_bounds__(256) k_energies(NetView nv, CondView cv, double* feat, int64_t fs, double* out,
                                                  int64_t ld_out) {
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= cv.n) return;
    double* f = feat + c;
    thermo_features(nv, cv.T[c * cv.sT], cv.p[c * cv.sp], cv.desc + c * cv.s_desc, cv.ld_desc, f, fs);
    const int rb = 2 + nv.D + 3 * nv.NTH;
    for (int r = 0; r < nv.NREG; ++r) out[r * ld_out + c] = f[(rb + r) * fs];
}

// ----------------------------------------------------------------------------
// per-lane setup shared by the solver and the evaluation kernels
// ----------------------------------------------------------------------------
// LDS per lane (stride = blockDim): kf_eff[R], kr_eff[R], inflow[NS]
template <int NS>
__device__ __forceinline__ void lane_setup(const NetView& nv, const CondView& cv, int64_t c, Lane<NS>& L, double& T,
                                           double* lds_lane, int ks) {
    T = cv.T[c * cv.sT];
    L.T = T;                          // reactor.py:34-41: CSTR row scaling is linear in T
    double* ins = lds_lane + (size_t)2 * nv.NRXN * ks;
    L.ins = ins;
#pragma unroll
    for (int i = 0; i < NS; ++i) {    // 1/residence_time on CSTR gas rows (reactor.py:154-156)
        if (nv.dyn[4 * i + 3] != 0.0) ins[i * ks] = cv.inflow ? cv.inflow[i * cv.ld_in + c * cv.s_in] : 0.0;
    }
}

__host__ __device__ inline size_t lds_bytes(int R, int NS, int B) {
    return sizeof(double) * (size_t)(2 * (R > 0 ? R : 1) + NS) * B;
}

// effective k (fixed species folded in, optional DRC perturbation) -> LDS
__device__ __forceinline__ void load_keff(const NetView& nv, const CondView& cv, int64_t c, const double* kf,
                                          const double* kr, int64_t ld_k, double* kfs, double* krs, int ks,
                                          int pj, double pfac) {
    for (int j = 0; j < nv.NRXN; ++j) {
        double a = kf[j * ld_k + c], b = kr[j * ld_k + c];
        for (int q = 0; q < nv.NFIX; ++q) {
            const int ea = nv.foldf[j * nv.NFIX + q], eb = nv.foldr[j * nv.NFIX + q];
            if (ea | eb) {
                const double x = cv.fixc[q * cv.ld_fix + c * cv.s_fix];
                if (ea) a *= ipow(x, ea);
                if (eb) b *= ipow(x, eb);
            }
        }
        if (j == pj) { a *= pfac; b *= pfac; }   // old_system.py:504-506: kf + eps*kf, kr*(1 + eps)
        kfs[j * ks] = a;
        krs[j * ks] = b;
    }
}

template <int NS>
__global__ void __launch_bounds__(128) k_species_rates(NetView nv, CondView cv, const double* kf, const double* kr,
                                                       int64_t ld_k, const double* y, int64_t ld_y, double* dydt) {
    extern __shared__ double lds[];
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= cv.n) return;
    double* kfs = lds + threadIdx.x;
    double* krs = lds + (size_t)nv.NRXN * blockDim.x + threadIdx.x;
    Lane<NS> L; double T;
    lane_setup<NS>(nv, cv, c, L, T, lds + threadIdx.x, blockDim.x);
    load_keff(nv, cv, c, kf, kr, ld_k, kfs, krs, blockDim.x, -1, 1.0);
    double yy[NS], f[NS];
#pragma unroll
    for (int i = 0; i < NS; ++i) yy[i] = y[i * ld_y + c];
    rhs<NS>(nv, L, kfs, krs, blockDim.x, yy, f);
#pragma unroll
    for (int i = 0; i < NS; ++i) dydt[i * ld_y + c] = f[i];
}

template <int NS>
__global__ void __launch_bounds__(128) k_jacobian(NetView nv, CondView cv, const double* kf, const double* kr,
                                                  int64_t ld_k, const double* y, int64_t ld_y, double* jo) {
    extern __shared__ double lds[];
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= cv.n) return;
    double* kfs = lds + threadIdx.x;
    double* krs = lds + (size_t)nv.NRXN * blockDim.x + threadIdx.x;
    Lane<NS> L; double T;
    lane_setup<NS>(nv, cv, c, L, T, lds + threadIdx.x, blockDim.x);
    load_keff(nv, cv, c, kf, kr, ld_k, kfs, krs, blockDim.x, -1, 1.0);
    double yy[NS], J[NS][NS];
#pragma unroll
    for (int i = 0; i < NS; ++i) yy[i] = y[i * ld_y + c];
    jac<NS>(nv, L, kfs, krs, blockDim.x, yy, J);
#pragma unroll
    for (int i = 0; i < NS; ++i)
#pragma unroll
        for (int k = 0; k < NS; ++k) jo[(i * NS + k) * ld_y + c] = J[i][k];
}

// ----------------------------------------------------------------------------
// kernel (3)+(4): solve
// ----------------------------------------------------------------------------
struct SolveArgs {
    double t0, t_end, rtol, atol, eps;
    int max_steps, newton, newton_iters, want_activity;
    double* y; int64_t ld_y;
    double* tof; int32_t* status; int32_t* nsteps;
    double* xi; int64_t ld_xi; double* tof0;   // DRC mode
    int G;                                     // lanes per condition (1, or DRC group size)
};

template <int NS>
__device__ __forceinline__ double rms_scaled(const double (&e)[NS], const double (&a)[NS], const double (&b)[NS],
                                             double atol, double rtol) {
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < NS; ++i) {
        const double sc = atol + rtol * fmax(fabs(a[i]), fabs(b[i]));
        const double r = e[i] / sc;
        s += r * r;
    }
    return sqrt(s / NS);
}

// RODAS4 (Hairer & Wanner, stiffly accurate 4(3) Rosenbrock, L-stable),
// autonomous form:  (I/(h g) - J) k_i = f(u_i) + sum_j C_ij k_j / h,
// u_{i+1} = y + sum_j a_ij k_j,  y_new = u_5 + k5 + k6,  error = k6.
namespace rodas4 {
constexpr double g = 0.25;
constexpr double a21 = 1.544, a31 = 0.9466785280815826, a32 = 0.2557011698983284;
constexpr double a41 = 3.314825187068521, a42 = 2.896124015972201, a43 = 0.9986419139977817;
constexpr double a51 = 1.221224509226641, a52 = 6.019134481288629, a53 = 12.53708332932087,
                 a54 = -0.6878860361058950;
constexpr double C21 = -5.6688, C31 = -2.430093356833875, C32 = -0.2063599157091915;
constexpr double C41 = -0.1073529058151375, C42 = -9.594562251023355, C43 = -20.47028614809616;
constexpr double C51 = 7.496443313967647, C52 = -10.24680431464352, C53 = -33.99990352819905,
                 C54 = 11.70890893206160;
constexpr double C61 = 8.083246795921522, C62 = -7.981132988064893, C63 = -31.52159432874371,
                 C64 = 16.31930543123136, C65 = -6.058818238834054;
}  // namespace rodas4

template <int NS>
__device__ int integrate(const NetView& nv, const Lane<NS>& L, const double* kfs, const double* krs, int ks,
                         double (&y)[NS], double t0, double t_end, double rtol, double atol, int max_steps,
                         int& nsteps) {
    using namespace rodas4;
    nsteps = 0;
    const double span = t_end - t0;
    if (!(span > 0.0)) return PCK_ST_OK;
    double F0[NS];
    rhs<NS>(nv, L, kfs, krs, ks, y, F0);
    double cons0[PCK_MAX_CONS];
    for (int l = 0; l < nv.NCONS; ++l) {
        double s = 0.0;
#pragma unroll
        for (int i = 0; i < NS; ++i) s += nv.C[l * NS + i] * y[i];
        cons0[l] = s;
    }
    // initial step (Hairer/Wanner heuristic, scipy's select_initial_step, order 4)
    double h;
    {
        double d0 = 0.0, d1 = 0.0;
#pragma unroll
        for (int i = 0; i < NS; ++i) {
            const double sc = atol + rtol * fabs(y[i]);
            d0 += (y[i] / sc) * (y[i] / sc);
            d1 += (F0[i] / sc) * (F0[i] / sc);
        }
        d0 = sqrt(d0 / NS); d1 = sqrt(d1 / NS);
        double h0 = (d0 < 1e-5 || d1 < 1e-5) ? 1e-6 : 0.01 * d0 / d1;
        h0 = fmin(h0, span);
        double y1[NS], F1[NS];
#pragma unroll
        for (int i = 0; i < NS; ++i) y1[i] = y[i] + h0 * F0[i];
        rhs<NS>(nv, L, kfs, krs, ks, y1, F1);
        double d2 = 0.0;
#pragma unroll
        for (int i = 0; i < NS; ++i) {
            const double sc = atol + rtol * fabs(y[i]);
            const double q = (F1[i] - F0[i]) / sc;
            d2 += q * q;
        }
        d2 = sqrt(d2 / NS) / h0;
        const double h1 = (d1 <= 1e-15 && d2 <= 1e-15) ? fmax(1e-6, h0 * 1e-3) : pow(0.01 / fmax(d1, d2), 0.2);
        h = fmin(fmin(100.0 * h0, h1), span);
    }
    double t = t0;
    double W[NS][NS];
    int piv[NS];
    while (t < t_end) {
        if (nsteps >= max_steps) return PCK_ST_MAXSTEPS;
        ++nsteps;
        bool last = false;
        if (t + h >= t_end) { h = t_end - t; last = true; }
        // W = I/(h g) - J
        jac<NS>(nv, L, kfs, krs, ks, y, W);
        const double ig = 1.0 / (h * g);
#pragma unroll
        for (int i = 0; i < NS; ++i) {
#pragma unroll
            for (int k = 0; k < NS; ++k) W[i][k] = -W[i][k];
            W[i][i] += ig;
        }
        if (!lu<NS>(W, piv)) { h *= 0.25; continue; }
        const double ih = 1.0 / h;
        double k1[NS], k2[NS], k3[NS], k4[NS], k5[NS], u[NS], fu[NS];
#pragma unroll
        for (int i = 0; i < NS; ++i) k1[i] = F0[i];
        lu_solve<NS>(W, piv, k1);
#pragma unroll
        for (int i = 0; i < NS; ++i) u[i] = y[i] + a21 * k1[i];
        rhs<NS>(nv, L, kfs, krs, ks, u, fu);
#pragma unroll
        for (int i = 0; i < NS; ++i) k2[i] = fu[i] + ih * (C21 * k1[i]);
        lu_solve<NS>(W, piv, k2);
#pragma unroll
        for (int i = 0; i < NS; ++i) u[i] = y[i] + a31 * k1[i] + a32 * k2[i];
        rhs<NS>(nv, L, kfs, krs, ks, u, fu);
#pragma unroll
        for (int i = 0; i < NS; ++i) k3[i] = fu[i] + ih * (C31 * k1[i] + C32 * k2[i]);
        lu_solve<NS>(W, piv, k3);
#pragma unroll
        for (int i = 0; i < NS; ++i) u[i] = y[i] + a41 * k1[i] + a42 * k2[i] + a43 * k3[i];
        rhs<NS>(nv, L, kfs, krs, ks, u, fu);
#pragma unroll
        for (int i = 0; i < NS; ++i) k4[i] = fu[i] + ih * (C41 * k1[i] + C42 * k2[i] + C43 * k3[i]);
        lu_solve<NS>(W, piv, k4);
#pragma unroll
        for (int i = 0; i < NS; ++i) u[i] = y[i] + a51 * k1[i] + a52 * k2[i] + a53 * k3[i] + a54 * k4[i];
        rhs<NS>(nv, L, kfs, krs, ks, u, fu);
#pragma unroll
        for (int i = 0; i < NS; ++i) k5[i] = fu[i] + ih * (C51 * k1[i] + C52 * k2[i] + C53 * k3[i] + C54 * k4[i]);
        lu_solve<NS>(W, piv, k5);
#pragma unroll
        for (int i = 0; i < NS; ++i) u[i] += k5[i];
        rhs<NS>(nv, L, kfs, krs, ks, u, fu);
        // reuse k5's slot for k6 once it has been folded into u
#pragma unroll
        for (int i = 0; i < NS; ++i)
            k5[i] = fu[i] + ih * (C61 * k1[i] + C62 * k2[i] + C63 * k3[i] + C64 * k4[i] + C65 * k5[i]);
        lu_solve<NS>(W, piv, k5);
        bool finite = true;
        double s = 0.0;
#pragma unroll
        for (int i = 0; i < NS; ++i) {
            u[i] += k5[i];
            finite = finite && isfinite(u[i]) && isfinite(k5[i]);
            const double sc = atol + rtol * fmax(fabs(y[i]), fabs(u[i]));
            const double r = k5[i] / sc;
            s += r * r;
        }
        const double en = finite ? sqrt(s / NS) : INFINITY;
        if (en <= 1.0) {
            t = last ? t_end : t + h;
#pragma unroll
            for (int i = 0; i < NS; ++i) y[i] = u[i];
            // Rosenbrock stages keep linear invariants only up to the rounding of
            // the stiff LU; rescale each non-negative site balance back onto its
            // initial total (multiplicative, so tiny coverages keep their digits)
            for (int l = 0; l < nv.NCONS; ++l) {
                double s = 0.0;
                bool pos = true;
#pragma unroll
                for (int i = 0; i < NS; ++i) {
                    const double cl = nv.C[l * NS + i];
                    pos = pos && (cl >= 0.0);
                    s += cl * y[i];
                }
                if (pos && s > 0.0) {
                    const double f = cons0[l] / s;
#pragma unroll
                    for (int i = 0; i < NS; ++i)
                        if (nv.C[l * NS + i] != 0.0) y[i] *= f;
                }
            }
            rhs<NS>(nv, L, kfs, krs, ks, y, F0);
            const double fac = (en > 0.0) ? 0.9 * rsqrt(sqrt(en)) : 6.0;   // 0.9 en^(-1/4)
            h *= fmin(6.0, fmax(0.2, fac));
        } else {
            h *= finite ? fmax(0.2, 0.9 * rsqrt(sqrt(en))) : 0.25;
        }
        if (!(h > 1e-15 * fmax(fabs(t), 1e-300)) && t < t_end) return PCK_ST_STEPFAIL;
    }
    return PCK_ST_OK;
}

// Newton on f(y) = 0 with the plan's conservation laws replacing their pivot
// rows (old_system.py:385-468 polishes with scipy least_squares; the root it
// converges to is the same).
template <int NS>
__device__ int newton(const NetView& nv, const Lane<NS>& L, const double* kfs, const double* krs, int ks,
                      double (&y)[NS], int iters) {
    double b[PCK_MAX_CONS];
    for (int l = 0; l < nv.NCONS; ++l) {
        double s = 0.0;
#pragma unroll
        for (int i = 0; i < NS; ++i) s += nv.C[l * NS + i] * y[i];
        b[l] = s;
    }
    double z[NS];
#pragma unroll
    for (int i = 0; i < NS; ++i) z[i] = y[i];
    bool conv = false;
    double prev = INFINITY, lastq = 1.0;
    int linear = 0;
    for (int it = 0; it < iters; ++it) {
        double G[NS], J[NS][NS];
        int piv[NS];
        rhs<NS>(nv, L, kfs, krs, ks, z, G);
        jac<NS>(nv, L, kfs, krs, ks, z, J);
        for (int l = 0; l < nv.NCONS; ++l) {
            const int p = nv.cpiv[l];
            double s = 0.0;
#pragma unroll
            for (int i = 0; i < NS; ++i) s += nv.C[l * NS + i] * z[i];
#pragma unroll
            for (int i = 0; i < NS; ++i) {
                if (i == p) {
                    G[i] = s - b[l];
#pragma unroll
                    for (int k = 0; k < NS; ++k) J[i][k] = nv.C[l * NS + k];
                }
            }
        }
        // row equilibration: rate rows (|J| ~ k p, up to 1e9) and the O(1)
        // conservation rows must carry comparable weight, or the LU's backward
        // error (eps * max row norm) leaks into the site balance
#pragma unroll
        for (int i = 0; i < NS; ++i) {
            double m = 0.0;
#pragma unroll
            for (int k = 0; k < NS; ++k) m = fmax(m, fabs(J[i][k]));
            const double sc = (m > 0.0) ? 1.0 / m : 1.0;
#pragma unroll
            for (int k = 0; k < NS; ++k) J[i][k] *= sc;
            G[i] = -G[i] * sc;
        }
        if (!lu<NS>(J, piv)) break;
        lu_solve<NS>(J, piv, G);
        // Newton with a multiplicity estimate: after two linear steps with
        // contraction q, step m = 1/(1-q) times (m = 2 on the halving of a
        // near-double root); never past a zero of a decreasing component
        double alpha = 1.0;
        if (linear >= 2 && lastq < 0.9) {
            alpha = fmin(4.0, 1.0 / (1.0 - lastq));
#pragma unroll
            for (int i = 0; i < NS; ++i)
                if (G[i] < 0.0 && z[i] > 0.0) alpha = fmin(alpha, 0.9 * z[i] / -G[i]);
            alpha = fmax(alpha, 1.0);
        }
        double rel = 0.0, zmax = 0.0;
        bool finite = true;
#pragma unroll
        for (int i = 0; i < NS; ++i) {
            G[i] *= alpha;
            z[i] += G[i];
            finite = finite && isfinite(z[i]);
            zmax = fmax(zmax, fabs(z[i]));
        }
        if (!finite) break;
        // components below 1e-12 of the largest are held to an absolute
        // 1e-24 * zmax: their relative digits sit under the residual's rounding
#pragma unroll
        for (int i = 0; i < NS; ++i) rel = fmax(rel, fabs(G[i]) / fmax(fabs(z[i]), 1e-12 * zmax + 1e-300));
        // converged: relative step at the 1e-12 level, or stagnated at the
        // rounding level of the residual (no 2x decrease once below 1e-7)
        if (rel < 1e-12 || (it >= 2 && rel < 1e-7 && rel > 0.5 * prev)) { conv = true; break; }
        // linear (halving) convergence = a degenerate root, e.g. a fully
        // poisoned surface approached algebraically: keep the transient state
        lastq = rel / prev;
        linear = (rel > 0.25 * prev) ? linear + 1 : 0;
        if (linear >= 12) break;
        prev = rel;
    }
    if (!conv) return PCK_ST_NEWTON;
    // accept only a physical root (no negative coverage / pressure): a root
    // with a component at -1e-30 is a vanishing species resolved below the
    // residual's rounding, i.e. not a regular steady state
#pragma unroll
    for (int i = 0; i < NS; ++i)
        if (z[i] < 0.0) return PCK_ST_NEWTON;
#pragma unroll
    for (int i = 0; i < NS; ++i) y[i] = z[i];
    return PCK_ST_OK;
}

template <int NS>
__device__ __forceinline__ double lane_tof(const NetView& nv, const Lane<NS>& L, const double* kfs,
                                           const double* krs, int ks, const double (&y)[NS]) {
    // old_system.py:482-488: sum of (r_fwd - r_rev) over tof_terms
    double c[NS];
#pragma unroll
    for (int i = 0; i < NS; ++i) c[i] = cfac(nv, i) * y[i];
    double tof = 0.0;
    for (int t = 0; t < nv.NTOF; ++t) {
        const int j = nv.tof[t];
        double rf = kfs[j * ks], rr = krs[j * ks];
#pragma unroll
        for (int i = 0; i < NS; ++i) {
            const int a = nv.expf[j * NS + i], b = nv.expr[j * NS + i];
            if (a) rf *= ipow(c[i], a);
            if (b) rr *= ipow(c[i], b);
        }
        tof += rf - rr;
    }
    return tof;
}

template <int NS>
__global__ void __launch_bounds__(128) k_solve(NetView nv, CondView cv, const double* kf, const double* kr,
                                               int64_t ld_k, SolveArgs a) {
    extern __shared__ double lds[];
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int G = a.G;
    const int64_t c = gid / G;
    const int q = (int)(gid % G);
    const int R = nv.NRXN;
    // DRC lanes: q = 0 base, q = 2j+1 -> k_j*(1+eps), q = 2j+2 -> k_j*(1-eps)
    const bool drc = (G > 1);
    const bool active = (c < cv.n) && (!drc || q <= 2 * R);
    double* kfs = lds + threadIdx.x;
    double* krs = lds + (size_t)R * blockDim.x + threadIdx.x;
    double tof = 0.0;
    int st = PCK_ST_OK;
    if (active) {
        int pj = -1;
        double pfac = 1.0;
        if (drc && q > 0) { pj = (q - 1) >> 1; pfac = (q & 1) ? 1.0 + a.eps : 1.0 - a.eps; }
        Lane<NS> L; double T;
        lane_setup<NS>(nv, cv, c, L, T, lds + threadIdx.x, blockDim.x);
        load_keff(nv, cv, c, kf, kr, ld_k, kfs, krs, blockDim.x, pj, pfac);
        double y[NS];
#pragma unroll
        for (int i = 0; i < NS; ++i) y[i] = cv.y0[i * cv.ld_y0 + c * cv.s_y0];
        int ns = 0;
        st = integrate<NS>(nv, L, kfs, krs, blockDim.x, y, a.t0, a.t_end, a.rtol, a.atol, a.max_steps, ns);
        if (st == PCK_ST_OK && a.newton) st = newton<NS>(nv, L, kfs, krs, blockDim.x, y, a.newton_iters);
        tof = lane_tof<NS>(nv, L, kfs, krs, blockDim.x, y);
        if (!drc) {
            bool fin = isfinite(tof);
#pragma unroll
            for (int i = 0; i < NS; ++i) fin = fin && isfinite(y[i]);
            if (!fin && st == PCK_ST_OK) st = PCK_ST_NONFINITE;
            if (a.y) {
#pragma unroll
                for (int i = 0; i < NS; ++i) a.y[i * a.ld_y + c] = y[i];
            }
            if (a.tof) {
                // old_system.py:526-527
                a.tof[c] = a.want_activity ? (log((hP * tof) / (kB * T)) * (Rgas * T)) * 1.0e-3 / eVtokJ : tof;
            }
            if (a.status) a.status[c] = st;
            if (a.nsteps) a.nsteps[c] = ns;
        }
    }
    if (drc) {
        // wavefront-shuffle combine: every lane of a condition's group lives in
        // the same wavefront (G divides 64)
        const int lane = threadIdx.x & 63;
        const int base = lane - q;
        const double t0 = __shfl(tof, base, 64);
        const double tm = __shfl(tof, lane + 1 < 64 ? lane + 1 : lane, 64);
        const int s0 = __shfl(st, base, 64);
        const int sm = __shfl(st, lane + 1 < 64 ? lane + 1 : lane, 64);
        if (active && (q & 1)) {
            const int j = (q - 1) >> 1;
            a.xi[j * a.ld_xi + c] = (tof - tm) / (2.0 * a.eps * t0);   // old_system.py:508
            // status of the group = worst member
            if (a.status && (st | sm)) atomicMax(&a.status[c], st > sm ? st : sm);
        }
        if (active && q == 0) {
            if (a.tof0) a.tof0[c] = tof;
            if (a.status && s0) atomicMax(&a.status[c], s0);
        }
    }
}

// ----------------------------------------------------------------------------
// C-ABI
// ----------------------------------------------------------------------------
extern "C" int pck_abi_version(void) { return PCK_ABI_VERSION; }
extern "C" const char* pck_last_error(void) { return g_err; }

extern "C" int pck_network_create(const int32_t* ip, int64_t n_ip, const double* dp, int64_t n_dp,
                                  pck_network** out) {
    if (!ip || !out || n_ip < PCK_IP_MIN) return fail(PCK_E_ARG, "int blob too short%s (%lld)", "", n_ip);
    if (ip[PCK_I_VERSION] != PCK_ABI_VERSION) return fail(PCK_E_ARG, "blob ABI version mismatch%s %lld", "", ip[0]);
    NetView nv;
    nv.D = ip[PCK_I_NDESC]; nv.NTH = ip[PCK_I_NTH]; nv.NREG = ip[PCK_I_NREG]; nv.NRXN = ip[PCK_I_NRXN];
    nv.NDYN = ip[PCK_I_NDYN]; nv.NFIX = ip[PCK_I_NFIX]; nv.NCONS = ip[PCK_I_NCONS]; nv.NTOF = ip[PCK_I_NTOF];
    nv.nfeat = 2 + nv.D + 3 * nv.NTH + nv.NREG;
    if (nv.D < 0 || nv.NTH < 0 || nv.NREG < 0 || nv.NRXN < 0 || nv.NFIX < 0 || nv.NCONS < 0 || nv.NTOF < 0)
        return fail(PCK_E_ARG, "negative dimension in blob%s", "");
    if (nv.NDYN < 0 || nv.NDYN > PCK_MAX_DYN_PLAN)
        return fail(PCK_E_SIZE, "NDYN out of range [0, 64]%s: %lld", "", nv.NDYN);
    if (nv.NRXN > PCK_MAX_RXN) return fail(PCK_E_SIZE, "too many reactions%s: %lld", "", nv.NRXN);
    if (nv.NCONS > PCK_MAX_CONS) return fail(PCK_E_SIZE, "too many conservation laws%s: %lld", "", nv.NCONS);
    if (nv.NTOF > PCK_MAX_TOF) return fail(PCK_E_SIZE, "too many TOF terms%s: %lld", "", nv.NTOF);
    // bounds of every int block
    const int64_t oth = ip[PCK_I_OFF_TH], oreg = ip[PCK_I_OFF_REG], orx = ip[PCK_I_OFF_RX];
    const int64_t oef = ip[PCK_I_OFF_EXPF], oer = ip[PCK_I_OFF_EXPR], off_ = ip[PCK_I_OFF_FOLDF];
    const int64_t ofr = ip[PCK_I_OFF_FOLDR], ocp = ip[PCK_I_OFF_CPIV], otf = ip[PCK_I_OFF_TOF];
    if (oreg + nv.NREG + 1 > n_ip) return fail(PCK_E_ARG, "reg block out of range%s", "");
    const int64_t nnz = ip[oreg + nv.NREG];
    struct { int64_t off, len; } blocks[] = {
        {oth, 4LL * nv.NTH}, {oreg, nv.NREG + 1 + nv.NREG + nnz}, {orx, 6LL * nv.NRXN},
        {oef, (int64_t)nv.NRXN * nv.NDYN}, {oer, (int64_t)nv.NRXN * nv.NDYN},
        {off_, (int64_t)nv.NRXN * nv.NFIX}, {ofr, (int64_t)nv.NRXN * nv.NFIX}, {ocp, nv.NCONS}, {otf, nv.NTOF}};
    for (auto& b : blocks)
        if (b.off < PCK_IP_MIN || b.off + b.len > n_ip) return fail(PCK_E_ARG, "int block out of range%s at %lld", "", b.off);
    int64_t doff[PCK_D_NBLK];
    for (int k = 0; k < PCK_D_NBLK; ++k) doff[k] = ip[PCK_D_OFF_SLOT0 + k];
    const int64_t dlen[PCK_D_NBLK] = {5LL * nv.NTH, 0, nnz, 3LL * nv.NRXN, (int64_t)nv.NDYN * nv.NRXN,
                                      4LL * nv.NDYN, (int64_t)nv.NCONS * nv.NDYN};
    for (int k = 0; k < PCK_D_NBLK; ++k)
        if (doff[k] < 0 || doff[k] + dlen[k] > n_dp) return fail(PCK_E_ARG, "float block out of range%s (%lld)", "", k);
    // every index inside the blocks
    for (int s = 0; s < nv.NTH; ++s) {
        const int f0 = ip[oth + 4 * s + 1], nf = ip[oth + 4 * s + 2];
        if (f0 < 0 || nf < 0 || doff[PCK_D_FREQ] + f0 + nf > n_dp) return fail(PCK_E_ARG, "freq range%s of state %lld", "", s);
    }
    for (int r = 0; r < nv.NREG; ++r) {
        const int a = ip[oreg + r], b = ip[oreg + r + 1];
        if (a < 0 || b < a || b > nnz) return fail(PCK_E_ARG, "reg_ptr%s not monotone at %lld", "", r);
        for (int q = a; q < b; ++q) {
            const int fi = ip[oreg + nv.NREG + 1 + nv.NREG + q];
            if (fi < 0 || fi >= 2 + nv.D + 3 * nv.NTH + r) return fail(PCK_E_ARG, "register%s reads feature out of order (%lld)", "", r);
        }
    }
    for (int j = 0; j < nv.NRXN; ++j) {
        for (int k = 2; k <= 4; ++k) {
            const int ri = ip[orx + 6 * j + k];
            if (ri >= nv.NREG) return fail(PCK_E_ARG, "reaction register index%s out of range (%lld)", "", j);
        }
        for (int i = 0; i < nv.NDYN; ++i)
            if (ip[oef + j * nv.NDYN + i] < 0 || ip[oer + j * nv.NDYN + i] < 0) return fail(PCK_E_ARG, "negative exponent%s", "");
    }
    for (int l = 0; l < nv.NCONS; ++l)
        if (ip[ocp + l] < 0 || ip[ocp + l] >= nv.NDYN) return fail(PCK_E_ARG, "conservation pivot%s out of range (%lld)", "", l);
    for (int t = 0; t < nv.NTOF; ++t)
        if (ip[otf + t] < 0 || ip[otf + t] >= nv.NRXN) return fail(PCK_E_ARG, "TOF term%s out of range (%lld)", "", t);

    pck_network* net = new (std::nothrow) pck_network();
    if (!net) return fail(PCK_E_ARG, "out of host memory%s", "");
    hipError_t e = hipMalloc(&net->d_ip, sizeof(int32_t) * n_ip);
    if (e == hipSuccess) e = hipMalloc(&net->d_dp, sizeof(double) * (n_dp > 0 ? n_dp : 1));
    if (e == hipSuccess) e = hipMemcpy(net->d_ip, ip, sizeof(int32_t) * n_ip, hipMemcpyHostToDevice);
    if (e == hipSuccess && n_dp > 0) e = hipMemcpy(net->d_dp, dp, sizeof(double) * n_dp, hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        hipFree(net->d_ip); hipFree(net->d_dp); delete net;
        return fail(PCK_E_HIP, "HIP error: %s (%lld)", hipGetErrorString(e), (long long)e);
    }
    const int32_t* I = net->d_ip;
    const double* Dp = net->d_dp;
    nv.th = I + oth;
    nv.reg_ptr = I + oreg;
    nv.reg_clamp = I + oreg + nv.NREG + 1;
    nv.reg_feat = I + oreg + nv.NREG + 1 + nv.NREG;
    nv.rx = I + orx; nv.expf = I + oef; nv.expr = I + oer; nv.foldf = I + off_; nv.foldr = I + ofr;
    nv.cpiv = I + ocp; nv.tof = I + otf;
    nv.thd = Dp + doff[PCK_D_TH]; nv.freq = Dp + doff[PCK_D_FREQ]; nv.reg_coef = Dp + doff[PCK_D_REGCOEF];
    nv.rxd = Dp + doff[PCK_D_RX]; nv.S = Dp + doff[PCK_D_STOICH]; nv.dyn = Dp + doff[PCK_D_DYN];
    nv.C = Dp + doff[PCK_D_CONS];
    net->nv = nv;
    *out = net;
    return PCK_OK;
}

extern "C" int pck_network_destroy(pck_network* net) {
    if (!net) return PCK_OK;
    hipFree(net->d_ip); hipFree(net->d_dp); hipFree(net->scratch); hipFree(net->kbuf);
    delete net;
    return PCK_OK;
}

extern "C" int pck_network_dims(const pck_network* net, int32_t* dims) {
    if (!net || !dims) return fail(PCK_E_ARG, "null argument%s", "");
    const NetView& v = net->nv;
    dims[0] = v.D; dims[1] = v.NTH; dims[2] = v.NREG; dims[3] = v.NRXN; dims[4] = v.NDYN;
    dims[5] = v.NFIX; dims[6] = v.NCONS; dims[7] = v.NTOF; dims[8] = v.nfeat;
    return PCK_OK;
}

static int check_cond(const pck_network* net, const pck_conditions* c, bool need_state) {
    if (!net || !c) return fail(PCK_E_ARG, "null network/conditions%s", "");
    if (c->n < 0) return fail(PCK_E_ARG, "negative condition count%s", "");
    if (c->n > 0 && (!c->T || !c->p)) return fail(PCK_E_ARG, "T and p are required%s", "");
    if (net->nv.D > 0 && c->n > 0 && !c->desc) return fail(PCK_E_ARG, "network needs %lld descriptors%s", "", net->nv.D);
    if (need_state && net->nv.NFIX > 0 && c->n > 0 && !c->fixc) return fail(PCK_E_ARG, "fixed-species concentrations required%s", "");
    return PCK_OK;
}

static int ensure(double** buf, int64_t* cap, int64_t need) {
    if (*cap >= need) return PCK_OK;
    hipFree(*buf);
    *buf = nullptr;
    *cap = 0;
    HIPCHK(hipMalloc(buf, sizeof(double) * (need > 0 ? need : 1)));
    *cap = need;
    return PCK_OK;
}

static int launch_rate_constants(pck_network* net, const pck_conditions* cond, double* kf, double* kr, int64_t ld_k,
                                 hipStream_t s) {
    const int64_t n = cond->n;
    if (n == 0) return PCK_OK;
    int rc = ensure(&net->scratch, &net->scratch_cap, (int64_t)net->nv.nfeat * n);
    if (rc) return rc;
    const int B = 256;
    hipLaunchKernelGGL(k_rate_constants, dim3((unsigned)((n + B - 1) / B)), dim3(B), 0, s, net->nv, cview(cond),
                       net->scratch, n, kf, kr, ld_k);
    HIPCHK(hipGetLastError());
    return PCK_OK;
}

extern "C" int pck_energies(const pck_network* net, const pck_conditions* cond, double* out, int64_t ld_out,
                            void* stream) {
    int rc = check_cond(net, cond, false);
    if (rc) return rc;
    const int64_t n = cond->n;
    if (n == 0 || net->nv.NREG == 0) return PCK_OK;
    if (!out || ld_out < n) return fail(PCK_E_ARG, "bad energies output%s (ld %lld)", "", ld_out);
    pck_network* nn = const_cast<pck_network*>(net);
    rc = ensure(&nn->scratch, &nn->scratch_cap, (int64_t)net->nv.nfeat * n);
    if (rc) return rc;
    const int B = 256;
    hipLaunchKernelGGL(k_energies, dim3((unsigned)((n + B - 1) / B)), dim3(B), 0, (hipStream_t)stream, net->nv,
                       cview(cond), nn->scratch, n, out, ld_out);
    HIPCHK(hipGetLastError());
    return PCK_OK;
}

extern "C" int pck_rate_constants(const pck_network* net, const pck_conditions* cond, double* kf, double* kr,
                                  int64_t ld_k, void* stream) {
    int rc = check_cond(net, cond, false);
    if (rc) return rc;
    if (cond->n > 0 && (!kf || !kr || ld_k < cond->n)) return fail(PCK_E_ARG, "bad kf/kr output%s (ld_k %lld)", "", ld_k);
    return launch_rate_constants(const_cast<pck_network*>(net), cond, kf, kr, ld_k, (hipStream_t)stream);
}

#define PCK_NS_SWITCH(NS, CALL)                                     \
    switch (NS) {                                                   \
    case 1: CALL(1); break; case 2: CALL(2); break;                 \
    case 3: CALL(3); break; case 4: CALL(4); break;                 \
    case 5: CALL(5); break; case 6: CALL(6); break;                 \
    case 7: CALL(7); break; case 8: CALL(8); break;                 \
    default: return fail(PCK_E_SIZE, "NDYN%s unsupported", "");     \
    }

extern "C" int pck_species_rates(const pck_network* net, const pck_conditions* cond, const double* kf,
                                 const double* kr, int64_t ld_k, const double* y, int64_t ld_y, double* dydt,
                                 void* stream) {
    int rc = check_cond(net, cond, true);
    if (rc) return rc;
    const int64_t n = cond->n;
    if (n == 0) return PCK_OK;
    if (!kf || !kr || !y || !dydt || ld_k < n || ld_y < n) return fail(PCK_E_ARG, "bad state/rate arrays%s", "");
    const int B = 128;
    const size_t shm = lds_bytes(net->nv.NRXN, net->nv.NDYN, B);
    dim3 g((unsigned)((n + B - 1) / B));
#define CALL(N) hipLaunchKernelGGL(k_species_rates<N>, g, dim3(B), shm, (hipStream_t)stream, net->nv, cview(cond), kf, kr, ld_k, y, ld_y, dydt)
    PCK_NS_SWITCH(net->nv.NDYN, CALL)
#undef CALL
    HIPCHK(hipGetLastError());
    return PCK_OK;
}

extern "C" int pck_jacobian(const pck_network* net, const pck_conditions* cond, const double* kf, const double* kr,
                            int64_t ld_k, const double* y, int64_t ld_y, double* jo, void* stream) {
    int rc = check_cond(net, cond, true);
    if (rc) return rc;
    const int64_t n = cond->n;
    if (n == 0) return PCK_OK;
    if (!kf || !kr || !y || !jo || ld_k < n || ld_y < n) return fail(PCK_E_ARG, "bad state/rate arrays%s", "");
    const int B = 128;
    const size_t shm = lds_bytes(net->nv.NRXN, net->nv.NDYN, B);
    dim3 g((unsigned)((n + B - 1) / B));
#define CALL(N) hipLaunchKernelGGL(k_jacobian<N>, g, dim3(B), shm, (hipStream_t)stream, net->nv, cview(cond), kf, kr, ld_k, y, ld_y, jo)
    PCK_NS_SWITCH(net->nv.NDYN, CALL)
#undef CALL
    HIPCHK(hipGetLastError());
    return PCK_OK;
}

static int check_params(const pck_solve_params* prm) {
    if (!prm) return fail(PCK_E_ARG, "null params%s", "");
    if (!(prm->t_end >= prm->t0)) return fail(PCK_E_ARG, "t_end < t0%s", "");
    if (!(prm->rtol > 0.0) || !(prm->atol > 0.0)) return fail(PCK_E_ARG, "tolerances must be positive%s", "");
    if (prm->max_steps < 1) return fail(PCK_E_ARG, "max_steps must be >= 1%s", "");
    if (prm->newton && (prm->newton_iters < 1 || prm->newton_iters > 200)) return fail(PCK_E_ARG, "newton_iters%s out of range", "");
    return PCK_OK;
}

static int launch_solve(pck_network* net, const pck_conditions* cond, const pck_solve_params* prm, SolveArgs a,
                        hipStream_t s) {
    const int64_t n = cond->n;
    if (n == 0) return PCK_OK;
    if (!cond->y0) return fail(PCK_E_ARG, "initial state y0 required%s", "");
    const int R = net->nv.NRXN;
    int rc = ensure(&net->kbuf, &net->kbuf_cap, 2LL * (R > 0 ? R : 1) * n);
    if (rc) return rc;
    double* kf = net->kbuf;
    double* kr = net->kbuf + (int64_t)(R > 0 ? R : 1) * n;
    rc = launch_rate_constants(net, cond, kf, kr, n, s);
    if (rc) return rc;
    a.t0 = prm->t0; a.t_end = prm->t_end; a.rtol = prm->rtol; a.atol = prm->atol; a.eps = prm->drc_eps;
    a.max_steps = prm->max_steps; a.newton = prm->newton; a.newton_iters = prm->newton_iters;
    a.want_activity = prm->want_activity;
    const int B = 128;
    const int64_t lanes = n * a.G;
    const size_t shm = lds_bytes(R, net->nv.NDYN, B);
    dim3 g((unsigned)((lanes + B - 1) / B));
#define CALL(N) hipLaunchKernelGGL(k_solve<N>, g, dim3(B), shm, s, net->nv, cview(cond), kf, kr, n, a)
    PCK_NS_SWITCH(net->nv.NDYN, CALL)
#undef CALL
    HIPCHK(hipGetLastError());
    return PCK_OK;
}

extern "C" int pck_solve(const pck_network* net, const pck_conditions* cond, const pck_solve_params* prm,
                         const pck_outputs* out, void* stream) {
    int rc = check_cond(net, cond, true);
    if (rc) return rc;
    rc = check_params(prm);
    if (rc) return rc;
    if (!out) return fail(PCK_E_ARG, "null outputs%s", "");
    if (out->y && out->ld_y < cond->n) return fail(PCK_E_ARG, "ld_y%s too small", "");
    SolveArgs a;
    memset(&a, 0, sizeof(a));
    a.y = out->y; a.ld_y = out->ld_y; a.tof = out->tof; a.status = out->status; a.nsteps = out->nsteps;
    a.G = 1;
    pck_network* nn = const_cast<pck_network*>(net);
    rc = launch_solve(nn, cond, prm, a, (hipStream_t)stream);
    if (rc) return rc;
    if ((out->kf || out->kr) && cond->n > 0) {
        if (out->ld_k < cond->n || !out->kf || !out->kr) return fail(PCK_E_ARG, "kf/kr dump needs both arrays%s", "");
        const int R = net->nv.NRXN;
        HIPCHK(hipMemcpy2DAsync(out->kf, sizeof(double) * out->ld_k, nn->kbuf, sizeof(double) * cond->n,
                                sizeof(double) * cond->n, R, hipMemcpyDeviceToDevice, (hipStream_t)stream));
        HIPCHK(hipMemcpy2DAsync(out->kr, sizeof(double) * out->ld_k, nn->kbuf + (int64_t)R * cond->n,
                                sizeof(double) * cond->n, sizeof(double) * cond->n, R, hipMemcpyDeviceToDevice,
                                (hipStream_t)stream));
    }
    return PCK_OK;
}

extern "C" int pck_drc(const pck_network* net, const pck_conditions* cond, const pck_solve_params* prm, double* xi,
                       int64_t ld_xi, double* tof0, int32_t* status, void* stream) {
    int rc = check_cond(net, cond, true);
    if (rc) return rc;
    rc = check_params(prm);
    if (rc) return rc;
    const int R = net->nv.NRXN;
    if (2 * R + 1 > 64) return fail(PCK_E_SIZE, "DRC needs 2R+1 <= 64 lanes%s (R=%lld)", "", R);
    if (!(prm->drc_eps > 0.0 && prm->drc_eps < 1.0)) return fail(PCK_E_ARG, "drc_eps must be in (0,1)%s", "");
    if (cond->n > 0 && (!xi || ld_xi < cond->n)) return fail(PCK_E_ARG, "bad xi output%s", "");
    int G = 1;
    while (G < 2 * R + 1) G <<= 1;
    if (status && cond->n > 0) HIPCHK(hipMemsetAsync(status, 0, sizeof(int32_t) * cond->n, (hipStream_t)stream));
    SolveArgs a;
    memset(&a, 0, sizeof(a));
    a.xi = xi; a.ld_xi = ld_xi; a.tof0 = tof0; a.status = status; a.G = G;
    return launch_solve(const_cast<pck_network*>(net), cond, prm, a, (hipStream_t)stream);
}
