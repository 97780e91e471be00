// Device-side building blocks of the batched MK solver (gfx950, fp64).
//
// Layout: one lane = one condition.  Per-condition inputs/outputs are
// structure-of-arrays in HBM (lane c reads element c of each row -> every
// wave-instruction is one contiguous 512-B segment).  The network plan is
// uniform across the grid; hipcc turns its reads into scalar loads.
// The dynamic state, the Rosenbrock stage vectors and the dense Jacobian /
// LU factors live in VGPRs (static indices only -- NS is a template
// parameter); the per-lane effective rate constants live in LDS so the
// reaction loop can stay a runtime loop over the plan.
#pragma once
#ifdef __HIPCC_RTC__
// run-time specialisation (mk_jit.h): hipRTC supplies the HIP built-ins and
// these headers come from the library's embedded copies
#include <stdint.h>
#include "pycatkin_amd.h"
#ifndef INFINITY
#define INFINITY __builtin_inf()
#endif
#else
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../include/pycatkin_amd.h"
#endif

namespace pck {

// pycatkin/constants/physical_constants.py:15-23
constexpr double kB = 1.380662e-23;
constexpr double hP = 6.626176e-34;
constexpr double JtoeV = 6.242e18;
constexpr double eVtokJ = 96.485;
constexpr double amutokg = 1.66053886e-27;
constexpr double amuA2tokgm2 = 1.66053907e-47;
constexpr double Rgas = 8.31446262;
constexpr double bartoPa = 1.0e5;
constexpr double EV2JMOL = eVtokJ * 1.0e3;
constexpr double PI = 3.14159265358979323846;

// Device view of an uploaded network (passed by value as a kernel argument).
struct NetView {
    int D, NTH, NREG, NRXN, NDYN, NFIX, NCONS, NTOF;
    int nfeat;                 // 2 + D + 3*NTH + NREG
    const int32_t* th;         // NTH x 4
    const int32_t* reg_ptr;    // NREG+1
    const int32_t* reg_clamp;  // NREG (1: max(v, 0))
    const int32_t* reg_feat;   // nnz
    const int32_t* rx;         // NRXN x 6
    const int32_t* expf;       // NRXN x NDYN
    const int32_t* expr;       // NRXN x NDYN
    const int32_t* foldf;      // NRXN x NFIX
    const int32_t* foldr;      // NRXN x NFIX
    const int32_t* cpiv;       // NCONS
    const int32_t* tof;        // NTOF
    const double* thd;         // NTH x 5
    const double* freq;
    const double* reg_coef;
    const double* rxd;         // NRXN x 3
    const double* S;           // NDYN x NRXN
    const double* dyn;         // NDYN x 4
    const double* C;           // NCONS x NDYN
};

struct CondView {
    int64_t n;
    const double* T; int64_t sT;
    const double* p; int64_t sp;
    const double* desc; int64_t ld_desc, s_desc;
    const double* fixc; int64_t ld_fix, s_fix;
    const double* y0; int64_t ld_y0, s_y0;
    const double* inflow; int64_t ld_in, s_in;
};

__device__ __forceinline__ double ipow(double c, int e) {
    // small non-negative integer powers (stoichiometric exponents)
    if (e == 0) return 1.0;
    if (e == 1) return c;
    if (e == 2) return c * c;
    double r = c * c * c;
    for (int k = 3; k < e; ++k) r *= c;
    return r;
}

// ---------------------------------------------------------------------------
// Kernel-1 body: thermochemistry features -> energy program -> k (one lane)
// State free energies: pycatkin/classes/state.py:266-386; rate constants:
// pycatkin/classes/reaction.py:94-168, pycatkin/functions/rate_constants.py.
// feat: this lane's feature column base; stride = lane stride of the scratch.
// ---------------------------------------------------------------------------
__device__ inline void thermo_features(const NetView& nv, double T, double p,
                                       const double* desc, int64_t ld_desc,
                                       double* feat, int64_t fs) {
    feat[0] = 1.0;
    feat[fs] = T;
    for (int k = 0; k < nv.D; ++k) feat[(2 + k) * fs] = desc[k * ld_desc];
    const double kT = kB * T;
    for (int s = 0; s < nv.NTH; ++s) {
        const int kind = nv.th[4 * s + 0];
        const int f0 = nv.th[4 * s + 1], nf = nv.th[4 * s + 2], shape = nv.th[4 * s + 3];
        const double zpe = nv.thd[5 * s + 0], mass = nv.thd[5 * s + 1];
        const double sigma = nv.thd[5 * s + 2], rotI = nv.thd[5 * s + 3], gvfix = nv.thd[5 * s + 4];
        double gv = 0.0, gt = 0.0, gr = 0.0;
        if (kind & PCK_TH_VIB) {
            if (gvfix == gvfix) {          // Gvibr given in the input (vibr_source 'inputfile')
                gv = gvfix;
            } else {
                double sl = 0.0, sf = 0.0;
                for (int q = 0; q < nf; ++q) {
                    const double nu = nv.freq[f0 + q];
                    sf += nu;
                    sl += log(1.0 - exp(-nu * hP / kT));
                }
                gv = (sf != 0.0) ? zpe + (kT * sl) * JtoeV : zpe;     // state.py:313-318
            }
        }
        if (kind & PCK_TH_GAS) {
            const double m = mass * amutokg;                          // state.py:329-331
            gt = (-kT * log((kT / p) * pow(2.0 * PI * m * kT / (hP * hP), 1.5))) * JtoeV;
            if (shape == 2) {                                         // state.py:351-358
                gr = (-kT * log(8.0 * PI * PI * kT * rotI / (sigma * hP * hP))) * JtoeV;
            } else {
                gr = (-kT * log((sqrt(PI) / sigma) * pow(8.0 * PI * PI * kT / (hP * hP), 1.5) * rotI)) * JtoeV;
            }
        }
        const int b = 2 + nv.D + 3 * s;
        feat[b * fs] = gv;
        feat[(b + 1) * fs] = gt;
        feat[(b + 2) * fs] = gr;
    }
    const int rb = 2 + nv.D + 3 * nv.NTH;
    for (int r = 0; r < nv.NREG; ++r) {
        double v = 0.0;
        for (int q = nv.reg_ptr[r]; q < nv.reg_ptr[r + 1]; ++q) v += nv.reg_coef[q] * feat[nv.reg_feat[q] * fs];
        if (nv.reg_clamp[r]) v = fmax(v, 0.0);   // e.g. np.max((ETS - EIS, 0.0)) in a volcano driver
        feat[(rb + r) * fs] = v;
    }
}

__device__ inline void rate_constants_from_feat(const NetView& nv, double T, const double* feat, int64_t fs,
                                                int j, double& kf, double& kr) {
    const int* rx = nv.rx + 6 * j;
    const int type = rx[0], rev = rx[1];
    const int rb = 2 + nv.D + 3 * nv.NTH;
    const double ga = rx[2] >= 0 ? feat[(rb + rx[2]) * fs] * EV2JMOL : 0.0;
    const double grxn = rx[3] >= 0 ? feat[(rb + rx[3]) * fs] * EV2JMOL : 0.0;
    const double erxn = rx[4] >= 0 ? feat[(rb + rx[4]) * fs] * EV2JMOL : 0.0;
    const double RT = Rgas * T;
    const double kads_c = nv.rxd[3 * j + 0], kdes_c = nv.rxd[3 * j + 1], kdes_e = nv.rxd[3 * j + 2];
    // reaction.py:121: "Arrhenius" or a non-zero free-energy barrier
    if (type == PCK_RX_ARRHENIUS || (rx[5] && ga != 0.0)) {
        kf = (kB * T / hP) * exp(-fmax(ga, 0.0) / RT);               // karr(prefactor(T), max(dGa,0))
        kr = rev ? kf / exp(-grxn / RT) : 0.0;                        // k_from_eq_rel(kf, keq_therm)
        return;
    }
    const double ka = kads_c / sqrt(T);                               // kads: area/sqrt(2 pi m kB T)
    switch (type) {
    case PCK_RX_ADS_KEQ:
        kf = ka; kr = rev ? ka / exp(-grxn / RT) : 0.0; break;
    case PCK_RX_DES_KEQ:
        kf = ka * exp(-grxn / RT); kr = rev ? ka : 0.0; break;
    case PCK_RX_ADS_KDES:
        kf = ka; kr = rev ? kdes_c * pow(T, kdes_e) * exp(erxn / RT) : 0.0; break;   // des_en = -dErxn
    case PCK_RX_DES_KDES:
        kf = kdes_c * pow(T, kdes_e) * exp(-erxn / RT); kr = rev ? ka : 0.0; break;
    default:
        kf = 0.0; kr = 0.0;
    }
}

// Reciprocal from v_rcp_f64 plus two Newton steps (the error of the hardware
// estimate squares each step: within 1 ulp, not always correctly rounded),
// 5 VALU ops instead of the ~10 of the IEEE divide sequence.  For positive or
// negative normal x; used where a last-bit difference only moves a step-size
// decision or a pivot reciprocal by rounding.
#ifndef PCK_FASTDIV
#define PCK_FASTDIV 1
#endif
__device__ __forceinline__ double rcp(double x) {
#if PCK_FASTDIV
    double r = __builtin_amdgcn_rcp(x);
    r = fma(fma(-x, r, 1.0), r, r);
    return fma(fma(-x, r, 1.0), r, r);
#else
    return 1.0 / x;
#endif
}

// One Newton step on the v_rcp_f64 estimate: the estimate's relative error
// is <= 4.6e-8, so one step leaves <= 2.3e-15 (two steps are correctly
// rounded on all 2^24 inputs of tools/rcp_accuracy.hip, measured on gfx950).
// 16 + 8 cycles instead of 16 + 16: for the lane integrator's step-size
// reciprocal, its stage LU pivots and the site-balance projection, where a
// few ulps only perturb the stage matrix or a scale factor by rounding
// (PCK_LANE_FAST below).
__device__ __forceinline__ double rcp1(double x) {
    const double r = __builtin_amdgcn_rcp(x);
    return fma(fma(-x, r, 1.0), r, r);
}

// Cheaper arithmetic in the one-lane integrator (mk_solver.h: integrate and
// the threshold-pivoting lu): the pivot reciprocals, 1/h and the projection
// factor from rcp1; the threshold rule's pivot search only where some lane of
// the wavefront needs it (one max per row and one compare per column on the
// common path); the step-size factor from v_log_f32 / v_exp_f32.  (The stage
// right-hand sides with the 1/h-scaled coefficients computed once per step
// saved 5 instructions and cost 8 VGPRs: not kept.)
// 0 = the round-4 arithmetic (A/B).  Results move by rounding only.
#ifndef PCK_LANE_FAST
#define PCK_LANE_FAST 1
#endif

// Double-double arithmetic (hi + lo, |lo| <= ulp(hi) / 2) for the Newton
// refinement's residual (mk_solver.h: newton): error-free products by FMA
// and Knuth's two-sum, so a balance of 1e11 / s fluxes that cancel to O(1)
// keeps ~30 digits instead of the ~5 the plain evaluation leaves.
struct dd {
    double hi, lo;
};
// no FMA contraction in these: the error terms must be computed as written
// (a contracted a*b feeding its own error term would cancel it)
#pragma clang fp contract(off)
__device__ __forceinline__ dd dd_of(double a) { return {a, 0.0}; }
__device__ __forceinline__ dd two_prod(double a, double b) {
    const double p = a * b;
    return {p, __builtin_fma(a, b, -p)};
}
__device__ __forceinline__ dd two_sum(double a, double b) {
    const double s = a + b;
    const double bb = s - a;
    return {s, (a - (s - bb)) + (b - bb)};
}
__device__ __forceinline__ dd quick_two_sum(double a, double b) {
    const double s = a + b;
    return {s, b - (s - a)};
}
__device__ __forceinline__ dd dd_add(dd a, dd b) {
    const dd s = two_sum(a.hi, b.hi);
    return quick_two_sum(s.hi, s.lo + (a.lo + b.lo));
}
__device__ __forceinline__ dd dd_neg(dd a) { return {-a.hi, -a.lo}; }
__device__ __forceinline__ dd dd_mul(dd a, double b) {
    const dd p = two_prod(a.hi, b);
    return quick_two_sum(p.hi, __builtin_fma(a.lo, b, p.lo));
}
__device__ __forceinline__ dd dd_mul(dd a, dd b) {
    const dd p = two_prod(a.hi, b.hi);
    return quick_two_sum(p.hi, __builtin_fma(a.hi, b.lo, __builtin_fma(a.lo, b.hi, p.lo)));
}
// c^e for a small non-negative integer e (ipow in double-double)
__device__ __forceinline__ dd dd_pow(dd c, int e) {
    dd r = dd_of(1.0);
    for (int q = 0; q < e; ++q) r = dd_mul(r, c);
    return r;
}
#pragma clang fp contract(fast)   // the build default (-ffp-contract=fast) again

// Step-size factor of the error controller, 0.9 en^(-1/4) with en^2 = q the
// mean squared scaled error, in fp32 (three single-instruction estimates
// instead of the fp64 sqrt / rsqrt sequences: the factor needs ~3 digits).
// q = 0 gives +inf and q = inf gives 0; callers clamp to [0.2, 6].
__device__ __forceinline__ double step_factor(double q) {
    const float qf = (float)q;
    return 0.9 * (double)__builtin_amdgcn_rsqf(__builtin_amdgcn_sqrtf(__builtin_amdgcn_sqrtf(qf)));
}

// the same factor from two fp32 transcendentals, 0.9 * 2^(-log2(q) / 8)
// (PCK_LANE_FAST: one fewer quarter-rate instruction on the controller's
// dependent chain)
__device__ __forceinline__ double step_factor_fast(double q) {
    const float qf = (float)q;
    return (double)(0.9f * __builtin_amdgcn_exp2f(-0.125f * __builtin_amdgcn_logf(qf)));
}

// In-register LU with threshold partial pivoting (row swaps by predicated
// selects so every register index stays static).  The diagonal is kept
// unless a row below is more than 1/PIVOT_TAU times larger (the classic
// threshold rule, growth bounded by (1 + 1/tau)^k); when no lane of the
// wavefront swaps at column k the select block is skipped (wave vote) and
// bit k of `swaps` stays clear for the solves.  Returns false on a zero pivot.
#ifndef PCK_PIVOT_TAU
#define PCK_PIVOT_TAU 0.1
#endif
constexpr double PIVOT_TAU = PCK_PIVOT_TAU;

// PARTIAL = true: plain partial pivoting (tau = 1), for the Newton polish,
// whose Jacobian is near-singular at a site-starved root (condition ~1e17):
// there the threshold rule's growth (up to (1 + 1/tau)^(NS-1)) costs the
// digits that decide whether Newton converges quadratically -- 60 of the 2 560
// volcano fixture nodes were classified degenerate by the device and regular
// by the oracle (LAPACK partial pivoting) from the same start state
// (tools/flip_probe.py).  The Rosenbrock matrices I/(h g) - J are
// diagonally dominant enough for the threshold rule, which swaps rarely.
template <int NS>
__device__ __forceinline__ void lu_swap_rows(double (&A)[NS][NS], int k, int p) {
    // the trailing columns only (LINPACK's dgefa): the multipliers of the
    // earlier columns stay in the rows they were computed in, which is what
    // lu_solve's forward sweep -- swap b[k], then eliminate with column k --
    // assumes.  Rounds 1-4 swapped whole rows here (LAPACK's storage, whose
    // solve applies every swap first), so a swap at column k >= 1 left the
    // solve with a wrong L: 95 % of random 5 x 5 systems solved to O(1) error
    // (DESIGN.md "LU").
#pragma unroll
    for (int r = k + 1; r < NS; ++r) {
        const bool sw = (p == r);
#pragma unroll
        for (int q = k; q < NS; ++q) {
            const double a = A[k][q], b = A[r][q];
            A[k][q] = sw ? b : a;
            A[r][q] = sw ? a : b;
        }
    }
}

template <int NS, bool PARTIAL = false>
__device__ __forceinline__ bool lu(double (&A)[NS][NS], int (&piv)[NS], unsigned& swaps) {
    bool ok = true;
    swaps = 0u;
#pragma unroll
    for (int k = 0; k < NS; ++k) {
        if (PCK_LANE_FAST && !PARTIAL) {
            // threshold rule, common path: the largest sub-diagonal entry of
            // column k against |A[k][k]| / tau; the search for the pivot row
            // runs only when some lane of the wavefront swaps (same pivots)
            const double dk = fabs(A[k][k]) * (1.0 / PIVOT_TAU);
            double m = 0.0;
#pragma unroll
            for (int r = k + 1; r < NS; ++r) m = fmax(m, fabs(A[r][k]));
            piv[k] = k;
            if (__any(m > dk)) {
                int p = k;
                double best = dk;
#pragma unroll
                for (int r = k + 1; r < NS; ++r) {
                    const double a = fabs(A[r][k]);
                    p = (a > best) ? r : p;
                    best = fmax(best, a);
                }
                piv[k] = p;
                swaps |= 1u << k;
                lu_swap_rows(A, k, p);
            }
            const double d = A[k][k];
            ok = ok && (d != 0.0) && (d == d);
            const double inv = rcp1(d);
#pragma unroll
            for (int r = k + 1; r < NS; ++r) {
                const double l = A[r][k] * inv;
                A[r][k] = l;
#pragma unroll
                for (int q = k + 1; q < NS; ++q) A[r][q] -= l * A[k][q];
            }
            A[k][k] = inv;
            continue;
        }
        int p = k;
        double best = fabs(A[k][k]) * (PARTIAL ? 1.0 : 1.0 / PIVOT_TAU);   // a multiply, not an IEEE divide
#pragma unroll
        for (int r = k + 1; r < NS; ++r) {
            const double a = fabs(A[r][k]);
            p = (a > best) ? r : p;      // one select + a max instead of selecting a double pair
            best = fmax(best, a);
        }
        piv[k] = p;
        if (__any(p != k)) {
            swaps |= 1u << k;
            lu_swap_rows(A, k, p);
        }
        const double d = A[k][k];
        ok = ok && (d != 0.0) && (d == d);
        const double inv = rcp(d);
#pragma unroll
        for (int r = k + 1; r < NS; ++r) {
            const double l = A[r][k] * inv;
            A[r][k] = l;
#pragma unroll
            for (int q = k + 1; q < NS; ++q) A[r][q] -= l * A[k][q];
        }
        A[k][k] = inv;     // the solves multiply by the stored reciprocal (one fp64 divide per pivot)
    }
    return ok;
}

template <int NS, bool SWAPS>
__device__ __forceinline__ void lu_solve_impl(const double (&A)[NS][NS], const int (&piv)[NS], unsigned swaps,
                                              double (&b)[NS]) {
#pragma unroll
    for (int k = 0; k < NS; ++k) {
        if (SWAPS && (swaps & (1u << k))) {
#pragma unroll
            for (int r = k + 1; r < NS; ++r) {
                const bool sw = (piv[k] == r);
                const double a = b[k], c = b[r];
                b[k] = sw ? c : a;
                b[r] = sw ? a : c;
            }
        }
#pragma unroll
        for (int r = k + 1; r < NS; ++r) b[r] -= A[r][k] * b[k];
    }
    // back substitution, each row's sum taken from the last column inward:
    // b[q] becomes final in that order, so only the b[k+1] term waits on the
    // row just solved and the chain is one FMA and one multiply per row (in
    // column order every term of the row waited on b[k+1]: the CSTR sweep,
    // bound by its slowest lane's step chain, 1.28 -> 1.08 ms per 1e4
    // temperatures; the volcano step unchanged, profiles/r6/ab_bsub/)
#pragma unroll
    for (int k = NS - 1; k >= 0; --k) {
        double v = b[k];
#pragma unroll
        for (int q = NS - 1; q > k; --q) v -= A[k][q] * b[q];
        b[k] = v * A[k][k];
    }
}

// `swaps` is wave-uniform (set under a wave vote in lu): readfirstlane makes
// that visible to the compiler, so the common no-swap case is one scalar
// branch to a select-free solve instead of speculated row selects
template <int NS>
__device__ __forceinline__ void lu_solve(const double (&A)[NS][NS], const int (&piv)[NS], unsigned swaps,
                                         double (&b)[NS]) {
    const unsigned sw = (unsigned)__builtin_amdgcn_readfirstlane((int)swaps);
    if (sw == 0u)
        lu_solve_impl<NS, false>(A, piv, 0u, b);
    else
        lu_solve_impl<NS, true>(A, piv, sw, b);
}

}  // namespace pck
