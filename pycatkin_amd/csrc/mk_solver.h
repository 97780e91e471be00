// Solver-side device code, templated on a network "plan policy":
//
//   PlanRT<NS>   reads the uploaded plan at run time (any network with NS <= 8);
//                the reaction loop is a runtime loop over uniform plan data,
//                k_eff lives in LDS.
//   PlanCT<Net>  a network compiled in (networks.h, generated from the same
//                plan by tools/gen_networks.py): every loop over reactions and
//                species is unrolled against constexpr tables, zero
//                stoichiometry / exponents vanish at compile time and k_eff
//                lives in VGPRs.  Selected at pck_network_create by the plan's
//                structural digest; results are identical to PlanRT.
//
// One lane = one condition (or one DRC perturbation of a condition).
#pragma once
#include "mk_device.h"
#include "networks.h"


namespace pck {

#ifdef PCK_TRACE
// diagnostic builds only (tools/trace_group.py, tools/trace_newton.py):
// records of one condition (lane-group integrator steps, lane Newton iterations)
#define PCK_TRACE_N 8192
#define PCK_TRACE_W 8
__device__ long long pck_trace_cond = -1;
__device__ int pck_trace_pos = 0;
__device__ double pck_trace_buf[PCK_TRACE_N * PCK_TRACE_W];
#endif

// Phase split of the lane integrator (diagnostic builds, -DPCK_PHASE=1;
// tools/phase_lane.py): shader-clock cycles of the waves whose block index
// is a multiple of PCK_PHASE_EVERY, per phase of a step, summed over those
// waves (lane 0 adds them up at the end of the solve):
//   [0 Jacobian + W, 1 LU, 2 six solves, 3 seven rhs, 4 stage combinations,
//    5 error norm / controller / projection / bookkeeping, 6 steps, 7 waves]
// Scheduling barriers around every stamp keep the phases in sequence; they
// cost the build its cross-phase overlap, so absolute cycles read high.
#ifndef PCK_PHASE
#define PCK_PHASE 0
#endif
#ifndef PCK_PHASE_EVERY
#define PCK_PHASE_EVERY 64
#endif
#if PCK_PHASE
__device__ double pck_lphase[8];
#define PCK_LPH_DECL                                                                   \
    double lph[8] = {0, 0, 0, 0, 0, 0, 0, 0};                                          \
    const bool lph_on = (blockIdx.x % PCK_PHASE_EVERY) == 0;                           \
    long long lph_t = 0
#define PCK_LPH(i, ...)                                                                \
    do {                                                                               \
        __builtin_amdgcn_sched_barrier(0);                                             \
        const long long t_ph0 = __builtin_readcyclecounter();                          \
        __builtin_amdgcn_sched_barrier(0);                                             \
        __VA_ARGS__;                                                                   \
        __builtin_amdgcn_sched_barrier(0);                                             \
        if (lph_on) lph[i] += (double)(__builtin_readcyclecounter() - t_ph0);          \
        __builtin_amdgcn_sched_barrier(0);                                             \
    } while (0)
#define PCK_LPH_STEP() do { if (lph_on) lph[6] += 1.0; } while (0)
#define PCK_LPH_MARK()                                                                 \
    do {                                                                               \
        __builtin_amdgcn_sched_barrier(0);                                             \
        lph_t = __builtin_readcyclecounter();                                          \
        __builtin_amdgcn_sched_barrier(0);                                             \
    } while (0)
#define PCK_LPH_UNTIL(i)                                                               \
    do {                                                                               \
        __builtin_amdgcn_sched_barrier(0);                                             \
        const long long t_ph1 = __builtin_readcyclecounter();                          \
        if (lph_on && lph_t) lph[i] += (double)(t_ph1 - lph_t);                        \
        lph_t = 0;                                                                     \
        __builtin_amdgcn_sched_barrier(0);                                             \
    } while (0)
#define PCK_LPH_FLUSH()                                                                \
    do {                                                                               \
        if (lph_on && (threadIdx.x & 63) == 0) {                                       \
            lph[7] = 1.0;                                                              \
            for (int q = 0; q < 8; ++q) atomicAdd(&pck_lphase[q], lph[q]);             \
        }                                                                              \
    } while (0)
#else
#define PCK_LPH_DECL
#define PCK_LPH(i, ...) __VA_ARGS__
#define PCK_LPH_STEP() do {} while (0)
#define PCK_LPH_MARK() do {} while (0)
#define PCK_LPH_UNTIL(i) do {} while (0)
#define PCK_LPH_FLUSH() do {} while (0)
#endif
// Wave timeline (diagnostic builds, -DPCK_WAVE_TIMES=1; tools/wave_timeline.py):
// every block of a lane-solver launch over the whole batch (no index list)
// records [start, end] on the constant-rate real-time clock and its hardware
// slot (HW_ID), for the first PCK_WT_N blocks of the last such launch
#ifndef PCK_WAVE_TIMES
#define PCK_WAVE_TIMES 0
#endif
#if PCK_WAVE_TIMES
#define PCK_WT_N 65536
__device__ long long pck_wtimes[3 * PCK_WT_N];
#endif

#define PCK_LRET(st)       \
    do {                   \
        PCK_LPH_FLUSH();   \
        return st;         \
    } while (0)

template <int NS_>
struct PlanRT {
    static constexpr int NS = NS_;
    static constexpr bool CT = false;
    static constexpr int RMAX = 1;
    const NetView& nv;
    __device__ explicit PlanRT(const NetView& v) : nv(v) {}
    __device__ int R() const { return nv.NRXN; }
    __device__ int ef(int j, int i) const { return nv.expf[j * NS + i]; }
    __device__ int er(int j, int i) const { return nv.expr[j * NS + i]; }
    __device__ double S(int i, int j) const { return nv.S[i * nv.NRXN + j]; }
    __device__ double cf(int i) const { return nv.dyn[4 * i + 0]; }
    __device__ double rs0(int i) const { return nv.dyn[4 * i + 1]; }
    __device__ double rsT(int i) const { return nv.dyn[4 * i + 2]; }
    __device__ double fl(int i) const { return nv.dyn[4 * i + 3]; }
    __device__ int ncons() const { return nv.NCONS; }
    __device__ double C(int l, int i) const { return nv.C[l * NS + i]; }
    __device__ int cpiv(int l) const { return nv.cpiv[l]; }
};

template <class Net>
struct PlanCT {
    static constexpr int NS = Net::NS;
    static constexpr bool CT = true;
    static constexpr int RMAX = Net::R;
    const NetView& nv;
    __device__ explicit PlanCT(const NetView& v) : nv(v) {}
    __device__ static constexpr int R() { return Net::R; }
    __device__ static constexpr int ef(int j, int i) { return Net::ef(j, i); }
    __device__ static constexpr int er(int j, int i) { return Net::er(j, i); }
    __device__ static constexpr double S(int i, int j) { return Net::S(i, j); }
    __device__ static constexpr double cf(int i) { return Net::dyn(i, 0); }
    __device__ static constexpr double rs0(int i) { return Net::dyn(i, 1); }
    __device__ static constexpr double rsT(int i) { return Net::dyn(i, 2); }
    __device__ static constexpr double fl(int i) { return Net::dyn(i, 3); }
    __device__ static constexpr int ncons() { return Net::NCONS; }
    __device__ static constexpr double C(int l, int i) { return Net::C(l, i); }
    __device__ static constexpr int cpiv(int l) { return Net::cpiv(l); }
};

// k_eff storage: LDS columns (runtime plans) or registers (compiled plans)
struct KLds {
    double* kf;
    double* kr;
    int ks;
    __device__ double f(int j) const { return kf[j * ks]; }
    __device__ double r(int j) const { return kr[j * ks]; }
    __device__ void set(int j, double a, double b) { kf[j * ks] = a; kr[j * ks] = b; }
};
template <int R>
struct KReg {
    double kf[R], kr[R];
    __device__ double f(int j) const { return kf[j]; }
    __device__ double r(int j) const { return kr[j]; }
    __device__ void set(int j, double a, double b) { kf[j] = a; kr[j] = b; }
};

// loop over reactions: unrolled for compiled plans, runtime otherwise
template <class P, class F>
__device__ __forceinline__ void for_rxn(const P& p, F&& body) {
    if constexpr (P::CT) {
#pragma unroll
        for (int j = 0; j < P::RMAX; ++j) body(j);
    } else {
        for (int j = 0; j < p.R(); ++j) body(j);
    }
}

template <int NS>
struct Lane {
    double T;
    const double* ins;   // this lane's inflow column in LDS (stride ks), flow rows only
    int ks;
#ifdef PCK_TRACE
    int64_t cidx;        // condition index (trace builds)
#endif
};

// ---------------------------------------------------------------------------
// Species rates / Jacobian.  pycatkin/classes/old_system.py:202-313 with
// reactor.py rhs/jacobian, and system.py:345-508 -- one mass-action form once
// the host folds fixed species and weights into the plan:
//   f_i = rs_i * sum_j S_ij (kf_j prod c^a - kr_j prod c^b) + fl_i (in_i - y_i),
//   c_i = cf_i y_i,  rs_i = rs0_i + rsT_i T.
// ---------------------------------------------------------------------------
// rf - rr: the lane solver lets the compiler contract the last product of
// rr into the subtraction (rounding it as written cost the volcano 4 % with
// unchanged step counts, profiles/r4; the lane-group kernels round it as
// written, mk_group.h: ct_sub, where the contraction noise cost DMTM
// transients 80x more steps -- DESIGN.md)
__device__ __forceinline__ double net_rate(double rf, double rr) { return rf - rr; }

template <class P, class K>
__device__ __forceinline__ void rhs(const P& p, const Lane<P::NS>& L, const K& k, const double (&y)[P::NS],
                                    double (&f)[P::NS]) {
    constexpr int NS = P::NS;
    double c[NS];
#pragma unroll
    for (int i = 0; i < NS; ++i) { c[i] = p.cf(i) * y[i]; f[i] = 0.0; }
    for_rxn(p, [&](int j) {
        double rf = k.f(j), rr = k.r(j);
#pragma unroll
        for (int i = 0; i < NS; ++i) {
            if (p.ef(j, i)) rf *= ipow(c[i], p.ef(j, i));
            if (p.er(j, i)) rr *= ipow(c[i], p.er(j, i));
        }
        const double net = net_rate(rf, rr);
#pragma unroll
        for (int i = 0; i < NS; ++i) {
            const double s = p.S(i, j);
            if (s != 0.0) f[i] += s * net;
        }
    });
#pragma unroll
    for (int i = 0; i < NS; ++i) {
        f[i] *= (p.rsT(i) != 0.0) ? p.rs0(i) + p.rsT(i) * L.T : p.rs0(i);
        if (p.fl(i) != 0.0) f[i] += p.fl(i) * (L.ins[i * L.ks] - y[i]);
    }
}

template <class P, class K>
__device__ __forceinline__ void jac(const P& p, const Lane<P::NS>& L, const K& k, const double (&y)[P::NS],
                                    double (&J)[P::NS][P::NS]) {
    constexpr int NS = P::NS;
    double c[NS];
#pragma unroll
    for (int i = 0; i < NS; ++i) {
        c[i] = p.cf(i) * y[i];
#pragma unroll
        for (int q = 0; q < NS; ++q) J[i][q] = 0.0;
    }
    for_rxn(p, [&](int j) {
        const double kf = k.f(j), kr = k.r(j);
        double d[NS];
#pragma unroll
        for (int q = 0; q < NS; ++q) {
            double v = 0.0;
            if (p.ef(j, q)) {
                double t = kf * (double)p.ef(j, q) * p.cf(q) * ipow(c[q], p.ef(j, q) - 1);
#pragma unroll
                for (int i = 0; i < NS; ++i)
                    if (i != q && p.ef(j, i)) t *= ipow(c[i], p.ef(j, i));
                v += t;
            }
            if (p.er(j, q)) {
                double t = kr * (double)p.er(j, q) * p.cf(q) * ipow(c[q], p.er(j, q) - 1);
#pragma unroll
                for (int i = 0; i < NS; ++i)
                    if (i != q && p.er(j, i)) t *= ipow(c[i], p.er(j, i));
                v -= t;
            }
            d[q] = v;
        }
#pragma unroll
        for (int i = 0; i < NS; ++i) {
            const double s = p.S(i, j);
            if (s != 0.0) {
#pragma unroll
                for (int q = 0; q < NS; ++q) J[i][q] += s * d[q];
            }
        }
    });
#pragma unroll
    for (int i = 0; i < NS; ++i) {
        const double rs = (p.rsT(i) != 0.0) ? p.rs0(i) + p.rsT(i) * L.T : p.rs0(i);
#pragma unroll
        for (int q = 0; q < NS; ++q) J[i][q] *= rs;
        J[i][i] -= p.fl(i);
    }
}

// ---------------------------------------------------------------------------
// per-lane setup: LDS per lane (stride = blockDim) = [kf_eff R][kr_eff R][inflow NS]
// ---------------------------------------------------------------------------
__host__ __device__ inline size_t lds_bytes(int R, int NS, int B) {
    return sizeof(double) * (size_t)(2 * (R > 0 ? R : 1) + NS) * B;
}

// every inflow slot is written (0 on rows without flow): PCK_INS_ALL=0 writes
// only the flow rows (the round-4 code, A/B)
#ifndef PCK_INS_ALL
#define PCK_INS_ALL 1
#endif
template <class P>
__device__ __forceinline__ void lane_setup(const P& p, const NetView& nv, const CondView& cv, int64_t c,
                                           Lane<P::NS>& L, double* lds_lane, int ks) {
    L.T = cv.T[c * cv.sT];           // reactor.py:34-41: CSTR row scaling is linear in T
    L.ks = ks;
#ifdef PCK_TRACE
    L.cidx = c;
#endif
    double* ins = lds_lane + (size_t)2 * nv.NRXN * ks;
    L.ins = ins;
#pragma unroll
    for (int i = 0; i < P::NS; ++i)  // 1/residence_time on CSTR gas rows (reactor.py:154-156)
        if (PCK_INS_ALL || p.fl(i) != 0.0)
            ins[i * ks] = (cv.inflow && p.fl(i) != 0.0) ? cv.inflow[i * cv.ld_in + c * cv.s_in] : 0.0;
}

// effective k (fixed species folded in, optional DRC perturbation)
template <class P, class K>
__device__ __forceinline__ void load_keff(const P& p, const NetView& nv, const CondView& cv, int64_t c,
                                          const double* kf, const double* kr, int64_t ld_k, K& k, int pj,
                                          double pfac) {
    for_rxn(p, [&](int j) {
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
        k.set(j, a, b);
    });
}

// Conservation rows in the stage system.  With site balances C f(y) = 0
// for every y, so C J = 0: the iteration matrix I/(h g) - J loses rank as h
// grows (t_end = 1e12 s in examples/DMTM) and its LU's error lands in the
// conserved directions.  The exact stage vectors satisfy C k_i = 0, so the
// pivot row of each law is replaced by that law (scaled to the row's size)
// and its right-hand side entry by 0: the same solution in exact
// arithmetic, a well-conditioned system at any h.
template <class P, int NS>
__device__ __forceinline__ void cons_rows(const P& p, double (&W)[NS][NS]) {
    for (int l = 0; l < p.ncons(); ++l) {
        const int pv = p.cpiv(l);
#pragma unroll
        for (int i = 0; i < NS; ++i) {
            if (i != pv) continue;
            double m = 0.0;
#pragma unroll
            for (int q = 0; q < NS; ++q) m = fmax(m, fabs(W[i][q]));
#pragma unroll
            for (int q = 0; q < NS; ++q) W[i][q] = p.C(l, q) * m;
        }
    }
}
template <class P, int NS>
__device__ __forceinline__ void cons_zero(const P& p, double (&b)[NS]) {
    for (int l = 0; l < p.ncons(); ++l) {
        const int pv = p.cpiv(l);
#pragma unroll
        for (int i = 0; i < NS; ++i)
            if (i == pv) b[i] = 0.0;
    }
}

// ---------------------------------------------------------------------------
// RODAS4P (Steinebach; by default, see rodas4 below) or RODAS4 (Hairer &
// Wanner): stiffly accurate 4(3) Rosenbrock methods, L-stable, same
// structure, autonomous form:  (I/(h g) - J) k_i = f(u_i) + sum_j C_ij k_j / h,
// u_{i+1} = y + sum_j a_ij k_j,  y_new = u_5 + k5 + k6,  error = k6.
// ---------------------------------------------------------------------------
// A rejected step with en^2 above PCK_BLOWUP_Q (error 1e6 x the tolerance)
// at a step size below 1e-4 t is catastrophic; more than PCK_MAX_BLOWUPS of
// them end the solve with PCK_ST_STEPFAIL (a healthy solve has a handful,
// while its first step size is being found; large-h rejections late in a
// long run, where I/(h g) - J loses rank along the site balances, do not
// count).
#define PCK_BLOWUP_Q 1e12
#define PCK_MAX_BLOWUPS 200
// Stagnation: more than PCK_STALL_STEPS consecutive steps with h below
// PCK_STALL_H * (t - t0) end the solve with PCK_ST_STEPFAIL.  The stalled
// solves of the synthetic network sit at h ~ 1e-6 t (scipy BDF fails on the
// same conditions); the slowest healthy solve measured (examples/DMTM at
// 400 K to 1e12 s at rtol 1e-10 / atol 1e-14, rounding-limited late in the
// run) keeps h above 2e-5 t.
#define PCK_STALL_STEPS 16384
#define PCK_STALL_H 1e-5
#define PCK_STALL_EVERY 64       // lane solver: tested every 64th step (power of 2)
// Positivity rule (reject steps that drive a component below -atol, clip
// falling tolerance-level negatives to 0): PCK_POSITIVITY=1.  Off, the
// integrator is plain Rodas4 like the reference's scipy BDF, which has no
// such rule.
#ifndef PCK_POSITIVITY
#define PCK_POSITIVITY 1
#endif
// Conservation rows in the lane solver's stage systems (cons_rows below): an
// A/B knob, compiled out by default (the runtime flag costs 3 % of the
// volcano step); the lane-group solver reads PCK_CONS_ROWS=1 at run time.
#ifndef PCK_CONS_ROWS
#define PCK_CONS_ROWS 0
#endif
// diagnostic builds: poison the dynamic LDS block at kernel start
#ifndef PCK_POISON_LDS
#define PCK_POISON_LDS 0
#endif
// integrate / newton are inlined into the kernel (see DESIGN.md "Runtime-plan
// fault"); -DPCK_LANE_INLINE=__noinline__ builds the call variant for study
#ifndef PCK_LANE_INLINE
#define PCK_LANE_INLINE __forceinline__
#endif

// Rosenbrock coefficients, in the transformed form (stages k_i solve
// (I/(h g) - J) k_i = f(u_i) + (1/h) sum_j C_ij k_j, u_i = y + sum_j a_ij k_j;
// stiffly accurate: y1 = y + a5. k + k5 + k6, error estimate k6).
// PCK_RODAS4P=1 (default): Steinebach's RODAS4P (1995), order 4 and free of
// the order reduction Rodas4 shows where a stiff mode is forced by a slowly
// varying solution (the Prothero-Robinson problem: Rodas4's error falls like
// h^1 there, RODAS4P's like h^3; tools/rodas_mirror.py).  On the volcano
// grid that regime is CO poisoning, sO decaying over ten decades under
// atol 1e-22: the slowest solve drops from 1 112 to 723 steps and the mean
// from 351 to 318 (DESIGN.md "Integrator").  PCK_RODAS4P=0: the
// Hairer-Wanner RODAS4 set of rounds 1-4.
#ifndef PCK_RODAS4P
#define PCK_RODAS4P 1
#endif
// largest step growth after an accepted step (Hairer-Wanner RODAS: 6).  10
// takes the steady-state transients through their first decades of t
// faster: volcano 320.0 M -> 315.0 M integrator steps per grid, 5.71 ->
// 5.63 ms (profiles/r4/ab_facmax10_*), CH4 and DMTM DRC unchanged or faster
#ifndef PCK_FACMAX
#define PCK_FACMAX 10.0
#endif
namespace rodas4 {
constexpr double g = 0.25;
#if PCK_RODAS4P
constexpr double a21 = 3.0, a31 = 1.831036793486759, a32 = 0.4955183967433795;
constexpr double a41 = 2.304376582692669, a42 = -0.05249275245743001, a43 = -1.176798761832782;
constexpr double a51 = -7.170454962423024, a52 = -4.741636671481785, a53 = -16.31002631330971,
                 a54 = -1.062004044111401;
constexpr double C21 = -12.0, C31 = -8.791795173947035, C32 = -2.207865586973518;
constexpr double C41 = 10.81793056857153, C42 = 6.780270611428266, C43 = 19.53485944642410;
constexpr double C51 = 34.19095006749676, C52 = 15.49671153725963, C53 = 54.74760875964130,
                 C54 = 14.16005392148534;
constexpr double C61 = 34.62605830930532, C62 = 15.30084976114473, C63 = 56.99955578662667,
                 C64 = 18.40807009793095, C65 = -5.714285714285717;
#else
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
#endif
}  // namespace rodas4

// Dense output: over an accepted step y0 -> y1 of size h,
//   y(t0 + s h) = (1-s) y0 + s (y1 + (1-s) (d2 + s d3)),
//   d2 = sum_j D2j k_j,  d3 = sum_j D3j k_j  (j = 1..5),
// the continuous extension sampled at the reference's log-spaced output
// times (old_system.py:359-376).  RODAS4P: D2 / D3 solve the four order-3
// conditions of the continuous weights plus d2 = d3 = 0 in the stiff limit
// (h lambda -> -inf on y' = lambda y), which leaves D3 = (32/7) e5 and
// D25 = -40/7 (tools/rodas_dense.py derives them; interior error O(h^4) on
// a nonstiff problem, 15-100x below the RODAS4 set's on Prothero-Robinson).
// RODAS4: the Hairer-Wanner set.  Checked in tools/rodas_mirror.py.
namespace rodas4_dense {
#if PCK_RODAS4P
constexpr double D21 = 26.549127843114945, D22 = 10.967258456569217, D23 = 35.997973167097996,
                 D24 = 8.496032352891316, D25 = -40.0 / 7.0;
constexpr bool D3_K5_ONLY = true;
constexpr double D31 = 0.0, D32 = 0.0, D33 = 0.0, D34 = 0.0, D35 = 32.0 / 7.0;
#else
constexpr double D21 = 10.12623508344586, D22 = -7.487995877610167, D23 = -34.80091861555747,
                 D24 = -7.992771707568823, D25 = 1.025137723295662;
constexpr bool D3_K5_ONLY = false;
constexpr double D31 = -0.6762803392801253, D32 = 6.087714651680015, D33 = 16.43084320892478,
                 D34 = 24.76722511418386, D35 = -6.594389125716872;
#endif
}  // namespace rodas4_dense

// Trajectory samples of one condition: state at the shared times t[0..n)
// into y[(k*NS + i)*ld + c]
struct TrajOut {
    const double* t;
    int n;
    double* y;
    int64_t ld;
    int64_t c;
};

template <bool TRAJ, class P, class K>
__device__ PCK_LANE_INLINE int integrate(const P& p, const Lane<P::NS>& L, const K& k, double (&y)[P::NS], double t0,
                         double t_end, double rtol, double atol, int max_steps, int& nsteps, bool crows,
                         const TrajOut& to) {
    using namespace rodas4;
    constexpr int NS = P::NS;
    PCK_LPH_DECL;
    int ko = 0;
    if constexpr (TRAJ) {
        for (; ko < to.n && to.t[ko] <= t0; ++ko) {
#pragma unroll
            for (int i = 0; i < NS; ++i) to.y[((int64_t)ko * NS + i) * to.ld + to.c] = y[i];
        }
    }
    nsteps = 0;
    const double span = t_end - t0;
    if (!(span > 0.0)) {
        if constexpr (TRAJ) {
            for (; ko < to.n; ++ko) {
#pragma unroll
                for (int i = 0; i < NS; ++i) to.y[((int64_t)ko * NS + i) * to.ld + to.c] = y[i];
            }
        }
        PCK_LRET(PCK_ST_OK);
    }
    double F0[NS];
    rhs(p, L, k, y, F0);
    double cons0[PCK_MAX_CONS];
    for (int l = 0; l < p.ncons(); ++l) {
        double s = 0.0;
#pragma unroll
        for (int i = 0; i < NS; ++i) s += p.C(l, i) * y[i];
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
        rhs(p, L, k, y1, F1);
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
    unsigned sw;
    int blowups = 0;
    int stall = 0;
    while (t < t_end) {
        if (__builtin_amdgcn_readfirstlane(nsteps) >= max_steps) PCK_LRET(PCK_ST_MAXSTEPS);
        ++nsteps;
        PCK_LPH_STEP();
        bool last = false;
        if (t + h >= t_end) { h = t_end - t; last = true; }
        double ih, ig;
        PCK_LPH(0, jac(p, L, k, y, W);                               // W = I/(h g) - J
               ih = PCK_LANE_FAST ? rcp1(h) : rcp(h); ig = ih * (1.0 / g);
               for (int i = 0; i < NS; ++i) {
                   for (int q = 0; q < NS; ++q) W[i][q] = -W[i][q];
                   W[i][i] += ig;
               });
        if (PCK_CONS_ROWS && crows) cons_rows(p, W);
        bool luok;
        PCK_LPH(1, luok = lu<NS>(W, piv, sw));
        if (!luok) {
            h *= 0.25;
            if (!(h > 2.220446049250313e-15 * fmax(fabs(t), 1e-300))) PCK_LRET(PCK_ST_STEPFAIL);
            continue;
        }
        double k1[NS], k2[NS], k3[NS], k4[NS], k5[NS], u[NS], fu[NS];
#pragma unroll
        for (int i = 0; i < NS; ++i) k1[i] = F0[i];
        if (PCK_CONS_ROWS && crows) cons_zero(p, k1);
        PCK_LPH(2, lu_solve<NS>(W, piv, sw, k1));
        PCK_LPH(4, for (int i = 0; i < NS; ++i) u[i] = y[i] + a21 * k1[i]);
        PCK_LPH(3, rhs(p, L, k, u, fu));
        PCK_LPH(4, for (int i = 0; i < NS; ++i) k2[i] = fu[i] + ih * (C21 * k1[i]));
        if (PCK_CONS_ROWS && crows) cons_zero(p, k2);
        PCK_LPH(2, lu_solve<NS>(W, piv, sw, k2));
        PCK_LPH(4, for (int i = 0; i < NS; ++i) u[i] = y[i] + a31 * k1[i] + a32 * k2[i]);
        PCK_LPH(3, rhs(p, L, k, u, fu));
        PCK_LPH(4, for (int i = 0; i < NS; ++i) k3[i] = fu[i] + ih * (C31 * k1[i] + C32 * k2[i]));
        if (PCK_CONS_ROWS && crows) cons_zero(p, k3);
        PCK_LPH(2, lu_solve<NS>(W, piv, sw, k3));
        PCK_LPH(4, for (int i = 0; i < NS; ++i) u[i] = y[i] + a41 * k1[i] + a42 * k2[i] + a43 * k3[i]);
        PCK_LPH(3, rhs(p, L, k, u, fu));
        PCK_LPH(4, for (int i = 0; i < NS; ++i) k4[i] = fu[i] + ih * (C41 * k1[i] + C42 * k2[i] + C43 * k3[i]));
        if (PCK_CONS_ROWS && crows) cons_zero(p, k4);
        PCK_LPH(2, lu_solve<NS>(W, piv, sw, k4));
        PCK_LPH(4, for (int i = 0; i < NS; ++i) u[i] = y[i] + a51 * k1[i] + a52 * k2[i] + a53 * k3[i] + a54 * k4[i]);
        PCK_LPH(3, rhs(p, L, k, u, fu));
        PCK_LPH(4, for (int i = 0; i < NS; ++i) k5[i] = fu[i] + ih * (C51 * k1[i] + C52 * k2[i] + C53 * k3[i] + C54 * k4[i]));
        if (PCK_CONS_ROWS && crows) cons_zero(p, k5);
        PCK_LPH(2, lu_solve<NS>(W, piv, sw, k5));
        double d2[TRAJ ? NS : 1], d3[TRAJ ? NS : 1];
        if constexpr (TRAJ) {
            using namespace rodas4_dense;
#pragma unroll
            for (int i = 0; i < NS; ++i) {
                d2[i] = D21 * k1[i] + D22 * k2[i] + D23 * k3[i] + D24 * k4[i] + D25 * k5[i];
                d3[i] = D3_K5_ONLY ? D35 * k5[i] : D31 * k1[i] + D32 * k2[i] + D33 * k3[i] + D34 * k4[i] + D35 * k5[i];
            }
        }
        PCK_LPH(4, for (int i = 0; i < NS; ++i) u[i] += k5[i]);
        PCK_LPH(3, rhs(p, L, k, u, fu));
        // k6 reuses k5's registers once k5 is folded into u
        PCK_LPH(4, for (int i = 0; i < NS; ++i)
                       k5[i] = fu[i] + ih * (C61 * k1[i] + C62 * k2[i] + C63 * k3[i] + C64 * k4[i] + C65 * k5[i]));
        if (PCK_CONS_ROWS && crows) cons_zero(p, k5);
        PCK_LPH(2, lu_solve<NS>(W, piv, sw, k5));
        PCK_LPH_MARK();
        double s = 0.0, umin = INFINITY, usum = 0.0;
#pragma unroll
        for (int i = 0; i < NS; ++i) {
            u[i] += k5[i];
            usum += u[i];
            umin = fmin(umin, u[i]);
            const double sc = atol + rtol * fmax(fabs(y[i]), fabs(u[i]));
            const double r = k5[i] * __builtin_amdgcn_rcp(sc);   // error weight: the v_rcp_f64 estimate suffices
            s += r * r;
        }
        // one finiteness test for the step: a non-finite stage value makes u
        // (which includes k6) non-finite, hence usum, and 0 * (inf or NaN) is NaN
        const bool finite = (0.0 * usum == 0.0);
        const double q = finite ? s * (1.0 / NS) : INFINITY;    // en^2
        // positivity (mass-action concentrations stay >= -atol): a step that
        // drives a component below -atol is rejected and retried at the
        // fraction of the step where that component reaches -atol
        const bool negv = PCK_POSITIVITY && umin < -atol;
        const double fac = PCK_LANE_FAST ? step_factor_fast(q) : step_factor(q);
        if (q <= 1.0 && !negv) {
            const double t_old = t;
            t = last ? t_end : t + h;
            double y_old[TRAJ ? NS : 1];
            if constexpr (TRAJ) {
#pragma unroll
                for (int i = 0; i < NS; ++i) y_old[i] = y[i];
            }
#pragma unroll
            for (int i = 0; i < NS; ++i) y[i] = u[i];
            // Rosenbrock stages keep linear invariants only up to the rounding of
            // the stiff LU; rescale each non-negative site balance back onto its
            // initial total (multiplicative, so tiny coverages keep their digits)
            for (int l = 0; l < p.ncons(); ++l) {
                double sm = 0.0;
                bool pos = true;
#pragma unroll
                for (int i = 0; i < NS; ++i) {
                    pos = pos && (p.C(l, i) >= 0.0);
                    sm += p.C(l, i) * y[i];
                }
                if (pos && sm > 0.0) {
                    const double fct = cons0[l] * (PCK_LANE_FAST ? rcp1(sm) : rcp(sm));
#pragma unroll
                    for (int i = 0; i < NS; ++i)
                        if (p.C(l, i) != 0.0) y[i] *= fct;
                }
            }
            if constexpr (TRAJ) {
                // samples inside (t_old, t]: the dense output of this step
                for (; ko < to.n && to.t[ko] <= t; ++ko) {
                    const double sv = fmin((to.t[ko] - t_old) / h, 1.0), s1 = 1.0 - sv;
#pragma unroll
                    for (int i = 0; i < NS; ++i)
                        to.y[((int64_t)ko * NS + i) * to.ld + to.c] =
                            y_old[i] * s1 + sv * (y[i] + s1 * (d2[i] + sv * d3[i]));
                }
            }
            PCK_LPH_UNTIL(5);
            PCK_LPH(3, rhs(p, L, k, y, F0));
            PCK_LPH_MARK();
            // a tolerance-level negative (>= -atol) that is still falling is set
            // to 0: left alone, a mass-action term of order >= 2 keeps driving it
            // down and the positivity rule then shrinks h to nothing; clipping
            // every negative instead perturbs the stiff modes at each step and
            // the error estimate rejects steps forever (tools/rodas_mirror.py
            // CLIPMODE, DESIGN.md "Positivity").  The common case costs one
            // min over the state and one wave vote.
            // the site-balance rescaling multiplies by a positive factor, so the
            // accepted state has a negative component exactly where u did
            if (PCK_POSITIVITY && __any(umin < 0.0)) {        // rare: one wave-uniform branch
                bool negf = false;
#pragma unroll
                for (int i = 0; i < NS; ++i)
                    if (y[i] < 0.0 && F0[i] < 0.0) { y[i] = 0.0; negf = true; }
                if (__any(negf)) rhs(p, L, k, y, F0);
            }
            h *= fmin(PCK_FACMAX, fmax(0.2, fac));
        } else {
            double pf = 1.0;
            if (__any(negv)) {              // rare: one wave-uniform branch
#pragma unroll
                for (int i = 0; i < NS; ++i)
                    if (u[i] < -atol) pf = fmin(pf, (y[i] + atol) / (y[i] - u[i]));
            }
            if (q <= 1.0) {
                h *= fmax(0.1, 0.9 * pf);
            } else {
                h *= finite ? fmax(0.2, fac) : 0.25;
                // repeated catastrophic rejections: see mk_group.h grp_integrate
                if (!(q < PCK_BLOWUP_Q) && h < 1e-4 * t && ++blowups > PCK_MAX_BLOWUPS) PCK_LRET(PCK_ST_STEPFAIL);
            }
        }
        // stagnation, sampled every PCK_STALL_EVERY steps (the active lanes of a
        // wave share the step counter: a scalar test)
        if ((__builtin_amdgcn_readfirstlane(nsteps) & (PCK_STALL_EVERY - 1)) == 0) {
            stall = (h < PCK_STALL_H * (t - t0)) ? stall + PCK_STALL_EVERY : 0;
            if (stall > PCK_STALL_STEPS) PCK_LRET(PCK_ST_STEPFAIL);
        }
        // scipy's BDF limit: a step below 10 ulp(t) is a failure
        if (!(h > 2.220446049250313e-15 * fmax(fabs(t), 1e-300)) && t < t_end) PCK_LRET(PCK_ST_STEPFAIL);
        PCK_LPH_UNTIL(5);
    }
    if constexpr (TRAJ) {
        // samples past t_end (a caller's log grid can round one ulp above it)
        // take the final state
        for (; ko < to.n; ++ko) {
#pragma unroll
            for (int i = 0; i < NS; ++i) to.y[((int64_t)ko * NS + i) * to.ld + to.c] = y[i];
        }
    }
    PCK_LRET(PCK_ST_OK);
}

// Is y a root, not an artefact of Newton's absolute floor?  Every species
// balance that is not a conservation pivot must hold to PCK_BALANCE_TOL of its
// gross flux (sum over reactions of |S_ij| (r_fwd + r_rev) times the row
// scale, plus the CSTR flow terms).  Newton's step test holds components below
// 1e-12 of the largest only to an absolute floor, so on an O-poisoned volcano
// node it can stop at coverages of 1e-41 that balance nothing (the trivial
// poisoned root approached, TOF ~1e-36 and undetermined).  Over the 2 560
// nodes of tests/golden/volcano_fixture.npz the oracle's accepted roots
// balance either to <= 1e-14 (2 216) or not at all (18, every non-pivot
// species off by 0.27 to 1 of its flux): the threshold sits in that gap,
// far from both.
#ifndef PCK_BALANCE_TOL
#define PCK_BALANCE_TOL 1e-3
#endif
template <class P, class K>
__device__ __forceinline__ void rhs_gross(const P& p, const Lane<P::NS>& L, const K& k, const double (&y)[P::NS],
                                          double (&f)[P::NS], double (&g)[P::NS]) {
    constexpr int NS = P::NS;
    double c[NS];
#pragma unroll
    for (int i = 0; i < NS; ++i) { c[i] = p.cf(i) * y[i]; f[i] = 0.0; g[i] = 0.0; }
    for_rxn(p, [&](int j) {
        double rf = k.f(j), rr = k.r(j);
#pragma unroll
        for (int i = 0; i < NS; ++i) {
            if (p.ef(j, i)) rf *= ipow(c[i], p.ef(j, i));
            if (p.er(j, i)) rr *= ipow(c[i], p.er(j, i));
        }
        const double net = net_rate(rf, rr), gross = fabs(rf) + fabs(rr);
#pragma unroll
        for (int i = 0; i < NS; ++i) {
            const double s = p.S(i, j);
            if (s != 0.0) { f[i] += s * net; g[i] += fabs(s) * gross; }
        }
    });
#pragma unroll
    for (int i = 0; i < NS; ++i) {
        const double rs = (p.rsT(i) != 0.0) ? p.rs0(i) + p.rsT(i) * L.T : p.rs0(i);
        f[i] *= rs;
        g[i] *= fabs(rs);
        if (p.fl(i) != 0.0) {
            f[i] += p.fl(i) * (L.ins[i * L.ks] - y[i]);
            g[i] += fabs(p.fl(i)) * (fabs(L.ins[i * L.ks]) + fabs(y[i]));
        }
    }
}

// f in double-double (mk_device.h: dd), rounded once at the end: the
// residual of the Newton refinement below.  The same terms as rhs; every
// product and sum error-free, so the result carries the rounding of the
// inputs (k_eff, the row scales, y) but not the cancellation of the fluxes.
template <class P, class K>
__device__ __forceinline__ void rhs_dd(const P& p, const Lane<P::NS>& L, const K& k, const double (&y)[P::NS],
                                       double (&f)[P::NS]) {
    constexpr int NS = P::NS;
    dd c[NS], acc[NS];
#pragma unroll
    for (int i = 0; i < NS; ++i) { c[i] = two_prod(p.cf(i), y[i]); acc[i] = dd_of(0.0); }
    for_rxn(p, [&](int j) {
        dd rf = dd_of(k.f(j)), rr = dd_of(k.r(j));
#pragma unroll
        for (int i = 0; i < NS; ++i) {
            if (p.ef(j, i)) rf = dd_mul(rf, dd_pow(c[i], p.ef(j, i)));
            if (p.er(j, i)) rr = dd_mul(rr, dd_pow(c[i], p.er(j, i)));
        }
        const dd net = dd_add(rf, dd_neg(rr));
#pragma unroll
        for (int i = 0; i < NS; ++i) {
            const double s = p.S(i, j);
            if (s != 0.0) acc[i] = dd_add(acc[i], dd_mul(net, s));
        }
        // one reaction at a time (the ILP scheduler would interleave them all
        // and raise the kernel's register count, i.e. lower its occupancy)
        __builtin_amdgcn_sched_barrier(0);
    });
#pragma unroll
    for (int i = 0; i < NS; ++i) {
        dd r = dd_mul(acc[i], (p.rsT(i) != 0.0) ? p.rs0(i) + p.rsT(i) * L.T : p.rs0(i));
        if (p.fl(i) != 0.0) r = dd_add(r, dd_mul(two_sum(L.ins[i * L.ks], -y[i]), p.fl(i)));
        f[i] = r.hi + r.lo;
    }
}

// every species balance except the conservation pivots within tol of its gross flux
template <class P>
__device__ __forceinline__ bool balanced(const P& p, const double (&f)[P::NS], const double (&g)[P::NS], double tol) {
    bool ok = true;
#pragma unroll
    for (int i = 0; i < P::NS; ++i) {
        bool pv = false;
        for (int l = 0; l < p.ncons(); ++l) pv = pv || (p.cpiv(l) == i);
        ok = ok && (pv || fabs(f[i]) <= tol * g[i]);
    }
    return ok;
}

// the largest |f_i| / gross_i over the species that are not conservation pivots
template <class P>
__device__ __forceinline__ double imbalance(const P& p, const double (&f)[P::NS], const double (&g)[P::NS]) {
    double m = 0.0;
#pragma unroll
    for (int i = 0; i < P::NS; ++i) {
        bool pv = false;
        for (int l = 0; l < p.ncons(); ++l) pv = pv || (p.cpiv(l) == i);
        if (!pv && f[i] != 0.0) m = fmax(m, fabs(f[i]) / g[i]);
    }
    return m;
}

template <class P, class K>
__device__ __forceinline__ bool resolved(const P& p, const Lane<P::NS>& L, const K& k, const double (&y)[P::NS]) {
    double f[P::NS], g[P::NS];
    rhs_gross(p, L, k, y, f, g);
    return balanced(p, f, g, PCK_BALANCE_TOL);
}

// Newton's stop at the rounding floor: once a Newton iterate balances every
// species to PCK_BALANCE_CONV of its gross flux, a next step that makes the
// balance worse is rounding noise amplified by the Jacobian's condition (up
// to 1e12 at a site-starved volcano root), not progress: the iteration keeps
// the better point and stops.  (1e-10 stopped some roots early enough to
// leave tiny TOFs with 3e-7 relative rounding; resolved roots balance to
// <= 1e-14.)  On fixture node 80 the device took such a
// step from the root, landed 10 % away on the 2.8e-10 free-site coverage and
// came back in a 12-iteration cycle until the iteration cap
// (tools/trace_newton.py), while LAPACK's solve in the oracle happened to
// land on the root.
#ifndef PCK_BALANCE_CONV
#define PCK_BALANCE_CONV 1e-12
#endif
// ... and the same stop in step terms: after a Newton step below
// PCK_STEP_FLOOR relative (quadratic convergence would make the next one
// ~1e-14), a LARGER step is residual rounding amplified by the Jacobian, not
// progress: the iteration returns the iterate before it as converged.  On
// volcano fixture node 2502 (an O-covered root, sO 0.99996, the O2 coverage
// 3.6e-5 set through the site balance) the step from the transient end was
// 2.5e-10 and the next 2.3e-4; the iteration then wandered at that noise
// level until the linear-convergence exit (tools/trace_newton.py), while the
// oracle's LAPACK solve happened to land inside 1e-12.
#ifndef PCK_STEP_FLOOR
#define PCK_STEP_FLOOR 1e-7
#endif
// Refinement of a converged root (mixed-precision iterative refinement):
// Newton steps from the root with the residual in double-double (rhs_dd),
// at most PCK_NEWTON_REFINE of them, stopped when the scaled residual stops
// falling.  The plain iteration stops where the residual's rounding (eps x
// the gross fluxes, amplified by a Jacobian condition up to 1e12) drowns the
// step -- on a site-starved root that leaves ~1e-7 of the answer to the
// rounding of one build, and two builds of one plan differed by 1.3e-6 in
// TOF.  With the residual exact to ~eps^2 the steps converge to the root of
// the rounded inputs in every well-determined direction, whatever order the
// build evaluates the fluxes in.  0 turns it off (A/B).
#ifndef PCK_NEWTON_REFINE
#define PCK_NEWTON_REFINE 2
#endif
#ifndef PCK_REFINE_MAXSTEP
#define PCK_REFINE_MAXSTEP 1e-6
#endif

// Newton on f(y) = 0 with the plan's conservation laws replacing their pivot
// rows (old_system.py:385-468 polishes with scipy least_squares; a regular
// root it converges to is the same).  Rows are equilibrated; a multiplicity
// estimate accelerates near-double roots; a root that stays linearly
// convergent (a site-starved surface approached algebraically) or lands on a
// negative component is not regular -> PCK_ST_NEWTON, transient state kept.
//
// dist > 0 (pck_solve_params.root_dist): the root is the answer only if the
// transient end y it started from has reached it -- every component within
// dist * |root| + atol -- i.e. the transient at t_end is at that steady
// state.  Otherwise PCK_ST_NEWTON with y unchanged: the transient end is the
// answer (old_system.py:517-529, what the volcano driver reports).  The test
// is a distance between two well-defined states, so where a device and a CPU
// implementation disagree on it the two answers they report are themselves
// within ~dist of each other (DESIGN.md "Steady state").
template <class P, class K>
__device__ PCK_LANE_INLINE int newton(const P& p, const Lane<P::NS>& L, const K& k, double (&y)[P::NS], int iters,
                                      double dist, double atol) {
    constexpr int NS = P::NS;
    double b[PCK_MAX_CONS];
    for (int l = 0; l < p.ncons(); ++l) {
        double s = 0.0;
#pragma unroll
        for (int i = 0; i < NS; ++i) s += p.C(l, i) * y[i];
        b[l] = s;
    }
    double z[NS], z_prev[NS];
#pragma unroll
    for (int i = 0; i < NS; ++i) z[i] = y[i];
    double bal_prev = INFINITY;
    bool conv = false;
    double prev = INFINITY, lastq = 1.0;
    int linear = 0;
    // newton_pinned: a species at exactly 0 whose rate is exactly 0 at the
    // transient end is held at 0 (its Newton steps are dropped here; the
    // group kernels give it a unit row and a zero residual).  Such a species
    // has no reaction that can produce it from the start state (every
    // producer involves another such species or a zero inflow / pressure):
    // the transient keeps it at 0 exactly, and the steady state on that
    // invariant subspace has it at 0.  Left free, its Jacobian row (tiny after
    // equilibration) loses the threshold pivot to a dense row, the LU's
    // rounding lands on it, and the balance test then fails on a 1e-33
    // residue (Butadiene with_jonas_byproducts: C4H9O2_2*, C4H8O2_3*, whose
    // only source is ethyl acetate at zero pressure; oracle: _set_reach).
    unsigned pinm = 0u;
    for (int it = 0; it < iters; ++it) {
        double G[NS], J[NS][NS];
        int piv[NS];
        {
            double Gg[NS];
            rhs_gross(p, L, k, z, G, Gg);
            if (it == 0) {
#pragma unroll
                for (int i = 0; i < NS; ++i) {
                    bool cp = false;
                    for (int l = 0; l < p.ncons(); ++l) cp = cp || (p.cpiv(l) == i);
                    if (!cp && z[i] == 0.0 && G[i] == 0.0) pinm |= 1u << i;
                }
            }
            const double bal = imbalance(p, G, Gg);
            if (it >= 2 && bal_prev <= PCK_BALANCE_CONV && bal > bal_prev) {   // the rounding floor
#pragma unroll
                for (int i = 0; i < NS; ++i) z[i] = z_prev[i];
                conv = true;
                break;
            }
            bal_prev = bal;
#pragma unroll
            for (int i = 0; i < NS; ++i) z_prev[i] = z[i];
        }
        jac(p, L, k, z, J);
        for (int l = 0; l < p.ncons(); ++l) {
            const int pv = p.cpiv(l);
            double s = 0.0;
#pragma unroll
            for (int i = 0; i < NS; ++i) s += p.C(l, i) * z[i];
#pragma unroll
            for (int i = 0; i < NS; ++i) {
                if (i == pv) {
                    G[i] = s - b[l];
#pragma unroll
                    for (int q = 0; q < NS; ++q) J[i][q] = p.C(l, q);
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
            for (int q = 0; q < NS; ++q) m = fmax(m, fabs(J[i][q]));
            const double sc = (m > 0.0) ? 1.0 / m : 1.0;
#pragma unroll
            for (int q = 0; q < NS; ++q) J[i][q] *= sc;
            G[i] = -G[i] * sc;
        }
        unsigned sw;
        if (!lu<NS, true>(J, piv, sw)) break;
        lu_solve<NS>(J, piv, sw, G);
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
            G[i] = (pinm & (1u << i)) ? 0.0 : G[i] * alpha;
            z[i] += G[i];
            finite = finite && isfinite(z[i]);
            zmax = fmax(zmax, fabs(z[i]));
        }
        if (!finite) break;
        // components below 1e-12 of the largest are held to an absolute
        // 1e-24 * zmax: their relative digits sit under the residual's rounding
#pragma unroll
        for (int i = 0; i < NS; ++i) rel = fmax(rel, fabs(G[i]) / fmax(fabs(z[i]), 1e-12 * zmax + 1e-300));
#ifdef PCK_TRACE
        if (L.cidx == pck_trace_cond) {           // [it, rel, alpha, z0..z4]
            double* rec = pck_trace_buf + (size_t)(pck_trace_pos % PCK_TRACE_N) * PCK_TRACE_W;
            rec[0] = it; rec[1] = rel; rec[2] = alpha;
#pragma unroll
            for (int i = 0; i < NS && i < PCK_TRACE_W - 3; ++i) rec[3 + i] = z[i];
            pck_trace_pos = pck_trace_pos + 1;
        }
#endif
        if (prev < PCK_STEP_FLOOR && rel > prev) {      // the step floor: undo the noise step
#pragma unroll
            for (int i = 0; i < NS; ++i) z[i] = z_prev[i];
            conv = true;
            break;
        }
        if (rel < 1e-12 || (it >= 2 && rel < 1e-7 && rel > 0.5 * prev)) { conv = true; break; }
        lastq = rel / prev;
        linear = (rel > 0.25 * prev) ? linear + 1 : 0;
        if (linear >= 12) break;
        prev = rel;
    }
#ifdef PCK_TRACE
    if (L.cidx == pck_trace_cond) {               // exit record: [-1, conv, min z, resolved]
        double* rec = pck_trace_buf + (size_t)(pck_trace_pos % PCK_TRACE_N) * PCK_TRACE_W;
        double zmin = z[0];
#pragma unroll
        for (int i = 1; i < NS; ++i) zmin = fmin(zmin, z[i]);
        rec[0] = -1.0; rec[1] = conv ? 1.0 : 0.0; rec[2] = zmin; rec[3] = resolved(p, L, k, z) ? 1.0 : 0.0;
        pck_trace_pos = pck_trace_pos + 1;
    }
#endif
    if (!conv) return PCK_ST_NEWTON;
    if (PCK_NEWTON_REFINE > 0) {
        // residual-refinement steps (PCK_NEWTON_REFINE): the Newton system of
        // the loop above at the current iterate, its right-hand side in
        // double-double.  Scheduling barriers keep the Jacobian / LU, the
        // double-double residual and the solve in sequence (interleaved by
        // the ILP scheduler they took the volcano kernel from 159 to 195
        // VGPRs, two waves per SIMD instead of three).
        double nprev = INFINITY;
#pragma unroll 1
        for (int r = 0; r <= PCK_NEWTON_REFINE; ++r) {
            double J[NS][NS], sc[NS], G[NS];
            int piv[NS];
            unsigned sw;
            jac(p, L, k, z, J);
            for (int l = 0; l < p.ncons(); ++l) {
                const int pv = p.cpiv(l);
#pragma unroll
                for (int i = 0; i < NS; ++i) {
                    if (i == pv) {
#pragma unroll
                        for (int q = 0; q < NS; ++q) J[i][q] = p.C(l, q);
                    }
                }
            }
#pragma unroll
            for (int i = 0; i < NS; ++i) {
                double m = 0.0;
#pragma unroll
                for (int q = 0; q < NS; ++q) m = fmax(m, fabs(J[i][q]));
                sc[i] = (m > 0.0) ? 1.0 / m : 1.0;
#pragma unroll
                for (int q = 0; q < NS; ++q) J[i][q] *= sc[i];
            }
            const bool luok = lu<NS, true>(J, piv, sw);
            __builtin_amdgcn_sched_barrier(0);
            rhs_dd(p, L, k, z, G);
            for (int l = 0; l < p.ncons(); ++l) {
                const int pv = p.cpiv(l);
                dd s = dd_of(-b[l]);
#pragma unroll
                for (int i = 0; i < NS; ++i) s = dd_add(s, two_prod(p.C(l, i), z[i]));
#pragma unroll
                for (int i = 0; i < NS; ++i)
                    if (i == pv) G[i] = s.hi + s.lo;
            }
            double nr = 0.0;
#pragma unroll
            for (int i = 0; i < NS; ++i) {
                G[i] = -G[i] * sc[i];
                nr = fmax(nr, fabs(G[i]));
            }
            __builtin_amdgcn_sched_barrier(0);
#ifdef PCK_TRACE
            if (L.cidx == pck_trace_cond) {           // refinement record: [100 + r, nr, luok, z0..z4]
                double* rec = pck_trace_buf + (size_t)(pck_trace_pos % PCK_TRACE_N) * PCK_TRACE_W;
                rec[0] = 100 + r; rec[1] = nr; rec[2] = luok ? 1.0 : 0.0;
#pragma unroll
                for (int i = 0; i < NS && i < PCK_TRACE_W - 3; ++i) rec[3 + i] = z[i];
                pck_trace_pos = pck_trace_pos + 1;
                double* rg = pck_trace_buf + (size_t)(pck_trace_pos % PCK_TRACE_N) * PCK_TRACE_W;
                rg[0] = 200 + r; rg[1] = sw; rg[2] = 0.0;         // [200 + r, swaps, 0, G0..G4 (scaled)]
#pragma unroll
                for (int i = 0; i < NS && i < PCK_TRACE_W - 3; ++i) rg[3 + i] = G[i];
                pck_trace_pos = pck_trace_pos + 1;
            }
#endif
            if (!(nr < nprev)) {                         // no longer falling: the previous iterate
                if (r > 0) {
#pragma unroll
                    for (int i = 0; i < NS; ++i) z[i] = z_prev[i];
                }
                break;
            }
            nprev = nr;
            if (r == PCK_NEWTON_REFINE || nr == 0.0 || !luok) break;
            lu_solve<NS>(J, piv, sw, G);
            bool fin = true;
            double zmax = 0.0, rel = 0.0;
#pragma unroll
            for (int i = 0; i < NS; ++i) zmax = fmax(zmax, fabs(z[i]));
#pragma unroll
            for (int i = 0; i < NS; ++i) {
                z_prev[i] = z[i];
                const double d = (pinm & (1u << i)) ? 0.0 : G[i];
                rel = fmax(rel, fabs(d) / fmax(fabs(z[i]), 1e-12 * zmax + 1e-300));
                z[i] += d;
                fin = fin && isfinite(z[i]);
            }
            // a refinement moves a converged root by rounding, not by 1e-6:
            // a larger step is the ill-conditioned direction speaking
            if (!fin || !(rel <= PCK_REFINE_MAXSTEP)) {
#pragma unroll
                for (int i = 0; i < NS; ++i) z[i] = z_prev[i];
                break;
            }
        }
    }
#pragma unroll
    for (int i = 0; i < NS; ++i)
        if (z[i] < 0.0) return PCK_ST_NEWTON;
    if (!resolved(p, L, k, z)) return PCK_ST_NEWTON;   // converged in absolute terms only
    if (dist > 0.0) {
        bool near = true;
#pragma unroll
        for (int i = 0; i < NS; ++i) near = near && (fabs(z[i] - y[i]) <= dist * fabs(z[i]) + atol);
        if (!near) return PCK_ST_NEWTON;                 // the transient has not reached this root
    }
#pragma unroll
    for (int i = 0; i < NS; ++i) y[i] = z[i];
    return PCK_ST_OK;
}

template <class P, class K>
__device__ __forceinline__ double lane_tof(const P& p, const NetView& nv, const K& k, const double (&y)[P::NS]) {
    // old_system.py:482-488: sum of (r_fwd - r_rev) over tof_terms
    constexpr int NS = P::NS;
    double c[NS];
#pragma unroll
    for (int i = 0; i < NS; ++i) c[i] = p.cf(i) * y[i];
    double tof = 0.0;
    for (int t = 0; t < nv.NTOF; ++t) {
        const int jt = nv.tof[t];
        for_rxn(p, [&](int j) {
            if (j != jt) return;
            double rf = k.f(j), rr = k.r(j);
#pragma unroll
            for (int i = 0; i < NS; ++i) {
                if (p.ef(j, i)) rf *= ipow(c[i], p.ef(j, i));
                if (p.er(j, i)) rr *= ipow(c[i], p.er(j, i));
            }
            tof += rf - rr;
        });
    }
    return tof;
}

// ---------------------------------------------------------------------------
// evaluation kernels (runtime plans): pck_species_rates / pck_jacobian
// ---------------------------------------------------------------------------
template <int NS, bool DD = false>
__global__ void __launch_bounds__(128) k_species_rates(NetView nv, CondView cv, const double* kf, const double* kr,
                                                       int64_t ld_k, const double* y, int64_t ld_y, double* dydt) {
    extern __shared__ double lds[];
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= cv.n) return;
    PlanRT<NS> p(nv);
    KLds k{lds + threadIdx.x, lds + (size_t)nv.NRXN * blockDim.x + threadIdx.x, (int)blockDim.x};
    Lane<NS> L;
    lane_setup(p, nv, cv, c, L, lds + threadIdx.x, blockDim.x);
    load_keff(p, nv, cv, c, kf, kr, ld_k, k, -1, 1.0);
    double yy[NS], f[NS];
#pragma unroll
    for (int i = 0; i < NS; ++i) yy[i] = y[i * ld_y + c];
    if constexpr (DD)
        rhs_dd(p, L, k, yy, f);           // the Newton refinement's residual (diagnostics: PCK_RATES_DD=1)
    else
        rhs(p, L, k, yy, f);
#pragma unroll
    for (int i = 0; i < NS; ++i) dydt[i * ld_y + c] = f[i];
}

template <int NS>
__global__ void __launch_bounds__(128) k_jacobian(NetView nv, CondView cv, const double* kf, const double* kr,
                                                  int64_t ld_k, const double* y, int64_t ld_y, double* jo) {
    extern __shared__ double lds[];
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= cv.n) return;
    PlanRT<NS> p(nv);
    KLds k{lds + threadIdx.x, lds + (size_t)nv.NRXN * blockDim.x + threadIdx.x, (int)blockDim.x};
    Lane<NS> L;
    lane_setup(p, nv, cv, c, L, lds + threadIdx.x, blockDim.x);
    load_keff(p, nv, cv, c, kf, kr, ld_k, k, -1, 1.0);
    double yy[NS], J[NS][NS];
#pragma unroll
    for (int i = 0; i < NS; ++i) yy[i] = y[i * ld_y + c];
    jac(p, L, k, yy, J);
#pragma unroll
    for (int i = 0; i < NS; ++i)
#pragma unroll
        for (int q = 0; q < NS; ++q) jo[(i * NS + q) * ld_y + c] = J[i][q];
}

// ---------------------------------------------------------------------------
// kernel (3)+(4): solve (+ TOF / activity, + DRC combine by wavefront shuffles)
// ---------------------------------------------------------------------------
struct SolveArgs {
    double t0, t_end, rtol, atol, eps;
    int max_steps, newton, newton_iters, want_activity;
    double* y; int64_t ld_y;
    double* tof; int32_t* status; int32_t* nsteps;
    double* xi; int64_t ld_xi; double* tof0;   // DRC mode
    int G;                                     // lanes per condition (1, or DRC group size)
    int cons_rows;                             // conservation rows in the stage systems (A/B: PCK_CONS_ROWS=1)
    double root_dist;                          // pck_solve_params.root_dist (newton: root only if the transient reached it)
    const double* t_out; int n_out;            // trajectory sample times (k_solve<P, true>)
    double* traj; int64_t ld_traj;             // [n_out][NS][ld_traj]
    // degenerate-root retry (pck_solve_params.retry_rtol), a second launch
    // over the compacted list of the conditions whose polish ended in
    // PCK_ST_NEWTON (mk_kernels.hip: launch_solve): lane i solves condition
    // idx[i] for i < *nidx, adds its steps to nsteps[c] and reports a
    // completed transient as PCK_ST_NEWTON.  idx == nullptr: lane i solves
    // condition i / G.  (Round 3 first ran the retry inside the first launch;
    // the pass loop kept ~70 more VGPRs live in every solver kernel -- the
    // volcano kernel went from 158 to 227, i.e. from 3 to 2 waves per SIMD.)
    const int64_t* idx; const int32_t* nidx;
    // 1: the degenerate-root retry above; 2: the screening pass's second
    // launch (pck_solve_params.screen_rtol): the listed conditions solved
    // exactly as a single pass would, nsteps adding the screening pass's
    int retry_pass;
    // cost-ordered dispatch (pck_solve_params.wave_order): block b of the lane
    // solver (one wavefront) solves the 64 conditions of wavefront worder[b]
    const int32_t* worder;
    // screening pass inside the solve (pck_solve_params.screen_rtol, one
    // launch): every lane first runs the rule at screen_rtol / screen_atol
    // with root distance screen_dist; a lane whose screening answer is not
    // an accepted root solves again from y0 at rtol / atol / root_dist, in
    // the same launch (screen_rtol 0: a single pass)
    double screen_rtol, screen_atol, screen_dist;
    // the screening trip's step cap (PCK_SCREEN_MAX_STEPS, default 2000, at
    // most max_steps): a trip past it is not accepted and the full solve runs
    // (an optimisation never costs more than this many steps per lane)
    int screen_max_steps;
    // screening with a screening-rule preview: a wavefront one of whose
    // preview samples was not accepted (k_wave_keys: wrej) runs the single
    // pass directly (its screening trip would lengthen the wave's critical
    // path for nothing); wrej == nullptr: never
    const int32_t* wrej;
};

// One condition's solve: transient from y0, then (with a.newton) the Newton
// polish.  Returns the status; ns = integrator steps.
template <bool TRAJ, class P, class K>
__device__ __forceinline__ int solve_lane(const P& p, const Lane<P::NS>& L, const K& k, const CondView& cv,
                                          int64_t c, const SolveArgs& a, double (&y)[P::NS], int& ns,
                                          const TrajOut& to, bool screen_on = true) {
    constexpr int NS = P::NS;
    // the screening trip and the full solve are two inlined copies of the
    // integrator (one copy in a two-trip loop kept the Newton polish's values
    // live through the integrator: 223 VGPRs against 165)
    int st, total = 0, nsp = 0;
    if (!TRAJ && a.screen_rtol > 0.0 && screen_on) {
#pragma unroll
        for (int i = 0; i < NS; ++i) y[i] = cv.y0[i * cv.ld_y0 + c * cv.s_y0];
        st = integrate<TRAJ>(p, L, k, y, a.t0, a.t_end, a.screen_rtol, a.screen_atol, a.screen_max_steps, nsp,
                             a.cons_rows != 0, to);
        // the acceptance test's absolute term is the caller's atol, not the
        // trip's scaled one (3e4 x larger): a trace species must be as close
        // to its root as the single pass requires
        if (st == PCK_ST_OK && a.newton) st = newton(p, L, k, y, a.newton_iters, a.screen_dist, a.atol);
        total = nsp;
        if (st == PCK_ST_OK) {
            ns = total;
            return st;
        }
    }
#pragma unroll
    for (int i = 0; i < NS; ++i) y[i] = cv.y0[i * cv.ld_y0 + c * cv.s_y0];
    st = integrate<TRAJ>(p, L, k, y, a.t0, a.t_end, a.rtol, a.atol, a.max_steps, nsp, a.cons_rows != 0, to);
    if (st == PCK_ST_OK && a.newton) st = newton(p, L, k, y, a.newton_iters, a.root_dist, a.atol);
    total += nsp;
    ns = total;
    return st;
}

// a DRC condition's status from the worst and the best of its 2R+1 solves:
// reached roots mixed with transient ends (the steady rule's two answers) are
// PCK_ST_DRC_MIXED; any integrator failure (1-3) stays the worst status
__host__ __device__ inline int drc_status(int worst, int best) {
    return ((worst == PCK_ST_NEWTON || worst == PCK_ST_NEWTON_LOOSE) && best == PCK_ST_OK) ? PCK_ST_DRC_MIXED
                                                                                          : worst;
}

// condition of a lane (or lane group) v: v / G, or the retry list's entry
// (cv.n past the list's end: the lane idles)
__device__ __forceinline__ int64_t cond_of(const SolveArgs& a, int64_t v, int G, int64_t n) {
    if (!a.idx) return v / G;
    const int64_t m = *a.nidx;
    return (v < m) ? a.idx[v] : n;
}

template <class P>
struct KFor {
    using type = KLds;
};
template <class Net>
struct KFor<PlanCT<Net>> {
    using type = KReg<Net::R>;
};

// threads per block of the lane solver: one wave per block schedules the
// uneven per-wave step counts at the finest grain (measured 3.7 % over 128)
#ifndef PCK_SOLVE_BLOCK
#define PCK_SOLVE_BLOCK 64
#endif

// occupancy floor of the solver (waves per SIMD); the VGPR budget follows
#ifndef PCK_SOLVE_WAVES
#define PCK_SOLVE_WAVES 1
#endif

template <class P, bool TRAJ = false>
__global__ void __launch_bounds__(PCK_SOLVE_BLOCK) __attribute__((amdgpu_waves_per_eu(PCK_SOLVE_WAVES))) k_solve(NetView nv, CondView cv, const double* kf, const double* kr,
                                               int64_t ld_k, SolveArgs a) {
    constexpr int NS = P::NS;
    extern __shared__ double lds[];
#if PCK_POISON_LDS
    {   // diagnostic builds (-DPCK_POISON_LDS=1): the dynamic LDS block starts as
        // NaN, so a read of an element no lane wrote this launch shows at once
        const int nd = (2 * (nv.NRXN > 0 ? nv.NRXN : 1) + NS) * (int)blockDim.x;
        for (int i = threadIdx.x; i < nd; i += blockDim.x) lds[i] = __builtin_nan("");
        __syncthreads();
    }
#endif
#if PCK_WAVE_TIMES
    const long long wt0 = __builtin_amdgcn_s_memrealtime();
#endif
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int G = a.G;
    const int64_t c = a.worder ? ((int64_t)a.worder[blockIdx.x] * PCK_SOLVE_BLOCK + threadIdx.x)
                               : cond_of(a, gid, G, cv.n);
    const int q = (int)(gid % G);
    const int R = nv.NRXN;
    P p(nv);
    // DRC lanes: q = 0 base, q = 2j+1 -> k_j*(1+eps), q = 2j+2 -> k_j*(1-eps)
    const bool drc = (G > 1);
    const bool active = (c < cv.n) && (!drc || q <= 2 * R);
    typename KFor<P>::type k;
    if constexpr (!P::CT) {
        k.kf = lds + threadIdx.x;
        k.kr = lds + (size_t)R * blockDim.x + threadIdx.x;
        k.ks = blockDim.x;
    }
    double tof = 0.0;
    int st = PCK_ST_OK;
    int ns = 0;
    double T = 0.0;
    if (active) {
        int pj = -1;
        double pfac = 1.0;
        if (drc && q > 0) { pj = (q - 1) >> 1; pfac = (q & 1) ? 1.0 + a.eps : 1.0 - a.eps; }
        Lane<NS> L;
        lane_setup(p, nv, cv, c, L, lds + threadIdx.x, blockDim.x);
        T = L.T;
        load_keff(p, nv, cv, c, kf, kr, ld_k, k, pj, pfac);
        double y[NS];
        TrajOut to{a.t_out, a.n_out, a.traj, a.ld_traj, c};
        const bool screen_on = !(a.wrej && a.worder && a.wrej[a.worder[blockIdx.x]]);
        st = solve_lane<TRAJ>(p, L, k, cv, c, a, y, ns, to, screen_on);
        tof = lane_tof(p, nv, k, y);
        bool fin = isfinite(tof);
#pragma unroll
        for (int i = 0; i < NS; ++i) fin = fin && isfinite(y[i]);
        if (!fin && st == PCK_ST_OK) st = PCK_ST_NONFINITE;
        if (!drc) {
            // retry pass: a completed transient is the degenerate root's answer;
            // a failed one keeps the first pass's outputs (PCK_ST_NEWTON_LOOSE)
            const bool keep = a.retry_pass == 1 && st != PCK_ST_OK;
            if (a.retry_pass == 1) st = keep ? PCK_ST_NEWTON_LOOSE : PCK_ST_NEWTON;
            if (a.y && !keep) {
#pragma unroll
                for (int i = 0; i < NS; ++i) a.y[i * a.ld_y + c] = y[i];
            }
            if (a.tof && !keep) {
                // old_system.py:526-527
                a.tof[c] = a.want_activity ? (log((hP * tof) / (kB * T)) * (Rgas * T)) * 1.0e-3 / eVtokJ : tof;
            }
            if (a.status) a.status[c] = st;
            if (a.nsteps) a.nsteps[c] = a.retry_pass ? a.nsteps[c] + ns : ns;
        }
    }
    if (drc) {
        // wavefront-shuffle combine: every lane of a condition's group lives in
        // the same wavefront (G divides 64); the group's status is the worst
        // member's and its step count the sum (butterfly over the G lanes, so
        // every lane holds the same values -- no atomics, no pre-zeroed output)
        const int lane = threadIdx.x & 63;
        const int base = lane - q;
        const double t0 = __shfl(tof, base, 64);
        const double tm = __shfl(tof, lane + 1 < 64 ? lane + 1 : lane, 64);
        int gst = active ? st : 0;
        int gmin = active ? st : 1 << 20;
        int gns = active ? ns : 0;
        for (int m = 1; m < G; m <<= 1) {
            gst = max(gst, __shfl_xor(gst, m, 64));
            gmin = min(gmin, __shfl_xor(gmin, m, 64));
            gns += __shfl_xor(gns, m, 64);
        }
        gst = drc_status(gst, gmin);
        if (active && (q & 1)) {
            const int j = (q - 1) >> 1;
            a.xi[j * a.ld_xi + c] = (tof - tm) / (2.0 * a.eps * t0);   // old_system.py:508
        }
        if (active && q == 0) {
            // a zero or non-finite base TOF makes every xi meaningless
            if (gst == PCK_ST_OK && !(isfinite(t0) && t0 != 0.0)) gst = PCK_ST_NONFINITE;
            if (a.tof0) a.tof0[c] = tof;
            if (a.status) a.status[c] = gst;
            if (a.nsteps) a.nsteps[c] = gns;
        }
    }
#if PCK_WAVE_TIMES
    {
        int wmax = active ? ns : 0;                  // the wave's largest step count
        for (int m = 1; m < 64; m <<= 1) wmax = max(wmax, __shfl_xor(wmax, m, 64));
        if (!a.idx && (threadIdx.x & 63) == 0 && blockIdx.x < PCK_WT_N) {
            const long long wt1 = __builtin_amdgcn_s_memrealtime();
            pck_wtimes[3 * blockIdx.x] = wt0;
            pck_wtimes[3 * blockIdx.x + 1] = wt1;
            // HW_ID (high word) and the step count
            pck_wtimes[3 * blockIdx.x + 2] =
                ((long long)(unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4) << 32) | (unsigned)wmax;
        }
    }
#endif
}

}  // namespace pck
