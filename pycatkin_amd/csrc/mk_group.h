// Lane-group solver: one condition per group of G = 16 / 32 / 64 lanes of a
// wavefront.  Used for networks with more than PCK_MAX_DYN_LANE dynamic
// species (DMTM: 11, test/CH4_input.json: 16, the 50-species synthetic
// network) and for networks whose reaction count does not fit the
// one-lane-per-condition LDS budget.
//
//   * lane i of a group owns species i: y_i, every Rosenbrock stage entry and
//     row i of the iteration matrix (NSP doubles in VGPRs, static indices);
//     NSP = NS exactly when the kernel is specialised for the network's size
//     at run time (csrc/mk_jit.h), else the next compiled-in size;
//   * rates: lane-per-reaction (reactions gl, gl+G, ...: balanced whatever the
//     species degrees) into the group's net-rate buffer in LDS, then every
//     row lane gathers its own row of S . net from the species CSR of the
//     stoichiometric matrix (pycatkin/classes/old_system.py:202-248,
//     system.py:345-416);
//   * Jacobian: lane-per-reaction derivatives d net_r / d y_q into LDS, then
//     every row lane accumulates its own row of S . D into a column block of
//     the group's Jacobian buffer, in P column passes (old_system.py:250-313,
//     system.py:437-508).  A buffer row is only ever touched by its owner
//     lane, whose LDS adds execute in program order: the sums are bitwise
//     reproducible (no cross-lane atomics);
//   * dense LU with partial pivoting across the group: the pivot is an integer
//     max-reduction of |a| (float bits, lane id in the low 6 bits), the pivot
//     row is broadcast through LDS, every free row eliminates its own entries
//     (unrolled: column k is the static register W[k]);
//   * triangular solves: one broadcast per column (v_readlane on a full
//     wavefront, __shfl on 16/32-lane groups);
//   * norms / step-size decisions are butterfly all-reductions, bitwise equal
//     on every lane, so control flow is group-uniform.
//
// LDS per group (doubles, each block even-sized): kf[R] kr[R] | c[NSP] |
// d[max(ND, R)] (net rates / derivatives) | J[NS][QB] | pb[NSP]
#pragma once
#include "mk_device.h"
#include "mk_solver.h"

namespace pck {

#ifdef PCK_TRACE
// shader-clock cycles of the traced condition's integrator phases:
// [jac, lu, solve, rhs, other, steps]
__device__ double pck_phase[8];
#define PCK_PH(i, expr)                                              \
    do {                                                             \
        const long long t_ph0 = __builtin_readcyclecounter();        \
        expr;                                                        \
        if (tr) pck_phase[i] += (double)(__builtin_readcyclecounter() - t_ph0); \
    } while (0)
#else
#define PCK_PH(i, expr) expr
#endif

#define PCK_GRP_MAX_PART 6   // dynamic participants (species with an exponent) per reaction
#define PCK_GRP_MAX_EXP 31

// Device tables of the lane-group plan (built by pck_network_create).
//   rx[R]: {w0, w1, w2, dptr | np << 16}; participant k < np is the 16-bit
//          field k of w0:w1:w2 = species | ef << 6 | er << 11, and its
//          derivative lives at d[dptr + k]
//   row[NS+1], ent[nnz(S)]: CSR of the stoichiometric matrix by species;
//          entry {a = r | np << 9 | dptr << 12 | q5 << 26,
//                 b = q0 | q1 << 6 | q2 << 12 | q3 << 18 | q4 << 24, s (lo, hi)}
//          with q0..q5 the participants of reaction r (as in rx[r])
//   sch[LS][G], xbe[2 NS], xrows[NXR]: the balanced walk of the CSR (LS > 0;
//          built by pck_network_create).  A species row longer than
//          ceil(NE / G) entries is cut into pieces; the pieces are packed onto
//          the G lanes of a group longest-first, so every lane walks at most
//          LS entries instead of the longest row (CH4: 35, synthetic: 56).
//          Word t of lane l: entry e (bits 0-13) | slot (14-23) | last entry
//          of its piece (30) | valid (31).  Slot i < NS is row i's first
//          piece, slot NS + x its extra piece x; row i's extras are
//          [xbe[2i], xbe[2i+1]), and xrows lists the rows that have any.
//          Sums run piece by piece in entry order, then over the pieces in
//          order: deterministic, the same in every build of one network.
struct GrpView {
    const uint4* rx;
    const int32_t* row;
    const uint4* ent;
    int ND;                  // total participants = size of the derivative buffer
    int NE;                  // entries of the species CSR (= row[NS])
    const uint32_t* sch;     // balanced walk (LS = 0: off, the per-row loops)
    const int32_t* xbe;
    const int32_t* xrows;
    int LS, NX, NXR;
};
// PCK_GRP_BAL: the balanced walk is decided at run time (-1, the compiled-in
// kernels), compiled in (1) or out (0) (the hipRTC build knows the network)
#ifndef PCK_GRP_BAL
#define PCK_GRP_BAL -1
#endif
#define PCK_GRP_BAL_ON(g) (PCK_GRP_BAL == 1 || (PCK_GRP_BAL == -1 && (g).LS > 0))
#define PCK_SCH_VALID 0x80000000u
#define PCK_SCH_LAST 0x40000000u

// The solver kernel (TAB = true) copies the tables into LDS once per block
// (shared by the block's groups): every rate / Jacobian evaluation walks
// them, and from LDS each dependent record fetch costs an LDS round trip
// instead of an L1/L2 one.  The host picks TAB only where the extra LDS does
// not lower the kernel's occupancy (csrc/mk_kernels.hip: grp_tables_pay).
// Layout (16-byte units): rx[max(R,1)] | ent[max(NE,1)] | row[NS+1] (int32)
// | sch[NSCH] (uint32, the balanced walk's words, NSCH = LS * G)
__host__ __device__ inline size_t grp_tab_doubles(int R, int NE, int NS, int NSCH = 0) {
    const size_t b = 16 * (size_t)(R > 0 ? R : 1) + 16 * (size_t)(NE > 0 ? NE : 1) + 4 * (size_t)(NS + 1) +
                     4 * (size_t)NSCH;
    return (b + 15) / 16 * 2;
}

__device__ __forceinline__ void wsync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// Group all-reductions.  Within each row of 16 lanes: xor-1 / xor-2 by DPP
// quad_perm, then row_half_mirror and row_mirror (4 DPP steps, no LDS); a
// 32- or 64-lane group then combines its rows' results read with v_readlane
// (uniform).  Every lane of a group gets the bitwise-same value (the same
// operands in the same order), so control flow on the result stays
// group-uniform.  Callers reduce at group-uniform points only: every lane of
// the group is active.
template <int CTRL>
__device__ __forceinline__ double dppd(double v) { return __builtin_amdgcn_update_dpp(v, v, CTRL, 0xf, 0xf, false); }
template <int CTRL>
__device__ __forceinline__ int dppi(int v) { return __builtin_amdgcn_update_dpp(v, v, CTRL, 0xf, 0xf, false); }
__device__ __forceinline__ double rlane(double v, int l) {
    return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), l),
                            __builtin_amdgcn_readlane(__double2loint(v), l));
}

#define PCK_ROW_REDUCE(v, OP, DPP)  \
    v = OP(v, DPP<0xB1>(v));       /* quad_perm [1,0,3,2] */ \
    v = OP(v, DPP<0x4E>(v));       /* quad_perm [2,3,0,1] */ \
    v = OP(v, DPP<0x141>(v));      /* row_half_mirror */     \
    v = OP(v, DPP<0x140>(v))       /* row_mirror */

__device__ __forceinline__ double rlane_t(double v, int l) { return rlane(v, l); }
__device__ __forceinline__ int rlane_t(int v, int l) { return __builtin_amdgcn_readlane(v, l); }

template <int G, class T, class F>
__device__ __forceinline__ T grows(T v, F op) {
    if constexpr (G == 64) {
        const T a = rlane_t(v, 0), b = rlane_t(v, 16), c = rlane_t(v, 32), d = rlane_t(v, 48);
        return op(op(a, b), op(c, d));
    } else if constexpr (G == 32) {
        const T a = rlane_t(v, 0), b = rlane_t(v, 16), c = rlane_t(v, 32), d = rlane_t(v, 48);
        return (threadIdx.x & 32) ? op(c, d) : op(a, b);
    } else {
        return v;
    }
}

__device__ __forceinline__ double op_add(double a, double b) { return a + b; }
__device__ __forceinline__ double op_max(double a, double b) { return fmax(a, b); }
__device__ __forceinline__ double op_min(double a, double b) { return fmin(a, b); }
__device__ __forceinline__ int op_maxi(int a, int b) { return max(a, b); }

template <int G>
__device__ __forceinline__ double gsum(double v) {
    PCK_ROW_REDUCE(v, op_add, dppd);
    return grows<G>(v, op_add);
}
template <int G>
__device__ __forceinline__ double gmax(double v) {
    PCK_ROW_REDUCE(v, op_max, dppd);
    return grows<G>(v, op_max);
}
template <int G>
__device__ __forceinline__ double gmin(double v) {
    PCK_ROW_REDUCE(v, op_min, dppd);
    return grows<G>(v, op_min);
}
template <int G>
__device__ __forceinline__ int gmaxi(int v) {
    PCK_ROW_REDUCE(v, op_maxi, dppi);
    return grows<G>(v, op_maxi);
}
// group sum in double-double (the Newton refinement's conservation rows);
// dd_add is commutative bit for bit, so every lane gets the same value
template <int CTRL>
__device__ __forceinline__ dd dppdd(dd v) { return {dppd<CTRL>(v.hi), dppd<CTRL>(v.lo)}; }
template <int G>
__device__ __forceinline__ dd gsum_dd(dd v) {
    v = dd_add(v, dppdd<0xB1>(v));
    v = dd_add(v, dppdd<0x4E>(v));
    v = dd_add(v, dppdd<0x141>(v));
    v = dd_add(v, dppdd<0x140>(v));
    if constexpr (G == 16) {
        return v;
    } else {
        const dd a{rlane(v.hi, 0), rlane(v.lo, 0)}, b{rlane(v.hi, 16), rlane(v.lo, 16)};
        const dd c{rlane(v.hi, 32), rlane(v.lo, 32)}, d{rlane(v.hi, 48), rlane(v.lo, 48)};
        if constexpr (G == 64) return dd_add(dd_add(a, b), dd_add(c, d));
        return (threadIdx.x & 32) ? dd_add(c, d) : dd_add(a, b);
    }
}

// lane K (compile-time after unrolling) of every row of 16: DPP row_newbcast
__device__ __forceinline__ double bc16(double v, int k) {
    switch (k) {
#define PCK_BC(K) case K: return __builtin_amdgcn_update_dpp(0.0, v, 0x150 + K, 0xf, 0xf, false);
        PCK_BC(0) PCK_BC(1) PCK_BC(2) PCK_BC(3) PCK_BC(4) PCK_BC(5) PCK_BC(6) PCK_BC(7)
        PCK_BC(8) PCK_BC(9) PCK_BC(10) PCK_BC(11) PCK_BC(12) PCK_BC(13) PCK_BC(14) PCK_BC(15)
#undef PCK_BC
        default: return 0.0;
    }
}

// broadcast lane `src` (group-uniform) of the group
template <int G>
__device__ __forceinline__ double gbcast(double v, int src) {
    if constexpr (G == 64) {
        const int s = __builtin_amdgcn_readfirstlane(src);
        const int lo = __builtin_amdgcn_readlane(__double2loint(v), s);
        const int hi = __builtin_amdgcn_readlane(__double2hiint(v), s);
        return __hiloint2double(hi, lo);
    } else {
        return __shfl(v, src, G);
    }
}

__device__ __forceinline__ int rx_np(const uint4& r) { return (int)((r.w >> 16) & 7u); }
__device__ __forceinline__ int rx_dptr(const uint4& r) { return (int)(r.w & 0xffffu); }
__device__ __forceinline__ int rx_field(const uint4& r, int k) {
    const uint32_t w = (k < 2) ? r.x : (k < 4) ? r.y : r.z;
    return (int)((w >> (16 * (k & 1))) & 0xffffu);
}
__device__ __forceinline__ double ent_s(const uint4& e) { return __hiloint2double((int)e.w, (int)e.z); }
__device__ __forceinline__ int ent_r(const uint4& e) { return (int)(e.x & 511u); }
__device__ __forceinline__ int ent_np(const uint4& e) { return (int)((e.x >> 9) & 7u); }
__device__ __forceinline__ int ent_dptr(const uint4& e) { return (int)((e.x >> 12) & 0x3fffu); }
__device__ __forceinline__ int ent_species(const uint4& e, int k) {
    return (k < 5) ? (int)((e.y >> (6 * k)) & 63u) : (int)(e.x >> 26);
}

// net rate of a reaction (record rec) from the group's concentrations
// Bounds of the record walk: the hipRTC build defines them from the network
// (most participants of one reaction, largest exponent; csrc/mk_jit.h), the
// compiled-in kernels use the format's limits.  Unused participant slots of a
// record are all-zero fields (species 0, exponents 0): they multiply by 1, so
// the walk runs the fixed bound without a data-dependent loop or branch.
#ifndef PCK_GRP_NPMAX
#define PCK_GRP_NPMAX PCK_GRP_MAX_PART
#endif
#ifndef PCK_GRP_EMAX
#define PCK_GRP_EMAX PCK_GRP_MAX_EXP
#endif
#ifndef PCK_GRP_DEGMAX
#define PCK_GRP_DEGMAX 0        // largest row degree of the species CSR (0: data-dependent row loops)
#endif

// x^e for 0 <= e <= PCK_GRP_EMAX, branch-free for the usual e <= 2
__device__ __forceinline__ double spow(double x, int e) {
    if constexpr (PCK_GRP_EMAX <= 2) {
        return ((e >= 1) ? x : 1.0) * ((e >= 2) ? x : 1.0);
    } else {
        return ipow(x, e);
    }
}

// net rate of a reaction (record rec) from the group's concentrations
__device__ __forceinline__ double rec_rate(const uint4& rec, double a, double b, const double* c) {
    // no FMA contraction: every build (exact-size hipRTC, padded compiled-in)
    // rounds the products and the difference the same way -- bitwise-equal results
#pragma clang fp contract(off)
#pragma unroll
    for (int k = 0; k < PCK_GRP_NPMAX; ++k) {
        const int f = rx_field(rec, k);
        const double x = c[f & 63];
        const int ef = (f >> 6) & 31, er = f >> 11;
        a *= spow(x, ef);
        b *= spow(x, er);
    }
    return a - b;
}

// d(net_r)/d(c_q) for participant k0 of the record's reaction
__device__ __forceinline__ double rec_drate(const uint4& rec, double kf, double kr, const double* c, int k0) {
#pragma clang fp contract(off)
    const int f0 = rx_field(rec, k0);
    const int ef0 = (f0 >> 6) & 31, er0 = f0 >> 11;
    const double x0 = c[f0 & 63];
    double a = (ef0 > 0) ? kf * (double)ef0 * spow(x0, ef0 - 1) : 0.0;
    double b = (er0 > 0) ? kr * (double)er0 * spow(x0, er0 - 1) : 0.0;
#pragma unroll
    for (int k = 0; k < PCK_GRP_NPMAX; ++k) {
        const int f = rx_field(rec, k);
        const double x = c[f & 63];
        const bool self = (k == k0);
        const int ef = self ? 0 : (f >> 6) & 31, er = self ? 0 : f >> 11;
        a *= spow(x, ef);
        b *= spow(x, er);
    }
    return a - b;
}

// every participant's d(net_r)/d(c_q) of a record at once (out[k] for slot
// k < np): prefix and suffix products of the per-slot factors instead of one
// NPMAX-long product per participant (rec_drate), O(NPMAX) instead of
// O(NPMAX^2).  Unused slots are factors of exactly 1, so the exact-size and
// padded builds still agree bitwise (no FMA contraction here either).
#ifndef PCK_GRP_PREFIX
#define PCK_GRP_PREFIX 1
#endif
__device__ __forceinline__ void rec_drates(const uint4& rec, double kf, double kr, const double* c, double* out,
                                           int np, const double* dyn) {
#pragma clang fp contract(off)
    double ff[PCK_GRP_NPMAX], fr[PCK_GRP_NPMAX], df[PCK_GRP_NPMAX], dr[PCK_GRP_NPMAX];
#pragma unroll
    for (int k = 0; k < PCK_GRP_NPMAX; ++k) {
        const int f = rx_field(rec, k);
        const double x = c[f & 63];
        const int ef = (f >> 6) & 31, er = f >> 11;
        ff[k] = spow(x, ef);
        fr[k] = spow(x, er);
        df[k] = (ef > 0) ? (double)ef * spow(x, ef - 1) : 0.0;
        dr[k] = (er > 0) ? (double)er * spow(x, er - 1) : 0.0;
    }
    // suffix products in place of ff / fr (sf[k] = prod_{j > k} f_j)
    double sf = 1.0, sr = 1.0;
    double sfk[PCK_GRP_NPMAX], srk[PCK_GRP_NPMAX];
#pragma unroll
    for (int k = PCK_GRP_NPMAX - 1; k >= 0; --k) {
        sfk[k] = sf;
        srk[k] = sr;
        sf *= ff[k];
        sr *= fr[k];
    }
    double pf = kf, pr = kr;
#pragma unroll
    for (int k = 0; k < PCK_GRP_NPMAX; ++k) {
        if (k < np) {
            const int q = rx_field(rec, k) & 63;
            out[k] = ((pf * df[k]) * sfk[k] - (pr * dr[k]) * srk[k]) * dyn[4 * q];     // x cf_q
        }
        pf *= ff[k];
        pr *= fr[k];
    }
}

__host__ __device__ constexpr int grp_even(int n) { return (n + 1) & ~1; }
__host__ __device__ inline size_t grp_lds_doubles(int R, int NSP, int NS, int ND, int QB, int LS = 0, int NX = 0) {
    const int r1 = R > 0 ? R : 1;
    return (size_t)2 * grp_even(r1) + grp_even(NSP) + grp_even(ND > r1 ? ND : r1) + grp_even(NS * QB) + grp_even(NSP) +
           (LS ? grp_even(NX * NS) + grp_even(NS + NX) : 0);
}

// Per-group context: LDS blocks and this lane's species row.
template <int NSP>
struct Grp {
    int gl, NS, R, QB;
    int64_t cidx;             // condition index (diagnostics)
    bool row;                 // gl < NS
    double* kf; double* kr;   // effective rate constants (fixed species folded, DRC perturbation)
    double* c;                // concentrations c_q = cf_q y_q
    double* d;                // net rates [R] / derivatives [ND]
    double* J;                // Jacobian column block: J[i*QB + j]
    double* pb;               // pivot-row broadcast
    double* Jx;               // balanced walk: Jacobian rows of the extra pieces [NX][NS]
    double* part;             // balanced walk: rate sums of the pieces [NS + NX]
    int xb, xe;               // balanced walk: this row's extra pieces
    int rb, re;               // this row's CSR range
    double cfi, rs, fl, in;   // this row's concentration factor, row scale, flow, inflow
};

// For networks on 64-lane groups (more than 32 species), the transient
// integration evaluates rates and Jacobian at the clamped state max(y, 0)
// instead of the positivity rule of the smaller networks (PCK_GRP_CLAMP,
// default on; the Newton polish and the TOF use the plain mass-action
// equations, whose root the reference's least_squares finds): a species at zero then has no consumption
// term, so tolerance-level negatives decay instead of feeding second-order
// terms of the wrong sign.  Large stiff networks (the synthetic 50 x 150 one)
// otherwise either oscillate around zero in sign-alternating steps (plain
// Rodas4, like scipy BDF, which fails outright on some of the same
// conditions) or chatter at h ~ 1e-8 t under a reject-below--atol rule; the
// CPU mirror (tools/rodas_mirror.py CLAMP=1) and the GPU both solve those
// conditions in ~1e3 steps with it.  Where every component is >= 0 it
// changes nothing.
// PCK_GRP_EXACT=1 (set by the hipRTC compile, csrc/mk_jit.h): NSP equals the
// network's species count, so every `k < NS` guard folds away at compile time
#ifndef PCK_GRP_EXACT
#define PCK_GRP_EXACT 0
#endif
#ifndef PCK_GRP_CLAMP
#define PCK_GRP_CLAMP 1
#endif
#ifndef PCK_CLAMP_CLIP_AFTER
#define PCK_CLAMP_CLIP_AFTER 4096
#endif

template <int NSP, bool CL = false>
__device__ __forceinline__ void put_c(const Grp<NSP>& x, double y) {
    wsync();                                   // previous readers of c / d are done
    if (x.row) x.c[x.gl] = x.cfi * ((CL && PCK_GRP_CLAMP) ? fmax(y, 0.0) : y);
    wsync();
}

// ---------------------------------------------------------------------------
// Compile-time network (the hipRTC build of csrc/mk_jit.h: jit_group_ct_kernel).
// With the network's tables constexpr (nets::Jit: exponents, stoichiometry,
// concentration factors), every lane of a group evaluates every reaction of
// its condition in straight-line code: the group's concentrations are
// broadcast into registers (DPP row_newbcast on 16-lane groups, v_readlane on
// a wavefront), the rates and their derivatives are products with compile-time
// exponents, and each lane keeps its own species row -- the row sums with
// compile-time coefficients.  No record decode, no CSR walk, no LDS traffic
// but the condition's k_eff (one broadcast read per reaction), no barrier.
// The record-table path (above: lane-per-reaction, then the CSR gather) does
// the same arithmetic in another order: the two agree to rounding.
// ---------------------------------------------------------------------------
typedef __attribute__((address_space(3))) const double lds_cdouble;
struct NoNet {};
template <class Net> struct IsCt { static constexpr bool v = true; };
template <> struct IsCt<NoNet> { static constexpr bool v = false; };

// compile-time loops: body(IC<k>{}) for k = B .. E-1, every index a constant
// expression (the #pragma unroll of a 58- or 150-reaction loop around an
// unrolled body gives up past LLVM's unroll threshold and leaves the table
// lookups and their branches at run time)
template <int V> struct IC { static constexpr int value = V; };
template <int B, int E, class F>
__device__ __forceinline__ void sfor(F&& body) {
    if constexpr (B < E) {
        body(IC<B>{});
        sfor<B + 1, E>(body);
    }
}

// lane q of the calling lane's group, q a compile-time constant
template <int G>
__device__ __forceinline__ double gbcast_k(double v, int q) {
    if constexpr (G == 16) {
        return bc16(v, q);
    } else if constexpr (G == 64) {
        return rlane(v, q);
    } else {
        const double a = rlane(v, q), b = rlane(v, 32 + q);
        return (threadIdx.x & 32) ? b : a;
    }
}

// row sums by per-row accumulators (cheaper for small networks) or by the
// lane's coefficient of each column (fewer registers)
#ifndef PCK_CT_ACC_MAX
#define PCK_CT_ACC_MAX 24
#endif
// Straight-line code over every reaction lets the scheduler hoist all the
// k_eff loads and products to the top (for CH4: 512 VGPRs, 830 spilled);
// a scheduling barrier every PCK_CT_CHUNK reactions bounds the live ranges
// to one chunk (the other waves of the SIMD hide the chunk's LDS latency).
#ifndef PCK_CT_CHUNK
#define PCK_CT_CHUNK 4
#endif
// the condition's k_eff from LDS, re-read at every evaluation: loop-invariant
// over the whole solve, LLVM would otherwise hoist all 2R loads out of the
// step loop and keep them live (CH4: 232 VGPRs)
__device__ __forceinline__ double ct_k(const double* p, int j) { return ((lds_cdouble*)p)[j]; }
// an evaluation starts with a compiler memory barrier: the k_eff loads below
// it cannot be hoisted out of the step loop (no instruction is emitted)
__device__ __forceinline__ void ct_reload() { asm volatile("" ::: "memory"); }
// At a chunk boundary the running sums pass through an empty asm: volatile
// asm statements keep their order, so every value a chunk computes is
// finished before the next chunk's loads issue (a memory clobber alone
// orders the loads but lets the selection-DAG scheduler sink the arithmetic
// below all of them).
template <int J, int N>
__device__ __forceinline__ void ct_fence(double (&v)[N]) {
    if constexpr ((J + 1) % PCK_CT_CHUNK == 0) {
#pragma unroll
        for (int i = 0; i < N; ++i) asm volatile("" : "+v"(v[i]) :: "memory");
    }
}

template <class Net, int NSP, int G, bool CL>
__device__ __forceinline__ void ct_conc(const Grp<NSP>& x, double y, double (&c)[Net::NS]) {
    if constexpr (G == 64) {
        // a wavefront's group: v_readlane would put all NS concentrations in
        // SGPRs (NS = 50: 100 of them, ~2 000 spilled); an LDS round trip
        // gives VGPRs (each read is one broadcast address)
        put_c<NSP, CL>(x, y);
        sfor<0, Net::NS>([&](auto qc) {
            constexpr int q = decltype(qc)::value;
            c[q] = ((lds_cdouble*)x.c)[q];
        });
    } else {
        const double v = (CL && PCK_GRP_CLAMP) ? fmax(y, 0.0) : y;
        sfor<0, Net::NS>([&](auto qc) {
            constexpr int q = decltype(qc)::value;
            c[q] = Net::dyn(q, 0) * gbcast_k<G>(v, q);
        });
    }
}

// S(gl, j): the calling lane's coefficient of column J (0 off its row).  gl
// is the lane's row as returned by ct_row(): the coefficients only depend on
// it, so LLVM would hoist all R of them out of the step loop and keep them
// live (CH4: 116 VGPRs, one wave per SIMD); ct_row() hides gl behind an
// empty asm at every evaluation, so they are recomputed (a few selects each).
__device__ __forceinline__ int ct_row(int gl) {
    asm volatile("" : "+v"(gl));
    return gl;
}
template <class Net, int J>
__device__ __forceinline__ double ct_coef(int gl) {
    double s = 0.0;
    sfor<0, Net::NS>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        if constexpr (Net::S(i, J) != 0.0) s = (gl == i) ? Net::S(i, J) : s;
    });
    return s;
}

template <class Net, int J>
__device__ __forceinline__ constexpr bool ct_col_used() {
    for (int i = 0; i < Net::NS; ++i)
        if (Net::S(i, J) != 0.0) return true;
    return false;
}

// x^E for a compile-time E >= 1
template <int E>
__device__ __forceinline__ double cpow(double x) {
    if constexpr (E == 1) return x;
    else if constexpr (E == 2) return x * x;
    else return x * cpow<E - 1>(x);
}

// rf - rr rounded as written: with contraction the difference would fold one
// product into an FMA and stop cancelling exactly where the two rates agree
// (mk_group.h rec_rate keeps contraction off for the same reason)
__device__ __forceinline__ double ct_sub(double a, double b) {
#pragma clang fp contract(off)
    return a - b;
}

// forward / reverse rate of reaction J (kf, kr: the condition's effective constants)
template <class Net, int J>
__device__ __forceinline__ void ct_rate(double kf, double kr, const double (&c)[Net::NS], double& rf, double& rr) {
#pragma clang fp contract(off)
    rf = kf;
    rr = kr;
    sfor<0, Net::NS>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        if constexpr (Net::ef(J, i) > 0) rf *= cpow<Net::ef(J, i)>(c[i]);
        if constexpr (Net::er(J, i) > 0) rr *= cpow<Net::er(J, i)>(c[i]);
    });
}

// f (and with GROSS the gross flux) of the calling lane's row
template <class Net, int NSP, int G, bool CL, bool GROSS = false>
__device__ __forceinline__ double ct_rhs(const Grp<NSP>& x, double y, double* gross = nullptr) {
    constexpr int NS = Net::NS, R = Net::R;
    ct_reload();
    const int gl = ct_row(x.gl);
    double c[NS];
    ct_conc<Net, NSP, G, CL>(x, y, c);
    double f = 0.0, gacc = 0.0;
    if constexpr (NS <= PCK_CT_ACC_MAX && !GROSS) {
        double acc[NS];
        sfor<0, NS>([&](auto ic) { acc[decltype(ic)::value] = 0.0; });
        sfor<0, R>([&](auto jc) {
            constexpr int j = decltype(jc)::value;
            if constexpr (ct_col_used<Net, j>()) {
                double rf, rr;
                ct_rate<Net, j>(ct_k(x.kf, j), ct_k(x.kr, j), c, rf, rr);
                const double net = ct_sub(rf, rr);
                sfor<0, NS>([&](auto ic) {
                    constexpr int i = decltype(ic)::value;
                    if constexpr (Net::S(i, j) != 0.0) acc[i] += Net::S(i, j) * net;
                });
                ct_fence<j>(acc);
            }
        });
        sfor<0, NS>([&](auto ic) {
            constexpr int i = decltype(ic)::value;
            f = (gl == i) ? acc[i] : f;
        });
    } else {
        sfor<0, R>([&](auto jc) {
            constexpr int j = decltype(jc)::value;
            if constexpr (ct_col_used<Net, j>()) {
                double rf, rr;
                ct_rate<Net, j>(ct_k(x.kf, j), ct_k(x.kr, j), c, rf, rr);
                const double s = ct_coef<Net, j>(gl);
                f = fma(s, ct_sub(rf, rr), f);
                if constexpr (GROSS) gacc = fma(fabs(s), fabs(rf) + fabs(rr), gacc);
                double fg[2] = {f, gacc};
                ct_fence<j>(fg);
                f = fg[0];
                gacc = fg[1];
            }
        });
    }
    if (!x.row) return 0.0;
    if constexpr (GROSS) *gross = gacc * fabs(x.rs) + fabs(x.fl) * (fabs(x.in) + fabs(y));
    return f * x.rs + x.fl * (x.in - y);
}

// the calling lane's row f in double-double, rounded once (mk_solver.h:
// rhs_dd; the Newton refinement's residual): concentrations as exact
// products cf_q y_q of the group's raw states, every reaction's rates and
// their difference error-free, one reaction per scheduling region
template <class Net, int NSP, int G>
__device__ __forceinline__ double ct_rhs_dd(const Grp<NSP>& x, double y) {
    constexpr int NS = Net::NS, R = Net::R;
    ct_reload();
    const int gl = ct_row(x.gl);
    if constexpr (G == 64) {
        wsync();
        if (x.row) x.c[x.gl] = y;                  // the raw state (put_c rewrites c before its next use)
        wsync();
    }
    // c_q = cf_q y_q exactly, fetched where a reaction uses it: the state
    // passes through an empty asm per reaction, so the broadcasts are not
    // shared across reactions (holding all NS concentrations in double-double
    // would cost 4 NS VGPRs: CH4 went to 256 with 4 spilled)
    dd acc = dd_of(0.0);
    sfor<0, R>([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        if constexpr (ct_col_used<Net, j>()) {
            double yv = y;
            asm volatile("" : "+v"(yv));
            auto conc = [&](auto qc) {
                constexpr int q = decltype(qc)::value;
                if constexpr (G == 64) return two_prod(Net::dyn(q, 0), ((lds_cdouble*)x.c)[q]);
                else return two_prod(Net::dyn(q, 0), gbcast_k<G>(yv, q));
            };
            dd rf = dd_of(ct_k(x.kf, j)), rr = dd_of(ct_k(x.kr, j));
            sfor<0, NS>([&](auto ic) {
                constexpr int i = decltype(ic)::value;
                if constexpr (Net::ef(j, i) > 0 || Net::er(j, i) > 0) {
                    const dd ci = conc(ic);
                    if constexpr (Net::ef(j, i) > 0) rf = dd_mul(rf, dd_pow(ci, Net::ef(j, i)));
                    if constexpr (Net::er(j, i) > 0) rr = dd_mul(rr, dd_pow(ci, Net::er(j, i)));
                }
            });
            acc = dd_add(acc, dd_mul(dd_add(rf, dd_neg(rr)), ct_coef<Net, j>(gl)));
            // the running sum passes through an empty asm (ct_fence): each
            // reaction is finished before the next one's loads issue
            asm volatile("" : "+v"(acc.hi), "+v"(acc.lo) :: "memory");
        }
    });
    if (!x.row) return 0.0;
    dd r = dd_mul(acc, x.rs);
    if (x.fl != 0.0) r = dd_add(r, dd_mul(two_sum(x.in, -y), x.fl));
    return r.hi + r.lo;
}

// d(prod_i c_i^E(J, i)) / d y_Q, times k (mk_solver.h: jac)
template <class Net, int J, int Q, bool FWD>
__device__ __forceinline__ double ct_dside(double k, const double (&c)[Net::NS]) {
    constexpr int eq = FWD ? Net::ef(J, Q) : Net::er(J, Q);
    double t = k * (double)eq * Net::dyn(Q, 0);
    if constexpr (eq > 1) t *= cpow<eq - 1>(c[Q]);
    sfor<0, Net::NS>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        constexpr int ei = FWD ? Net::ef(J, i) : Net::er(J, i);
        if constexpr (i != Q && ei > 0) t *= cpow<ei>(c[i]);
    });
    return t;
}

// W[q] = sgn * dF_i/dy_q + (q == i ? shift : 0) on the calling lane's row i
template <class Net, int NSP, int G, bool CL>
__device__ __forceinline__ void ct_jac(const Grp<NSP>& x, double y, double sgn, double shift, double (&W)[NSP]) {
    constexpr int NS = Net::NS, R = Net::R;
    ct_reload();
    const int gl = ct_row(x.gl);
    double c[NS];
    ct_conc<Net, NSP, G, CL>(x, y, c);
    double jr[NS];
    sfor<0, NS>([&](auto qc) { jr[decltype(qc)::value] = 0.0; });
    sfor<0, R>([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        if constexpr (ct_col_used<Net, j>()) {
            const double s = ct_coef<Net, j>(gl);
            const double kf = ct_k(x.kf, j), kr = ct_k(x.kr, j);
            sfor<0, NS>([&](auto qc) {
                constexpr int q = decltype(qc)::value;
                if constexpr (Net::ef(j, q) > 0 || Net::er(j, q) > 0) {
                    double v = 0.0;
                    if constexpr (Net::ef(j, q) > 0) v += ct_dside<Net, j, q, true>(kf, c);
                    if constexpr (Net::er(j, q) > 0) v -= ct_dside<Net, j, q, false>(kr, c);
                    jr[q] = fma(s, v, jr[q]);
                }
            });
            ct_fence<j>(jr);
        }
    });
    const double sc = sgn * x.rs;
    const double dg = shift - sgn * x.fl;
#pragma unroll
    for (int q = 0; q < NSP; ++q) W[q] = (x.row && q < NS) ? sc * jr[q < NS ? q : 0] + (q == x.gl ? dg : 0.0) : 0.0;
}

// f_i = rs_i * sum_r S_ir net_r + fl_i (in_i - y_i)   (row lanes; 0 elsewhere)
template <int NSP, int G, bool CL = false, class Net = NoNet>
__device__ __forceinline__ double grp_rhs(const GrpView& g, const Grp<NSP>& x, double y) {
    if constexpr (IsCt<Net>::v) return ct_rhs<Net, NSP, G, CL>(x, y);
    put_c<NSP, CL>(x, y);
    for (int r = x.gl; r < x.R; r += G) x.d[r] = rec_rate(g.rx[r], x.kf[r], x.kr[r], x.c);
    wsync();
    double f = 0.0;
    if (PCK_GRP_BAL_ON(g)) {
        // balanced walk: every lane sums its pieces, the row's lane adds them up
        // the next word and its entry are fetched one iteration ahead (an
        // invalid word's entry index is 0: a harmless load)
        double acc = 0.0;
        uint32_t w = g.sch[x.gl];
        uint4 q = g.ent[w & 0x3fffu];
        for (int t = 0; t < g.LS; ++t) {
            const uint32_t wn = (t + 1 < g.LS) ? g.sch[(t + 1) * G + x.gl] : 0u;
            const uint4 qn = g.ent[wn & 0x3fffu];
            if (w & PCK_SCH_VALID) {
                acc = fma(ent_s(q), x.d[ent_r(q)], acc);
                if (w & PCK_SCH_LAST) {
                    x.part[(w >> 14) & 0x3ffu] = acc;
                    acc = 0.0;
                }
            }
            w = wn;
            q = qn;
        }
        wsync();
        if (x.row) {
            f = (x.re > x.rb) ? x.part[x.gl] : 0.0;
            for (int p = x.xb; p < x.xe; ++p) f += x.part[x.NS + p];
            f = f * x.rs + x.fl * (x.in - y);
        }
        return f;
    }
    if (x.row) {
        // two partial sums keep several entry loads in flight
        double f2 = 0.0;
#if PCK_GRP_DEGMAX > 0
        // hipRTC build: the trip count is the network's largest row degree,
        // the same for every lane (scalar loop control)
#pragma unroll 2
        for (int i = 0; i < PCK_GRP_DEGMAX; i += 2) {
            const int e = x.rb + i;
            if (e + 1 < x.re) {                 // lanes past their row's end are masked: no LDS traffic
                const uint4 q = g.ent[e], q2 = g.ent[e + 1];
                f = fma(ent_s(q), x.d[ent_r(q)], f);
                f2 = fma(ent_s(q2), x.d[ent_r(q2)], f2);
            } else if (e < x.re) {
                const uint4 q = g.ent[e];
                f = fma(ent_s(q), x.d[ent_r(q)], f);
            }
        }
#else
        int e = x.rb;
#pragma unroll 2
        for (; e + 1 < x.re; e += 2) {
            const uint4 q = g.ent[e], q2 = g.ent[e + 1];
            f = fma(ent_s(q), x.d[ent_r(q)], f);
            f2 = fma(ent_s(q2), x.d[ent_r(q2)], f2);
        }
        if (e < x.re) {
            const uint4 q = g.ent[e];
            f = fma(ent_s(q), x.d[ent_r(q)], f);
        }
#endif
        f = (f + f2) * x.rs + x.fl * (x.in - y);
    }
    return f;
}

// The row's f in double-double (ct_rhs_dd) for the record-table kernels:
// lane-per-reaction rates in double-double, their high parts gathered along
// the species CSR with error-free products and sums, then their low parts
// (the per-row loops, also where the balanced walk is compiled in: this runs
// a few times per solve)
template <int NSP, int G>
__device__ __forceinline__ double tab_rhs_dd(const NetView& nv, const GrpView& g, const Grp<NSP>& x, double y) {
    wsync();
    if (x.row) x.c[x.gl] = y;                      // the raw state (put_c rewrites c before its next use)
    wsync();
    auto rate = [&](int r) {
        const uint4 rec = g.rx[r];
        dd a = dd_of(x.kf[r]), b = dd_of(x.kr[r]);
#pragma unroll
        for (int k = 0; k < PCK_GRP_NPMAX; ++k) {
            const int f = rx_field(rec, k);
            const int q = f & 63, ef = (f >> 6) & 31, er = f >> 11;
            if (ef | er) {
                const dd cq = two_prod(nv.dyn[4 * q], x.c[q]);
                if (ef) a = dd_mul(a, dd_pow(cq, ef));
                if (er) b = dd_mul(b, dd_pow(cq, er));
            }
        }
        return dd_add(a, dd_neg(b));
    };
    for (int r = x.gl; r < x.R; r += G) x.d[r] = rate(r).hi;
    wsync();
    dd acc = dd_of(0.0);
    if (x.row) {
        for (int e = x.rb; e < x.re; ++e) {
            const uint4 q = g.ent[e];
            acc = dd_add(acc, two_prod(ent_s(q), x.d[ent_r(q)]));
        }
    }
    wsync();
    for (int r = x.gl; r < x.R; r += G) x.d[r] = rate(r).lo;
    wsync();
    if (x.row) {
        double lo = 0.0;
        for (int e = x.rb; e < x.re; ++e) {
            const uint4 q = g.ent[e];
            lo = fma(ent_s(q), x.d[ent_r(q)], lo);
        }
        acc = dd_add(acc, dd_of(lo));
    }
    wsync();
    if (!x.row) return 0.0;
    dd r = dd_mul(acc, x.rs);
    if (x.fl != 0.0) r = dd_add(r, dd_mul(two_sum(x.in, -y), x.fl));
    return r.hi + r.lo;
}

template <int NSP, int G, class Net = NoNet>
__device__ __forceinline__ double grp_rhs_dd(const NetView& nv, const GrpView& g, const Grp<NSP>& x, double y) {
    if constexpr (IsCt<Net>::v) return ct_rhs_dd<Net, NSP, G>(x, y);
    else return tab_rhs_dd<NSP, G>(nv, g, x, y);
}

// W[q] = sgn * dF_i/dy_q + (q == i ? shift : 0), with dF/dy including the flow
// diagonal (-fl_i); 0 on lanes without a row
template <int NSP, int G, int P, bool CL = false, class Net = NoNet>
__device__ __forceinline__ void grp_jac(const NetView& nv, const GrpView& g, const Grp<NSP>& x, double y, double sgn,
                                        double shift, double (&W)[NSP]) {
    if constexpr (IsCt<Net>::v) {
        ct_jac<Net, NSP, G, CL>(x, y, sgn, shift, W);
        return;
    }
    constexpr int QB = (NSP + P - 1) / P;
    put_c<NSP, CL>(x, y);
    for (int r = x.gl; r < x.R; r += G) {
        const uint4 rec = g.rx[r];
        const int np = rx_np(rec), dp = rx_dptr(rec);
        const double a = x.kf[r], b = x.kr[r];
        if constexpr (PCK_GRP_PREFIX) {
            rec_drates(rec, a, b, x.c, x.d + dp, np, nv.dyn);
        } else {
#pragma unroll
            for (int k = 0; k < PCK_GRP_NPMAX; ++k) {
                if (k < np) {
                    const int q = rx_field(rec, k) & 63;
                    x.d[dp + k] = rec_drate(rec, a, b, x.c, k) * nv.dyn[4 * q];     // x cf_q
                }
            }
        }
    }
    wsync();
    const double sc = sgn * x.rs;
    const double dg = shift - sgn * x.fl;
    if (P == 1 && PCK_GRP_BAL_ON(g)) {
        // balanced walk: each lane adds its pieces' terms into their rows (a
        // row's first piece into J, extras into Jx: every target row has one
        // writer), then the extras are folded into J per (row, column)
        uint32_t w = g.sch[x.gl];
        uint4 q = g.ent[w & 0x3fffu];
        for (int t = 0; t < g.LS; ++t) {
            const uint32_t wn = (t + 1 < g.LS) ? g.sch[(t + 1) * G + x.gl] : 0u;
            const uint4 qn = g.ent[wn & 0x3fffu];
            if (w & PCK_SCH_VALID) {
                const int slot = (int)((w >> 14) & 0x3ffu);
                double* dst = (slot < x.NS) ? x.J + slot * QB : x.Jx + (slot - x.NS) * x.NS;
                const double s = ent_s(q);
                const int np = ent_np(q), dp = ent_dptr(q);
#pragma unroll
                for (int k = 0; k < PCK_GRP_NPMAX; ++k) {
                    if (k < np) {
                        // one writer lane per target row: its LDS adds land in
                        // program order (fire-and-forget ds_add, no read back)
                        const int sp = ent_species(q, k);
                        atomicAdd(dst + sp, s * x.d[dp + k]);
                    }
                }
            }
            w = wn;
            q = qn;
        }
        wsync();
        for (int it = x.gl; it < g.NXR * x.NS; it += G) {
            const int i = g.xrows[it / x.NS], j = it % x.NS;
            double v = x.J[i * QB + j];
            for (int p = g.xbe[2 * i]; p < g.xbe[2 * i + 1]; ++p) {
                v += x.Jx[p * x.NS + j];
                x.Jx[p * x.NS + j] = 0.0;
            }
            x.J[i * QB + j] = v;
        }
        wsync();
#pragma unroll
        for (int q = 0; q < NSP; ++q) {
            double v = 0.0;
            if (x.row && q < x.NS) {
                v = x.J[x.gl * QB + q];
                x.J[x.gl * QB + q] = 0.0;
            }
            W[q] = x.row ? sc * v + (q == x.gl ? dg : 0.0) : 0.0;
        }
        return;
    }
#pragma unroll
    for (int pass = 0; pass < P; ++pass) {
        const int q0 = pass * QB;
        if (x.row) {
            double* jr = x.J + x.gl * QB - q0;
#if PCK_GRP_DEGMAX > 0
#pragma unroll 2
            for (int i = 0; i < PCK_GRP_DEGMAX; ++i) {
                if (x.rb + i >= x.re) continue;      // masked lanes: no LDS traffic
                const uint4 q = g.ent[x.rb + i];
                const double s = ent_s(q);
                const int np = ent_np(q), dp = ent_dptr(q);
#pragma unroll
                for (int k = 0; k < PCK_GRP_NPMAX; ++k) {
                    const int sp = ent_species(q, k);
                    // only the owner lane adds to its row: program order = summation order
                    if (k < np && (P == 1 || (sp >= q0 && sp < q0 + QB))) atomicAdd(jr + sp, s * x.d[dp + k]);
                }
            }
#else
#pragma unroll 4
            for (int e = x.rb; e < x.re; ++e) {
                const uint4 q = g.ent[e];
                const double s = ent_s(q);
                const int np = ent_np(q), dp = ent_dptr(q);
                for (int k = 0; k < np; ++k) {
                    const int sp = ent_species(q, k);
                    // only the owner lane adds to its row: program order = summation order
                    if (P == 1 || (sp >= q0 && sp < q0 + QB)) atomicAdd(jr + sp, s * x.d[dp + k]);
                }
            }
#endif
        }
        wsync();
#pragma unroll
        for (int j = 0; j < QB; ++j) {
            const int q = q0 + j;
            if (q < NSP) {
                double v = 0.0;
                if (x.row && q < x.NS) {
                    v = x.J[x.gl * QB + j];
                    x.J[x.gl * QB + j] = 0.0;
                }
                W[q] = x.row ? sc * v + (q == x.gl ? dg : 0.0) : 0.0;
            }
        }
    }
}

// pivot sequence, 4 lane ids per register
template <int NSP>
struct Perm {
    uint32_t w[(NSP + 3) / 4];
    __device__ __forceinline__ void set(int k, int p) {
        const int s = 8 * (k & 3);
        w[k >> 2] = (w[k >> 2] & ~(255u << s)) | ((uint32_t)p << s);
    }
    __device__ __forceinline__ int get(int k) const { return (int)((w[k >> 2] >> (8 * (k & 3))) & 255u); }
};

// LU factors of the group's rows: multipliers in the eliminated rows'
// columns, U in the pivot rows with 1/U_kk in the pivot column; pk[k] = lane
// of the pivot row of column k; step = column at which this row was pivot.
template <int NSP>
struct LU {
    double W[NSP];
    Perm<NSP> pk;
    int step;
    int src;        // 16- and 64-lane groups (physical row swaps): original row now held by this lane
    bool swp;       // 64-lane groups: some rows were interchanged (wave-uniform)
};

// 16-lane groups (one row of the wavefront per condition): LU with partial
// pivoting by PHYSICAL row interchanges, so the pivot row of column k always
// sits in lane k and every broadcast has a compile-time source lane: DPP
// row_newbcast (one v_mov_b64_dpp, no LDS, no barrier).  The interchange
// itself moves both rows' registers with ds_bpermute, only in waves where
// some group swaps (wave vote).  Same pivots and the same operations in the
// same order as the lane-indexed form below: identical factors.
template <int NSP>
__device__ __forceinline__ bool grp_lu16(const Grp<NSP>& x, LU<NSP>& F) {
    bool ok = true;
    F.src = x.gl;
#pragma unroll
    for (int k = 0; k < NSP; ++k) {
        if (k < x.NS) {
            const float mag = (float)fabs(F.W[k]);
            int key = (x.row && x.gl >= k) ? (int)((__float_as_uint(mag) & ~63u) | (uint32_t)x.gl) : -1;
            key = gmaxi<16>(key);
            const int p = key & 63;
            ok = ok && key >= 0;
            if (__any(p != k)) {
                const int from = (x.gl == k) ? p : (x.gl == p) ? k : x.gl;
#pragma unroll
                for (int j = 0; j < NSP; ++j) F.W[j] = __shfl(F.W[j], from, 16);
                F.src = __shfl(F.src, from, 16);
            }
            const double piv = bc16(F.W[k], k);
            ok = ok && piv != 0.0 && isfinite(piv);
            const double inv = rcp(piv);
            const bool below = x.gl > k;            // padding lanes hold zero rows: updates are no-ops
            const double l = F.W[k] * inv;
            // the multiplier is 0 on the rows at and above k, whose trailing
            // entries the fma then leaves as they are (one VALU op per column
            // instead of an fma and a select)
            const double lm = below ? -l : 0.0;
            if (x.gl == k) F.W[k] = inv;
            if (below) F.W[k] = l;
#pragma unroll
            for (int j = k + 1; j < NSP; ++j) {
                if (j < x.NS) {
                    const double pj = bc16(F.W[j], k);
                    F.W[j] = fma(lm, pj, F.W[j]);
                }
            }
        }
    }
    return ok;
}

template <int NSP>
__device__ __forceinline__ double grp_solve16(const Grp<NSP>& x, const LU<NSP>& F, double b) {
    b = __shfl(b, F.src, 16);                      // the row interchanges of the factorisation
#pragma unroll
    for (int k = 0; k < NSP; ++k) {
        if (k < x.NS) {
            const double bk = bc16(b, k);
            if (x.gl > k) b = fma(-F.W[k], bk, b);
        }
    }
#pragma unroll
    for (int kk = 0; kk < NSP; ++kk) {
        const int k = NSP - 1 - kk;
        if (k < x.NS) {
            const double xk = bc16(b * F.W[k], k);
            if (x.gl < k) b = fma(-F.W[k], xk, b);
            if (x.gl == k) b = xk;
        }
    }
    return x.row ? b : 0.0;
}

// 64-lane groups (one condition per wavefront; round 5): threshold pivoting
// as the lane solver (mk_device.h: lu, PCK_PIVOT_TAU) with physical row
// interchanges, so row k of the factors sits in lane k and every broadcast of
// the LU and both substitutions is a v_readlane from a constant lane -- no
// pivot-index extraction, no readfirstlane, no SGPR lane operands.  Rows are
// interchanged only where some row below the diagonal is 1/tau times larger
// (wave vote, rare); the pivot row is then the largest one, as in partial
// pivoting.  The trailing update of a column runs in chunks of PCK_LU64_CHUNK
// entries: an empty asm at each chunk boundary takes the chunk's results and
// the next chunk's sources, so the next readlanes cannot be hoisted above the
// chunk's FMAs (all 2 (NS - k) of them at once overflow the SGPRs and spill).
// PCK_GRP_TPIV64=0 keeps the partial-pivoting form below.
#ifndef PCK_GRP_TPIV64
#define PCK_GRP_TPIV64 1
#endif
#ifndef PCK_LU64_CHUNK
#define PCK_LU64_CHUNK 8
#endif
#ifndef PCK_LU64_TAU
#define PCK_LU64_TAU PCK_PIVOT_TAU
#endif
template <int NSP>
__device__ __forceinline__ bool grp_lu64(const Grp<NSP>& x, LU<NSP>& F) {
    bool ok = true;
    // the lane index through an empty asm: the per-column lane masks (gl > k,
    // gl == k) are recomputed at each use instead of hoisted for the whole
    // kernel into SGPR pairs that then spill (ct_row, same trick)
    const int gl = ct_row(x.gl);
    F.src = gl;
    F.swp = false;
    // the column loop by template recursion (every k a constant: LLVM's full
    // unroll gives up on the nest and the factors go to scratch), the
    // updates of one column by a plain unrolled loop
    sfor<0, NSP>([&](auto kc) {
        constexpr int k = decltype(kc)::value;
        if (k < x.NS) {
            const double dk = fabs(rlane(F.W[k], k)) * (1.0 / PCK_LU64_TAU);
            if (__any(x.row && gl > k && fabs(F.W[k]) > dk)) {      // rare: wave-uniform
                const float mag = (float)fabs(F.W[k]);
                int key = (x.row && gl >= k) ? (int)((__float_as_uint(mag) & ~63u) | (uint32_t)gl) : -1;
                key = gmaxi<64>(key);
                const int p = __builtin_amdgcn_readfirstlane(key & 63);
                if (p != k) {
                    // rows k and p through LDS: row k into the concentration
                    // buffer, row p into the pivot buffer (both free outside
                    // the rate evaluations, which rewrite c first), then each
                    // reads the other's -- 2 NS LDS accesses on the two lanes
                    // instead of 2 NS ds_bpermute on the wavefront (code size:
                    // this block is unrolled per column and per call site)
                    const int from = (gl == k) ? p : (gl == p) ? k : gl;
                    const bool mover = (gl == k) || (gl == p);
                    double* mine = (gl == k) ? x.c : x.pb;
                    const double* theirs = (gl == k) ? x.pb : x.c;
                    wsync();
                    if (mover) {
#pragma unroll
                        for (int j = 0; j < NSP; ++j) mine[j] = F.W[j];
                    }
                    wsync();
                    if (mover) {
#pragma unroll
                        for (int j = 0; j < NSP; ++j) F.W[j] = theirs[j];
                    }
                    wsync();
                    F.src = __shfl(F.src, from, 64);
                    F.swp = true;
                }
            }
            const double piv = rlane(F.W[k], k);
            ok = ok && piv != 0.0 && isfinite(piv);
            const double inv = rcp(piv);
            const bool below = gl > k;                 // padding lanes hold zero rows: updates are no-ops
            const double l = F.W[k] * inv;
            const double lm = below ? -l : 0.0;        // 0 at and above row k: the fma leaves them as they are
            if (gl == k) F.W[k] = inv;
            if (below) F.W[k] = l;
#pragma unroll
            for (int j = k + 1; j < NSP; ++j) {
                if ((j - k - 1) % PCK_LU64_CHUNK == 0 && j > k + 1) {
                    // chunk boundary: the previous chunk's results, then this chunk's sources
#pragma unroll
                    for (int q = j - PCK_LU64_CHUNK; q < j + PCK_LU64_CHUNK && q < NSP; ++q)
                        asm volatile("" : "+v"(F.W[q]));
                }
                if (j < x.NS) F.W[j] = fma(lm, rlane(F.W[j], k), F.W[j]);
            }
        }
    });
    return ok;
}

template <int NSP>
__device__ __forceinline__ double grp_solve64(const Grp<NSP>& x, const LU<NSP>& F, double b) {
    if (F.swp) b = __shfl(b, F.src, 64);                // the row interchanges of the factorisation
    const int gl = ct_row(x.gl);                        // see grp_lu64
#pragma unroll
    for (int k = 0; k < NSP; ++k) {
        if (k < x.NS) {
            const double bk = rlane(b, k);
            b = fma((gl > k) ? -F.W[k] : 0.0, bk, b);   // a select: exec-mask branches measured 2 % slower
        }
    }
#pragma unroll
    for (int kk = 0; kk < NSP; ++kk) {
        const int k = NSP - 1 - kk;
        if (k < x.NS) {
            const double xk = rlane(b * F.W[k], k);
            b = fma((gl < k) ? -F.W[k] : 0.0, xk, b);
            if (gl == k) b = xk;
        }
    }
    return x.row ? b : 0.0;
}

#ifndef PCK_GRP_READLANE
#define PCK_GRP_READLANE 1
#endif
template <int NSP, int G>
__device__ __forceinline__ bool grp_lu(const Grp<NSP>& x, LU<NSP>& F) {
    if constexpr (G == 16 && NSP <= 16) return grp_lu16<NSP>(x, F);
    // (exact-size hipRTC kernels only: the padded compiled-in fallback keeps
    // the partial-pivoting form, whose unrolled interchanges at run-time NS
    // took the split build's 64-lane unit past 10 minutes)
    if constexpr (G == 64 && PCK_GRP_TPIV64 && PCK_GRP_EXACT) return grp_lu64<NSP>(x, F);
    bool fre = x.row;
    bool ok = true;
    F.step = NSP;
#pragma unroll
    for (int k = 0; k < NSP; ++k) {
        if (k < x.NS) {
            const float mag = (float)fabs(F.W[k]);
            int key = fre ? (int)((__float_as_uint(mag) & ~63u) | (uint32_t)x.gl) : -1;
            key = gmaxi<G>(key);
            const int p = key & 63;
            if constexpr (G == 64 && PCK_GRP_READLANE) {
                // full wavefront: the pivot row is read straight out of the
                // pivot lane's registers (v_readlane into SGPRs, used as the
                // scalar operand of the FMAs) -- no LDS round trip, no copy
                const int ps = __builtin_amdgcn_readfirstlane(p);
                const double piv = gbcast<64>(F.W[k], ps);
                ok = ok && key >= 0 && piv != 0.0 && isfinite(piv);
                const bool elim = ok && fre && x.gl != ps;
                if (x.gl == ps) {
                    F.W[k] = rcp(F.W[k]);
                    fre = false;
                    F.step = k;
                }
                if (elim) {
                    const double l = F.W[k] * rcp(piv);
                    F.W[k] = l;
#pragma unroll
                    for (int j = k + 1; j < NSP; ++j) F.W[j] -= l * gbcast<64>(F.W[j], ps);
                }
            } else {
                wsync();                           // readers of the previous pivot row are done
                if (x.gl == p) {
#pragma unroll
                    for (int j = k; j < NSP; ++j) x.pb[j - k] = F.W[j];
                }
                wsync();
                const double piv = x.pb[0];
                ok = ok && key >= 0 && piv != 0.0 && isfinite(piv);
                if (x.gl == p) {
                    F.W[k] = rcp(F.W[k]);
                    fre = false;
                    F.step = k;
                }
                if (ok && fre) {
                    const double l = F.W[k] * rcp(piv);
                    F.W[k] = l;
#pragma unroll
                    for (int j = k + 1; j < NSP; ++j) F.W[j] -= l * x.pb[j - k];
                }
            }
            F.pk.set(k, p);
        }
    }
    return ok;
}

// Solve (LU) x = b for the group; b_i on lane i in, x_i on lane i out.
template <int NSP, int G>
__device__ __forceinline__ double grp_solve(const Grp<NSP>& x, const LU<NSP>& F, double b) {
    if constexpr (G == 16 && NSP <= 16) return grp_solve16<NSP>(x, F, b);
    if constexpr (G == 64 && PCK_GRP_TPIV64 && PCK_GRP_EXACT) return grp_solve64<NSP>(x, F, b);
#pragma unroll
    for (int k = 0; k < NSP; ++k) {
        if (k < x.NS) {
            const double bk = gbcast<G>(b, F.pk.get(k));
            if (F.step > k) b -= F.W[k] * bk;
        }
    }
    double out = 0.0;
#pragma unroll
    for (int kk = 0; kk < NSP; ++kk) {
        const int k = NSP - 1 - kk;
        if (k < x.NS) {
            const double xk = gbcast<G>(b * F.W[k], F.pk.get(k));
            if (F.step < k) b -= F.W[k] * xk;
            if (x.gl == k) out = xk;
        }
    }
    return x.row ? out : 0.0;
}

// ---------------------------------------------------------------------------
// RODAS4P on the group (same scheme, controller, projection and positivity
// rule as mk_solver.h: integrate)
// ---------------------------------------------------------------------------
// removal of the stage increments' conserved-total drift along y (see grp_integrate)
#ifndef PCK_GRP_KPROJ
#define PCK_GRP_KPROJ 1
#endif
template <int NSP, int G, int P, bool TRAJ = false, class Net = NoNet>
__device__ __forceinline__ int grp_integrate(const NetView& nv, const GrpView& gv, const Grp<NSP>& x, double& y,
                                             double t0, double t_end, double rtol, double atol, int max_steps,
                                             int& nsteps, bool crows, const TrajOut& to, LU<NSP>& F) {
    using namespace rodas4;
    constexpr bool CLAMP = PCK_GRP_CLAMP && G == 64;    // see put_c
    const int NS = x.NS;
    int ko = 0;
    if constexpr (TRAJ) {                       // samples at or before t0: the initial state
        for (; ko < to.n && to.t[ko] <= t0; ++ko)
            if (x.row) to.y[((int64_t)ko * NS + x.gl) * to.ld + to.c] = y;
    }
    const double invNS = 1.0 / NS;
    nsteps = 0;
    const double span = t_end - t0;
    if (!(span > 0.0)) {
        if constexpr (TRAJ) {
            for (; ko < to.n; ++ko)
                if (x.row) to.y[((int64_t)ko * NS + x.gl) * to.ld + to.c] = y;
        }
        return PCK_ST_OK;
    }
    double F0 = grp_rhs<NSP, G, CLAMP, Net>(gv, x, y);
    double cons0[PCK_MAX_CONS];
    double ci[PCK_MAX_CONS];
    bool cpos[PCK_MAX_CONS];
#pragma unroll
    for (int l = 0; l < PCK_MAX_CONS; ++l) {
        if (l < nv.NCONS) {
            ci[l] = x.row ? nv.C[l * NS + x.gl] : 0.0;
            cons0[l] = gsum<G>(ci[l] * y);
            cpos[l] = gmin<G>(ci[l]) >= 0.0;
        }
    }
    // stage increments keep the conserved totals (PCK_GRP_KPROJ): C k = 0
    // holds exactly for the ODE (C f = 0, C J = 0), but in floating point
    // C f is the rounding of the species balances, ~eps x the gross fluxes
    // (1e11 / s on DMTM), and the stage solve multiplies it by h g along the
    // Jacobian's null direction -- at h ~ 1e9 s on a steady state that drift
    // swamps the tolerance and the step is rejected over and over.  The
    // drift is removed along y restricted to the law's own species (the
    // direction of the multiplicative projection after the step, so a
    // species' correction scales with its size, and a species outside the law
    // -- a CSTR gas, another site type -- is left alone); an orthogonal
    // projection spreads the large species' rounding onto the tiny ones and
    // stalls the solve (tools/rodas_mirror.py KPROJ).
    double icy[PCK_MAX_CONS];                  // this lane's y / (c . y) on the law's species, else 0
    auto kproj = [&](double k) {
        if (PCK_GRP_KPROJ && !crows) {
#pragma unroll
            for (int l = 0; l < PCK_MAX_CONS; ++l)
                if (l < nv.NCONS && cpos[l]) k -= gsum<G>(ci[l] * k) * icy[l];
        }
        return k;
    };
    double h;
    {
        const double sc = atol + rtol * fabs(y);
        const double d0 = sqrt(gsum<G>(x.row ? (y / sc) * (y / sc) : 0.0) * invNS);
        const double d1 = sqrt(gsum<G>(x.row ? (F0 / sc) * (F0 / sc) : 0.0) * invNS);
        double h0 = (d0 < 1e-5 || d1 < 1e-5) ? 1e-6 : 0.01 * d0 / d1;
        h0 = fmin(h0, span);
        const double F1 = grp_rhs<NSP, G, CLAMP, Net>(gv, x, y + h0 * F0);
        const double q = (F1 - F0) / sc;
        const double d2 = sqrt(gsum<G>(x.row ? q * q : 0.0) * invNS) / h0;
        const double h1 = (d1 <= 1e-15 && d2 <= 1e-15) ? fmax(1e-6, h0 * 1e-3) : pow(0.01 / fmax(d1, d2), 0.2);
        h = fmin(fmin(100.0 * h0, h1), span);
    }
    double t = t0;
    int blowups = 0;
    int stall = 0;
    int cpv = -1;                                              // conservation law whose pivot row is this lane's
    for (int l = 0; l < nv.NCONS; ++l)
        if (crows && x.row && nv.cpiv[l] == x.gl) cpv = l;
    const double keep = (cpv >= 0) ? 0.0 : 1.0;                // its stage right-hand sides are 0
    while (t < t_end) {
        if (nsteps >= max_steps) return PCK_ST_MAXSTEPS;
        ++nsteps;
        bool last = false;
        if (t + h >= t_end) { h = t_end - t; last = true; }
        const double ih = rcp(h);
        const double ig = ih * (1.0 / g);
#ifdef PCK_TRACE
        const bool tr = (x.cidx == pck_trace_cond) && x.gl == 0;
        if (tr) pck_phase[5] += 1.0;
#endif
        PCK_PH(0, (grp_jac<NSP, G, P, CLAMP, Net>(nv, gv, x, y, -1.0, ig, F.W)));       // W = I/(h g) - J
        if (cpv >= 0) {                                        // conservation rows (mk_solver.h: cons_rows)
            double m = 0.0;
#pragma unroll
            for (int q = 0; q < NSP; ++q) m = fmax(m, fabs(F.W[q]));
#pragma unroll
            for (int q = 0; q < NSP; ++q) F.W[q] = (q < NS) ? nv.C[cpv * NS + q] * m : 0.0;
        }
#ifdef PCK_TRACE
        const double ymin = gmin<G>(x.row ? y : INFINITY);
        auto trace = [&](double q, double luok) {
            if (!tr) return;
            const int pos = pck_trace_pos % PCK_TRACE_N;
            double* rec = pck_trace_buf + (size_t)pos * PCK_TRACE_W;
            rec[0] = nsteps; rec[1] = t; rec[2] = h; rec[3] = q; rec[4] = luok; rec[5] = ymin;
            rec[6] = F0; rec[7] = y;
            pck_trace_pos = pck_trace_pos + 1;
        };
#else
        auto trace = [&](double, double) {};
#endif
        bool luok;
        PCK_PH(1, (luok = grp_lu<NSP, G>(x, F)));
        if (!luok) {
            trace(-1.0, 0.0);
            h *= 0.25;
            if (!(h > 2.220446049250313e-15 * fmax(fabs(t), 1e-300))) return PCK_ST_STEPFAIL;
            continue;
        }
        if (PCK_GRP_KPROJ && !crows) {
#pragma unroll
            for (int l = 0; l < PCK_MAX_CONS; ++l) {
                if (l < nv.NCONS && cpos[l]) {
                    const double cy = gsum<G>(ci[l] * y);
                    icy[l] = (cy > 0.0 && ci[l] != 0.0) ? y / cy : 0.0;
                }
            }
        }
        double k1, k2, k3, k4, k5, k6, fu, u;
        if constexpr (IsCt<Net>::v) {
            // the straight-line network code is large: one rhs and one solve
            // site for the five stages (the same stage formulas, unused
            // coefficients zero; u_6 = u_5 + k5 as a sixth row)
            PCK_PH(2, (k1 = kproj(grp_solve<NSP, G>(x, F, keep * F0))));
            k2 = k3 = k4 = k5 = k6 = 0.0;
#pragma unroll 1
            for (int st = 2; st <= 6; ++st) {
                double b1, b2, b3, b4, b5, e1, e2, e3, e4, e5;
                switch (st) {
                    case 2: b1 = a21; b2 = b3 = b4 = b5 = 0.0; e1 = C21; e2 = e3 = e4 = e5 = 0.0; break;
                    case 3: b1 = a31; b2 = a32; b3 = b4 = b5 = 0.0; e1 = C31; e2 = C32; e3 = e4 = e5 = 0.0; break;
                    case 4: b1 = a41; b2 = a42; b3 = a43; b4 = b5 = 0.0; e1 = C41; e2 = C42; e3 = C43; e4 = e5 = 0.0; break;
                    case 5: b1 = a51; b2 = a52; b3 = a53; b4 = a54; b5 = 0.0; e1 = C51; e2 = C52; e3 = C53; e4 = C54;
                            e5 = 0.0; break;
                    default: b1 = a51; b2 = a52; b3 = a53; b4 = a54; b5 = 1.0; e1 = C61; e2 = C62; e3 = C63; e4 = C64;
                             e5 = C65; break;
                }
                u = y + b1 * k1 + b2 * k2 + b3 * k3 + b4 * k4 + b5 * k5;
                PCK_PH(3, (fu = grp_rhs<NSP, G, CLAMP, Net>(gv, x, u)));
                double kn;
                PCK_PH(2, (kn = kproj(grp_solve<NSP, G>(x, F, keep * (fu + ih * (e1 * k1 + e2 * k2 + e3 * k3 +
                                                                                 e4 * k4 + e5 * k5))))));
                k2 = (st == 2) ? kn : k2;
                k3 = (st == 3) ? kn : k3;
                k4 = (st == 4) ? kn : k4;
                k5 = (st == 5) ? kn : k5;
                k6 = (st == 6) ? kn : k6;
            }
        } else {
        PCK_PH(2, (k1 = kproj(grp_solve<NSP, G>(x, F, keep * F0))));
        PCK_PH(3, (fu = grp_rhs<NSP, G, CLAMP, Net>(gv, x, y + a21 * k1)));
        PCK_PH(2, (k2 = kproj(grp_solve<NSP, G>(x, F, keep * (fu + ih * (C21 * k1))))));
        PCK_PH(3, (fu = grp_rhs<NSP, G, CLAMP, Net>(gv, x, y + a31 * k1 + a32 * k2)));
        PCK_PH(2, (k3 = kproj(grp_solve<NSP, G>(x, F, keep * (fu + ih * (C31 * k1 + C32 * k2))))));
        PCK_PH(3, (fu = grp_rhs<NSP, G, CLAMP, Net>(gv, x, y + a41 * k1 + a42 * k2 + a43 * k3)));
        PCK_PH(2, (k4 = kproj(grp_solve<NSP, G>(x, F, keep * (fu + ih * (C41 * k1 + C42 * k2 + C43 * k3))))));
        u = y + a51 * k1 + a52 * k2 + a53 * k3 + a54 * k4;
        PCK_PH(3, (fu = grp_rhs<NSP, G, CLAMP, Net>(gv, x, u)));
        PCK_PH(2, (k5 = kproj(grp_solve<NSP, G>(x, F, keep * (fu + ih * (C51 * k1 + C52 * k2 + C53 * k3 +
                                                                          C54 * k4))))));
        u += k5;
        PCK_PH(3, (fu = grp_rhs<NSP, G, CLAMP, Net>(gv, x, u)));
        PCK_PH(2, (k6 = kproj(grp_solve<NSP, G>(x, F, keep * (fu + ih * (C61 * k1 + C62 * k2 + C63 * k3 +
                                                                          C64 * k4 + C65 * k5))))));
        }
        double d2 = 0.0, d3 = 0.0;                 // dense output (mk_solver.h: rodas4_dense)
        if constexpr (TRAJ) {
            using namespace rodas4_dense;
            d2 = D21 * k1 + D22 * k2 + D23 * k3 + D24 * k4 + D25 * k5;
            d3 = D3_K5_ONLY ? D35 * k5 : D31 * k1 + D32 * k2 + D33 * k3 + D34 * k4 + D35 * k5;
        }
        u += k6;
        const double sc = atol + rtol * fmax(fabs(y), fabs(u));
        const double r = k6 * __builtin_amdgcn_rcp(sc);     // error weight: the v_rcp_f64 estimate suffices
        // the finiteness test rides on the error sum: a non-finite stage value
        // makes u (which includes k6) non-finite, and 0 * (inf or NaN) is NaN;
        // for finite u the added term is an exact zero
        const double s = gsum<G>(x.row ? r * r + 0.0 * u : 0.0);
        const double fin = (s == s) ? 1.0 : 0.0;
        const double q = (fin > 0.0) ? s * invNS : INFINITY;     // en^2
        // positivity (mass-action concentrations stay >= -atol): a step that
        // drives a component below -atol is rejected and retried at the
        // fraction of the step where that component reaches -atol
        const double pf = (PCK_POSITIVITY && !CLAMP) ? gmin<G>((x.row && u < -atol) ? (y + atol) / (y - u) : 1.0) : 1.0;
        const double fac = step_factor(q);
        trace(q, 1.0);
        if (q <= 1.0 && pf >= 1.0) {
            const double t_old = t, y_old = y;
            t = last ? t_end : t + h;
            // clamped-state rates: a negative component enters every rate as
            // 0, so the clamped flow never leaves y >= 0 and a negative is
            // discretisation error.  A tolerance-level one (>= -atol) kept
            // makes the state and the Jacobian (taken at max(y, 0)) disagree
            // for good: on synthetic condition 39547 a -5e-11 component held
            // the error estimate at the controller's fixed point (en^2 =
            // 0.9^8, h = 0.034 s) for 99 160 steps
            // (profiles/r2/synthetic/trace_39547.log).  Set to 0 it changes
            // no rate -- they already saw 0.  It is a rescue, applied only to
            // a solve already past PCK_CLAMP_CLIP_AFTER steps (the synthetic
            // network's p99 is ~1 800): applied from the first step it turned
            // 0.14 % of 1e6 conditions into step failures; zeroing larger
            // negatives too left 239 of 512 at the step budget.
            const bool clip = CLAMP && nsteps > PCK_CLAMP_CLIP_AFTER;
            y = x.row ? ((clip && u < 0.0 && u >= -atol) ? 0.0 : u) : 0.0;
#pragma unroll
            for (int l = 0; l < PCK_MAX_CONS; ++l) {
                if (l < nv.NCONS) {
                    const double sm = gsum<G>(ci[l] * y);
                    if (cpos[l] && sm > 0.0) {
                        const double fct = cons0[l] * rcp(sm);
                        if (ci[l] != 0.0) y *= fct;
                    }
                }
            }
            if constexpr (TRAJ) {
                for (; ko < to.n && to.t[ko] <= t; ++ko) {
                    const double sv = fmin((to.t[ko] - t_old) / h, 1.0), s1 = 1.0 - sv;
                    if (x.row)
                        to.y[((int64_t)ko * NS + x.gl) * to.ld + to.c] =
                            y_old * s1 + sv * (y + s1 * (d2 + sv * d3));
                }
            }
            PCK_PH(3, (F0 = grp_rhs<NSP, G, CLAMP, Net>(gv, x, y)));
            // falling tolerance-level negatives to 0 (mk_solver.h: integrate)
            const bool negf = x.row && y < 0.0 && F0 < 0.0;
            if (PCK_POSITIVITY && !CLAMP && gmaxi<G>(negf ? 1 : 0) > 0) {
                if (negf) y = 0.0;
                PCK_PH(3, (F0 = grp_rhs<NSP, G, CLAMP, Net>(gv, x, y)));
            }
            h *= fmin(PCK_FACMAX, fmax(0.2, fac));
        } else if (q <= 1.0) {
            h *= fmax(0.1, 0.9 * pf);
        } else {
            h *= (fin > 0.0) ? fmax(0.2, fac) : 0.25;
            // a step whose error is 1e6x the tolerance (or not finite) means
            // I/(h g) - J was near singular -- the step size sits on an
            // explosive mode of J; a solve that keeps growing h back into it
            // cannot advance (scipy BDF stops with "step size less than
            // spacing" on the same conditions)
            if (!(q < PCK_BLOWUP_Q) && h < 1e-4 * t && ++blowups > PCK_MAX_BLOWUPS) return PCK_ST_STEPFAIL;
        }
        stall = (h < PCK_STALL_H * (t - t0)) ? stall + 1 : 0;
        if (stall > PCK_STALL_STEPS) return PCK_ST_STEPFAIL;
        // scipy's BDF limit: a step below 10 ulp(t) is a failure
        if (!(h > 2.220446049250313e-15 * fmax(fabs(t), 1e-300)) && t < t_end) return PCK_ST_STEPFAIL;
    }
    if constexpr (TRAJ) {                       // samples past t_end (rounding of the caller's grid)
        for (; ko < to.n; ++ko)
            if (x.row) to.y[((int64_t)ko * NS + x.gl) * to.ld + to.c] = y;
    }
    return PCK_ST_OK;
}

// forward + reverse rate of a record's reaction (its gross flux)
__device__ __forceinline__ double rec_gross(const uint4& rec, double a, double b, const double* c) {
#pragma unroll
    for (int k = 0; k < PCK_GRP_NPMAX; ++k) {
        const int f = rx_field(rec, k);
        const double x = c[f & 63];
        const int ef = (f >> 6) & 31, er = f >> 11;
        a *= spow(x, ef);
        b *= spow(x, er);
    }
    return fabs(a) + fabs(b);
}

// mk_solver.h: imbalance -- the largest |f_i| / gross_i over the rows that are
// not conservation pivots (group-uniform); f = the row's rate (grp_rhs)
template <int NSP, int G, class Net = NoNet>
__device__ __forceinline__ double grp_imbalance(const NetView& nv, const GrpView& g, const Grp<NSP>& x, double y,
                                                double& f) {
    if constexpr (IsCt<Net>::v) {
        double gr = 0.0;
        f = ct_rhs<Net, NSP, G, false, true>(x, y, &gr);
        bool pv = false;
        for (int l = 0; l < nv.NCONS; ++l) pv = pv || (nv.cpiv[l] == x.gl);
        return gmax<G>((x.row && !pv && f != 0.0) ? fabs(f) / gr : 0.0);
    }
    f = grp_rhs<NSP, G>(g, x, y);
    wsync();                                   // the rows' reads of the net rates are done
    for (int r = x.gl; r < x.R; r += G) x.d[r] = rec_gross(g.rx[r], x.kf[r], x.kr[r], x.c);
    wsync();
    double gr = 0.0;
    if (x.row) {
        for (int e = x.rb; e < x.re; ++e) {
            const uint4 q = g.ent[e];
            gr += fabs(ent_s(q)) * x.d[ent_r(q)];
        }
        gr = gr * fabs(x.rs) + fabs(x.fl) * (fabs(x.in) + fabs(y));
    }
    bool pv = false;
    for (int l = 0; l < nv.NCONS; ++l) pv = pv || (nv.cpiv[l] == x.gl);
    return gmax<G>((x.row && !pv && f != 0.0) ? fabs(f) / gr : 0.0);
}

template <int NSP, int G, class Net = NoNet>
__device__ __forceinline__ bool grp_resolved(const NetView& nv, const GrpView& g, const Grp<NSP>& x, double y) {
    double f;
    return grp_imbalance<NSP, G, Net>(nv, g, x, y, f) <= PCK_BALANCE_TOL;
}

// Newton steady-state polish (same rules as mk_solver.h: newton)
template <int NSP, int G, int P, class Net = NoNet>
__device__ __forceinline__ int grp_newton(const NetView& nv, const GrpView& gv, const Grp<NSP>& x, double& y,
                                          int iters, LU<NSP>& F, double dist, double atol) {
    const int NS = x.NS;
    double b[PCK_MAX_CONS], ci[PCK_MAX_CONS];
    int piv_l[PCK_MAX_CONS];
#pragma unroll
    for (int l = 0; l < PCK_MAX_CONS; ++l) {
        if (l < nv.NCONS) {
            ci[l] = x.row ? nv.C[l * NS + x.gl] : 0.0;
            b[l] = gsum<G>(ci[l] * y);
            piv_l[l] = nv.cpiv[l];
        }
    }
    double z = y, z_prev = y, bal_prev = INFINITY;
    double scl = 1.0;                          // this row's scale in the last factorisation (F)
    bool conv = false;
    double prev = INFINITY, lastq = 1.0;
    int linear = 0;
    bool pv = false;
#pragma unroll
    for (int l = 0; l < PCK_MAX_CONS; ++l) pv = pv || (l < nv.NCONS && x.gl == piv_l[l]);
    // mk_solver.h: newton_pinned -- a species at exactly 0 with an exactly
    // zero rate at the transient end is held at 0 (its Newton steps dropped)
    bool pin = false;
    for (int it = 0; it < iters; ++it) {
        double Gv;
        // the rounding floor (mk_solver.h: PCK_BALANCE_CONV)
        const double bal = grp_imbalance<NSP, G, Net>(nv, gv, x, z, Gv);
        if (it == 0) pin = x.row && !pv && z == 0.0 && Gv == 0.0;
        if (it >= 2 && bal_prev <= PCK_BALANCE_CONV && bal > bal_prev) { z = z_prev; conv = true; break; }
        bal_prev = bal;
        z_prev = z;
        grp_jac<NSP, G, P, false, Net>(nv, gv, x, z, 1.0, 0.0, F.W);
#pragma unroll
        for (int l = 0; l < PCK_MAX_CONS; ++l) {
            if (l < nv.NCONS) {
                const double s = gsum<G>(ci[l] * z);
                if (x.gl == piv_l[l]) {
                    Gv = s - b[l];
#pragma unroll
                    for (int q = 0; q < NSP; ++q) F.W[q] = (q < NS) ? nv.C[l * NS + q] : 0.0;
                }
            }
        }
        // row equilibration (rate rows up to 1e9, conservation rows O(1))
        double m = 0.0;
#pragma unroll
        for (int q = 0; q < NSP; ++q) m = fmax(m, fabs(F.W[q]));
        scl = (m > 0.0) ? 1.0 / m : 1.0;
#pragma unroll
        for (int q = 0; q < NSP; ++q) F.W[q] *= scl;
        Gv = -Gv * scl;
        if (!grp_lu<NSP, G>(x, F)) break;
        double dz = grp_solve<NSP, G>(x, F, Gv);
        if (pin) dz = 0.0;
        double alpha = 1.0;
        if (linear >= 2 && lastq < 0.9) {
            alpha = fmin(4.0, 1.0 / (1.0 - lastq));
            const double cand = (x.row && dz < 0.0 && z > 0.0) ? 0.9 * z / -dz : INFINITY;
            alpha = fmax(fmin(alpha, gmin<G>(cand)), 1.0);
        }
        dz *= alpha;
        z += dz;
        const double fin = gmin<G>((!x.row || isfinite(z)) ? 1.0 : 0.0);
        if (!(fin > 0.0)) break;
        const double zmax = gmax<G>(x.row ? fabs(z) : 0.0);
        const double rel = gmax<G>(x.row ? fabs(dz) / fmax(fabs(z), 1e-12 * zmax + 1e-300) : 0.0);
        if (prev < PCK_STEP_FLOOR && rel > prev) { z = z_prev; conv = true; break; }   // mk_solver.h: the step floor
        if (rel < 1e-12 || (it >= 2 && rel < 1e-7 && rel > 0.5 * prev)) { conv = true; break; }
        lastq = rel / prev;
        linear = (rel > 0.25 * prev) ? linear + 1 : 0;
        if (linear >= 12) break;
        prev = rel;
    }
    if (!conv) return PCK_ST_NEWTON;
    if (PCK_NEWTON_REFINE > 0) {
        // residual refinement (mk_solver.h: newton), on the loop's last
        // factorisation (F) and row scale: a second Jacobian and LU in this
        // kernel took CH4 from 197 to 256 VGPRs and DMTM from 3 to 2 waves
        // per SIMD.  A Jacobian one step old converges linearly at a rate of
        // that step times the condition; steps above PCK_REFINE_MAXSTEP are
        // refused.
        double nprev = INFINITY, zp = z;
#pragma unroll 1
        for (int r = 0; r <= PCK_NEWTON_REFINE; ++r) {
            double Gv = grp_rhs_dd<NSP, G, Net>(nv, gv, x, z);
#pragma unroll
            for (int l = 0; l < PCK_MAX_CONS; ++l) {
                if (l < nv.NCONS) {
                    const dd s = dd_add(gsum_dd<G>(two_prod(ci[l], z)), dd_of(-b[l]));
                    if (x.gl == piv_l[l]) Gv = s.hi + s.lo;
                }
            }
            Gv = -Gv * scl;
            const double nr = gmax<G>(x.row ? fabs(Gv) : 0.0);
            if (!(nr < nprev)) {                        // no longer falling: the previous iterate
                if (r > 0) z = zp;
                break;
            }
            nprev = nr;
            if (r == PCK_NEWTON_REFINE || nr == 0.0) break;
            const double dz = pin ? 0.0 : grp_solve<NSP, G>(x, F, Gv);
            const double zmax = gmax<G>(x.row ? fabs(z) : 0.0);
            const double rel = gmax<G>(x.row ? fabs(dz) / fmax(fabs(z), 1e-12 * zmax + 1e-300) : 0.0);
            zp = z;
            z += dz;
            if (!(gmin<G>((!x.row || isfinite(z)) ? 1.0 : 0.0) > 0.0) || !(rel <= PCK_REFINE_MAXSTEP)) {
                z = zp;
                break;
            }
        }
    }
    if (gmin<G>((x.row && z < 0.0) ? -1.0 : 1.0) < 0.0) return PCK_ST_NEWTON;
    if (!grp_resolved<NSP, G, Net>(nv, gv, x, z)) return PCK_ST_NEWTON;   // converged in absolute terms only
    // mk_solver.h: newton -- the root only if the transient end reached it
    if (dist > 0.0 && gmin<G>((x.row && !(fabs(z - y) <= dist * fabs(z) + atol)) ? -1.0 : 1.0) < 0.0)
        return PCK_ST_NEWTON;
    y = z;
    return PCK_ST_OK;
}

// ---------------------------------------------------------------------------
// group setup + kernels
// ---------------------------------------------------------------------------
template <int NSP, int G>
__device__ __forceinline__ void grp_setup(const NetView& nv, const GrpView& gv, const CondView& cv, int64_t c,
                                          const double* kf, const double* kr, int64_t ld_k, int pj, double pfac,
                                          double* base, int QB, Grp<NSP>& x, double& T) {
    const int R = nv.NRXN;
    const int r1 = R > 0 ? R : 1;
    x.gl = threadIdx.x % G;
    x.cidx = c;
    x.NS = PCK_GRP_EXACT ? NSP : nv.NDYN;   // hipRTC kernels are instantiated at the network's exact size
    x.R = R;
    x.QB = QB;
    x.row = x.gl < x.NS;
    x.kf = base;
    x.kr = x.kf + grp_even(r1);
    x.c = x.kr + grp_even(r1);
    x.d = x.c + grp_even(NSP);
    x.J = x.d + grp_even(gv.ND > r1 ? gv.ND : r1);
    x.pb = x.J + grp_even(x.NS * QB);
    x.Jx = x.pb + grp_even(NSP);
    x.part = x.Jx + grp_even(gv.NX * x.NS);
    x.xb = x.xe = 0;
    if (gv.LS) {
        for (int i = x.gl; i < gv.NX * x.NS; i += G) x.Jx[i] = 0.0;
        if (x.gl < x.NS) { x.xb = gv.xbe[2 * x.gl]; x.xe = gv.xbe[2 * x.gl + 1]; }
    }
    T = cv.T[c * cv.sT];
    for (int j = x.gl; j < R; j += G) {
        double a = kf[j * ld_k + c], b = kr[j * ld_k + c];
        for (int q = 0; q < nv.NFIX; ++q) {
            const int ea = nv.foldf[j * nv.NFIX + q], eb = nv.foldr[j * nv.NFIX + q];
            if (ea | eb) {
                const double v = cv.fixc[q * cv.ld_fix + c * cv.s_fix];
                if (ea) a *= ipow(v, ea);
                if (eb) b *= ipow(v, eb);
            }
        }
        if (j == pj) { a *= pfac; b *= pfac; }   // old_system.py:504-506
        x.kf[j] = a;
        x.kr[j] = b;
    }
    x.cfi = x.rs = x.fl = x.in = 0.0;
    x.rb = x.re = 0;
    if (x.row) {
        for (int j = 0; j < QB; ++j) x.J[x.gl * QB + j] = 0.0;
        const double* d = nv.dyn + 4 * x.gl;
        x.cfi = d[0];
        x.rs = (d[2] != 0.0) ? d[1] + d[2] * T : d[1];   // reactor.py:34-41
        x.fl = d[3];
        if (x.fl != 0.0 && cv.inflow) x.in = cv.inflow[x.gl * cv.ld_in + c * cv.s_in];
        x.rb = gv.row[x.gl];
        x.re = gv.row[x.gl + 1];
    }
    wsync();
}

// TOF of the group's state (old_system.py:482-488), valid on every lane
template <int NSP, int G>
__device__ __forceinline__ double grp_tof(const NetView& nv, const GrpView& g, const Grp<NSP>& x, double y) {
    put_c(x, y);
    double t = 0.0;
    for (int k = x.gl; k < nv.NTOF; k += G) {
        const int r = nv.tof[k];
        t += rec_rate(g.rx[r], x.kf[r], x.kr[r], x.c);
    }
    return gsum<G>(t);
}

struct GrpArgs {
    int M;              // groups per condition: 1, or 2R+1 in DRC mode
    int QB;             // Jacobian column block (= ceil(NSP / P))
    double* tofbuf;     // DRC mode: [M][n] TOF per perturbation
    int32_t* stbuf;     // DRC mode: [M][n] status per perturbation
    int32_t* nsbuf;     // DRC mode: [M][n] integrator steps per perturbation
};

// occupancy floor of the 64-lane-group solver (waves per SIMD; the VGPR
// budget follows: 2 -> 256 VGPRs, the NS = 50 kernel then spills in the
// Newton polish); PCK_GRP_WAVES16 the same for 16/32-lane groups (3 -> 168
// VGPRs: measured 20 % slower on CH4 than the unconstrained allocation)
#ifndef PCK_GRP_WAVES
#define PCK_GRP_WAVES 1
#endif
#ifndef PCK_GRP_WAVES16
#define PCK_GRP_WAVES16 1
#endif
template <int NSP, int G, int P, bool TRAJ = false, bool TAB = false, class Net = NoNet>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(G == 64 ? PCK_GRP_WAVES : PCK_GRP_WAVES16))) k_solve_grp(NetView nv, GrpView gv, CondView cv, const double* kf,
                                                  const double* kr, int64_t ld_k, SolveArgs a, GrpArgs ga) {
    extern __shared__ double lds[];
#if PCK_POISON_LDS
    {   // diagnostic builds: the whole dynamic LDS block starts as NaN (mk_solver.h: k_solve)
        const size_t nd = (TAB ? grp_tab_doubles(nv.NRXN, gv.NE, nv.NDYN, gv.LS * G) : 0) +
                          (size_t)(64 / G) * grp_lds_doubles(nv.NRXN, NSP, nv.NDYN, gv.ND, ga.QB, gv.LS, gv.NX);
        for (size_t i = threadIdx.x; i < nd; i += 64) lds[i] = __builtin_nan("");
        wsync();
    }
#endif
    const int grp = threadIdx.x / G;
    const int64_t v = (int64_t)blockIdx.x * (64 / G) + grp;
    const int64_t slot = cond_of(a, v, ga.M, cv.n);
    const int q = (int)(v % ga.M);
    const int R1 = nv.NRXN > 0 ? nv.NRXN : 1, NE1 = gv.NE > 0 ? gv.NE : 1;
    GrpView gl = gv;                                // TAB: the tables, copied to LDS by the whole block (one wave)
    if constexpr (TAB) {
        uint4* trx = (uint4*)lds;
        uint4* tent = trx + R1;
        int32_t* trow = (int32_t*)(tent + NE1);
        for (int i = threadIdx.x; i < nv.NRXN; i += 64) trx[i] = gv.rx[i];
        for (int i = threadIdx.x; i < gv.NE; i += 64) tent[i] = gv.ent[i];
        for (int i = threadIdx.x; i <= nv.NDYN; i += 64) trow[i] = gv.row[i];
        uint32_t* tsch = (uint32_t*)(trow + nv.NDYN + 1);
        for (int i = threadIdx.x; i < gv.LS * G; i += 64) tsch[i] = gv.sch[i];
        wsync();
        gl.rx = trx;
        gl.ent = tent;
        gl.row = trow;
        if (gv.LS) gl.sch = tsch;
    }
    if (slot >= cv.n) return;                       // group-uniform exit; no block barriers below
    const int64_t c = slot;
    int pj = -1;
    double pfac = 1.0;
    if (q > 0) { pj = (q - 1) >> 1; pfac = (q & 1) ? 1.0 + a.eps : 1.0 - a.eps; }
    Grp<NSP> x;
    double T;
    grp_setup<NSP, G>(nv, gl, cv, c, kf, kr, ld_k, pj, pfac,
                      lds + (TAB ? grp_tab_doubles(nv.NRXN, gv.NE, nv.NDYN, gv.LS * G) : 0) +
                          (size_t)grp * grp_lds_doubles(nv.NRXN, NSP, nv.NDYN, gv.ND, ga.QB, gv.LS, gv.NX), ga.QB, x, T);
    double y = 0.0;
    int ns = 0;
    TrajOut to{a.t_out, a.n_out, a.traj, a.ld_traj, c};
    LU<NSP> F;                  // one factorisation storage for the transient and the Newton polish
    // transient and polish (a degenerate root's retry transient is a second
    // launch over the compacted list, mk_solver.h: SolveArgs::idx); with the
    // screening pass (SolveArgs::screen_rtol, mk_solver.h: solve_lane) first
    // the rule at the screening tolerance, and the full solve only where it
    // is not accepted (the decision is group-uniform)
    int st = PCK_ST_NEWTON;
    bool done = false;
    // (64-lane groups run the single pass: screening is a small-network
    // optimisation -- System.solve_batch screens networks of at most 8
    // species -- and a second inlined integrator doubles the 64-lane kernel's
    // code, whose unrolled LU and substitutions are most of it)
    if (!TRAJ && G != 64 && a.screen_rtol > 0.0) {
        y = x.row ? cv.y0[x.gl * cv.ld_y0 + c * cv.s_y0] : 0.0;
        st = grp_integrate<NSP, G, P, TRAJ, Net>(nv, gl, x, y, a.t0, a.t_end, a.screen_rtol, a.screen_atol,
                                                 a.screen_max_steps, ns, a.cons_rows != 0, to, F);
        if (st == PCK_ST_OK && a.newton)
            st = grp_newton<NSP, G, P, Net>(nv, gl, x, y, a.newton_iters, F, a.screen_dist, a.atol);
        done = (st == PCK_ST_OK);
    }
    if (!done) {
        int nsp = 0;
        y = x.row ? cv.y0[x.gl * cv.ld_y0 + c * cv.s_y0] : 0.0;
        st = grp_integrate<NSP, G, P, TRAJ, Net>(nv, gl, x, y, a.t0, a.t_end, a.rtol, a.atol, a.max_steps, nsp,
                                                 a.cons_rows != 0, to, F);
        if (st == PCK_ST_OK && a.newton)
            st = grp_newton<NSP, G, P, Net>(nv, gl, x, y, a.newton_iters, F, a.root_dist, a.atol);
        ns += nsp;
    }
    const double tof = grp_tof<NSP, G>(nv, gl, x, y);
    const bool fin = gmin<G>((!x.row || isfinite(y)) ? 1.0 : 0.0) > 0.0 && isfinite(tof);
    if (!fin && st == PCK_ST_OK) st = PCK_ST_NONFINITE;
    if (ga.M > 1) {
        if (x.gl == 0) {
            ga.tofbuf[(int64_t)q * cv.n + c] = tof;
            ga.stbuf[(int64_t)q * cv.n + c] = st;
            ga.nsbuf[(int64_t)q * cv.n + c] = ns;
        }
        return;
    }
    // retry pass (mk_solver.h: k_solve): a failed tight transient keeps the
    // first pass's outputs
    const bool keep = a.retry_pass && st != PCK_ST_OK;
    if (a.retry_pass) st = keep ? PCK_ST_NEWTON_LOOSE : PCK_ST_NEWTON;
    if (a.y && x.row && !keep) a.y[x.gl * a.ld_y + c] = y;
    if (x.gl == 0) {
        if (a.tof && !keep)
            a.tof[c] = a.want_activity ? (log((hP * tof) / (kB * T)) * (Rgas * T)) * 1.0e-3 / eVtokJ : tof;
        if (a.status) a.status[c] = st;
        if (a.nsteps) a.nsteps[c] = a.retry_pass ? a.nsteps[c] + ns : ns;
    }
}

// (not in the kernel-only translation units of the split build, csrc/mk_inst.h:
// a non-template kernel is defined once, with the C-ABI)
#ifndef PCK_KERNEL_TU
// DRC combine (old_system.py:490-515): xi_j = (TOF_j+ - TOF_j-) / (2 eps TOF_0)
__global__ void __launch_bounds__(256) k_drc_combine(int64_t n, int R, double eps, const double* tofbuf,
                                                     const int32_t* stbuf, const int32_t* nsbuf, double* xi,
                                                     int64_t ld_xi, double* tof0, int32_t* status, int32_t* nsteps) {
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= n) return;
    const double t0 = tofbuf[c];
    int st = stbuf[c], stmin = st;
    int ns = nsbuf[c];
    for (int j = 0; j < R; ++j) {
        const double tp = tofbuf[(int64_t)(2 * j + 1) * n + c], tm = tofbuf[(int64_t)(2 * j + 2) * n + c];
        xi[j * ld_xi + c] = (tp - tm) / (2.0 * eps * t0);
        const int sp = stbuf[(int64_t)(2 * j + 1) * n + c], sm = stbuf[(int64_t)(2 * j + 2) * n + c];
        st = max(st, max(sp, sm));
        stmin = min(stmin, min(sp, sm));
        ns += nsbuf[(int64_t)(2 * j + 1) * n + c] + nsbuf[(int64_t)(2 * j + 2) * n + c];
    }
    st = drc_status(st, stmin);
    // a zero or non-finite base TOF makes every xi meaningless
    if (st == PCK_ST_OK && !(isfinite(t0) && t0 != 0.0)) st = PCK_ST_NONFINITE;
    if (tof0) tof0[c] = t0;
    if (status) status[c] = st;
    if (nsteps) nsteps[c] = ns;
}
#endif  // PCK_KERNEL_TU

template <int NSP, int G, int P>
__global__ void __launch_bounds__(64) k_rates_grp(NetView nv, GrpView gv, CondView cv, const double* kf,
                                                  const double* kr, int64_t ld_k, const double* yin, int64_t ld_y,
                                                  double* out, int jac, int QB) {
    extern __shared__ double lds[];
    const int grp = threadIdx.x / G;
    const int64_t c = (int64_t)blockIdx.x * (64 / G) + grp;
    if (c >= cv.n) return;
    Grp<NSP> x;
    double T;
    grp_setup<NSP, G>(nv, gv, cv, c, kf, kr, ld_k, -1, 1.0,
                      lds + (size_t)grp * grp_lds_doubles(nv.NRXN, NSP, nv.NDYN, gv.ND, QB, gv.LS, gv.NX), QB, x, T);
    const double y = x.row ? yin[x.gl * ld_y + c] : 0.0;
    if (!jac) {
        const double f = grp_rhs<NSP, G>(gv, x, y);
        if (x.row) out[x.gl * ld_y + c] = f;
    } else {
        double W[NSP];
        grp_jac<NSP, G, P>(nv, gv, x, y, 1.0, 0.0, W);
        if (x.row) {
#pragma unroll
            for (int q = 0; q < NSP; ++q)
                if (q < x.NS) out[((int64_t)x.gl * x.NS + q) * ld_y + c] = W[q];
        }
    }
}

}  // namespace pck
