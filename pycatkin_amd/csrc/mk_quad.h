// Quad-group solver: one condition per QUAD of lanes (4 lanes), each lane
// owning 4 species rows (row i = 4 * lane + slot), for networks of 9..16
// dynamic species with the network compiled in (hipRTC, nets::Jit).  Round 5.
//
// Why: the 16-lane group kernel with the network compiled in (mk_group.h:
// ct_rhs / ct_jac) evaluates every reaction on every lane of its group, so a
// rate evaluation of test/CH4_input.json (58 reactions) is issued 16 times
// per condition.  Here a lane evaluates them once for its 4 rows: 4x less
// redundancy, 16 conditions per wavefront instead of 4.  Every broadcast of
// the dense linear algebra is a DPP quad_perm (any lane of a quad, one
// v_mov_dpp per dword, no LDS), and the rows a step must not touch are left
// out by exec masks on the lane (gl > K) and compile-time slot ranges, not by
// selects.
//
// Same integrator as the lane-group kernel (mk_group.h: grp_integrate):
// RODAS4P with RMS error control, the positivity rule, the conserved totals'
// drift removal from the stage increments (PCK_GRP_KPROJ) and the
// multiplicative site-balance projection after each step.  The LU is
// threshold-pivoted like the lane solver's (mk_device.h: lu, tau 0.1): the
// diagonal is kept unless a row below is 10x larger; where a quad of the
// wavefront needs a swap (wave vote) its rows are exchanged physically
// (whole rows, LAPACK storage) and the solves apply the row permutation to
// the right-hand side first.
//
// Scope: every group solve of a network of at most 16 dynamic species --
// transients (the BASELINE CH4 SteadyStateSolver transient to 1e4 s, the
// DMTM DRC's 2R+1 transients per condition), steady solves with the quad
// Newton polish (q_newton) and trajectories (TRAJ, RODAS4P dense output);
// each is its own instantiation k_solve_q4<Net, NEWTON, TRAJ>.  An explicit
// screening pass (SolveArgs::screen_rtol) and PCK_CONS_ROWS run on the
// 16-lane kernel instead (csrc/mk_kernels.hip: run_solver).
#pragma once
#include "mk_group.h"

namespace pck {

// lane L of every quad, L a compile-time constant
template <int L>
__device__ __forceinline__ double qb(double v) {
    return __builtin_amdgcn_update_dpp(0.0, v, L | (L << 2) | (L << 4) | (L << 6), 0xf, 0xf, false);
}
template <int L>
__device__ __forceinline__ int qbi(int v) {
    return __builtin_amdgcn_update_dpp(0, v, L | (L << 2) | (L << 4) | (L << 6), 0xf, 0xf, false);
}
// quad all-reductions (bitwise the same value on the 4 lanes)
__device__ __forceinline__ double qsum(double v) {
    v = v + dppd<0xB1>(v);
    return v + dppd<0x4E>(v);
}
__device__ __forceinline__ double qmax(double v) {
    v = fmax(v, dppd<0xB1>(v));
    return fmax(v, dppd<0x4E>(v));
}
__device__ __forceinline__ double qmin(double v) {
    v = fmin(v, dppd<0xB1>(v));
    return fmin(v, dppd<0x4E>(v));
}
__device__ __forceinline__ int qmaxi(int v) {
    v = max(v, dppi<0xB1>(v));
    return max(v, dppi<0x4E>(v));
}

// the value of slot s (quad-uniform, run time) of this lane: selects on
// four scalars (an array indexed at run time would go to scratch)
__device__ __forceinline__ double slot4(double v0, double v1, double v2, double v3, int s) {
    const double lo = (s == 1) ? v1 : v0, hi = (s == 3) ? v3 : v2;
    return (s >= 2) ? hi : lo;
}

// rate sums of the lane's 4 rows only (see q_rhs)
#ifndef PCK_QUAD_ACC4
#define PCK_QUAD_ACC4 0
#endif

// the network's rows have no flow term (no CSTR in/outflow) / unit row scale
// (no T-dependent scale): compile-time, so those per-slot registers and
// their arithmetic fold away (DMTM, CH4)
template <class Net>
__device__ constexpr bool q_has_flow() {
    for (int i = 0; i < Net::NS; ++i)
        if (Net::dyn(i, 3) != 0.0) return true;
    return false;
}
template <class Net>
__device__ constexpr bool q_unit_rs() {
    for (int i = 0; i < Net::NS; ++i)
        if (Net::dyn(i, 1) != 1.0 || Net::dyn(i, 2) != 0.0) return false;
    return true;
}
template <class Net>
__device__ __forceinline__ double q_row_f(const struct Quad& x, int s, double acc, double y);

// per-lane context of a quad
struct Quad {
    int gl;                      // lane of the quad (0..3): rows 4 gl + s
    int64_t cidx;
    const double* kf;            // the condition's effective rate constants (LDS)
    const double* kr;
    double rs[4], fl[4], in[4];  // row scale, flow, inflow of the lane's rows
};

// f_i of slot s from its reaction sum: rs_i sum + fl_i (in_i - y_i)
template <class Net>
__device__ __forceinline__ double q_row_f(const Quad& x, int s, double acc, double y) {
    const double r = q_unit_rs<Net>() ? acc : acc * x.rs[s];
    return q_has_flow<Net>() ? r + x.fl[s] * (x.in[s] - y) : r;
}

// f of the lane's 4 rows: every reaction once (compile-time network), the
// per-species sums selected for the lane's rows at the end
template <class Net>
__device__ __forceinline__ void q_rhs(const Quad& x, const double (&y)[4], double (&f)[4]) {
    constexpr int NS = Net::NS, R = Net::R;
    ct_reload();
    const int gl = ct_row(x.gl);
    double c[NS];
    sfor<0, NS>([&](auto qc) {
        constexpr int q = decltype(qc)::value;
        c[q] = Net::dyn(q, 0) * qb<q / 4>(y[q % 4]);
    });
#if PCK_QUAD_ACC4
    // the lane's 4 rows only: each term S_ij net_j added with the coefficient
    // selected for the lane (S_ij on the lane owning row i, else 0) -- more
    // instructions, 24 fewer VGPRs than the per-species sums
    double acc[4] = {0.0, 0.0, 0.0, 0.0};
    sfor<0, R>([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        if constexpr (ct_col_used<Net, j>()) {
            double rf, rr;
            ct_rate<Net, j>(ct_k(x.kf, j), ct_k(x.kr, j), c, rf, rr);
            const double net = ct_sub(rf, rr);
            sfor<0, NS>([&](auto ic) {
                constexpr int i = decltype(ic)::value;
                if constexpr (Net::S(i, j) != 0.0) acc[i % 4] = fma((gl == i / 4) ? Net::S(i, j) : 0.0, net, acc[i % 4]);
            });
            ct_fence<j>(acc);
        }
    });
    sfor<0, 4>([&](auto sc) {
        constexpr int s = decltype(sc)::value;
        f[s] = q_row_f<Net>(x, s, acc[s], y[s]);
    });
#else
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
    sfor<0, 4>([&](auto sc) {
        constexpr int s = decltype(sc)::value;
        double v = 0.0;
        sfor<0, 4>([&](auto gc) {
            constexpr int g = decltype(gc)::value;
            constexpr int i = 4 * g + s;
            if constexpr (i < NS) v = (gl == g) ? acc[i] : v;
        });
        f[s] = q_row_f<Net>(x, s, v, y[s]);
    });
#endif
}

// some row 4 g + s (g = 0..3) has a nonzero coefficient in reaction j
template <class Net, int j, int s>
__device__ constexpr bool q_slot_used() {
    for (int g = 0; g < 4; ++g)
        if (4 * g + s < Net::NS && Net::S(4 * g + s, j) != 0.0) return true;
    return false;
}

// the lane's 4 rows of W = ig I - J (J = d f / d y, rows scaled by rs, the
// flow on the diagonal); padding rows (>= NS) are zero
template <class Net>
__device__ __forceinline__ void q_jac(const Quad& x, const double (&y)[4], double ig, double (&W)[4][Net::NS]) {
    constexpr int NS = Net::NS, R = Net::R;
    ct_reload();
    const int gl = ct_row(x.gl);
    double c[NS];
    sfor<0, NS>([&](auto qc) {
        constexpr int q = decltype(qc)::value;
        c[q] = Net::dyn(q, 0) * qb<q / 4>(y[q % 4]);
    });
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int q = 0; q < NS; ++q) W[s][q] = 0.0;
    sfor<0, R>([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        if constexpr (ct_col_used<Net, j>()) {
            const double kf = ct_k(x.kf, j), kr = ct_k(x.kr, j);
            // the lane's coefficient S(4 gl + s, j) of each slot
            double cs[4];
            sfor<0, 4>([&](auto sc) {
                constexpr int s = decltype(sc)::value;
                double v = 0.0;
                sfor<0, 4>([&](auto gc) {
                    constexpr int g = decltype(gc)::value;
                    constexpr int i = 4 * g + s;
                    if constexpr (i < NS) {
                        if constexpr (Net::S(i, j) != 0.0) v = (gl == g) ? Net::S(i, j) : v;
                    }
                });
                cs[s] = v;
            });
            sfor<0, NS>([&](auto qc) {
                constexpr int q = decltype(qc)::value;
                if constexpr (Net::ef(j, q) > 0 || Net::er(j, q) > 0) {
                    double v = 0.0;
                    if constexpr (Net::ef(j, q) > 0) v += ct_dside<Net, j, q, true>(kf, c);
                    if constexpr (Net::er(j, q) > 0) v -= ct_dside<Net, j, q, false>(kr, c);
                    // only the slots some lane's row of reaction j falls in
                    sfor<0, 4>([&](auto sc) {
                        constexpr int s = decltype(sc)::value;
                        if constexpr (q_slot_used<Net, j, s>()) W[s][q] = fma(cs[s], v, W[s][q]);
                    });
                }
            });
            if constexpr ((j + 1) % PCK_CT_CHUNK == 0) {
#pragma unroll
                for (int s = 0; s < 4; ++s) ct_fence<PCK_CT_CHUNK - 1>(W[s]);
            }
        }
    });
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        const double rs = q_unit_rs<Net>() ? -1.0 : -x.rs[s];
#pragma unroll
        for (int q = 0; q < NS; ++q) W[s][q] *= rs;
        // the diagonal: column 4 gl + s
        const double dg = q_has_flow<Net>() ? ig + x.fl[s] : ig;
#pragma unroll
        for (int g = 0; g < 4; ++g)
            if (4 * g + s < NS) W[s][4 * g + s] += (gl == g) ? dg : 0.0;
    }
}

// Threshold-pivoted LU of the quad's NS x NS matrix, rows distributed 4 per
// lane.  src[s]: original row of slot s (the solves' permutation); swapped:
// some quad of the wavefront exchanged rows (wave-uniform).  Returns false on
// a zero or non-finite pivot.
template <int NS>
__device__ __forceinline__ bool q_lu(int gl, double (&W)[4][NS], int (&src)[4], bool& swapped) {
    bool ok = true;
    swapped = false;
#pragma unroll
    for (int s = 0; s < 4; ++s) src[s] = 4 * gl + s;
    sfor<0, NS>([&](auto kc) {
        constexpr int k = decltype(kc)::value;
        constexpr int K = k / 4, KR = k % 4;
        // the largest |a_ik| below the diagonal against |a_kk| / tau
        double m = 0.0;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const int i = 4 * gl + s;
            if (i < NS) m = fmax(m, (i > k) ? fabs(W[s][k]) : 0.0);
        }
        m = qmax(m);
        const double dk = fabs(qb<K>(W[KR][k])) * (1.0 / PIVOT_TAU);
        if (__any(m > dk)) {
            // rare: partial pivoting on the quads that need it -- the row of
            // the largest |a_ik|, i >= k, exchanged with row k (whole rows)
            int key = -1;
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                const int i = 4 * gl + s;
                if (i < NS && i >= k) {
                    const float mag = (float)fabs(W[s][k]);
                    key = max(key, (int)((__float_as_uint(mag) & ~63u) | (uint32_t)i));
                }
            }
            key = qmaxi(key);
            int p = key & 63;
            if (!(m > dk)) p = k;                   // this quad keeps its diagonal
            swapped = true;
            const int ps = p & 3, pl = p >> 2;
#pragma unroll
            for (int j = 0; j < NS; ++j) {
                {
                    const double ak = qb<K>(W[KR][j]);
                    const double ap =
                        __shfl(slot4(W[0][j], W[1][j], W[2][j], W[3][j], ps), (int)(threadIdx.x & ~3u) | pl, 64);
                    if (p != k) {
                        if (gl == K) W[KR][j] = ap;
#pragma unroll
                        for (int s = 0; s < 4; ++s)
                            if (gl == pl && s == ps) W[s][j] = ak;
                    }
                }
            }
            {
                const int ik = qbi<K>(src[KR]);
                const int ip = __shfl(ps == 0 ? src[0] : ps == 1 ? src[1] : ps == 2 ? src[2] : src[3],
                                      (int)(threadIdx.x & ~3u) | pl, 64);
                if (p != k) {
                    if (gl == K) src[KR] = ip;
#pragma unroll
                    for (int s = 0; s < 4; ++s)
                        if (gl == pl && s == ps) src[s] = ik;
                }
            }
        }
        const double akk = qb<K>(W[KR][k]);
        ok = ok && (akk != 0.0) && (akk == akk);
        const double inv = rcp1(akk);
        // multipliers of the rows below k (0 on the rows at and above it, whose
        // trailing entries the updates then leave as they are: no exec-mask
        // branches per column), the stored reciprocal on row k
        double mk[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const bool below = (gl > K) || (gl == K && s > KR);
            const double m_s = W[s][k] * inv;
            mk[s] = below ? -m_s : 0.0;
            W[s][k] = below ? m_s : ((gl == K && s == KR) ? inv : W[s][k]);
        }
#pragma unroll
        for (int j = k + 1; j < NS; ++j) {
            const double pj = qb<K>(W[KR][j]);
#pragma unroll
            for (int s = 0; s < 4; ++s) W[s][j] = fma(mk[s], pj, W[s][j]);
        }
    });
    swapped = __any(swapped);
    return ok;
}

// Solve (LU) x = b for the quad; b, x: the lane's 4 rows
template <int NS>
__device__ __forceinline__ void q_solve(int gl, const double (&W)[4][NS], const int (&src)[4], bool swapped,
                                        double (&b)[4]) {
    if (swapped) {                               // wave-uniform: b <- P b
        double nb[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const int o = src[s];
            // slot o & 3 of lane o >> 2: every lane offers all 4 slots, the
            // reader picks
            const double v0 = __shfl(b[0], (int)(threadIdx.x & ~3u) | (o >> 2), 64);
            const double v1 = __shfl(b[1], (int)(threadIdx.x & ~3u) | (o >> 2), 64);
            const double v2 = __shfl(b[2], (int)(threadIdx.x & ~3u) | (o >> 2), 64);
            const double v3 = __shfl(b[3], (int)(threadIdx.x & ~3u) | (o >> 2), 64);
            nb[s] = slot4(v0, v1, v2, v3, o & 3);
        }
#pragma unroll
        for (int s = 0; s < 4; ++s) b[s] = nb[s];
    }
    // 4 x 4 blocks: the diagonal block on its own lane, then one broadcast of
    // its 4 values and the update of the other lanes' rows -- 2 exec-mask
    // branches and one DPP round per block instead of per column; every row
    // still subtracts its terms in column order (the same rounding)
    constexpr int NB = (NS + 3) / 4;
    // forward: unit lower triangle
    sfor<0, NB>([&](auto Kc) {
        constexpr int K = decltype(Kc)::value;
        if (gl == K) {
            sfor<1, 4>([&](auto sc) {
                constexpr int s = decltype(sc)::value;
                if constexpr (4 * K + s < NS) {
#pragma unroll
                    for (int r = 0; r < s; ++r) b[s] = fma(-W[s][4 * K + r], b[r], b[s]);
                }
            });
        }
        if constexpr (K + 1 < NB) {
            double bk[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) bk[r] = qb<K>(b[r]);
            if (gl > K) {
#pragma unroll
                for (int s = 0; s < 4; ++s) {
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        if (4 * K + r < NS) b[s] = fma(-W[s][4 * K + r], bk[r], b[s]);
                }
            }
        }
    });
    // backward: U with the stored reciprocals of its diagonal
    sfor<0, NB>([&](auto Kc) {
        constexpr int K = NB - 1 - decltype(Kc)::value;
        if (gl == K) {
            sfor<0, 4>([&](auto rc) {
                constexpr int r = 3 - decltype(rc)::value;
                if constexpr (4 * K + r < NS) {
                    b[r] = b[r] * W[r][4 * K + r];
#pragma unroll
                    for (int s = 0; s < r; ++s) b[s] = fma(-W[s][4 * K + r], b[r], b[s]);
                }
            });
        }
        if constexpr (K > 0) {
            double xk[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) xk[r] = qb<K>(b[r]);
            if (gl < K) {
#pragma unroll
                for (int s = 0; s < 4; ++s) {
#pragma unroll
                    for (int r = 3; r >= 0; --r)
                        if (4 * K + r < NS) b[s] = fma(-W[s][4 * K + r], xk[r], b[s]);
                }
            }
        }
    });
}

// RODAS4P on the quad (mk_group.h: grp_integrate, transient only)
template <class Net, bool TRAJ = false>
__device__ __forceinline__ int q_integrate(const Quad& x, double (&y)[4], double t0, double t_end, double rtol,
                                           double atol, int max_steps, int& nsteps, const TrajOut& to = TrajOut{}) {
    using namespace rodas4;
    constexpr int NS = Net::NS;
    constexpr int NC = Net::NCONS;
    const int gl = x.gl;
    bool real[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) real[s] = (4 * gl + s) < NS;
    // trajectory samples (mk_group.h: grp_integrate): the lane's rows of
    // sample k at to.y[(k NS + i) ld + c]
    int ko = 0;
    auto put = [&](int k, const double (&v)[4]) {
#pragma unroll
        for (int s = 0; s < 4; ++s)
            if (real[s]) to.y[((int64_t)k * NS + 4 * gl + s) * to.ld + to.c] = v[s];
    };
    if constexpr (TRAJ) {
        for (; ko < to.n && to.t[ko] <= t0; ++ko) put(ko, y);
    }
    const double invNS = 1.0 / NS;
    nsteps = 0;
    const double span = t_end - t0;
    if (!(span > 0.0)) {
        if constexpr (TRAJ) {
            for (; ko < to.n; ++ko) put(ko, y);
        }
        return PCK_ST_OK;
    }
    double F0[4];
    q_rhs<Net>(x, y, F0);
    // conservation laws: the lane's coefficients (small integers: exact in
    // fp32, half the registers), initial totals
    float ci[NC > 0 ? NC : 1][4];
    double cons0[NC > 0 ? NC : 1];
    bool cpos[NC > 0 ? NC : 1];
    sfor<0, NC>([&](auto lc) {
        constexpr int l = decltype(lc)::value;
        bool pos = true;
        for (int i = 0; i < NS; ++i) pos = pos && (Net::C(l, i) >= 0.0);
        cpos[l] = pos;
        double sm = 0.0;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            double v = 0.0;
#pragma unroll
            for (int g = 0; g < 4; ++g)
                if (4 * g + s < NS) v = (gl == g) ? Net::C(l, (4 * g + s) < NS ? 4 * g + s : 0) : v;
            ci[l][s] = (float)v;
            sm += v * y[s];
        }
        cons0[l] = qsum(sm);
    });
    // 1 / (c . y) of each law at the step's start (the drift removal's
    // direction y / (c . y) on the law's species, mk_group.h: kproj)
    double icy[NC > 0 ? NC : 1];
    auto kproj = [&](double (&k)[4]) {
        if (PCK_GRP_KPROJ) {
            sfor<0, NC>([&](auto lc) {
                constexpr int l = decltype(lc)::value;
                if (cpos[l]) {
                    double sm = 0.0;
#pragma unroll
                    for (int s = 0; s < 4; ++s) sm += (double)ci[l][s] * k[s];
                    sm = qsum(sm) * icy[l];
#pragma unroll
                    for (int s = 0; s < 4; ++s)
                        if (ci[l][s] != 0.0f) k[s] -= sm * y[s];
                }
            });
        }
    };
    double h;
    {
        double d0 = 0.0, d1 = 0.0, sc[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            sc[s] = atol + rtol * fabs(y[s]);
            if (real[s]) { d0 += (y[s] / sc[s]) * (y[s] / sc[s]); d1 += (F0[s] / sc[s]) * (F0[s] / sc[s]); }
        }
        d0 = sqrt(qsum(d0) * invNS);
        d1 = sqrt(qsum(d1) * invNS);
        double h0 = (d0 < 1e-5 || d1 < 1e-5) ? 1e-6 : 0.01 * d0 / d1;
        h0 = fmin(h0, span);
        double y1[4], F1[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) y1[s] = y[s] + h0 * F0[s];
        q_rhs<Net>(x, y1, F1);
        double d2 = 0.0;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const double q = (F1[s] - F0[s]) / sc[s];
            if (real[s]) d2 += q * q;
        }
        d2 = sqrt(qsum(d2) * invNS) / h0;
        const double h1 = (d1 <= 1e-15 && d2 <= 1e-15) ? fmax(1e-6, h0 * 1e-3) : pow(0.01 / fmax(d1, d2), 0.2);
        h = fmin(fmin(100.0 * h0, h1), span);
    }
    double t = t0;
    int blowups = 0, stall = 0;
    double W[4][NS];        // the network's columns only (DMTM: 11, 40 VGPRs fewer than 16)
    int src[4];
    bool sw;
    while (t < t_end) {
        if (nsteps >= max_steps) return PCK_ST_MAXSTEPS;
        ++nsteps;
        bool last = false;
        if (t + h >= t_end) { h = t_end - t; last = true; }
        const double ih = rcp(h);
        const double ig = ih * (1.0 / g);
        q_jac<Net>(x, y, ig, W);
        if (!q_lu<NS>(gl, W, src, sw)) {
            h *= 0.25;
            if (!(h > 2.220446049250313e-15 * fmax(fabs(t), 1e-300))) return PCK_ST_STEPFAIL;
            continue;
        }
        if (PCK_GRP_KPROJ) {
            sfor<0, NC>([&](auto lc) {
                constexpr int l = decltype(lc)::value;
                if (cpos[l]) {
                    double cy = 0.0;
#pragma unroll
                    for (int s = 0; s < 4; ++s) cy += (double)ci[l][s] * y[s];
                    cy = qsum(cy);
                    icy[l] = (cy > 0.0) ? 1.0 / cy : 0.0;
                }
            });
        }
        double k1[4], k2[4], k3[4], k4[4], k5[4], u[4], fu[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) k1[s] = F0[s];
        q_solve<NS>(gl, W, src, sw, k1);
        kproj(k1);
#pragma unroll
        for (int s = 0; s < 4; ++s) u[s] = y[s] + a21 * k1[s];
        q_rhs<Net>(x, u, fu);
#pragma unroll
        for (int s = 0; s < 4; ++s) k2[s] = fu[s] + ih * (C21 * k1[s]);
        q_solve<NS>(gl, W, src, sw, k2);
        kproj(k2);
#pragma unroll
        for (int s = 0; s < 4; ++s) u[s] = y[s] + a31 * k1[s] + a32 * k2[s];
        q_rhs<Net>(x, u, fu);
#pragma unroll
        for (int s = 0; s < 4; ++s) k3[s] = fu[s] + ih * (C31 * k1[s] + C32 * k2[s]);
        q_solve<NS>(gl, W, src, sw, k3);
        kproj(k3);
#pragma unroll
        for (int s = 0; s < 4; ++s) u[s] = y[s] + a41 * k1[s] + a42 * k2[s] + a43 * k3[s];
        q_rhs<Net>(x, u, fu);
#pragma unroll
        for (int s = 0; s < 4; ++s) k4[s] = fu[s] + ih * (C41 * k1[s] + C42 * k2[s] + C43 * k3[s]);
        q_solve<NS>(gl, W, src, sw, k4);
        kproj(k4);
#pragma unroll
        for (int s = 0; s < 4; ++s) u[s] = y[s] + a51 * k1[s] + a52 * k2[s] + a53 * k3[s] + a54 * k4[s];
        q_rhs<Net>(x, u, fu);
#pragma unroll
        for (int s = 0; s < 4; ++s) k5[s] = fu[s] + ih * (C51 * k1[s] + C52 * k2[s] + C53 * k3[s] + C54 * k4[s]);
        q_solve<NS>(gl, W, src, sw, k5);
        kproj(k5);
        double d2[TRAJ ? 4 : 1], d3[TRAJ ? 4 : 1];     // dense output (mk_solver.h: rodas4_dense)
        if constexpr (TRAJ) {
            using namespace rodas4_dense;
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                d2[s] = D21 * k1[s] + D22 * k2[s] + D23 * k3[s] + D24 * k4[s] + D25 * k5[s];
                d3[s] = D3_K5_ONLY ? D35 * k5[s] : D31 * k1[s] + D32 * k2[s] + D33 * k3[s] + D34 * k4[s] + D35 * k5[s];
            }
        }
#pragma unroll
        for (int s = 0; s < 4; ++s) u[s] += k5[s];
        q_rhs<Net>(x, u, fu);
        // k6 in k5's registers
#pragma unroll
        for (int s = 0; s < 4; ++s)
            k5[s] = fu[s] + ih * (C61 * k1[s] + C62 * k2[s] + C63 * k3[s] + C64 * k4[s] + C65 * k5[s]);
        q_solve<NS>(gl, W, src, sw, k5);
        kproj(k5);
        double es = 0.0, pfl = 1.0;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            u[s] += k5[s];
            const double sc = atol + rtol * fmax(fabs(y[s]), fabs(u[s]));
            const double r = k5[s] * __builtin_amdgcn_rcp(sc);
            if (real[s]) {
                es += r * r + 0.0 * u[s];        // a non-finite stage makes the sum NaN
                if (PCK_POSITIVITY && u[s] < -atol) pfl = fmin(pfl, (y[s] + atol) / (y[s] - u[s]));
            }
        }
        es = qsum(es);
        const double fin = (es == es) ? 1.0 : 0.0;
        const double q = (fin > 0.0) ? es * invNS : INFINITY;
        const double pf = PCK_POSITIVITY ? qmin(pfl) : 1.0;
        const double fac = step_factor(q);
        if (q <= 1.0 && pf >= 1.0) {
            const double t_old = t;
            double y_old[TRAJ ? 4 : 1];
            if constexpr (TRAJ) {
#pragma unroll
                for (int s = 0; s < 4; ++s) y_old[s] = y[s];
            }
            t = last ? t_end : t + h;
#pragma unroll
            for (int s = 0; s < 4; ++s) y[s] = real[s] ? u[s] : 0.0;
            sfor<0, NC>([&](auto lc) {
                constexpr int l = decltype(lc)::value;
                double sm = 0.0;
#pragma unroll
                for (int s = 0; s < 4; ++s) sm += (double)ci[l][s] * y[s];
                sm = qsum(sm);
                if (cpos[l] && sm > 0.0) {
                    const double fct = cons0[l] * rcp(sm);
#pragma unroll
                    for (int s = 0; s < 4; ++s)
                        if (ci[l][s] != 0.0f) y[s] *= fct;
                }
            });
            if constexpr (TRAJ) {
                // samples inside (t_old, t]: the dense output of this step
                for (; ko < to.n && to.t[ko] <= t; ++ko) {
                    const double sv = fmin((to.t[ko] - t_old) / h, 1.0), s1 = 1.0 - sv;
                    double v[4];
#pragma unroll
                    for (int s = 0; s < 4; ++s) v[s] = y_old[s] * s1 + sv * (y[s] + s1 * (d2[s] + sv * d3[s]));
                    put(ko, v);
                }
            }
            q_rhs<Net>(x, y, F0);
            // falling tolerance-level negatives to 0 (mk_solver.h: integrate)
            bool negf = false;
#pragma unroll
            for (int s = 0; s < 4; ++s) negf = negf || (real[s] && y[s] < 0.0 && F0[s] < 0.0);
            if (PCK_POSITIVITY && __any(negf)) {
                const double anyq = qmax(negf ? 1.0 : 0.0);
#pragma unroll
                for (int s = 0; s < 4; ++s)
                    if (real[s] && y[s] < 0.0 && F0[s] < 0.0) y[s] = 0.0;
                if (anyq > 0.0) q_rhs<Net>(x, y, F0);
            }
            h *= fmin(PCK_FACMAX, fmax(0.2, fac));
        } else if (q <= 1.0) {
            h *= fmax(0.1, 0.9 * pf);
        } else {
            h *= (fin > 0.0) ? fmax(0.2, fac) : 0.25;
            if (!(q < PCK_BLOWUP_Q) && h < 1e-4 * t && ++blowups > PCK_MAX_BLOWUPS) return PCK_ST_STEPFAIL;
        }
        stall = (h < PCK_STALL_H * (t - t0)) ? stall + 1 : 0;
        if (stall > PCK_STALL_STEPS) return PCK_ST_STEPFAIL;
        if (!(h > 2.220446049250313e-15 * fmax(fabs(t), 1e-300)) && t < t_end) return PCK_ST_STEPFAIL;
    }
    if constexpr (TRAJ) {
        // samples past t_end (a log grid can round one ulp above it): the final state
        for (; ko < to.n; ++ko) put(ko, y);
    }
    return PCK_ST_OK;
}

// ---------------------------------------------------------------------------
// Newton steady-state polish on the quad (mk_group.h: grp_newton, the same
// rules: rounding-floor and step-floor stops, linear-convergence
// extrapolation, double-double residual refinement on the last
// factorisation, the balance test and the steady rule against the transient
// end).  Round 5; PCK_GRP_QUAD_NEWTON=0 keeps steady solves on the 16-lane
// kernel.
// ---------------------------------------------------------------------------

// coefficient of row 4 gl + s in a compile-time table T(i) (0 on padding rows)
template <class Net, int S, class F>
__device__ __forceinline__ double q_slot_coef(int gl, F tab) {
    double v = 0.0;
    sfor<0, 4>([&](auto gc) {
        constexpr int g = decltype(gc)::value;
        if constexpr (4 * g + S < Net::NS) {
            constexpr double t = tab(4 * g + S);
            if constexpr (t != 0.0) v = (gl == g) ? t : v;
        }
    });
    return v;
}

// f and the gross flux sum_j |S_ij| (|rf_j| + |rr_j|) of the lane's rows
template <class Net>
__device__ __forceinline__ void q_fgross(const Quad& x, const double (&y)[4], double (&f)[4], double (&gr)[4]) {
    constexpr int NS = Net::NS, R = Net::R;
    ct_reload();
    const int gl = ct_row(x.gl);
    double c[NS];
    sfor<0, NS>([&](auto qc) {
        constexpr int q = decltype(qc)::value;
        c[q] = Net::dyn(q, 0) * qb<q / 4>(y[q % 4]);
    });
    double acc[4] = {0.0, 0.0, 0.0, 0.0}, gacc[4] = {0.0, 0.0, 0.0, 0.0};
    sfor<0, R>([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        if constexpr (ct_col_used<Net, j>()) {
            double rf, rr;
            ct_rate<Net, j>(ct_k(x.kf, j), ct_k(x.kr, j), c, rf, rr);
            const double net = ct_sub(rf, rr), gro = fabs(rf) + fabs(rr);
            sfor<0, 4>([&](auto sc) {
                constexpr int s = decltype(sc)::value;
                if constexpr (q_slot_used<Net, j, s>()) {
                    const double v = q_slot_coef<Net, s>(gl, [](int i) constexpr { return Net::S(i, j); });
                    acc[s] = fma(v, net, acc[s]);
                    gacc[s] = fma(fabs(v), gro, gacc[s]);
                }
            });
            ct_fence<j>(acc);
        }
    });
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        f[s] = q_row_f<Net>(x, s, acc[s], y[s]);
        double g = q_unit_rs<Net>() ? gacc[s] : gacc[s] * fabs(x.rs[s]);
        if (q_has_flow<Net>()) g += fabs(x.fl[s]) * (fabs(x.in[s]) + fabs(y[s]));
        gr[s] = g;
    }
}

// f of the lane's rows in double-double, rounded once (mk_group.h: ct_rhs_dd)
template <class Net>
__device__ __forceinline__ void q_rhs_dd(const Quad& x, const double (&y)[4], double (&f)[4]) {
    constexpr int NS = Net::NS, R = Net::R;
    ct_reload();
    const int gl = ct_row(x.gl);
    dd acc[4] = {dd_of(0.0), dd_of(0.0), dd_of(0.0), dd_of(0.0)};
    sfor<0, R>([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        if constexpr (ct_col_used<Net, j>()) {
            double yv[4] = {y[0], y[1], y[2], y[3]};
#pragma unroll
            for (int s = 0; s < 4; ++s) asm volatile("" : "+v"(yv[s]));
            dd rf = dd_of(ct_k(x.kf, j)), rr = dd_of(ct_k(x.kr, j));
            sfor<0, NS>([&](auto ic) {
                constexpr int i = decltype(ic)::value;
                if constexpr (Net::ef(j, i) > 0 || Net::er(j, i) > 0) {
                    const dd ci = two_prod(Net::dyn(i, 0), qb<i / 4>(yv[i % 4]));
                    if constexpr (Net::ef(j, i) > 0) rf = dd_mul(rf, dd_pow(ci, Net::ef(j, i)));
                    if constexpr (Net::er(j, i) > 0) rr = dd_mul(rr, dd_pow(ci, Net::er(j, i)));
                }
            });
            const dd net = dd_add(rf, dd_neg(rr));
            sfor<0, 4>([&](auto sc) {
                constexpr int s = decltype(sc)::value;
                if constexpr (q_slot_used<Net, j, s>()) {
                    const double v = q_slot_coef<Net, s>(gl, [](int i) constexpr { return Net::S(i, j); });
                    acc[s] = dd_add(acc[s], dd_mul(net, v));
                }
            });
#pragma unroll
            for (int s = 0; s < 4; ++s) asm volatile("" : "+v"(acc[s].hi), "+v"(acc[s].lo) :: "memory");
        }
    });
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        dd r = q_unit_rs<Net>() ? acc[s] : dd_mul(acc[s], x.rs[s]);
        if (q_has_flow<Net>() && x.fl[s] != 0.0) r = dd_add(r, dd_mul(two_sum(x.in[s], -y[s]), x.fl[s]));
        f[s] = r.hi + r.lo;
    }
}

template <int CTRL>
__device__ __forceinline__ dd q_dppdd(dd v) { return {dppd<CTRL>(v.hi), dppd<CTRL>(v.lo)}; }
__device__ __forceinline__ dd q_sum_dd(dd v) {
    v = dd_add(v, q_dppdd<0xB1>(v));
    return dd_add(v, q_dppdd<0x4E>(v));
}

template <class Net>
__device__ __forceinline__ int q_newton(const Quad& x, double (&y)[4], int iters, double dist, double atol) {
    constexpr int NS = Net::NS, NC = Net::NCONS;
    const int gl = x.gl;
    bool real[4], pv[4], pin[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        real[s] = (4 * gl + s) < NS;
        pv[s] = false;
        pin[s] = false;
    }
    // conservation laws: the lane's coefficients, totals at the transient end,
    // the pivot rows (compile-time rows, the lane that holds them at run time)
    double ci[NC > 0 ? NC : 1][4], b[NC > 0 ? NC : 1];
    sfor<0, NC>([&](auto lc) {
        constexpr int l = decltype(lc)::value;
        double sm = 0.0;
        sfor<0, 4>([&](auto sc) {
            constexpr int s = decltype(sc)::value;
            ci[l][s] = q_slot_coef<Net, s>(gl, [](int i) constexpr { return Net::C(l, i); });
            sm += ci[l][s] * y[s];
        });
        b[l] = qsum(sm);
        constexpr int pr = Net::cpiv(l);
#pragma unroll
        for (int s = 0; s < 4; ++s) pv[s] = pv[s] || (4 * gl + s == pr);
    });
    auto imbalance = [&](const double (&z)[4], double (&f)[4]) {
        double gr[4];
        q_fgross<Net>(x, z, f, gr);
        double m = 0.0;
#pragma unroll
        for (int s = 0; s < 4; ++s)
            if (real[s] && !pv[s] && f[s] != 0.0) m = fmax(m, fabs(f[s]) / gr[s]);
        return qmax(m);
    };
    double z[4], zp[4], scl[4] = {1.0, 1.0, 1.0, 1.0};
#pragma unroll
    for (int s = 0; s < 4; ++s) z[s] = zp[s] = y[s];
    double bal_prev = INFINITY, prev = INFINITY, lastq = 1.0;
    int linear = 0;
    bool conv = false;
    double W[4][NS];
    int src[4];
    bool sw = false;
    for (int it = 0; it < iters; ++it) {
        double Gv[4];
        const double bal = imbalance(z, Gv);
        if (it == 0) {
            // mk_solver.h: newton_pinned -- zero species with a zero rate stay 0
#pragma unroll
            for (int s = 0; s < 4; ++s) pin[s] = real[s] && !pv[s] && z[s] == 0.0 && Gv[s] == 0.0;
        }
        if (it >= 2 && bal_prev <= PCK_BALANCE_CONV && bal > bal_prev) {
#pragma unroll
            for (int s = 0; s < 4; ++s) z[s] = zp[s];
            conv = true;
            break;
        }
        bal_prev = bal;
#pragma unroll
        for (int s = 0; s < 4; ++s) zp[s] = z[s];
        q_jac<Net>(x, z, 0.0, W);                     // -J
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
            for (int q = 0; q < NS; ++q) W[s][q] = -W[s][q];
        sfor<0, NC>([&](auto lc) {
            constexpr int l = decltype(lc)::value;
            constexpr int pr = Net::cpiv(l);
            double sm = 0.0;
#pragma unroll
            for (int s = 0; s < 4; ++s) sm += ci[l][s] * z[s];
            sm = qsum(sm);
            if (gl == pr / 4) {
                Gv[pr % 4] = sm - b[l];
                sfor<0, NS>([&](auto qc) {
                    constexpr int q = decltype(qc)::value;
                    W[pr % 4][q] = Net::C(l, q);
                });
            }
        });
        // row equilibration (rate rows up to 1e9, conservation rows O(1))
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            double m = 0.0;
#pragma unroll
            for (int q = 0; q < NS; ++q) m = fmax(m, fabs(W[s][q]));
            scl[s] = (m > 0.0) ? 1.0 / m : 1.0;
#pragma unroll
            for (int q = 0; q < NS; ++q) W[s][q] *= scl[s];
            Gv[s] = -Gv[s] * scl[s];
        }
        if (!q_lu<NS>(gl, W, src, sw)) break;
        q_solve<NS>(gl, W, src, sw, Gv);              // Gv <- dz
        double alpha = 1.0;
        if (linear >= 2 && lastq < 0.9) {
            alpha = fmin(4.0, 1.0 / (1.0 - lastq));
            double cand = INFINITY;
#pragma unroll
            for (int s = 0; s < 4; ++s)
                if (real[s] && Gv[s] < 0.0 && z[s] > 0.0) cand = fmin(cand, 0.9 * z[s] / -Gv[s]);
            alpha = fmax(fmin(alpha, qmin(cand)), 1.0);
        }
        bool fin = true;
        double zmax = 0.0;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            Gv[s] = pin[s] ? 0.0 : Gv[s] * alpha;
            z[s] += Gv[s];
            if (real[s]) {
                fin = fin && isfinite(z[s]);
                zmax = fmax(zmax, fabs(z[s]));
            }
        }
        if (!(qmin(fin ? 1.0 : 0.0) > 0.0)) break;
        zmax = qmax(zmax);
        double rl = 0.0;
#pragma unroll
        for (int s = 0; s < 4; ++s)
            if (real[s]) rl = fmax(rl, fabs(Gv[s]) / fmax(fabs(z[s]), 1e-12 * zmax + 1e-300));
        const double rel = qmax(rl);
        if (prev < PCK_STEP_FLOOR && rel > prev) {     // mk_solver.h: the step floor
#pragma unroll
            for (int s = 0; s < 4; ++s) z[s] = zp[s];
            conv = true;
            break;
        }
        if (rel < 1e-12 || (it >= 2 && rel < 1e-7 && rel > 0.5 * prev)) { conv = true; break; }
        lastq = rel / prev;
        linear = (rel > 0.25 * prev) ? linear + 1 : 0;
        if (linear >= 12) break;
        prev = rel;
    }
    if (!conv) return PCK_ST_NEWTON;
    if (PCK_NEWTON_REFINE > 0) {
        // residual refinement on the loop's last factorisation and row scale
        double nprev = INFINITY, zq[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) zq[s] = z[s];
#pragma unroll 1
        for (int r = 0; r <= PCK_NEWTON_REFINE; ++r) {
            double Gv[4];
            q_rhs_dd<Net>(x, z, Gv);
            sfor<0, NC>([&](auto lc) {
                constexpr int l = decltype(lc)::value;
                constexpr int pr = Net::cpiv(l);
                dd sm = dd_of(0.0);
#pragma unroll
                for (int s = 0; s < 4; ++s) sm = dd_add(sm, two_prod(ci[l][s], z[s]));
                const dd t = dd_add(q_sum_dd(sm), dd_of(-b[l]));
                if (gl == pr / 4) Gv[pr % 4] = t.hi + t.lo;
            });
            double nr = 0.0;
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                Gv[s] = -Gv[s] * scl[s];
                if (real[s]) nr = fmax(nr, fabs(Gv[s]));
            }
            nr = qmax(nr);
            if (!(nr < nprev)) {                        // no longer falling: the previous iterate
                if (r > 0) {
#pragma unroll
                    for (int s = 0; s < 4; ++s) z[s] = zq[s];
                }
                break;
            }
            nprev = nr;
            if (r == PCK_NEWTON_REFINE || nr == 0.0) break;
            q_solve<NS>(gl, W, src, sw, Gv);
            double zmax = 0.0;
#pragma unroll
            for (int s = 0; s < 4; ++s)
                if (real[s]) zmax = fmax(zmax, fabs(z[s]));
            zmax = qmax(zmax);
            double rl = 0.0;
            bool fin = true;
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                if (pin[s]) Gv[s] = 0.0;
                if (real[s]) rl = fmax(rl, fabs(Gv[s]) / fmax(fabs(z[s]), 1e-12 * zmax + 1e-300));
                zq[s] = z[s];
                z[s] += Gv[s];
                if (real[s]) fin = fin && isfinite(z[s]);
            }
            const double rel = qmax(rl);
            if (!(qmin(fin ? 1.0 : 0.0) > 0.0) || !(rel <= PCK_REFINE_MAXSTEP)) {
#pragma unroll
                for (int s = 0; s < 4; ++s) z[s] = zq[s];
                break;
            }
        }
    }
    bool neg = false, far = false;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        if (real[s]) {
            neg = neg || z[s] < 0.0;
            far = far || !(fabs(z[s] - y[s]) <= dist * fabs(z[s]) + atol);
        }
    }
    if (qmax(neg ? 1.0 : 0.0) > 0.0) return PCK_ST_NEWTON;
    {
        double f[4];
        if (!(imbalance(z, f) <= PCK_BALANCE_TOL)) return PCK_ST_NEWTON;   // converged in absolute terms only
    }
    // mk_solver.h: newton -- the root only if the transient end reached it
    if (dist > 0.0 && qmax(far ? 1.0 : 0.0) > 0.0) return PCK_ST_NEWTON;
#pragma unroll
    for (int s = 0; s < 4; ++s) y[s] = real[s] ? z[s] : 0.0;
    return PCK_ST_OK;
}

// TOF of the quad's state (old_system.py:482-488): the listed reactions'
// net rates, every lane the same value
template <class Net>
__device__ __forceinline__ double q_tof(const NetView& nv, const Quad& x, const double (&y)[4]) {
    constexpr int NS = Net::NS, R = Net::R;
    double c[NS];
    sfor<0, NS>([&](auto qc) {
        constexpr int q = decltype(qc)::value;
        c[q] = Net::dyn(q, 0) * qb<q / 4>(y[q % 4]);
    });
    double tof = 0.0;
    sfor<0, R>([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        bool in = false;
        for (int t = 0; t < nv.NTOF; ++t) in = in || (nv.tof[t] == j);
        if (in) {
            double rf, rr;
            ct_rate<Net, j>(x.kf[j], x.kr[j], c, rf, rr);
            tof += rf - rr;
        }
    });
    return tof;
}

// occupancy floor (waves per SIMD) of the quad kernel; the VGPR budget follows
#ifndef PCK_QUAD_WAVES
#define PCK_QUAD_WAVES 1
#endif
// one condition (or one DRC perturbation of one) per quad; 16 per block
template <class Net, bool NEWTON = false, bool TRAJ = false>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(PCK_QUAD_WAVES))) k_solve_q4(NetView nv, CondView cv, const double* kf, const double* kr,
                                                 int64_t ld_k, SolveArgs a, GrpArgs ga) {
    static_assert(Net::NS <= 16, "quad-group solver: at most 16 dynamic species");
    constexpr int NS = Net::NS, R = Net::R;
    extern __shared__ double lds[];
    const int quad = threadIdx.x >> 2;
    const int gl = threadIdx.x & 3;
    const int64_t v = (int64_t)blockIdx.x * 16 + quad;
    const int64_t slot = cond_of(a, v, ga.M, cv.n);
    const int q = (int)(v % ga.M);
    Quad x;
    x.gl = gl;
    x.cidx = slot;
    double* kb = lds + (size_t)quad * 2 * R;
    x.kf = kb;
    x.kr = kb + R;
    if (slot >= cv.n) return;                    // quad-uniform; no block barriers below
    const int64_t c = slot;
    int pj = -1;
    double pfac = 1.0;
    if (q > 0) { pj = (q - 1) >> 1; pfac = (q & 1) ? 1.0 + a.eps : 1.0 - a.eps; }
    const double T = cv.T[c * cv.sT];
    for (int j = gl; j < R; j += 4) {
        double aa = kf[j * ld_k + c], bb = kr[j * ld_k + c];
        for (int f = 0; f < nv.NFIX; ++f) {
            const int ea = nv.foldf[j * nv.NFIX + f], eb = nv.foldr[j * nv.NFIX + f];
            if (ea | eb) {
                const double w = cv.fixc[f * cv.ld_fix + c * cv.s_fix];
                if (ea) aa *= ipow(w, ea);
                if (eb) bb *= ipow(w, eb);
            }
        }
        if (j == pj) { aa *= pfac; bb *= pfac; }   // old_system.py:504-506
        kb[j] = aa;
        kb[R + j] = bb;
    }
    double y[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        const int i = 4 * gl + s;
        x.rs[s] = x.fl[s] = x.in[s] = 0.0;
        y[s] = 0.0;
        if (i < NS) {
            const double* d = nv.dyn + 4 * i;
            x.rs[s] = (d[2] != 0.0) ? d[1] + d[2] * T : d[1];     // reactor.py:34-41
            x.fl[s] = d[3];
            if (x.fl[s] != 0.0 && cv.inflow) x.in[s] = cv.inflow[i * cv.ld_in + c * cv.s_in];
            y[s] = cv.y0[i * cv.ld_y0 + c * cv.s_y0];
        }
    }
    wsync();
    int ns = 0;
    // (a screening pass is not run here: System.solve_batch screens networks
    // of at most 8 species, all of them on the lane solver; a single pass
    // gives the same answers)
    const TrajOut to{a.t_out, a.n_out, a.traj, a.ld_traj, c};
    int st = q_integrate<Net, TRAJ>(x, y, a.t0, a.t_end, a.rtol, a.atol, a.max_steps, ns, to);
    if constexpr (NEWTON) {
        if (st == PCK_ST_OK && a.newton) st = q_newton<Net>(x, y, a.newton_iters, a.root_dist, a.atol);
    }
    const double tof = q_tof<Net>(nv, x, y);
    bool fin = isfinite(tof);
#pragma unroll
    for (int s = 0; s < 4; ++s) fin = fin && isfinite(y[s]);
    fin = qmin(fin ? 1.0 : 0.0) > 0.0;
    if (!fin && st == PCK_ST_OK) st = PCK_ST_NONFINITE;
    if (ga.M > 1) {
        if (gl == 0) {
            ga.tofbuf[(int64_t)q * cv.n + c] = tof;
            ga.stbuf[(int64_t)q * cv.n + c] = st;
            ga.nsbuf[(int64_t)q * cv.n + c] = ns;
        }
        return;
    }
    const bool keep = a.retry_pass == 1 && st != PCK_ST_OK;
    if (a.retry_pass == 1) st = keep ? PCK_ST_NEWTON_LOOSE : PCK_ST_NEWTON;
    if (a.y && !keep) {
#pragma unroll
        for (int s = 0; s < 4; ++s)
            if (4 * gl + s < NS) a.y[(4 * gl + s) * a.ld_y + c] = y[s];
    }
    if (gl == 0) {
        if (a.tof && !keep)
            a.tof[c] = a.want_activity ? (log((hP * tof) / (kB * T)) * (Rgas * T)) * 1.0e-3 / eVtokJ : tof;
        if (a.status) a.status[c] = st;
        if (a.nsteps) a.nsteps[c] = a.retry_pass ? a.nsteps[c] + ns : ns;
    }
}

}  // namespace pck
