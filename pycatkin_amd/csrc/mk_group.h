// Lane-group solver: one condition per group of G = 16 / 32 / 64 lanes of a
// wavefront, one species row per lane.  Used for networks with more than
// PCK_MAX_DYN_LANE dynamic species (DMTM: 11, test/CH4_input.json: 16, the
// 50-species synthetic network) and for networks whose reaction count does
// not fit the one-lane-per-condition LDS budget.
//
//   lane i of a group owns species i: y_i, every Rosenbrock stage entry,
//   row i of the iteration matrix (NSP doubles in VGPRs, static indices).
//   Rates are evaluated from the concentration vector the group keeps in
//   LDS, over the sparse plan (participants of each reaction, CSR of S by
//   species) -- pycatkin/classes/old_system.py:202-313, system.py:345-508.
//   The Jacobian row is scattered into an LDS column block, then loaded into
//   registers.  Dense LU with partial pivoting across the group: the pivot is
//   an integer max-reduction (|a| as float bits, lane id in the low 6 bits),
//   the pivot row is broadcast through LDS, every row lane eliminates its own
//   row.  Triangular solves broadcast one entry per column by __shfl.
//   Norms / step-size decisions are butterfly all-reductions, bitwise equal
//   on every lane of the group, so control flow is group-uniform.
//
// LDS per group (doubles): kf[R] kr[R] | c[NSP] | pivot row[NSP] | J[NSP][NSP]
#pragma once
#include "mk_device.h"
#include "mk_solver.h"

namespace pck {

// Sparse plan (built by pck_network_create from the dense blocks).
struct GrpView {
    const int32_t* rx_ptr;   // NRXN+1: participants of reaction r
    const int32_t* rx_sp;    // participant species
    const int32_t* rx_e;     // (forward exponent << 8) | reverse exponent
    const double* rx_cf;     // participant's concentration factor cf
    const int32_t* row_ptr;  // NDYN+1: CSR of S by species
    const int32_t* row_rx;   // reaction
    const double* row_s;     // S[i][r]
};

__device__ __forceinline__ void wsync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

template <int G>
__device__ __forceinline__ double gsum(double v) {
#pragma unroll
    for (int m = G / 2; m >= 1; m >>= 1) v += __shfl_xor(v, m, G);
    return v;
}
template <int G>
__device__ __forceinline__ double gmax(double v) {
#pragma unroll
    for (int m = G / 2; m >= 1; m >>= 1) v = fmax(v, __shfl_xor(v, m, G));
    return v;
}
template <int G>
__device__ __forceinline__ double gmin(double v) {
#pragma unroll
    for (int m = G / 2; m >= 1; m >>= 1) v = fmin(v, __shfl_xor(v, m, G));
    return v;
}
template <int G>
__device__ __forceinline__ int gmaxi(int v) {
#pragma unroll
    for (int m = G / 2; m >= 1; m >>= 1) v = max(v, __shfl_xor(v, m, G));
    return v;
}

// Per-group context: LDS blocks and this lane's species row.
template <int NSP>
struct Grp {
    int gl, NS, R;
    bool row;                 // gl < NS
    double* kf; double* kr;   // effective rate constants (fixed species folded, DRC perturbation)
    double* c;                // concentrations c_q = cf_q y_q
    double* pb;               // pivot-row broadcast
    double* J;                // Jacobian scatter block, column-major: J[q*NSP + i]
    double cf, rs, fl, in;    // this row's concentration factor, row scale, flow, inflow
};

__device__ __forceinline__ double rate_net(const GrpView& g, const double* kf, const double* kr, const double* c,
                                           int r) {
    double a = kf[r], b = kr[r];
    const int p1 = g.rx_ptr[r + 1];
    for (int p = g.rx_ptr[r]; p < p1; ++p) {
        const double x = c[g.rx_sp[p]];
        const int e = g.rx_e[p];
        const int ef = e >> 8, er = e & 255;
        if (ef) a *= ipow(x, ef);
        if (er) b *= ipow(x, er);
    }
    return a - b;
}

// d(net_r)/d(y_q) for participant slot p0 of reaction r
__device__ __forceinline__ double drate_net(const GrpView& g, const double* kf, const double* kr, const double* c,
                                            int r, int p0) {
    const int e0 = g.rx_e[p0];
    const int ef0 = e0 >> 8, er0 = e0 & 255;
    const double x0 = c[g.rx_sp[p0]];
    double a = ef0 ? kf[r] * (double)ef0 * ipow(x0, ef0 - 1) : 0.0;
    double b = er0 ? kr[r] * (double)er0 * ipow(x0, er0 - 1) : 0.0;
    const int p1 = g.rx_ptr[r + 1];
    for (int p = g.rx_ptr[r]; p < p1; ++p) {
        if (p == p0) continue;
        const double x = c[g.rx_sp[p]];
        const int e = g.rx_e[p];
        const int ef = e >> 8, er = e & 255;
        if (ef) a *= ipow(x, ef);
        if (er) b *= ipow(x, er);
    }
    return (a - b) * g.rx_cf[p0];
}

// f_i = rs_i * sum_r S_ir net_r + fl_i (in_i - y_i)   (row lanes; 0 elsewhere)
template <int NSP>
__device__ __forceinline__ double grp_rhs(const GrpView& g, const Grp<NSP>& x, double y) {
    wsync();                                   // previous readers of c are done
    if (x.row) x.c[x.gl] = x.cf * y;
    wsync();
    double f = 0.0;
    if (x.row) {
        const int e1 = g.row_ptr[x.gl + 1];
        for (int e = g.row_ptr[x.gl]; e < e1; ++e) f += g.row_s[e] * rate_net(g, x.kf, x.kr, x.c, g.row_rx[e]);
        f = f * x.rs + x.fl * (x.in - y);
    }
    return f;
}

// W[q] = sgn * dF_i/dy_q + (q == i ? shift : 0), with dF/dy including the flow
// diagonal (-fl_i).  The scatter block is read back and cleared.
template <int NSP>
__device__ __forceinline__ void grp_jac(const GrpView& g, const Grp<NSP>& x, double y, double sgn, double shift,
                                        double (&W)[NSP]) {
    wsync();
    if (x.row) x.c[x.gl] = x.cf * y;
    wsync();
    if (x.row) {
        const int e1 = g.row_ptr[x.gl + 1];
        for (int e = g.row_ptr[x.gl]; e < e1; ++e) {
            const int r = g.row_rx[e];
            const double s = g.row_s[e];
            const int p1 = g.rx_ptr[r + 1];
            for (int p = g.rx_ptr[r]; p < p1; ++p) {
                const double d = drate_net(g, x.kf, x.kr, x.c, r, p);
                x.J[g.rx_sp[p] * NSP + x.gl] += s * d;
            }
        }
    }
    const double sc = sgn * x.rs;
    const double dg = shift - sgn * x.fl;
#pragma unroll
    for (int q = 0; q < NSP; ++q) {
        const double v = x.J[q * NSP + x.gl];
        x.J[q * NSP + x.gl] = 0.0;
        W[q] = sc * v + (q == x.gl ? dg : 0.0);
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

// In-place LU of the group's rows with partial pivoting.  step = column at
// which this lane's row became the pivot (NSP: padding lane).  Multipliers
// stay in the eliminated rows' columns, the pivot row keeps U and stores
// 1/U_kk in its pivot column.  Returns false on a zero / non-finite pivot.
template <int NSP, int G>
__device__ __forceinline__ bool grp_lu(const Grp<NSP>& x, double (&W)[NSP], Perm<NSP>& pk, int& step) {
    bool fre = x.row;
    bool ok = true;
    step = NSP;
#pragma unroll
    for (int i = 0; i < (NSP + 3) / 4; ++i) pk.w[i] = 0u;
    // single-exit loops with group-uniform guards, so the column index stays static
#pragma unroll
    for (int k = 0; k < NSP; ++k) {
        if (k < x.NS && ok) {
            const float mag = (float)fabs(W[k]);
            int key = fre ? (int)((__float_as_uint(mag) & ~63u) | (uint32_t)x.gl) : -1;
            key = gmaxi<G>(key);
            const int p = key & 63;
            wsync();
            if (x.gl == p) {
#pragma unroll
                for (int j = k; j < NSP; ++j) x.pb[j] = W[j];
                fre = false;
                step = k;
            }
            wsync();
            pk.set(k, p);
            const double piv = x.pb[k];
            ok = key >= 0 && piv != 0.0 && isfinite(piv);
            const double inv = 1.0 / piv;
            if (fre && ok) {
                const double l = W[k] * inv;
                W[k] = l;
#pragma unroll
                for (int j = k + 1; j < NSP; ++j) W[j] -= l * x.pb[j];
            }
            if (x.gl == p) W[k] = inv;
        }
    }
    return ok;
}

// Solve LU x = b for the group; b_i on lane i in, x_i on lane i out.
template <int NSP, int G>
__device__ __forceinline__ double grp_solve(const Grp<NSP>& x, const double (&W)[NSP], const Perm<NSP>& pk,
                                            int step, double b) {
#pragma unroll
    for (int k = 0; k < NSP; ++k) {
        if (k < x.NS) {
            const double bk = __shfl(b, pk.get(k), G);
            if (step > k) b -= W[k] * bk;
        }
    }
    double out = 0.0;
#pragma unroll
    for (int kk = 0; kk < NSP; ++kk) {
        const int k = NSP - 1 - kk;
        if (k < x.NS) {
            const double xk = __shfl(b * W[k], pk.get(k), G);
            if (step < k) b -= W[k] * xk;
            if (x.gl == k) out = xk;
        }
    }
    return out;
}

// ---------------------------------------------------------------------------
// RODAS4 on the group (same scheme, controller and projection as mk_solver.h)
// ---------------------------------------------------------------------------
template <int NSP, int G>
__device__ __forceinline__ int grp_integrate(const NetView& nv, const GrpView& gv, const Grp<NSP>& x, double& y, double t0,
                             double t_end, double rtol, double atol, int max_steps, int& nsteps) {
    using namespace rodas4;
    const int NS = x.NS;
    const double invNS = 1.0 / NS;
    nsteps = 0;
    const double span = t_end - t0;
    if (!(span > 0.0)) return PCK_ST_OK;
    double F0 = grp_rhs(gv, x, y);
    double cons0[PCK_MAX_CONS];
    double ci[PCK_MAX_CONS];
    bool cpos[PCK_MAX_CONS];
#pragma unroll
    for (int l = 0; l < PCK_MAX_CONS; ++l) if (l < nv.NCONS) {
        ci[l] = x.row ? nv.C[l * NS + x.gl] : 0.0;
        cons0[l] = gsum<G>(ci[l] * y);
        cpos[l] = gmin<G>(ci[l]) >= 0.0;
    }
    double h;
    {
        const double sc = atol + rtol * fabs(y);
        const double d0 = sqrt(gsum<G>(x.row ? (y / sc) * (y / sc) : 0.0) * invNS);
        const double d1 = sqrt(gsum<G>(x.row ? (F0 / sc) * (F0 / sc) : 0.0) * invNS);
        double h0 = (d0 < 1e-5 || d1 < 1e-5) ? 1e-6 : 0.01 * d0 / d1;
        h0 = fmin(h0, span);
        const double F1 = grp_rhs(gv, x, y + h0 * F0);
        const double q = (F1 - F0) / sc;
        const double d2 = sqrt(gsum<G>(x.row ? q * q : 0.0) * invNS) / h0;
        const double h1 = (d1 <= 1e-15 && d2 <= 1e-15) ? fmax(1e-6, h0 * 1e-3) : pow(0.01 / fmax(d1, d2), 0.2);
        h = fmin(fmin(100.0 * h0, h1), span);
    }
    double t = t0;
    double W[NSP];
    Perm<NSP> pk;
    int step;
    while (t < t_end) {
        if (nsteps >= max_steps) return PCK_ST_MAXSTEPS;
        ++nsteps;
        bool last = false;
        if (t + h >= t_end) { h = t_end - t; last = true; }
        const double ig = 1.0 / (h * g);
        grp_jac(gv, x, y, -1.0, ig, W);                  // W = I/(h g) - J
        if (!grp_lu<NSP, G>(x, W, pk, step)) { h *= 0.25; continue; }
        const double ih = 1.0 / h;
        const double k1 = grp_solve<NSP, G>(x, W, pk, step, F0);
        double fu = grp_rhs(gv, x, y + a21 * k1);
        const double k2 = grp_solve<NSP, G>(x, W, pk, step, fu + ih * (C21 * k1));
        fu = grp_rhs(gv, x, y + a31 * k1 + a32 * k2);
        const double k3 = grp_solve<NSP, G>(x, W, pk, step, fu + ih * (C31 * k1 + C32 * k2));
        fu = grp_rhs(gv, x, y + a41 * k1 + a42 * k2 + a43 * k3);
        const double k4 = grp_solve<NSP, G>(x, W, pk, step, fu + ih * (C41 * k1 + C42 * k2 + C43 * k3));
        double u = y + a51 * k1 + a52 * k2 + a53 * k3 + a54 * k4;
        fu = grp_rhs(gv, x, u);
        const double k5 = grp_solve<NSP, G>(x, W, pk, step, fu + ih * (C51 * k1 + C52 * k2 + C53 * k3 + C54 * k4));
        u += k5;
        fu = grp_rhs(gv, x, u);
        const double k6 =
            grp_solve<NSP, G>(x, W, pk, step, fu + ih * (C61 * k1 + C62 * k2 + C63 * k3 + C64 * k4 + C65 * k5));
        u += k6;
        const bool fin_l = !x.row || (isfinite(u) && isfinite(k6));
        const double fin = gmin<G>(fin_l ? 1.0 : 0.0);
        const double sc = atol + rtol * fmax(fabs(y), fabs(u));
        const double r = k6 / sc;
        const double s = gsum<G>(x.row ? r * r : 0.0);
        const double en = (fin > 0.0) ? sqrt(s * invNS) : INFINITY;
        if (en <= 1.0) {
            t = last ? t_end : t + h;
            y = x.row ? u : 0.0;
        #pragma unroll
    for (int l = 0; l < PCK_MAX_CONS; ++l) if (l < nv.NCONS) {
                const double sm = gsum<G>(ci[l] * y);
                if (cpos[l] && sm > 0.0) {
                    const double fct = cons0[l] / sm;
                    if (ci[l] != 0.0) y *= fct;
                }
            }
            F0 = grp_rhs(gv, x, y);
            const double fac = (en > 0.0) ? 0.9 * rsqrt(sqrt(en)) : 6.0;
            h *= fmin(6.0, fmax(0.2, fac));
        } else {
            h *= (fin > 0.0) ? fmax(0.2, 0.9 * rsqrt(sqrt(en))) : 0.25;
        }
        if (!(h > 1e-15 * fmax(fabs(t), 1e-300)) && t < t_end) return PCK_ST_STEPFAIL;
    }
    return PCK_ST_OK;
}

// Newton steady-state polish (same rules as mk_solver.h: newton)
template <int NSP, int G>
__device__ __forceinline__ int grp_newton(const NetView& nv, const GrpView& g, const Grp<NSP>& x, double& y, int iters) {
    const int NS = x.NS;
    double b[PCK_MAX_CONS], ci[PCK_MAX_CONS];
    int piv_l[PCK_MAX_CONS];
#pragma unroll
    for (int l = 0; l < PCK_MAX_CONS; ++l) if (l < nv.NCONS) {
        ci[l] = x.row ? nv.C[l * NS + x.gl] : 0.0;
        b[l] = gsum<G>(ci[l] * y);
        piv_l[l] = nv.cpiv[l];
    }
    double z = y;
    bool conv = false;
    double prev = INFINITY, lastq = 1.0;
    int linear = 0;
    double W[NSP];
    Perm<NSP> pk;
    int step;
    for (int it = 0; it < iters; ++it) {
        double Gv = grp_rhs(g, x, z);
        grp_jac(g, x, z, 1.0, 0.0, W);
    #pragma unroll
    for (int l = 0; l < PCK_MAX_CONS; ++l) if (l < nv.NCONS) {
            const double s = gsum<G>(ci[l] * z);
            if (x.gl == piv_l[l]) {
                Gv = s - b[l];
#pragma unroll
                for (int q = 0; q < NSP; ++q) W[q] = (q < NS) ? nv.C[l * NS + q] : 0.0;
            }
        }
        double m = 0.0;
#pragma unroll
        for (int q = 0; q < NSP; ++q) m = fmax(m, fabs(W[q]));
        const double sc = (m > 0.0) ? 1.0 / m : 1.0;
#pragma unroll
        for (int q = 0; q < NSP; ++q) W[q] *= sc;
        Gv = -Gv * sc;
        if (!grp_lu<NSP, G>(x, W, pk, step)) break;
        double dz = grp_solve<NSP, G>(x, W, pk, step, Gv);
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
        if (rel < 1e-12 || (it >= 2 && rel < 1e-7 && rel > 0.5 * prev)) { conv = true; break; }
        lastq = rel / prev;
        linear = (rel > 0.25 * prev) ? linear + 1 : 0;
        if (linear >= 12) break;
        prev = rel;
    }
    if (!conv) return PCK_ST_NEWTON;
    if (gmin<G>((x.row && z < 0.0) ? -1.0 : 1.0) < 0.0) return PCK_ST_NEWTON;
    y = z;
    return PCK_ST_OK;
}

// ---------------------------------------------------------------------------
// group setup + kernels
// ---------------------------------------------------------------------------
__host__ __device__ inline size_t grp_lds_doubles(int R, int NSP) {
    return (size_t)2 * (R > 0 ? R : 1) + 2 * (size_t)NSP + (size_t)NSP * NSP;
}

template <int NSP, int G>
__device__ __forceinline__ void grp_setup(const NetView& nv, const CondView& cv, int64_t c, const double* kf,
                                          const double* kr, int64_t ld_k, int pj, double pfac, double* base,
                                          Grp<NSP>& x, double& T) {
    const int R = nv.NRXN;
    x.gl = threadIdx.x % G;
    x.NS = nv.NDYN;
    x.R = R;
    x.row = x.gl < x.NS;
    x.kf = base;
    x.kr = base + (R > 0 ? R : 1);
    x.c = x.kr + (R > 0 ? R : 1);
    x.pb = x.c + NSP;
    x.J = x.pb + NSP;
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
#pragma unroll
    for (int q = 0; q < NSP; ++q) x.J[q * NSP + x.gl] = 0.0;
    x.cf = x.rs = x.fl = x.in = 0.0;
    if (x.row) {
        const double* d = nv.dyn + 4 * x.gl;
        x.cf = d[0];
        x.rs = (d[2] != 0.0) ? d[1] + d[2] * T : d[1];   // reactor.py:34-41
        x.fl = d[3];
        if (x.fl != 0.0 && cv.inflow) x.in = cv.inflow[x.gl * cv.ld_in + c * cv.s_in];
    }
    wsync();
}

// TOF of the group's state (old_system.py:482-488), valid on every lane
template <int NSP, int G>
__device__ __forceinline__ double grp_tof(const NetView& nv, const GrpView& g, const Grp<NSP>& x, double y) {
    wsync();
    if (x.row) x.c[x.gl] = x.cf * y;
    wsync();
    double t = 0.0;
    for (int k = x.gl; k < nv.NTOF; k += G) t += rate_net(g, x.kf, x.kr, x.c, nv.tof[k]);
    return gsum<G>(t);
}

struct GrpArgs {
    int M;              // groups per condition: 1, or 2R+1 in DRC mode
    double* tofbuf;     // DRC mode: [M][n] TOF per perturbation
    int32_t* stbuf;     // DRC mode: [M][n] status per perturbation
};

template <int NSP, int G>
__global__ void __launch_bounds__(64) k_solve_grp(NetView nv, GrpView gv, CondView cv, const double* kf,
                                                  const double* kr, int64_t ld_k, SolveArgs a, GrpArgs ga) {
    extern __shared__ double lds[];
    const int grp = threadIdx.x / G;
    const int64_t v = (int64_t)blockIdx.x * (64 / G) + grp;
    const int64_t c = v / ga.M;
    const int q = (int)(v % ga.M);
    if (c >= cv.n) return;                          // group-uniform exit; no block barriers below
    int pj = -1;
    double pfac = 1.0;
    if (q > 0) { pj = (q - 1) >> 1; pfac = (q & 1) ? 1.0 + a.eps : 1.0 - a.eps; }
    Grp<NSP> x;
    double T;
    grp_setup<NSP, G>(nv, cv, c, kf, kr, ld_k, pj, pfac, lds + (size_t)grp * grp_lds_doubles(nv.NRXN, NSP), x, T);
    double y = x.row ? cv.y0[x.gl * cv.ld_y0 + c * cv.s_y0] : 0.0;
    int ns = 0;
    int st = grp_integrate<NSP, G>(nv, gv, x, y, a.t0, a.t_end, a.rtol, a.atol, a.max_steps, ns);
    if (st == PCK_ST_OK && a.newton) st = grp_newton<NSP, G>(nv, gv, x, y, a.newton_iters);
    const double tof = grp_tof<NSP, G>(nv, gv, x, y);
    const bool fin = gmin<G>((!x.row || isfinite(y)) ? 1.0 : 0.0) > 0.0 && isfinite(tof);
    if (!fin && st == PCK_ST_OK) st = PCK_ST_NONFINITE;
    if (ga.M > 1) {
        if (x.gl == 0) {
            ga.tofbuf[(int64_t)q * cv.n + c] = tof;
            ga.stbuf[(int64_t)q * cv.n + c] = st;
        }
        return;
    }
    if (a.y && x.row) a.y[x.gl * a.ld_y + c] = y;
    if (x.gl == 0) {
        if (a.tof) a.tof[c] = a.want_activity ? (log((hP * tof) / (kB * T)) * (Rgas * T)) * 1.0e-3 / eVtokJ : tof;
        if (a.status) a.status[c] = st;
        if (a.nsteps) a.nsteps[c] = ns;
    }
}

// DRC combine (old_system.py:490-515): xi_j = (TOF_j+ - TOF_j-) / (2 eps TOF_0)
__global__ void __launch_bounds__(256) k_drc_combine(int64_t n, int R, double eps, const double* tofbuf,
                                                     const int32_t* stbuf, double* xi, int64_t ld_xi, double* tof0,
                                                     int32_t* status) {
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= n) return;
    const double t0 = tofbuf[c];
    int st = stbuf[c];
    for (int j = 0; j < R; ++j) {
        const double tp = tofbuf[(int64_t)(2 * j + 1) * n + c], tm = tofbuf[(int64_t)(2 * j + 2) * n + c];
        xi[j * ld_xi + c] = (tp - tm) / (2.0 * eps * t0);
        st = max(st, max(stbuf[(int64_t)(2 * j + 1) * n + c], stbuf[(int64_t)(2 * j + 2) * n + c]));
    }
    if (tof0) tof0[c] = t0;
    if (status) status[c] = st;
}

template <int NSP, int G>
__global__ void __launch_bounds__(64) k_rates_grp(NetView nv, GrpView gv, CondView cv, const double* kf,
                                                  const double* kr, int64_t ld_k, const double* yin, int64_t ld_y,
                                                  double* out, int jac) {
    extern __shared__ double lds[];
    const int grp = threadIdx.x / G;
    const int64_t c = (int64_t)blockIdx.x * (64 / G) + grp;
    if (c >= cv.n) return;
    Grp<NSP> x;
    double T;
    grp_setup<NSP, G>(nv, cv, c, kf, kr, ld_k, -1, 1.0, lds + (size_t)grp * grp_lds_doubles(nv.NRXN, NSP), x, T);
    const double y = x.row ? yin[x.gl * ld_y + c] : 0.0;
    if (!jac) {
        const double f = grp_rhs(gv, x, y);
        if (x.row) out[x.gl * ld_y + c] = f;
    } else {
        double W[NSP];
        grp_jac(gv, x, y, 1.0, 0.0, W);
        if (x.row) {
#pragma unroll
            for (int q = 0; q < NSP; ++q)
                if (q < x.NS) out[((int64_t)x.gl * x.NS + q) * ld_y + c] = W[q];
        }
    }
}

}  // namespace pck
