// HIP kernels + C-ABI entry points of pycatkin_amd (gfx950 / MI355X).
//
//   k_rate_constants   kernel (1): thermochemistry -> energy program -> kf/kr,
//                      one lane per condition (reaction.py:94, state.py:367)
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
#include <stdlib.h>
#include <string.h>
#include <algorithm>
#include <atomic>
#include <mutex>
#include <new>
#include <vector>
#include "mk_device.h"
#include "mk_group.h"
#include "mk_jit.h"

using namespace pck;

struct pck_network {
    NetView nv;
    int32_t* d_ip = nullptr;
    double* d_dp = nullptr;
    void* d_grp = nullptr;          // lane-group plan (mk_group.h): reaction records, species CSR of S
    int grp_ok = 0;                 // every reaction fits a record (<= 6 participants, exponents <= 31)
    int grp_npmax = 0, grp_emax = 0;  // most participants of a reaction / largest exponent (hipRTC bounds)
    int grp_degmax = 0;               // largest row degree of the species CSR (hipRTC bound)
    GrpView gv;
    int spec = 0;                   // id of the compiled-in plan (networks.h) or 0
    int plan_mode = PCK_PLAN_AUTO;  // pck_network_set_plan_mode
    unsigned long long digest = 0;
    std::string jit_src;            // mk_jit.h: constexpr plan source for hipRTC (lane networks without a compiled plan)
    std::string jit_grp_src;        // the same tables for the lane-group solver's compile-time network (mk_group.h: ct_rhs)
    // diagnostics of the last solve (pck_network_dims), the only fields a solve
    // writes: atomic, so calls from several host threads stay race-free
    mutable std::atomic<bool> jit_on{false};      // the last lane solve ran the hipRTC-compiled plan
    mutable std::atomic<bool> grp_jit_on{false};  // the last lane-group solve ran the exact-size hipRTC kernel
    mutable std::atomic<bool> grp_ct_on{false};   // ... with the network compiled in (mk_group.h: ct_rhs)
    mutable std::atomic<bool> grp_quad_on{false}; // ... the quad-group kernel (mk_quad.h)
    mutable std::atomic<int> grp_lanes{0};        // lanes per condition of the last lane-group solve
};

// FNV-1a 64 over the solver-side structure (network.py: structural_digest)
static unsigned long long fnv1a(unsigned long long h, const void* p, size_t n) {
    const unsigned char* b = (const unsigned char*)p;
    for (size_t i = 0; i < n; ++i) { h ^= b[i]; h *= 0x100000001b3ULL; }
    return h;
}

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
// feat == nullptr: this block's feature columns in LDS (stride blockDim.x),
// else column c of the HBM scratch (stride fs)
__global__ void __launch_bounds__(64) k_rate_constants(NetView nv, CondView cv, double* feat, int64_t fs,
                                                       double* kf, double* kr, int64_t ld_k) {
    extern __shared__ double lds_feat[];
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= cv.n) return;
    const double T = cv.T[c * cv.sT];
    const double p = cv.p[c * cv.sp];
    double* f = feat ? feat + c : lds_feat + threadIdx.x;
    if (!feat) fs = blockDim.x;
    thermo_features(nv, T, p, cv.desc + c * cv.s_desc, cv.ld_desc, f, fs);
    for (int j = 0; j < nv.NRXN; ++j) {
        double a, b;
        rate_constants_from_feat(nv, T, f, fs, j, a, b);
        kf[j * ld_k + c] = a;
        kr[j * ld_k + c] = b;
    }
}

// energy-program registers only (free / reaction energies in eV)
__global__ void __launch_bounds__(64) k_energies(NetView nv, CondView cv, double* feat, int64_t fs, double* out,
                                                 int64_t ld_out) {
    extern __shared__ double lds_feat[];
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= cv.n) return;
    double* f = feat ? feat + c : lds_feat + threadIdx.x;
    if (!feat) fs = blockDim.x;
    thermo_features(nv, cv.T[c * cv.sT], cv.p[c * cv.sp], cv.desc + c * cv.s_desc, cv.ld_desc, f, fs);
    const int rb = 2 + nv.D + 3 * nv.NTH;
    for (int r = 0; r < nv.NREG; ++r) out[r * ld_out + c] = f[(rb + r) * fs];
}

#include "mk_solver.h"

// The solver kernels are compiled in translation units of their own in the
// product build (csrc/mk_inst.h, csrc/tu_*.hip): here they are only declared.
#ifndef PCK_SPLIT_TU
#define PCK_SPLIT_TU 0
#endif
#if PCK_SPLIT_TU
#include "mk_inst.h"
namespace pck {
#define PCK_X(N) PCK_DO_LANE_RT(extern, N)
PCK_INST_LANE_RT(PCK_X)
#undef PCK_X
#define PCK_X(id, T) PCK_DO_LANE_CT(extern, id, T)
PCK_COMPILED_NETWORKS(PCK_X)
#undef PCK_X
#define PCK_X(NP, GG, PP) PCK_DO_GRP(extern, NP, GG, PP)
PCK_INST_GRP(PCK_X)
#undef PCK_X
}  // namespace pck
#endif

// forward / reverse rate of every active reaction at states y, fixed species
// folded in (System._calc_rates, system.py:345-376; old_system.py:202-225
// reaction_terms).  One lane per condition; not on the solve path.
__global__ void __launch_bounds__(64) k_reaction_rates(NetView nv, CondView cv, const double* kf, const double* kr,
                                                       int64_t ld_k, const double* y, int64_t ld_y, double* rf,
                                                       double* rr, int64_t ld_r) {
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= cv.n) return;
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
        for (int i = 0; i < nv.NDYN; ++i) {
            const int ea = nv.expf[j * nv.NDYN + i], eb = nv.expr[j * nv.NDYN + i];
            if (ea | eb) {
                const double x = nv.dyn[4 * i] * y[i * ld_y + c];
                if (ea) a *= ipow(x, ea);
                if (eb) b *= ipow(x, eb);
            }
        }
        rf[j * ld_r + c] = a;
        rr[j * ld_r + c] = b;
    }
}

// ----------------------------------------------------------------------------
// C-ABI
// ----------------------------------------------------------------------------
extern "C" int pck_abi_version(void) { return PCK_ABI_VERSION; }

#ifdef PCK_TRACE
// diagnostic builds only: trace the lane-group integrator of one condition
extern "C" int pck_trace_set(long long cond) {
    int zero = 0;
    HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(pck_trace_cond), &cond, sizeof(cond)));
    HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(pck_trace_pos), &zero, sizeof(zero)));
    const double ph0[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(pck_phase), ph0, sizeof(ph0)));
    return PCK_OK;
}
extern "C" int pck_phase_get(double* host8) {
    HIPCHK(hipDeviceSynchronize());
    HIPCHK(hipMemcpyFromSymbol(host8, HIP_SYMBOL(pck_phase), sizeof(double) * 8));
    return PCK_OK;
}
extern "C" int pck_trace_get(double* host, int* pos) {
    HIPCHK(hipDeviceSynchronize());
    HIPCHK(hipMemcpyFromSymbol(pos, HIP_SYMBOL(pck_trace_pos), sizeof(int)));
    HIPCHK(hipMemcpyFromSymbol(host, HIP_SYMBOL(pck_trace_buf), sizeof(double) * PCK_TRACE_N * PCK_TRACE_W));
    return PCK_OK;
}
#endif
#if PCK_PHASE
// diagnostic builds only (-DPCK_PHASE=1): the lane integrator's phase
// counters (mk_solver.h: PCK_LPH), zeroed / read by tools/phase_lane.py
extern "C" int pck_lphase_reset(void) {
    const double z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(pck_lphase), z, sizeof(z)));
    return PCK_OK;
}
extern "C" int pck_lphase_get(double* host8) {
    HIPCHK(hipDeviceSynchronize());
    HIPCHK(hipMemcpyFromSymbol(host8, HIP_SYMBOL(pck_lphase), sizeof(double) * 8));
    return PCK_OK;
}
#endif
#if PCK_WAVE_TIMES
// diagnostic builds only (-DPCK_WAVE_TIMES=1): the lane solver's wave
// timeline (mk_solver.h), read by tools/wave_timeline.py
extern "C" int pck_wtimes_get(long long* host, int n) {
    HIPCHK(hipDeviceSynchronize());
    HIPCHK(hipMemcpyFromSymbol(host, HIP_SYMBOL(pck_wtimes), sizeof(long long) * 3 * (size_t)(n < PCK_WT_N ? n : PCK_WT_N)));
    return PCK_OK;
}
#endif
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
        for (int i = 0; i < nv.NDYN; ++i) {
            const int ea = ip[oef + j * nv.NDYN + i], eb = ip[oer + j * nv.NDYN + i];
            if (ea < 0 || eb < 0) return fail(PCK_E_ARG, "negative exponent%s", "");
            if (ea > PCK_MAX_EXP || eb > PCK_MAX_EXP) return fail(PCK_E_SIZE, "exponent%s above %lld", "", PCK_MAX_EXP);
        }
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
        (void)hipFree(net->d_ip); (void)hipFree(net->d_dp); delete net;
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
    // lane-group plan (mk_group.h): one 16-byte record per reaction (packed
    // participants + offset of their derivatives) and the species CSR of S
    // whose entries carry the reaction's participants
    {
        const int R = nv.NRXN, NS = nv.NDYN;
        const double* S = dp + doff[PCK_D_STOICH];
        std::vector<uint32_t> rx(4 * (size_t)(R > 0 ? R : 1), 0u);
        std::vector<int> npv(R > 0 ? R : 1, 0), dpv(R > 0 ? R : 1, 0), spv(6 * (size_t)(R > 0 ? R : 1), 0);
        net->grp_ok = (R <= 511) ? 1 : 0;
        int ND = 0;
        for (int j = 0; j < R; ++j) {
            uint32_t w[3] = {0, 0, 0};
            int n = 0;
            for (int i = 0; i < NS; ++i) {
                const int ea = ip[oef + j * NS + i], eb = ip[oer + j * NS + i];
                if (!(ea | eb)) continue;
                if (n == PCK_GRP_MAX_PART || ea > PCK_GRP_MAX_EXP || eb > PCK_GRP_MAX_EXP) {
                    net->grp_ok = 0;
                    continue;
                }
                net->grp_emax = std::max(net->grp_emax, std::max(ea, eb));
                const uint32_t f = (uint32_t)i | ((uint32_t)ea << 6) | ((uint32_t)eb << 11);
                w[n >> 1] |= f << (16 * (n & 1));
                spv[6 * j + n] = i;
                ++n;
            }
            npv[j] = n;
            net->grp_npmax = std::max(net->grp_npmax, n);
            dpv[j] = ND;
            ND += n;
            rx[4 * j + 0] = w[0]; rx[4 * j + 1] = w[1]; rx[4 * j + 2] = w[2];
            rx[4 * j + 3] = (uint32_t)ND - (uint32_t)n | ((uint32_t)n << 16);
        }
        if (ND > 0x3fff) net->grp_ok = 0;
        std::vector<int32_t> row(NS + 1, 0);
        std::vector<uint32_t> ent;
        for (int i = 0; i < NS; ++i) {
            row[i] = (int32_t)(ent.size() / 4);
            for (int j = 0; j < R; ++j) {
                const double sv = S[i * R + j];
                if (sv == 0.0) continue;
                const int n = npv[j];
                uint32_t a = (uint32_t)j | ((uint32_t)n << 9) | ((uint32_t)dpv[j] << 12);
                if (n > 5) a |= (uint32_t)spv[6 * j + 5] << 26;
                uint32_t bb = 0;
                for (int k = 0; k < n && k < 5; ++k) bb |= (uint32_t)spv[6 * j + k] << (6 * k);
                uint32_t sw[2];
                memcpy(sw, &sv, sizeof(sv));
                ent.push_back(a); ent.push_back(bb); ent.push_back(sw[0]); ent.push_back(sw[1]);
            }
        }
        row[NS] = (int32_t)(ent.size() / 4);
        for (int i = 0; i < NS; ++i) net->grp_degmax = std::max(net->grp_degmax, row[i + 1] - row[i]);
        // balanced walk of the CSR (mk_group.h: GrpView::sch): rows longer than
        // K = ceil(NE / G) entries are cut into near-equal pieces, the pieces
        // packed onto the G lanes longest-first (least-loaded lane, lowest id on
        // ties); PCK_GRP_BALANCE=0: off
        std::vector<uint32_t> sch;
        std::vector<int32_t> xbe(2 * (size_t)NS, 0), xrows;
        int LS = 0, NX = 0;
        {
            const int NE = row[NS];
            const int G = NS <= 16 ? 16 : NS <= 32 ? 32 : 64;      // csrc: grp_g
            const char* eb = getenv("PCK_GRP_BALANCE");
            if (!(eb && eb[0] == '0') && NE > 0 && NE <= 0x3fff && NS > 0) {
                const int K = std::max(1, (NE + G - 1) / G);
                struct Piece { int b, e, slot; };
                std::vector<Piece> pcs;
                for (int i = 0; i < NS; ++i) {
                    const int deg = row[i + 1] - row[i];
                    if (deg == 0) continue;
                    const int m = (deg + K - 1) / K;
                    xbe[2 * i] = NX;
                    for (int p = 0; p < m; ++p)
                        pcs.push_back({row[i] + deg * p / m, row[i] + deg * (p + 1) / m, p == 0 ? i : NS + NX++});
                    xbe[2 * i + 1] = NX;
                    if (m > 1) xrows.push_back(i);
                }
                std::vector<int> ord(pcs.size());
                for (size_t k = 0; k < ord.size(); ++k) ord[k] = (int)k;
                std::stable_sort(ord.begin(), ord.end(), [&](int a, int b2) {
                    return pcs[a].e - pcs[a].b > pcs[b2].e - pcs[b2].b;
                });
                std::vector<int> load(G, 0);
                std::vector<std::vector<int>> lane(G);
                for (int k : ord) {
                    int l = 0;
                    for (int j = 1; j < G; ++j)
                        if (load[j] < load[l]) l = j;
                    lane[l].push_back(k);
                    load[l] += pcs[k].e - pcs[k].b;
                }
                for (int l = 0; l < G; ++l) LS = std::max(LS, load[l]);
                // taken where the longest row is at least 3x the balanced walk:
                // the per-row rate loop takes two entries per iteration, and
                // on CH4 (35 -> 17 entries) the balanced walk measured 1.5x
                // slower per step; on the synthetic network (56 -> 10) 11 %
                // faster (runs r3y / r3za)
                if ((3 * LS > net->grp_degmax && !(eb && eb[0] == '2')) || NS + NX > 1023) {   // 2: always (tests)
                    LS = 0;                                 // no gain (or too many slots): the per-row loops
                } else {
                    sch.assign((size_t)LS * G, 0u);
                    for (int l = 0; l < G; ++l) {
                        int t = 0;
                        for (int k : lane[l])
                            for (int e2 = pcs[k].b; e2 < pcs[k].e; ++e2, ++t)
                                sch[(size_t)t * G + l] = (uint32_t)e2 | ((uint32_t)pcs[k].slot << 14) | PCK_SCH_VALID |
                                                         (e2 == pcs[k].e - 1 ? PCK_SCH_LAST : 0u);
                    }
                }
            }
            if (!LS) { NX = 0; xrows.clear(); }
        }
        if (sch.empty()) sch.assign(1, 0u);
        if (xrows.empty()) xrows.assign(1, 0);
        if (xbe.empty()) xbe.assign(2, 0);
        if (ent.empty()) ent.assign(4, 0u);
        const size_t brx = sizeof(uint32_t) * rx.size(), bent = sizeof(uint32_t) * ent.size();
        const size_t brow = sizeof(int32_t) * row.size(), bsch = sizeof(uint32_t) * sch.size();
        const size_t bxbe = sizeof(int32_t) * xbe.size(), bxr = sizeof(int32_t) * xrows.size();
        char* buf = nullptr;
        e = hipMalloc((void**)&buf, brx + bent + brow + bsch + bxbe + bxr);
        if (e == hipSuccess) e = hipMemcpy(buf, rx.data(), brx, hipMemcpyHostToDevice);
        if (e == hipSuccess) e = hipMemcpy(buf + brx, ent.data(), bent, hipMemcpyHostToDevice);
        if (e == hipSuccess) e = hipMemcpy(buf + brx + bent, row.data(), brow, hipMemcpyHostToDevice);
        size_t o = brx + bent + brow;
        if (e == hipSuccess) e = hipMemcpy(buf + o, sch.data(), bsch, hipMemcpyHostToDevice);
        if (e == hipSuccess) e = hipMemcpy(buf + o + bsch, xbe.data(), bxbe, hipMemcpyHostToDevice);
        if (e == hipSuccess) e = hipMemcpy(buf + o + bsch + bxbe, xrows.data(), bxr, hipMemcpyHostToDevice);
        net->gv.sch = (const uint32_t*)(buf + o);
        net->gv.xbe = (const int32_t*)(buf + o + bsch);
        net->gv.xrows = (const int32_t*)(buf + o + bsch + bxbe);
        net->gv.LS = LS;
        net->gv.NX = NX;
        net->gv.NXR = LS ? (int)xrows.size() : 0;
        net->d_grp = buf;
        if (e != hipSuccess) {
            (void)hipFree(net->d_ip); (void)hipFree(net->d_dp); (void)hipFree(buf);
            delete net;
            return fail(PCK_E_HIP, "HIP error: %s (%lld)", hipGetErrorString(e), (long long)e);
        }
        net->gv.rx = (const uint4*)buf;
        net->gv.ent = (const uint4*)(buf + brx);
        net->gv.row = (const int32_t*)(buf + brx + bent);
        net->gv.ND = ND;
        net->gv.NE = row[NS];
    }
    // structural digest -> compiled-in plan (same bytes as network.py: structural_digest)
    {
        const int32_t hdr3[3] = {nv.NDYN, nv.NRXN, nv.NCONS};
        unsigned long long h = 0xcbf29ce484222325ULL;
        h = fnv1a(h, hdr3, sizeof(hdr3));
        h = fnv1a(h, ip + oef, sizeof(int32_t) * nv.NRXN * nv.NDYN);
        h = fnv1a(h, ip + oer, sizeof(int32_t) * nv.NRXN * nv.NDYN);
        h = fnv1a(h, dp + doff[PCK_D_STOICH], sizeof(double) * nv.NDYN * nv.NRXN);
        h = fnv1a(h, dp + doff[PCK_D_DYN], sizeof(double) * 4 * nv.NDYN);
        h = fnv1a(h, dp + doff[PCK_D_CONS], sizeof(double) * nv.NCONS * nv.NDYN);
        h = fnv1a(h, ip + ocp, sizeof(int32_t) * nv.NCONS);
        net->digest = h;
#define PCK_MATCH(id, T) \
        if (h == T::DIGEST && nv.NDYN == T::NS && nv.NRXN == T::R && nv.NCONS == T::NCONS) net->spec = id;
        PCK_COMPILED_NETWORKS(PCK_MATCH)
#undef PCK_MATCH
        if (nv.NDYN >= 1 && nv.NDYN <= PCK_MAX_DYN_LANE)        // hipRTC plan (also for trajectory solves)
            net->jit_src = jit_source(nv.NDYN, nv.NRXN, nv.NCONS, ip + oef, ip + oer, dp + doff[PCK_D_STOICH],
                                      dp + doff[PCK_D_DYN], dp + doff[PCK_D_CONS], ip + ocp);
        if (nv.NDYN >= 1 && net->grp_ok)
            net->jit_grp_src = nv.NDYN <= PCK_MAX_DYN_LANE
                                   ? net->jit_src
                                   : jit_source(nv.NDYN, nv.NRXN, nv.NCONS, ip + oef, ip + oer,
                                                dp + doff[PCK_D_STOICH], dp + doff[PCK_D_DYN], dp + doff[PCK_D_CONS],
                                                ip + ocp);
    }
    *out = net;
    return PCK_OK;
}

extern "C" int pck_network_destroy(pck_network* net) {
    if (!net) return PCK_OK;
    (void)hipFree(net->d_ip); (void)hipFree(net->d_dp); (void)hipFree(net->d_grp);
    delete net;
    return PCK_OK;
}

extern "C" int pck_network_dims(const pck_network* net, int32_t* dims) {
    if (!net || !dims) return fail(PCK_E_ARG, "null argument%s", "");
    const NetView& v = net->nv;
    dims[0] = v.D; dims[1] = v.NTH; dims[2] = v.NREG; dims[3] = v.NRXN; dims[4] = v.NDYN;
    dims[5] = v.NFIX; dims[6] = v.NCONS; dims[7] = v.NTOF; dims[8] = v.nfeat;
    dims[9] = net->spec ? net->spec : net->jit_on.load(std::memory_order_relaxed) ? PCK_SPEC_JIT : 0;
    dims[10] = net->grp_quad_on.load(std::memory_order_relaxed) ? 3
               : net->grp_ct_on.load(std::memory_order_relaxed) ? 2
               : net->grp_jit_on.load(std::memory_order_relaxed) ? 1 : 0;
    return PCK_OK;
}

extern "C" int pck_network_group_lanes(const pck_network* net, int32_t* lanes) {
    if (!net || !lanes) return fail(PCK_E_ARG, "null argument%s", "");
    *lanes = net->grp_lanes.load(std::memory_order_relaxed);
    return PCK_OK;
}

extern "C" int pck_network_set_plan_mode(pck_network* net, int mode) {
    if (!net) return fail(PCK_E_ARG, "null network%s", "");
    if (mode < PCK_PLAN_AUTO || mode > PCK_PLAN_GROUP) return fail(PCK_E_ARG, "unknown plan mode%s %lld", "", mode);
    net->plan_mode = mode;
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

// Per-call device scratch, stream-ordered: allocated on the caller's stream
// before the launches that use it and released on the same stream after them
// (hipFreeAsync in the destructor, on every return path).  Calls on different
// streams -- or on one stream, back to back -- never share a buffer, so the
// network handle is read-only after pck_network_create.  The default pool of
// the device keeps freed blocks (release threshold raised once per device),
// so repeated calls do not go back to the driver.
struct StreamScratch {
    void* p = nullptr;
    hipStream_t s = nullptr;
    StreamScratch() = default;
    StreamScratch(const StreamScratch&) = delete;
    StreamScratch& operator=(const StreamScratch&) = delete;
    ~StreamScratch() { if (p) (void)hipFreeAsync(p, s); }
    template <class T> T* as() const { return static_cast<T*>(p); }
};

static void pool_keep_blocks() {
    static std::mutex mu;
    static unsigned long long done = 0;     // bit per device
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return;
    std::lock_guard<std::mutex> lk(mu);
    if (done & (1ULL << dev)) return;
    done |= 1ULL << dev;
    hipMemPool_t pool;
    if (hipDeviceGetDefaultMemPool(&pool, dev) == hipSuccess) {
        uint64_t thr = ~0ULL;
        (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &thr);
    }
}

static int salloc(StreamScratch& b, size_t bytes, hipStream_t s) {
    pool_keep_blocks();
    b.s = s;
    HIPCHK(hipMallocAsync(&b.p, bytes > 0 ? bytes : 8, s));
    return PCK_OK;
}

// kernel (1): the feature columns of a block live in LDS when they fit
// (nfeat x 64 lanes x 8 B <= 64 KiB), else in per-call HBM scratch
static constexpr int RC_BLOCK = 64;
static inline bool rc_feat_in_lds(int nfeat) { return (size_t)nfeat * RC_BLOCK * sizeof(double) <= 64 * 1024; }

static int launch_rate_constants(const pck_network* net, const pck_conditions* cond, double* kf, double* kr,
                                 int64_t ld_k, hipStream_t s) {
    const int64_t n = cond->n;
    if (n == 0) return PCK_OK;
    const int nfeat = net->nv.nfeat;
    StreamScratch scr;
    size_t shm = 0;
    double* feat = nullptr;
    int64_t fs = 0;
    if (rc_feat_in_lds(nfeat)) {
        shm = sizeof(double) * (size_t)nfeat * RC_BLOCK;
    } else {
        int rc = salloc(scr, sizeof(double) * (size_t)nfeat * n, s);
        if (rc) return rc;
        feat = scr.as<double>();
        fs = n;
    }
    hipLaunchKernelGGL(k_rate_constants, dim3((unsigned)((n + RC_BLOCK - 1) / RC_BLOCK)), dim3(RC_BLOCK), shm, s,
                       net->nv, cview(cond), feat, fs, kf, kr, ld_k);
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
    const int nfeat = net->nv.nfeat;
    StreamScratch scr;
    size_t shm = 0;
    double* feat = nullptr;
    int64_t fs = 0;
    if (rc_feat_in_lds(nfeat)) {
        shm = sizeof(double) * (size_t)nfeat * RC_BLOCK;
    } else {
        rc = salloc(scr, sizeof(double) * (size_t)nfeat * n, (hipStream_t)stream);
        if (rc) return rc;
        feat = scr.as<double>();
        fs = n;
    }
    hipLaunchKernelGGL(k_energies, dim3((unsigned)((n + RC_BLOCK - 1) / RC_BLOCK)), dim3(RC_BLOCK), shm,
                       (hipStream_t)stream, net->nv, cview(cond), feat, fs, out, ld_out);
    HIPCHK(hipGetLastError());
    return PCK_OK;
}

extern "C" int pck_rate_constants(const pck_network* net, const pck_conditions* cond, double* kf, double* kr,
                                  int64_t ld_k, void* stream) {
    int rc = check_cond(net, cond, false);
    if (rc) return rc;
    if (cond->n > 0 && (!kf || !kr || ld_k < cond->n)) return fail(PCK_E_ARG, "bad kf/kr output%s (ld_k %lld)", "", ld_k);
    return launch_rate_constants(net, cond, kf, kr, ld_k, (hipStream_t)stream);
}

#define PCK_NS_SWITCH(NS, CALL)                                     \
    switch (NS) {                                                   \
    case 1: CALL(1); break; case 2: CALL(2); break;                 \
    case 3: CALL(3); break; case 4: CALL(4); break;                 \
    case 5: CALL(5); break; case 6: CALL(6); break;                 \
    case 7: CALL(7); break; case 8: CALL(8); break;                 \
    default: return fail(PCK_E_SIZE, "NDYN%s unsupported", "");     \
    }

// Lane-group path (mk_group.h) for networks beyond the one-lane-per-condition
// limits: more than PCK_MAX_DYN_LANE dynamic species, a k_eff block that does
// not fit LDS at 128 lanes per block, or DRC needing more than 64 lanes.
static bool use_group(const pck_network* net, int lanes_per_cond) {
    const NetView& v = net->nv;
    return net->plan_mode == PCK_PLAN_GROUP || v.NDYN > PCK_MAX_DYN_LANE || lds_bytes(v.NRXN, v.NDYN, 128) > 64 * 1024 ||
           lanes_per_cond > 64;
}
// Lane-group kernels: compiled-in sizes <NSP, G, P> (NS <= NSP) and the
// exact-size specialisation hipRTC compiles at the first solve (mk_jit.h).
static inline int grp_g(int NS) { return NS <= 16 ? 16 : NS <= 32 ? 32 : 64; }
// Jacobian column passes: the whole NS x NS block in LDS (one pass, 20 KiB
// at NS = 50) -- measured 2.3x faster per Jacobian than 4 passes over a
// 6 KiB block at NS = 50 (tools/phase_group.py).
static inline int grp_p(int) { return 1; }
#define PCK_GRP_SWITCH(NS, CALL)              \
    if ((NS) <= 16) { CALL(16, 16, 1); }       \
    else if ((NS) <= 32) { CALL(32, 32, 1); }  \
    else { CALL(64, 64, 1); }
static inline int grp_nsp_ct(int NS) { return NS <= 16 ? 16 : NS <= 32 ? 32 : 64; }
static inline int grp_p_ct(int) { return 1; }

static int grp_shape(const pck_network* net, int nsp, int P, size_t* shm, int* QB, bool tables = false) {
    const int NS = net->nv.NDYN;
    const int per = 64 / grp_g(NS);
    *QB = (nsp + P - 1) / P;
    *shm = sizeof(double) * per * grp_lds_doubles(net->nv.NRXN, nsp, NS, net->gv.ND, *QB, net->gv.LS, net->gv.NX);
    if (tables) *shm += sizeof(double) * grp_tab_doubles(net->nv.NRXN, net->gv.NE, NS, net->gv.LS * grp_g(NS));
    if (*shm > 64 * 1024)
        return fail(PCK_E_SIZE, "lane-group solver: network needs %s%lld bytes of LDS per wavefront", "", (long long)*shm);
    return PCK_OK;
}

// LDS copies of the network tables (k_solve_grp<..., TAB = true>) pay when
// they do not lower the resident waves per CU: min(VGPR-limited waves,
// LDS-limited blocks) with the tables >= the same without (blocks are one
// wavefront; 512 VGPRs per lane per SIMD, 160 KiB of LDS per CU on gfx950).
// resident wavefronts per SIMD the kernel's VGPR count allows (0 if unknown)
static int grp_waves(hipFunction_t f) {
    int regs = 0;
    if (hipFuncGetAttribute(&regs, HIP_FUNC_ATTRIBUTE_NUM_REGS, f) != hipSuccess || regs <= 0) return 0;
    return std::min(8, 512 / ((regs + 7) / 8 * 8));
}

static bool grp_tables_pay(hipFunction_t f, size_t shm, size_t shm_tab) {
    const int per_simd = grp_waves(f);
    if (per_simd <= 0) return false;
    const long vgpr_waves = 4L * per_simd;
    const long lds = 160L * 1024;
    const long w0 = std::min(vgpr_waves, shm ? lds / (long)shm : vgpr_waves);
    const long w1 = std::min(vgpr_waves, lds / (long)shm_tab);
    return w1 >= w0;
}

static int launch_grp_rates(const pck_network* net, const pck_conditions* cond, const double* kf, const double* kr,
                            int64_t ld_k, const double* y, int64_t ld_y, double* out, int jac, hipStream_t s) {
    if (!net->grp_ok) return fail(PCK_E_SIZE, "lane-group solver: a reaction has more than 6 dynamic participants%s", "");
    const int NS = net->nv.NDYN;
    const int per = 64 / grp_g(NS);
    dim3 g((unsigned)((cond->n + per - 1) / per));
    size_t shm;
    int QB;
    int rc = grp_shape(net, grp_nsp_ct(NS), grp_p_ct(NS), &shm, &QB);
    if (rc) return rc;
#define CALL(NP, GG, PP) hipLaunchKernelGGL((k_rates_grp<NP, GG, PP>), g, dim3(64), shm, s, net->nv, net->gv, cview(cond), kf, kr, ld_k, y, ld_y, out, jac, QB)
    PCK_GRP_SWITCH(NS, CALL)
#undef CALL
    HIPCHK(hipGetLastError());
    return PCK_OK;
}

extern "C" int pck_species_rates(const pck_network* net, const pck_conditions* cond, const double* kf,
                                 const double* kr, int64_t ld_k, const double* y, int64_t ld_y, double* dydt,
                                 void* stream) {
    int rc = check_cond(net, cond, true);
    if (rc) return rc;
    const int64_t n = cond->n;
    if (n == 0) return PCK_OK;
    if (!kf || !kr || !y || !dydt || ld_k < n || ld_y < n) return fail(PCK_E_ARG, "bad state/rate arrays%s", "");
    if (use_group(net, 1)) return launch_grp_rates(net, cond, kf, kr, ld_k, y, ld_y, dydt, 0, (hipStream_t)stream);
    const int B = 128;
    const size_t shm = lds_bytes(net->nv.NRXN, net->nv.NDYN, B);
    dim3 g((unsigned)((n + B - 1) / B));
    const char* edd = getenv("PCK_RATES_DD");     // diagnostics: the double-double residual of the Newton refinement
    if (edd && edd[0] == '1') {
#define CALL(N) hipLaunchKernelGGL((k_species_rates<N, true>), g, dim3(B), shm, (hipStream_t)stream, net->nv, cview(cond), kf, kr, ld_k, y, ld_y, dydt)
        PCK_NS_SWITCH(net->nv.NDYN, CALL)
#undef CALL
    } else {
#define CALL(N) hipLaunchKernelGGL((k_species_rates<N, false>), g, dim3(B), shm, (hipStream_t)stream, net->nv, cview(cond), kf, kr, ld_k, y, ld_y, dydt)
        PCK_NS_SWITCH(net->nv.NDYN, CALL)
#undef CALL
    }
    HIPCHK(hipGetLastError());
    return PCK_OK;
}

extern "C" int pck_reaction_rates(const pck_network* net, const pck_conditions* cond, const double* kf,
                                  const double* kr, int64_t ld_k, const double* y, int64_t ld_y, double* rf,
                                  double* rr, int64_t ld_r, void* stream) {
    int rc = check_cond(net, cond, true);
    if (rc) return rc;
    const int64_t n = cond->n;
    if (n == 0 || net->nv.NRXN == 0) return PCK_OK;
    if (!kf || !kr || !y || !rf || !rr || ld_k < n || ld_y < n || ld_r < n)
        return fail(PCK_E_ARG, "bad state/rate arrays%s", "");
    hipLaunchKernelGGL(k_reaction_rates, dim3((unsigned)((n + 63) / 64)), dim3(64), 0, (hipStream_t)stream, net->nv,
                       cview(cond), kf, kr, ld_k, y, ld_y, rf, rr, ld_r);
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
    if (use_group(net, 1)) return launch_grp_rates(net, cond, kf, kr, ld_k, y, ld_y, jo, 1, (hipStream_t)stream);
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
    if (!(prm->root_dist >= 0.0 && prm->root_dist < 1.0)) return fail(PCK_E_ARG, "root_dist must be in [0, 1)%s", "");
    if (prm->retry_rtol != 0.0 && !(prm->retry_rtol > 0.0 && prm->retry_atol > 0.0))
        return fail(PCK_E_ARG, "retry tolerances must both be positive (or retry_rtol 0)%s", "");
    if (!(prm->screen_rtol >= 0.0) || !(prm->screen_margin >= 0.0 && prm->screen_margin <= 1.0))
        return fail(PCK_E_ARG, "screen_rtol must be >= 0 and screen_margin in [0, 1]%s", "");
    if (prm->screen_rtol > 0.0 && prm->retry_rtol > 0.0)
        return fail(PCK_E_ARG, "screen_rtol and retry_rtol are exclusive%s", "");
    return PCK_OK;
}

// Retry list: the indices c < n with status[c] == want, appended per
// wavefront (one ballot, one vector atomic on the list length per wave that
// has any), so the 64 conditions of a grid patch stay together in the list.
// The list's order across wavefronts follows the atomics; every lane's solve
// is independent of which lanes share its wavefront, so results do not
// depend on it.
// want < 0: every status but PCK_ST_OK (the screening pass's rejects)
__global__ void __launch_bounds__(256) k_select_status(int64_t n, const int32_t* status, int32_t want,
                                                       int64_t* idx, int32_t* cnt) {
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool f = (c < n) && (want < 0 ? status[c] != PCK_ST_OK : status[c] == want);
    const unsigned long long m = __ballot(f);
    if (m == 0ull) return;                             // wave-uniform
    const int lane = threadIdx.x & 63;
    int base = 0;
    if (lane == 0) base = atomicAdd(cnt, (int)__popcll(m));
    base = __shfl(base, 0, 64);
    if (f) idx[base + __popcll(m & ((1ull << lane) - 1ull))] = c;
}

// Cost-ordered dispatch of the lane solver (pck_solve_params.wave_order).
// A wavefront's time is its slowest lane's; the hardware dispatches blocks in
// launch order, so long wavefronts launched last leave the machine idle in a
// tail (the wave-scheduling model puts the volcano launch at 1.19x its ideal,
// longest-first at 1.17x faster: tools/sched_sim.py).  The preview solves 4
// lanes of every wavefront (its first and last two: the corners of a 16 x 4
// volcano patch) as a loose transient; max of their step counts is the
// wavefront's key (tools/predictor_eval.py: 1.167x in the model against 1.170x
// for the true costs).
// With the screening pass (round 5) a wavefront's cost is its screening
// trips plus the full solves of the lanes the screening does not accept, so
// the preview runs the screening trip itself (transient, Newton, the rule at
// the screening distance) and a sample it does not accept adds
// PCK_PREVIEW_REJECT_STEPS (400; 200 / 800 within noise) steps to the key.
// With the transient-only preview, wavefronts whose screening rejected lanes
// started mid-launch and ended the launch 0.5 ms after the rest
// (tools/wave_timeline.py, profiles/r5/wave_timeline_*): 2.71 -> 2.52 ms per
// 2^20 volcano step.  (8 samples per wavefront instead of its 4 corners:
// 2.57 ms, the longer preview costs more than the extra samples find.)
constexpr int PCK_PREVIEW_REJECT_STEPS = 400;
// the preview lanes, the wavefront sort and k_solve's
// worder mapping all take one block of the lane solver to be one wavefront
static_assert(PCK_SOLVE_BLOCK == 64, "cost-ordered dispatch assumes one wavefront per lane-solver block");
__device__ __forceinline__ int preview_lane(int k, int) {
    return (k < 2) ? 3 * k : 60 + 3 * (k - 2);                     // 0, 3, 60, 63
}

__global__ void __launch_bounds__(256) k_preview_list(int64_t n, int64_t W, int np, int64_t* list, int32_t* cnt) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < W * np) {
        const int64_t c = (i / np) * PCK_SOLVE_BLOCK + preview_lane((int)(i % np), np);
        list[i] = (c < n) ? c : n - 1;      // a short last wavefront samples its last condition
    }
    if (i == 0) *cnt = (int32_t)(W * np);
}

// (A grid-wide histogram / scan / scatter sort took 0.17 ms against the one-
// block sort's 0.07 ms -- its global atomics contend on a few hundred bins --
// and its order inside a bin cost the first pass 0.15 ms more:
// profiles/r3/wave_sort_ab.)
// the sort key of every wavefront (the max preview step count of its samples),
// gathered from the scattered preview outputs by the whole grid, so that the
// one-block sort below reads W contiguous keys (it read 4 W scattered lines
// itself: ~28 of its 70 us)
// st (screening previews): a sample whose screening trip is not accepted
// counts `reject` more steps, and its wavefront's wrej flag is set (the
// solve skips that wavefront's screening trip, mk_solver.h: k_solve)
__global__ void __launch_bounds__(256) k_wave_keys(int64_t n, int64_t W, int np, const int32_t* ns,
                                                   const int32_t* st, int reject, int32_t* wkey, int32_t* wrej) {
    const int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= W) return;
    int k = 0;
    bool rej = false;
    for (int l = 0; l < np; ++l) {
        int64_t c = w * PCK_SOLVE_BLOCK + preview_lane(l, np);
        c = (c < n) ? c : n - 1;
        const bool r = st && st[c] != PCK_ST_OK;
        rej = rej || r;
        k = max(k, ns[c] + (r ? reject : 0));
    }
    wkey[w] = min(max(k, 0), 1023);
    wrej[w] = rej ? 1 : 0;
}

// descending counting sort of the wavefronts by their key (one block).
__global__ void __launch_bounds__(1024) k_wave_order(int64_t W, const int32_t* wkey, int32_t* order) {
    __shared__ int hist[1024];
    __shared__ int base[1024];
    const int tid = threadIdx.x;
    hist[tid] = 0;
    __syncthreads();
    for (int64_t w = tid; w < W; w += 1024) atomicAdd(&hist[wkey[w]], 1);
    __syncthreads();
    // exclusive scan over the bins, descending (heaviest first): Hillis-Steele
    // on the reversed histogram, one bin per thread
    const int v = hist[1023 - tid];
    base[tid] = v;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {
        const int add = (tid >= off) ? base[tid - off] : 0;
        __syncthreads();
        base[tid] += add;
        __syncthreads();
    }
    hist[1023 - tid] = base[tid] - v;           // each bin's start: the wavefronts in heavier bins
    __syncthreads();
    for (int64_t w = tid; w < W; w += 1024) order[atomicAdd(&hist[wkey[w]], 1)] = (int32_t)w;
}

// One solver launch over the batch (lane or lane-group path).
// lanes > 0 (lane path with an index list of known length): launch only that
// many lanes instead of n * G
static int run_solver(const pck_network* net, const pck_conditions* cond, const SolveArgs& a_in, bool grp,
                      GrpArgs& ga, bool traj, const double* kf, const double* kr, hipStream_t s,
                      int64_t lanes_override = 0) {
    SolveArgs a = a_in;
    const int64_t n = cond->n;
    int rc;
    if (grp) {
        const int NS = net->nv.NDYN;
        const int G = grp_g(NS);
        const int per = 64 / G;
        const int64_t groups = n * ga.M;
        // solves of networks of at most 16 species: the quad-group kernel
        // (mk_quad.h), four lanes per condition (steady solves with its Newton
        // polish unless PCK_GRP_QUAD_NEWTON=0)
        // (an explicit screening pass runs on the 16-lane kernel, which has it)
        if (NS <= 16 && (!a.newton || grp_quad_newton_enabled()) && !a.cons_rows && a.screen_rtol <= 0.0 &&
            net->plan_mode != PCK_PLAN_RUNTIME && jit_enabled() &&
            grp_quad_enabled(NS, net->nv.NRXN) && grp_ct_enabled(G, net->nv.NRXN) && !net->jit_grp_src.empty()) {
            hipFunction_t fq =
                jit_group_quad_kernel(net->digest, net->jit_grp_src, net->grp_npmax, net->grp_emax, a.newton != 0, traj);
            if (fq) {
                const int R1 = net->nv.NRXN > 0 ? net->nv.NRXN : 1;
                const size_t shm = sizeof(double) * 16 * 2 * (size_t)R1;
                if (shm > 64 * 1024)
                    return fail(PCK_E_SIZE, "quad-group solver: %s%lld bytes of LDS per block", "", (long long)shm);
                NetView nv = net->nv;
                CondView cv = cview(cond);
                const double* kfp = kf;
                const double* krp = kr;
                int64_t ldk = n;
                void* args[] = {&nv, &cv, &kfp, &krp, &ldk, &a, &ga};
                const unsigned nb = (unsigned)((groups + 15) / 16);
                HIPCHK(hipModuleLaunchKernel(fq, nb, 1, 1, 64, 1, 1, (unsigned)shm, s, args, nullptr));
                net->grp_jit_on.store(true, std::memory_order_relaxed);
                net->grp_ct_on.store(false, std::memory_order_relaxed);
                net->grp_quad_on.store(true, std::memory_order_relaxed);
                net->grp_lanes.store(4, std::memory_order_relaxed);
                HIPCHK(hipGetLastError());
                return PCK_OK;
            }
        }
        net->grp_quad_on.store(false, std::memory_order_relaxed);
        net->grp_lanes.store(G, std::memory_order_relaxed);
        dim3 g((unsigned)((groups + per - 1) / per));
        hipFunction_t f = nullptr;
        int P = grp_p(NS);
        int degmax = 0;
        const int bal = net->gv.LS > 0 ? 1 : 0;
        bool ct = false;
        if ((net->plan_mode != PCK_PLAN_RUNTIME || traj) && jit_enabled() && grp_ct_enabled(G, net->nv.NRXN) &&
            !net->jit_grp_src.empty() && P == 1) {
            // the compile-time network (mk_group.h: ct_rhs / ct_jac)
            f = jit_group_ct_kernel(net->digest, net->jit_grp_src, NS, G, P, traj, net->grp_npmax, net->grp_emax);
            ct = f != nullptr;
        }
        if (!ct && (net->plan_mode != PCK_PLAN_RUNTIME || traj) && jit_enabled()) {
            // (row loops bounded by the largest row degree measured slower:
            // CH4 100.6 k -> 83.6 k solves/s, profiles/r2/configs/ab_degmax.txt)
            f = jit_group_kernel(NS, G, P, traj, false, net->grp_npmax, net->grp_emax, 0, bal);
        }
        if (traj && !f) return fail(PCK_E_HIP, "hipRTC compile of the trajectory kernel failed%s", "");
        size_t shm;
        if (f) {
            rc = grp_shape(net, NS, P, &shm, &ga.QB);
            if (rc) return rc;
            size_t shm_t;
            int qb_t;
            const char* et = getenv("PCK_GRP_TAB");              // A/B: 0 = tables stay in global memory
            if (!ct && !(et && et[0] == '0') && grp_shape(net, NS, P, &shm_t, &qb_t, true) == PCK_OK &&
                grp_tables_pay(f, shm, shm_t)) {
                hipFunction_t ft = jit_group_kernel(NS, G, P, traj, true, net->grp_npmax, net->grp_emax, degmax, bal);
                if (ft) { f = ft; shm = shm_t; }
            }
            NetView nv = net->nv;
            GrpView gv = net->gv;
            CondView cv = cview(cond);
            const double* kfp = kf;
            const double* krp = kr;
            int64_t ldk = n;
            void* args[] = {&nv, &gv, &cv, &kfp, &krp, &ldk, &a, &ga};
            HIPCHK(hipModuleLaunchKernel(f, g.x, 1, 1, 64, 1, 1, (unsigned)shm, s, args, nullptr));
        } else {
            rc = grp_shape(net, grp_nsp_ct(NS), grp_p_ct(NS), &shm, &ga.QB);
            if (rc) return rc;
#define CALL(NP, GG, PP) hipLaunchKernelGGL((k_solve_grp<NP, GG, PP>), g, dim3(64), shm, s, net->nv, net->gv, cview(cond), kf, kr, n, a, ga)
            PCK_GRP_SWITCH(NS, CALL)
#undef CALL
        }
        net->grp_jit_on.store(f != nullptr, std::memory_order_relaxed);
        net->grp_ct_on.store(ct, std::memory_order_relaxed);
        HIPCHK(hipGetLastError());
        return PCK_OK;
    }
    const int B = PCK_SOLVE_BLOCK;
    const int R = net->nv.NRXN;
    const int64_t lanes = (lanes_override > 0 && !grp) ? lanes_override : n * a.G;
    const size_t shm = lds_bytes(R, net->nv.NDYN, B);
    dim3 g((unsigned)((lanes + B - 1) / B));
    if (traj) {
        hipFunction_t f = net->jit_src.empty() ? nullptr : jit_kernel(net->digest, net->jit_src, true);
        if (!f) return fail(PCK_E_HIP, "hipRTC compile of the trajectory kernel failed%s", "");
        NetView nv = net->nv;
        CondView cv = cview(cond);
        const double* kfp = kf;
        const double* krp = kr;
        int64_t ldk = n;
        void* args[] = {&nv, &cv, &kfp, &krp, &ldk, &a};
        HIPCHK(hipModuleLaunchKernel(f, g.x, 1, 1, B, 1, 1, (unsigned)shm, s, args, nullptr));
    } else if (net->spec && net->plan_mode == PCK_PLAN_AUTO) {
#define PCK_LAUNCH_CT(id, T)                                                                           \
        if (net->spec == id)                                                                          \
            hipLaunchKernelGGL(k_solve<PlanCT<T>>, g, dim3(B), shm, s, net->nv, cview(cond), kf, kr, n, a);
        PCK_COMPILED_NETWORKS(PCK_LAUNCH_CT)
#undef PCK_LAUNCH_CT
    } else {
        hipFunction_t f = nullptr;
        if (net->plan_mode == PCK_PLAN_AUTO && !net->jit_src.empty() && jit_enabled())
            f = jit_kernel(net->digest, net->jit_src);
        net->jit_on.store(f != nullptr, std::memory_order_relaxed);
        if (f) {
            NetView nv = net->nv;
            CondView cv = cview(cond);
            const double* kfp = kf;
            const double* krp = kr;
            int64_t ldk = n;
            void* args[] = {&nv, &cv, &kfp, &krp, &ldk, &a};
            HIPCHK(hipModuleLaunchKernel(f, g.x, 1, 1, B, 1, 1, (unsigned)shm, s, args, nullptr));
        } else {
#define CALL(N) hipLaunchKernelGGL(k_solve<PlanRT<N>>, g, dim3(B), shm, s, net->nv, cview(cond), kf, kr, n, a)
            PCK_NS_SWITCH(net->nv.NDYN, CALL)
#undef CALL
        }
    }
    HIPCHK(hipGetLastError());
    return PCK_OK;
}

// kf / kr of the batch go to `kscr` (per-call, stream-ordered): [2][R][n]
static int launch_solve(const pck_network* net, const pck_conditions* cond, const pck_solve_params* prm, SolveArgs a,
                        hipStream_t s, StreamScratch& kscr, int drc_groups = 0) {
    const int64_t n = cond->n;
    if (n == 0) return PCK_OK;
    if (!cond->y0) return fail(PCK_E_ARG, "initial state y0 required%s", "");
    const int R = net->nv.NRXN;
    int rc = salloc(kscr, sizeof(double) * 2 * (size_t)(R > 0 ? R : 1) * n, s);
    if (rc) return rc;
    double* kf = kscr.as<double>();
    double* kr = kf + (int64_t)(R > 0 ? R : 1) * n;
    rc = launch_rate_constants(net, cond, kf, kr, n, s);
    if (rc) return rc;
    a.t0 = prm->t0; a.t_end = prm->t_end; a.rtol = prm->rtol; a.atol = prm->atol; a.eps = prm->drc_eps;
    a.max_steps = prm->max_steps; a.newton = prm->newton; a.newton_iters = prm->newton_iters;
    a.want_activity = prm->want_activity;
    a.root_dist = prm->root_dist;
    a.idx = nullptr; a.nidx = nullptr; a.retry_pass = 0; a.worder = nullptr;
    // degenerate roots (status 4) are re-integrated by a second launch over
    // their compacted list (pck_solve only: G == 1, no DRC groups)
    bool retry = prm->newton && prm->retry_rtol > 0.0 && !drc_groups && a.G == 1;
    const bool traj = (prm->n_out > 0 && a.traj != nullptr);
    // screening pass (pck_solve_params.screen_rtol): the steady rule at a
    // loose tolerance with a tighter acceptance, then the single pass at the
    // caller's tolerances over the rest (one-lane path, pck_solve only)
    bool screen = prm->newton && prm->root_dist > 0.0 && prm->screen_rtol > 0.0 && prm->screen_rtol > prm->rtol &&
                  !traj;
    if (traj) {
        if (!prm->t_out) return fail(PCK_E_ARG, "n_out > 0 without t_out%s", "");
        if (drc_groups || a.G != 1) return fail(PCK_E_ARG, "trajectory output is for pck_solve only%s", "");
        if (!jit_enabled()) return fail(PCK_E_ARG, "trajectory output needs the hipRTC kernels (PCK_JIT=0 is set)%s", "");
        a.t_out = prm->t_out;
        a.n_out = (int)prm->n_out;
    }
    {
        // conservation rows in the stage systems (mk_solver.h: cons_rows) are
        // off by default: measured on examples/DMTM at 400 K they cost 1.5x
        // (GPU) to 2.6x (numpy restatement) more steps -- the pivot species
        // inherits the cancellation of the other coverages' increments
        const char* e = getenv("PCK_CONS_ROWS");
        a.cons_rows = (e && e[0] == '1');
    }
    const bool grp = drc_groups || use_group(net, a.G);
    // the screening pass inside the solve: a lane or group that fails it
    // solves again at once, so the slow second solves overlap the bulk of the
    // first pass (as two launches, the second latency-bound on its slowest
    // solve, it was 3.26 against 2.93 ms per volcano step; DESIGN.md
    // "Screening pass")
    {
        a.screen_max_steps = std::min(a.max_steps, 2000);
        const char* e = getenv("PCK_SCREEN_MAX_STEPS");
        if (e && atoi(e) > 0) a.screen_max_steps = std::min(a.max_steps, atoi(e));
    }
    if (screen) {
        // the 64-lane group kernel carries one integrator copy (mk_group.h:
        // k_solve_grp): a screening request there is refused, not ignored
        if (grp && grp_g(net->nv.NDYN) == 64)
            return fail(PCK_E_ARG, "screen_rtol: no screening pass on networks of more than 32 dynamic species%s", "");
        a.screen_rtol = prm->screen_rtol;
        a.screen_atol = a.atol * (prm->screen_rtol / a.rtol);
        a.screen_dist = a.root_dist * (prm->screen_margin > 0.0 ? prm->screen_margin : 0.1);
    }
    if (grp && !net->grp_ok)
        return fail(PCK_E_SIZE, "lane-group solver: a reaction has more than 6 dynamic participants%s", "");
    GrpArgs ga;
    ga.M = drc_groups ? drc_groups : 1;
    ga.QB = 1;
    ga.tofbuf = nullptr;
    ga.stbuf = nullptr;
    ga.nsbuf = nullptr;
    StreamScratch dscr;
    if (drc_groups) {
        const int64_t m = (int64_t)drc_groups * n;
        rc = salloc(dscr, sizeof(double) * m + 2 * sizeof(int32_t) * m, s);
        if (rc) return rc;
        ga.tofbuf = dscr.as<double>();
        ga.stbuf = (int32_t*)(ga.tofbuf + m);
        ga.nsbuf = ga.stbuf + m;
    }
    // cost-ordered dispatch: preview, order, then the first pass in that order
    // (auto from 131 072 conditions: the volcano grid's N = 8 shard runs 1.31
    // ms with it against 1.38 ms without, round 6; a uniform-cost sweep is
    // better off without it -- pck_solve_params.wave_order = -1)
    StreamScratch oscr;
    const bool order = !grp && !traj && a.G == 1 && !drc_groups &&
                       (prm->wave_order > 0 || (prm->wave_order == 0 && n >= 131072));
    if (order) {
        const int64_t W = (n + PCK_SOLVE_BLOCK - 1) / PCK_SOLVE_BLOCK;
        const int np = 4;
        // the preview runs the screening trip where the solve screens
        const bool pscreen = a.screen_rtol > 0.0;
        const size_t b_list = sizeof(int64_t) * (size_t)W * np, b_ns = sizeof(int32_t) * (size_t)n;
        rc = salloc(oscr, b_list + 64 + 2 * b_ns + 3 * sizeof(int32_t) * (size_t)W, s);
        if (rc) return rc;
        int64_t* list = oscr.as<int64_t>();
        int32_t* cnt = (int32_t*)((char*)list + b_list);
        int32_t* pns = (int32_t*)((char*)list + b_list + 64);
        int32_t* pst = pns + n;                     // screening previews: the samples' statuses
        int32_t* wo = pst + n;
        int32_t* wkey = wo + W;                     // per-wavefront sort key, compact
        int32_t* wrej = wkey + W;                   // per wavefront: a screening sample was not accepted
        hipLaunchKernelGGL(k_preview_list, dim3((unsigned)((W * np + 255) / 256)), dim3(256), 0, s,
                           n, W, np, list, cnt);
        HIPCHK(hipGetLastError());
        SolveArgs pv = a;
        pv.screen_rtol = 0.0;
        // the preview's rtol floor: 1e-2 (the preview is latency-bound on its
        // slowest sample: ~80 steps there against ~120 at 1e-3; the volcano
        // step 5.71 -> 5.65 ms with the coarser order, profiles/r4/ab_preview_*);
        // PCK_PREVIEW_RTOL overrides it (A/B)
        pv.rtol = fmax(a.rtol, 1e-2);
        {
            const char* e = getenv("PCK_PREVIEW_RTOL");
            if (e) pv.rtol = fmax(a.rtol, atof(e));
        }
        pv.atol = a.atol * (pv.rtol / a.rtol);       // the same atol / rtol ratio
        pv.newton = 0;
        if (pscreen) {
            // the screening trip at a coarser rtol (0.2, atol scaled alike):
            // its verdict orders the wavefronts and flags those that skip
            // the trip; a cheaper preview that flags a few more of them
            // measured 2.43 / 2.46 -> 2.38 / 2.38 ms per volcano step at 0.1,
            // and 2.28 / 2.25 -> 2.23 / 2.22 ms at 0.2 with the screening
            // margin 0.5 (0.05: 2.24 / 2.25, 0.3: 2.26;
            // profiles/r6/ab_preview_screen_rtol.txt).
            // PCK_PREVIEW_SCREEN_RTOL overrides it (A/B).
            double prt = 0.2;
            {
                const char* e = getenv("PCK_PREVIEW_SCREEN_RTOL");
                if (e && atof(e) > 0.0) prt = atof(e);
            }
            prt = fmax(prt, a.screen_rtol);
            pv.rtol = prt;
            pv.atol = a.screen_atol * (prt / a.screen_rtol);
            pv.newton = a.newton;
            pv.root_dist = a.screen_dist;
        }
        // the transient preview's cap; a screening preview runs its trip with
        // the solve's own trip cap
        // (lower caps, 30 / 50 steps, flagged most wavefronts: 2.9x the steps)
        pv.max_steps = pscreen ? a.screen_max_steps : (a.max_steps < 1000 ? a.max_steps : 1000);
        pv.y = nullptr; pv.tof = nullptr; pv.status = pscreen ? pst : nullptr; pv.nsteps = pns;
        pv.idx = list; pv.nidx = cnt; pv.retry_pass = 0; pv.worder = nullptr;
        rc = run_solver(net, cond, pv, grp, ga, traj, kf, kr, s, W * np);
        if (rc) return rc;
        hipLaunchKernelGGL(k_wave_keys, dim3((unsigned)((W + 255) / 256)), dim3(256), 0, s, n, W, np, pns,
                           pscreen ? pst : nullptr, PCK_PREVIEW_REJECT_STEPS, wkey, wrej);
        HIPCHK(hipGetLastError());
        hipLaunchKernelGGL(k_wave_order, dim3(1), dim3(1024), 0, s, W, wkey, wo);
        HIPCHK(hipGetLastError());
        a.worder = wo;
        // wavefronts with a rejected preview sample skip the screening trip
        // (their critical path is the full solve of a rejected lane; its
        // screening trip only delays it): 2.53 -> 2.40 ms per 2^20 volcano
        // step.  Their accepted lanes then report the root reached from the
        // full transient instead of the screening one: the same root to the
        // refinement's rounding (~1e-13).
        if (pscreen) a.wrej = wrej;
    }
    StreamScratch rscr;
    if (retry) {
        // the retry list (int64 per condition), its length, and a status
        // array when the caller passed none
        // (W wavefronts' worth of entries: the overlapped split keeps two lists)
        const size_t nl = (size_t)((n + PCK_SOLVE_BLOCK - 1) / PCK_SOLVE_BLOCK) * PCK_SOLVE_BLOCK;
        const size_t bytes = sizeof(int64_t) * nl + 64 + (a.status ? 0 : sizeof(int32_t) * (size_t)n);
        rc = salloc(rscr, bytes, s);
        if (rc) return rc;
        if (!a.status) a.status = (int32_t*)(rscr.as<char>() + sizeof(int64_t) * nl + 64);
    }
    {
        rc = run_solver(net, cond, a, grp, ga, traj, kf, kr, s);
        if (rc) return rc;
    }
    if (retry) {
        int64_t* idx = rscr.as<int64_t>();
        int32_t* cnt = (int32_t*)(idx + ((n + PCK_SOLVE_BLOCK - 1) / PCK_SOLVE_BLOCK) * PCK_SOLVE_BLOCK);
        HIPCHK(hipMemsetAsync(cnt, 0, sizeof(int32_t), s));
        hipLaunchKernelGGL(k_select_status, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, n, a.status,
                           (int32_t)PCK_ST_NEWTON, idx, cnt);
        HIPCHK(hipGetLastError());
        // pass 1: the same grid (the list's length stays on the device); lanes
        // past *cnt idle at once
        SolveArgs r = a;
        r.rtol = prm->retry_rtol;
        r.atol = prm->retry_atol;
        r.newton = 0;
        r.idx = idx;
        r.nidx = cnt;
        r.retry_pass = 1;
        r.worder = nullptr;
        // the trajectory stays the first pass's: a retry that fails keeps the
        // first pass's outputs, and a partly rewritten trajectory would mix the two
        r.traj = nullptr; r.t_out = nullptr; r.n_out = 0;
        rc = run_solver(net, cond, r, grp, ga, false, kf, kr, s);
        if (rc) return rc;
    }
    if (drc_groups) {
        hipLaunchKernelGGL(k_drc_combine, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, n, R, a.eps,
                           ga.tofbuf, ga.stbuf, ga.nsbuf, a.xi, a.ld_xi, a.tof0, a.status, a.nsteps);
        HIPCHK(hipGetLastError());
    }
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
    if (prm->n_out > 0 && out->traj) {
        if (out->ld_traj < cond->n) return fail(PCK_E_ARG, "ld_traj%s too small", "");
        a.traj = out->traj;
        a.ld_traj = out->ld_traj;
    }
    if ((out->kf || out->kr) && cond->n > 0 && (out->ld_k < cond->n || !out->kf || !out->kr))
        return fail(PCK_E_ARG, "kf/kr dump needs both arrays%s", "");
    StreamScratch kscr;
    rc = launch_solve(net, cond, prm, a, (hipStream_t)stream, kscr);
    if (rc) return rc;
    if ((out->kf || out->kr) && cond->n > 0) {
        const int R = net->nv.NRXN;
        const double* kb = kscr.as<double>();
        HIPCHK(hipMemcpy2DAsync(out->kf, sizeof(double) * out->ld_k, kb, sizeof(double) * cond->n,
                                sizeof(double) * cond->n, R, hipMemcpyDeviceToDevice, (hipStream_t)stream));
        HIPCHK(hipMemcpy2DAsync(out->kr, sizeof(double) * out->ld_k, kb + (int64_t)(R > 0 ? R : 1) * cond->n,
                                sizeof(double) * cond->n, sizeof(double) * cond->n, R, hipMemcpyDeviceToDevice,
                                (hipStream_t)stream));
    }
    return PCK_OK;
}

extern "C" int pck_drc(const pck_network* net, const pck_conditions* cond, const pck_solve_params* prm, double* xi,
                       int64_t ld_xi, double* tof0, int32_t* status, int32_t* nsteps, void* stream) {
    int rc = check_cond(net, cond, true);
    if (rc) return rc;
    rc = check_params(prm);
    if (rc) return rc;
    const int R = net->nv.NRXN;
    if (!(prm->drc_eps > 0.0 && prm->drc_eps < 1.0)) return fail(PCK_E_ARG, "drc_eps must be in (0,1)%s", "");
    if (cond->n > 0 && (!xi || ld_xi < cond->n)) return fail(PCK_E_ARG, "bad xi output%s", "");
    int G = 1;
    while (G < 2 * R + 1) G <<= 1;
    SolveArgs a;
    memset(&a, 0, sizeof(a));
    a.xi = xi; a.ld_xi = ld_xi; a.tof0 = tof0; a.status = status; a.nsteps = nsteps; a.G = G;
    StreamScratch kscr;
    // lane-group networks: one group per (condition, perturbation), combined after
    if (use_group(net, G)) return launch_solve(net, cond, prm, a, (hipStream_t)stream, kscr, 2 * R + 1);
    return launch_solve(net, cond, prm, a, (hipStream_t)stream, kscr);
}
