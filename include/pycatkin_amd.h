/* pycatkin_amd C-ABI: batched mean-field microkinetic (MK) solves on MI355X.
 *
 * One "condition" = one independent MK model instance (a temperature /
 * pressure / descriptor-grid point).  Every per-condition array is
 * structure-of-arrays, device-resident, fp64: element (k, c) of an array with
 * leading dimension ld and condition stride s lives at ptr[k*ld + c*s]; a
 * stride of 0 broadcasts one column to every condition.
 *
 * The network is compiled host-side (pycatkin_amd/network.py) into two flat
 * blobs -- int32 `ip` and float64 `dp` -- whose layout is given by the
 * PCK_I_* / PCK_D_* header slots below, and uploaded once with
 * pck_network_create().
 *
 * Each entry point replaces one reference (PyCatKin) Python routine that a
 * ctypes / FFI binding would call for the whole batch:
 *
 *   pck_rate_constants  <- Reaction.calc_rate_constants      pycatkin/classes/reaction.py:94
 *                          (+ State.calc_free_energy          pycatkin/classes/state.py:367,
 *                             ScalingState.calc_free_energy   state.py:519,
 *                             UserDefinedReaction.calc_reaction_energy reaction.py:222)
 *   pck_species_rates   <- System.species_odes + Reactor.rhs  pycatkin/classes/old_system.py:227,
 *                                                             pycatkin/classes/reactor.py:91,141
 *                          System.get_dydt / _fun_ss          pycatkin/classes/system.py:396,528
 *   pck_jacobian        <- System.species_jacobian + Reactor.jacobian old_system.py:293, reactor.py:103,161
 *                          System.get_jacobian / _jac_ss      system.py:493,547
 *   pck_reaction_rates  <- System._calc_rates                 system.py:345
 *                          System.reaction_terms              old_system.py:202
 *   pck_solve           <- System.solve_odes (+ find_steady)  old_system.py:315 (385)
 *                          SteadyStateSolver.solve_ode        pycatkin/classes/solver.py:374
 *                          System.run_and_return_tof / activity old_system.py:470,517
 *   pck_drc             <- System.degree_of_rate_control      old_system.py:490
 *
 * All functions return 0 on success and a negative PCK_E_* code on failure;
 * pck_last_error() returns a message for the calling thread.  Device pointers
 * only; `stream` is a hipStream_t (NULL = default stream).  Launches are
 * asynchronous on `stream` unless noted.  A network handle is read-only after
 * pck_network_create: every call allocates its own scratch in stream order
 * on `stream` (hipMallocAsync / hipFreeAsync), so calls on different streams
 * may share one network.
 */
#ifndef PYCATKIN_AMD_H
#define PYCATKIN_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PCK_ABI_VERSION 6

/* error codes */
#define PCK_OK 0
#define PCK_E_ARG (-1)      /* bad argument / blob layout */
#define PCK_E_HIP (-2)      /* HIP runtime error */
#define PCK_E_SIZE (-3)     /* network exceeds the compiled kernel limits */

/* kernel limits.  Networks with up to PCK_MAX_DYN_LANE dynamic species run
 * one condition per lane (state, Jacobian and LU in VGPRs); larger ones (up to
 * PCK_MAX_DYN) run one condition per lane group of 16/32/64 lanes, one
 * species row per lane (csrc/mk_group.h). */
#define PCK_MAX_DYN 64      /* dynamic species per condition (solver kernels) */
#define PCK_MAX_DYN_LANE 8  /* ... on the one-lane-per-condition path */
#define PCK_MAX_DYN_PLAN 64 /* dynamic species a plan may hold (rate constants / energies) */
#define PCK_MAX_RXN 256     /* active reactions */
#define PCK_MAX_EXP 255     /* stoichiometric exponent */
#define PCK_MAX_CONS 4      /* conservation laws */
#define PCK_MAX_TOF 16      /* TOF terms */

/* int32 blob header slots (ip[0..PCK_I_HDR)) */
enum {
    PCK_I_VERSION = 0, /* == PCK_ABI_VERSION */
    PCK_I_NDESC,       /* D: descriptors per condition */
    PCK_I_NTH,         /* thermo states (vib/tran/rot features) */
    PCK_I_NREG,        /* energy-program registers */
    PCK_I_NRXN,        /* active reactions R */
    PCK_I_NDYN,        /* dynamic species NS */
    PCK_I_NFIX,        /* fixed (non-dynamic) species F */
    PCK_I_NCONS,       /* conservation laws m */
    PCK_I_NTOF,        /* TOF terms */
    PCK_I_OFF_TH,      /* -> th: NTH x {kind, freq_off, freq_cnt, rot_shape} */
    PCK_I_OFF_REG,     /* -> reg_ptr[NREG+1], reg_clamp[NREG], reg_feat[nnz] */
    PCK_I_OFF_RX,      /* -> rx: NRXN x {type, reversible, reg_ga, reg_grxn, reg_erxn, arr_if_barrier} */
    PCK_I_OFF_EXPF,    /* -> forward exponents  [NRXN][NDYN] */
    PCK_I_OFF_EXPR,    /* -> reverse exponents  [NRXN][NDYN] */
    PCK_I_OFF_FOLDF,   /* -> forward fixed-species exponents [NRXN][NFIX] */
    PCK_I_OFF_FOLDR,   /* -> reverse fixed-species exponents [NRXN][NFIX] */
    PCK_I_OFF_CPIV,    /* -> pivot row of each conservation law [NCONS] */
    PCK_I_OFF_TOF,     /* -> active-reaction index of each TOF term [NTOF] */
    PCK_I_HDR
};

/* float64 blob header-less layout: offsets are stored in the int blob */
enum {
    PCK_D_OFF_SLOT0 = PCK_I_HDR, /* ip[PCK_D_OFF_SLOT0 + k] = dp offset of block k: */
    PCK_D_TH = 0,    /* th: NTH x {zpe [eV], mass [amu], sigma, rotI = sqrt(prod nonzero I) [kg m^2], Gvibr given (NaN = compute)} */
    PCK_D_FREQ,      /* frequency table (Hz) */
    PCK_D_REGCOEF,   /* reg_coef[nnz] */
    PCK_D_RX,        /* rx: NRXN x {kads_c, kdes_c, kdes_texp} */
    PCK_D_STOICH,    /* S[NDYN][NRXN] (weights incl. scaling / site density) */
    PCK_D_DYN,       /* dyn: NDYN x {conc_factor, rowscale0, rowscale_T, flow_rate} */
    PCK_D_CONS,      /* C[NCONS][NDYN] */
    PCK_D_NBLK
};
#define PCK_IP_MIN (PCK_I_HDR + PCK_D_NBLK)

/* register feature index space: 0 = constant 1, 1 = T, 2 .. 2+D-1 = descriptors,
 * then 3 per thermo state (vib, tran, rot), then earlier registers. */

/* reaction rate-constant types (reaction.py:94-168) */
enum {
    PCK_RX_ARRHENIUS = 0,  /* kf = kBT/h exp(-max(dGa,0)/RT); kr = kf/exp(-dGrxn/RT) */
    PCK_RX_ADS_KEQ = 1,    /* kf = kads;  kr = kads/exp(-dGrxn/RT) (classic) */
    PCK_RX_DES_KEQ = 2,    /* kr = kads;  kf = kads*exp(-dGrxn/RT) (classic) */
    PCK_RX_ADS_KDES = 3,   /* kf = kads;  kr = kdes(-dErxn) (reaction.py:135-147) */
    PCK_RX_DES_KDES = 4    /* kf = kdes(dErxn); kr = kads (reaction.py:150-162) */
};

/* thermo state kinds (bit flags) */
#define PCK_TH_VIB 1
#define PCK_TH_GAS 2

typedef struct pck_network pck_network;

/* Per-condition inputs (device pointers; see stride rule above). */
typedef struct {
    int64_t n;                       /* number of conditions */
    const double* T;  int64_t sT;    /* temperature [K] */
    const double* p;  int64_t sp;    /* pressure [Pa] (free energies only) */
    const double* desc; int64_t ld_desc, s_desc;   /* [D][..] descriptor values (eV) */
    const double* fixc; int64_t ld_fix, s_fix;     /* [F][..] fixed-species concentrations */
    const double* y0; int64_t ld_y0, s_y0;         /* [NS][..] initial dynamic state */
    const double* inflow; int64_t ld_in, s_in;     /* [NS][..] inflow (CSTR gas rows) */
} pck_conditions;

typedef struct {
    double t0, t_end;      /* integrate from t0 to t_end */
    double rtol, atol;     /* local error control (RMS norm) */
    int32_t max_steps;     /* per condition */
    int32_t newton;        /* 1: polish to f(y)=0 after the transient (find_steady) */
    int32_t newton_iters;  /* max Newton iterations */
    int32_t want_activity; /* 1: write activity (eV) instead of TOF into tof_out */
    double drc_eps;        /* pck_drc only: relative k perturbation */
    const double* t_out;   /* pck_solve: n_out ascending sample times in [t0, t_end] (device), or NULL */
    int64_t n_out;         /*   the state at each is written to pck_outputs.traj (dense output) */
    double retry_rtol;     /* with newton: a condition whose polish meets a degenerate root */
    double retry_atol;     /*   (PCK_ST_NEWTON) is integrated again, t0..t_end, at these tolerances,
                            *   by a second launch over the compacted list of such conditions on
                            *   the same stream (pck_solve only; 0: off); its y / tof become that
                            *   transient end,
                            *   the reference's System.activity semantics (old_system.py:517-529),
                            *   status stays PCK_ST_NEWTON and nsteps adds the retry's steps; a
                            *   retry that fails keeps the first pass's y / tof (PCK_ST_NEWTON_LOOSE) */
    int32_t wave_order;    /* pck_solve on the lane solver: dispatch the 64-condition wavefronts in
                            *   descending cost, predicted by a preview of 4 lanes of each (a loose
                            *   transient, or the screening trip at rtol 0.2 when the solve screens:
                            *   a wavefront with a sample it does not accept skips its trip);
                            *   1 on, -1 off, 0 auto (on for n >= 131072).  It pays where costs vary
                            *   across the batch and is overhead on a uniform-cost sweep.  Results
                            *   do not depend on it beyond rounding: the same 64 conditions share a
                            *   wavefront either way, and a skipped trip's lanes answer from the
                            *   full solve (the same root to ~1e-13). */
    double root_dist;      /* with newton (> 0): the Newton root is reported (PCK_ST_OK) only if the
                            *   transient end it started from lies within root_dist * |root_i| + atol
                            *   of it in every dynamic species -- the transient has reached that steady
                            *   state by t_end; otherwise the transient end is reported with
                            *   PCK_ST_NEWTON (old_system.py:517-529 System.activity semantics).
                            *   0: any converged, balanced, non-negative root is reported
                            *   (old_system.py:385-468 find_steady from a given state). */
    double screen_rtol;    /* with newton and root_dist > 0 (no trajectory): a screening pass at
                            *   rtol = screen_rtol (atol scaled alike) whose Newton root is accepted
                            *   (PCK_ST_OK) only if the screening transient's end lies within
                            *   screen_margin * root_dist * |root_i| + atol (the caller's atol) of
                            *   it; every other condition solves again from y0 at rtol / atol in the
                            *   same launch, exactly as without screening (y, tof, status of that
                            *   solve; nsteps adds the two trips).  A transient that has settled on
                            *   a root ends on it at any tolerance, so the accepted conditions report
                            *   the root the single pass would (DESIGN.md "Screening pass").  Runs on
                            *   the one-lane solver and the 16- and 32-lane group kernels, pck_solve
                            *   and pck_drc; a network of <= 16 species then leaves the quad-group
                            *   kernel for the 16-lane one; networks of > 32 species (64-lane
                            *   groups) refuse it with PCK_E_ARG.  0: off. */
    double screen_margin;  /*   fraction of root_dist for the screening pass's acceptance (0: 0.1) */
} pck_solve_params;

/* Outputs of pck_solve (device pointers; any may be NULL). */
typedef struct {
    double* y; int64_t ld_y;   /* [NS][ld_y] final dynamic state */
    double* tof;               /* [n] TOF (1/s) or activity (eV) */
    int32_t* status;           /* [n] PCK_ST_* */
    int32_t* nsteps;           /* [n] accepted + rejected steps */
    double* kf; double* kr;    /* [NRXN][ld_k] optional rate-constant dump */
    int64_t ld_k;
    double* traj; int64_t ld_traj;   /* [n_out][NS][ld_traj] states at pck_solve_params.t_out
                                      * (System.solve_odes' solution, old_system.py:350-376);
                                      * needs the hipRTC-specialised kernels (PCK_JIT != 0) */
} pck_outputs;

/* per-condition status codes */
#define PCK_ST_OK 0
#define PCK_ST_MAXSTEPS 1
#define PCK_ST_STEPFAIL 2
#define PCK_ST_NONFINITE 3
/* no steady state reached by t_end (with root_dist: the transient has not
 * reached a root; without: Newton met a degenerate root): y / tof are the
 * transient end at t_end */
#define PCK_ST_NEWTON 4
/* a degenerate root whose tight retry transient failed (step budget / step
 * size): y and tof are the first pass's transient end at the caller's
 * tolerances -- what the reference's own lsoda path reports */
#define PCK_ST_NEWTON_LOOSE 5
/* pck_drc with newton: the 2R+1 solves of a condition fall on both sides of
 * the steady rule (some report a reached root, PCK_ST_OK, others the
 * transient end, PCK_ST_NEWTON / _LOOSE): the central differences then mix
 * two definitions of the answer and xi measures the rule switching, not rate
 * control.  xi / tof0 are still written. */
#define PCK_ST_DRC_MIXED 6

int pck_abi_version(void);
const char* pck_last_error(void);

/* Upload a compiled network (host blobs) to the current device. */
int pck_network_create(const int32_t* ip, int64_t n_ip, const double* dp, int64_t n_dp,
                       pck_network** out);
int pck_network_destroy(pck_network* net);
/* Sizes of a created network: dims[0..10] = D, NTH, NREG, NRXN, NDYN, NFIX, NCONS, NTOF,
 * n_features, plan id: a compiled-in plan (csrc/networks.h), PCK_PLAN_ID_JIT once a
 * lane solve ran the plan hipRTC specialised for this network (csrc/mk_jit.h;
 * PCK_JIT=0 in the environment disables it), 0 = runtime plan; and the kernel of the
 * last lane-group solve: 0 compiled-in record tables, 1 hipRTC exact-size record
 * tables, 2 hipRTC with the network compiled in (PCK_GRP_CT=0 disables it). */
#define PCK_PLAN_ID_JIT 100
int pck_network_dims(const pck_network* net, int32_t* dims);
/* Lanes per condition of the last lane-group solve (networks beyond the
 * one-lane limits): 4 for the quad-group kernel (csrc/mk_quad.h, <= 16
 * species), else the group width G = 16, 32 or 64 (csrc/mk_group.h: grp_g);
 * 0 before any group solve.  Diagnostic: which kernel answered. */
int pck_network_group_lanes(const pck_network* net, int32_t* lanes);
/* Solver selection (A/B checks): PCK_PLAN_AUTO (default: compiled-in plan when
 * the structural digest matches, else the runtime plan, lane-group solver
 * beyond the one-lane limits), PCK_PLAN_RUNTIME (never the compiled-in plan),
 * PCK_PLAN_GROUP (always the lane-group solver). */
#define PCK_PLAN_AUTO 0
#define PCK_PLAN_RUNTIME 1
#define PCK_PLAN_GROUP 2
int pck_network_set_plan_mode(pck_network* net, int mode);

/* Energy-program registers (eV) per condition: out[r][ld_out], r < NREG.
 * Replaces State.get_free_energy (state.py:388) / Reaction.get_reaction_energy
 * (reaction.py:171) / get_reaction_barriers (reaction.py:182) for a batch.
 * Networks with NDYN == 0 are accepted for this call and pck_rate_constants. */
int pck_energies(const pck_network* net, const pck_conditions* cond, double* out, int64_t ld_out,
                 void* stream);

/* kf, kr: [NRXN][ld_k] outputs (1/s or 1/(s Pa^n) as the reference's). */
int pck_rate_constants(const pck_network* net, const pck_conditions* cond,
                       double* kf, double* kr, int64_t ld_k, void* stream);

/* Effective rates of the dynamic species at states y ([NS][ld_y]):
 * dydt[NS][ld_y] = rowscale * (S . net_rates) + flow.  kf/kr as produced by
 * pck_rate_constants (fixed species are folded in here). */
int pck_species_rates(const pck_network* net, const pck_conditions* cond,
                      const double* kf, const double* kr, int64_t ld_k,
                      const double* y, int64_t ld_y, double* dydt, void* stream);

/* Forward and reverse rate of every active reaction at states y ([NS][ld_y]),
 * fixed-species concentrations folded in: rf, rr [NRXN][ld_r].
 * Replaces System._calc_rates (pycatkin/classes/system.py:345) and
 * System.reaction_terms (pycatkin/classes/old_system.py:202). */
int pck_reaction_rates(const pck_network* net, const pck_conditions* cond,
                       const double* kf, const double* kr, int64_t ld_k,
                       const double* y, int64_t ld_y, double* rf, double* rr, int64_t ld_r,
                       void* stream);

/* Jacobian d(dydt)/dy: jac[(i*NS + k)][ld_y] (row-major per condition). */
int pck_jacobian(const pck_network* net, const pck_conditions* cond,
                 const double* kf, const double* kr, int64_t ld_k,
                 const double* y, int64_t ld_y, double* jac, void* stream);

/* Fused: rate constants -> stiff integration t0..t_end (L-stable Rosenbrock
 * W-method) -> optional Newton steady-state polish -> TOF / activity. */
int pck_solve(const pck_network* net, const pck_conditions* cond,
              const pck_solve_params* prm, const pck_outputs* out, void* stream);

/* Degree of rate control for every active reaction (old_system.py:490):
 * xi[j][ld_xi] = (TOF(k_j*(1+eps)) - TOF(k_j*(1-eps))) / (2 eps TOF0).
 * tof0 (optional) receives the unperturbed TOF; status (optional) the worst
 * status of the 2R+1 solves (PCK_ST_NONFINITE also for a zero / non-finite
 * TOF0; PCK_ST_DRC_MIXED where they mix reached roots and transient ends);
 * nsteps (optional) the sum of their integrator steps. */
int pck_drc(const pck_network* net, const pck_conditions* cond,
            const pck_solve_params* prm, double* xi, int64_t ld_xi,
            double* tof0, int32_t* status, int32_t* nsteps, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* PYCATKIN_AMD_H */
