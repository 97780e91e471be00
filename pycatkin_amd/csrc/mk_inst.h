// Solver-kernel instantiations of the library, one list per family.  The
// product build (__graft_entry__.build, PCK_SPLIT_TU=1) compiles each family
// in a translation unit of its own (csrc/tu_*.hip, compiled in parallel and
// linked with mk_kernels.hip): mk_kernels.hip then only declares them
// (extern template) and launches them.  A single-TU build (PCK_SPLIT_TU=0,
// the diagnostic builds of tools/ab_build.sh, whose __device__ counters must
// live in the translation unit that reads them back) instantiates them where
// they are launched, as before.
#pragma once
#include "mk_group.h"

// k_solve over the runtime plan of NS = 1..8 dynamic species, with the
// evaluation kernels of the same NS
#define PCK_INST_LANE_RT_A(X) X(1) X(2) X(3) X(4)
#define PCK_INST_LANE_RT_B(X) X(5) X(6) X(7) X(8)
#define PCK_INST_LANE_RT(X) PCK_INST_LANE_RT_A(X) PCK_INST_LANE_RT_B(X)
// lane-group kernels: (NSP, G, P) of PCK_GRP_SWITCH
#define PCK_INST_GRP(X) X(16, 16, 1) X(32, 32, 1) X(64, 64, 1)

#define PCK_SIG_SOLVE NetView, CondView, const double*, const double*, int64_t, SolveArgs
#define PCK_SIG_RATES NetView, CondView, const double*, const double*, int64_t, const double*, int64_t, double*
#define PCK_SIG_SOLVE_GRP NetView, GrpView, CondView, const double*, const double*, int64_t, SolveArgs, GrpArgs
#define PCK_SIG_RATES_GRP                                                                              \
    NetView, GrpView, CondView, const double*, const double*, int64_t, const double*, int64_t, double*, int, int

#define PCK_DO_LANE_RT(EXT, N)                                                   \
    EXT template __global__ void k_solve<PlanRT<N>, false>(PCK_SIG_SOLVE);        \
    EXT template __global__ void k_species_rates<N, true>(PCK_SIG_RATES);         \
    EXT template __global__ void k_species_rates<N, false>(PCK_SIG_RATES);        \
    EXT template __global__ void k_jacobian<N>(PCK_SIG_RATES);
#define PCK_DO_LANE_CT(EXT, id, T) EXT template __global__ void k_solve<PlanCT<T>, false>(PCK_SIG_SOLVE);
#define PCK_DO_GRP(EXT, NP, GG, PP)                                                      \
    EXT template __global__ void k_solve_grp<NP, GG, PP>(PCK_SIG_SOLVE_GRP);              \
    EXT template __global__ void k_rates_grp<NP, GG, PP>(PCK_SIG_RATES_GRP);
