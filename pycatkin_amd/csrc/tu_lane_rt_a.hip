// Translation unit of the runtime-plan lane kernels of NS = 1..4 (csrc/mk_inst.h; the
// parallel product build of __graft_entry__.build).
#define PCK_KERNEL_TU 1
#include "mk_inst.h"
namespace pck {
#define PCK_X(N) PCK_DO_LANE_RT(, N)
PCK_INST_LANE_RT_A(PCK_X)
#undef PCK_X
}  // namespace pck
