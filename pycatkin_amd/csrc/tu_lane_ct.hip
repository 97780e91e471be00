// Translation unit of the compiled-in lane plans (csrc/networks.h,
// csrc/mk_inst.h; the parallel product build of __graft_entry__.build).
#define PCK_KERNEL_TU 1
#include "mk_inst.h"
namespace pck {
#define PCK_X(id, T) PCK_DO_LANE_CT(, id, T)
PCK_COMPILED_NETWORKS(PCK_X)
#undef PCK_X
}  // namespace pck
