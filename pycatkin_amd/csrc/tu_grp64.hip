// Translation unit of the 64-lane group kernels (csrc/mk_inst.h; the
// parallel product build of __graft_entry__.build).
#define PCK_KERNEL_TU 1
#include "mk_inst.h"
namespace pck {
PCK_DO_GRP(, 64, 64, 1)
}  // namespace pck
