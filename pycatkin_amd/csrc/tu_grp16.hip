// Translation unit of the 16-lane group kernels (csrc/mk_inst.h; the
// parallel product build of __graft_entry__.build).
#define PCK_KERNEL_TU 1
#include "mk_inst.h"
namespace pck {
PCK_DO_GRP(, 16, 16, 1)
}  // namespace pck
