// Instantiations of the gfx950 kernels for op::BitOR (integer types only: it does not compile for floats, mpi.h:106-111) (include/core/mpi.h:85-112).
#include "rdc_kernels_impl.h"

namespace rdc_amd {
bool pick_bitor(int dtype, KernelSet* ks) { return pick_int<RDC_OP_BITOR>(dtype, ks); }
}  // namespace rdc_amd
