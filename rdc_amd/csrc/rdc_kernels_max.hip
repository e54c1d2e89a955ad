// Instantiations of the gfx950 kernels for op::Max (include/core/mpi.h:85-112).
#include "rdc_kernels_impl.h"

namespace rdc_amd {
bool pick_max(int dtype, KernelSet* ks) { return pick_arith<RDC_OP_MAX>(dtype, ks); }
}  // namespace rdc_amd
