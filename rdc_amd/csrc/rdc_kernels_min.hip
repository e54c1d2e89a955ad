// Instantiations of the gfx950 kernels for op::Min (include/core/mpi.h:85-112).
#include "rdc_kernels_impl.h"

namespace rdc_amd {
bool pick_min(int dtype, KernelSet* ks) { return pick_arith<RDC_OP_MIN>(dtype, ks); }
}  // namespace rdc_amd
