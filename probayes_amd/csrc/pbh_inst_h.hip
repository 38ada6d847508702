// pbh_inst_h.hip -- kernel instantiations for d in [32].
#include "pbh_kernels_impl.h"

namespace pbh {
PBH_INSTANTIATE(32)
}  // namespace pbh
