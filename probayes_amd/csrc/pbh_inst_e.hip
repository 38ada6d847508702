// pbh_inst_e.hip -- kernel instantiations for d in [16].
#include "pbh_kernels_impl.h"

namespace pbh {
PBH_INSTANTIATE(16)
}  // namespace pbh
