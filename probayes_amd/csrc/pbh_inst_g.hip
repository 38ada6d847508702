// pbh_inst_g.hip -- kernel instantiations for d in [24].
#include "pbh_kernels_impl.h"

namespace pbh {
PBH_INSTANTIATE(24)
}  // namespace pbh
