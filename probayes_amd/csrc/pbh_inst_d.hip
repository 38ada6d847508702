// pbh_inst_d.hip -- kernel instantiations for d in [11, 12].
#include "pbh_kernels_impl.h"

namespace pbh {
PBH_INSTANTIATE(11)
PBH_INSTANTIATE(12)
}  // namespace pbh
