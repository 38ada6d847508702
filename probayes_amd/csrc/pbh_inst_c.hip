// pbh_inst_c.hip -- kernel instantiations for d in [9, 10].
#include "pbh_kernels_impl.h"

namespace pbh {
PBH_INSTANTIATE(9)
PBH_INSTANTIATE(10)
}  // namespace pbh
