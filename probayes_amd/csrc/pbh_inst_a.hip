// pbh_inst_a.hip -- kernel instantiations for d in [1, 2, 3, 4].
#include "pbh_kernels_impl.h"

namespace pbh {
PBH_INSTANTIATE(1)
PBH_INSTANTIATE(2)
PBH_INSTANTIATE(3)
PBH_INSTANTIATE(4)
}  // namespace pbh
