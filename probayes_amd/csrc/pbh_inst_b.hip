// pbh_inst_b.hip -- kernel instantiations for d in [5, 6, 7, 8].
#include "pbh_kernels_impl.h"

namespace pbh {
PBH_INSTANTIATE(5)
PBH_INSTANTIATE(6)
PBH_INSTANTIATE(7)
PBH_INSTANTIATE(8)
}  // namespace pbh
