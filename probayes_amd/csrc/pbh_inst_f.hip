// pbh_inst_f.hip -- kernel instantiations for d in [20].
#include "pbh_kernels_impl.h"

namespace pbh {
PBH_INSTANTIATE(20)
}  // namespace pbh
