// pbh_dispatch.cpp -- runtime dim -> compiled kernel instantiation.
// The kernels are instantiated per dimension in pbh_inst_*.hip so that the
// gfx950 code objects compile in parallel.
#include "pbh_kernels.h"
#include "../../include/pbhip.h"

namespace pbh {

template <int D>
hipError_t launch_mh_d(const KArgs &a, hipStream_t st, size_t lds);
template <int D>
hipError_t launch_gibbs_d(const KArgs &a, hipStream_t st);

#define PBH_DIMS(X) \
  X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(16) X(20) X(24) X(32)

bool mh_dim_supported(int d) {
  switch (d) {
#define PBH_CASE(D) case D:
    PBH_DIMS(PBH_CASE)
#undef PBH_CASE
    return true;
    default:
      return false;
  }
}

hipError_t launch_mh(const KArgs &a, hipStream_t s, size_t lds) {
  switch (a.d) {
#define PBH_CASE(D) \
  case D:           \
    return launch_mh_d<D>(a, s, lds);
    PBH_DIMS(PBH_CASE)
#undef PBH_CASE
    default:
      return hipErrorInvalidValue;
  }
}

hipError_t launch_gibbs(const KArgs &a, hipStream_t s) {
  switch (a.d) {
#define PBH_CASE(D) \
  case D:           \
    return launch_gibbs_d<D>(a, s);
    PBH_DIMS(PBH_CASE)
#undef PBH_CASE
    default:
      return hipErrorInvalidValue;
  }
}

}  // namespace pbh
