// pbh_dispatch.cpp -- runtime dim -> compiled kernel instantiation.
// The kernels are instantiated per dimension in pbh_inst_*.hip so that the
// gfx950 code objects compile in parallel.
#include "pbh_kernels.h"
#include "pbh_device.h"
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

// xoshiro128** seeding: stream (chain c, lane half h) gets the 128-bit state
// of two SplitMix64 outputs started at seed * phi ^ (2 * (off + c) + h), the
// seeding Blackman & Vigna recommend; stream ids are global chain ids, so a
// chain's draws do not depend on how chains are sharded over GPUs.
__global__ void xo_seed_kernel(uint32_t *xo, int64_t n, int64_t off,
                               uint64_t seed) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= 2 * n) return;
  const int64_t h = i / n, c = i % n;
  uint64_t z = (seed * 0x9E3779B97F4A7C15ull) ^ (uint64_t)(2 * (off + c) + h);
  const uint64_t u = splitmix64(z), v = splitmix64(z);
  uint32_t w[4] = {(uint32_t)u, (uint32_t)(u >> 32), (uint32_t)v,
                   (uint32_t)(v >> 32)};
  if ((w[0] | w[1] | w[2] | w[3]) == 0u) w[0] = 1u;   // never the zero state
  for (int k = 0; k < 4; ++k) xo[(k * 2 + h) * n + c] = w[k];
}

hipError_t launch_xo_seed(uint32_t *xo, int64_t n, int64_t off, uint64_t seed,
                          hipStream_t s) {
  const int64_t m = 2 * n;
  hipLaunchKernelGGL(xo_seed_kernel, dim3((unsigned)((m + 255) / 256)),
                     dim3(256), 0, s, xo, n, off, seed);
  return hipGetLastError();
}

}  // namespace pbh
