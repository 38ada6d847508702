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

// Diagnostic: the production acceptance filter against the exact ratio form
// on caller-supplied (lp, lp', t) triples.  out[i] bit 0 = exact decision,
// bit 1 = the filter decided (no fallback needed), bit 2 = filter decision.
__global__ void check_accept_kernel(int64_t n, const double *lp,
                                    const double *lpp, const uint32_t *t0,
                                    const uint32_t *t1, int32_t lin,
                                    double log_npi, uint8_t *out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double t = u01(t0[i], t1[i]);
  const bool ex = ratio_accept(lpp[i], lp[i], t, lin != 0, log_npi);
  const Decision d = accept_filter(lpp[i], lp[i], t0[i], lin != 0);
  out[i] = (uint8_t)((ex ? 1 : 0) | (d.need ? 0 : 2) | (d.acc ? 4 : 0));
}

hipError_t launch_check_accept(int64_t n, const double *lp, const double *lpp,
                               const uint32_t *t0, const uint32_t *t1,
                               int32_t lin, double log_npi, uint8_t *out) {
  hipLaunchKernelGGL(check_accept_kernel, dim3((unsigned)((n + 255) / 256)),
                     dim3(256), 0, 0, n, lp, lpp, t0, t1, lin, log_npi, out);
  return hipGetLastError();
}

// Diagnostic: box_muller_fast against box_muller on caller-supplied blocks.
__global__ void check_normals_kernel(int64_t n, const uint32_t *words,
                                     double *fast, double *ref) {
  __shared__ BMTables t;
  bm_tables_init(&t);
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const u32x4 w{words[4 * i], words[4 * i + 1], words[4 * i + 2], words[4 * i + 3]};
  box_muller_tab(w, &t, fast[2 * i], fast[2 * i + 1]);
  box_muller(w, ref[2 * i], ref[2 * i + 1]);
}

hipError_t launch_check_normals(int64_t n, const uint32_t *words, double *fast,
                                double *ref) {
  hipLaunchKernelGGL(check_normals_kernel, dim3((unsigned)((n + 255) / 256)),
                     dim3(256), 0, 0, n, words, fast, ref);
  return hipGetLastError();
}

}  // namespace pbh
