// pbh_dispatch.cpp -- runtime dim -> compiled kernel instantiation.
// The kernels are instantiated per dimension in pbh_inst_*.hip so that the
// gfx950 code objects compile in parallel.
#include <cstring>
#include <cmath>
#include <cstdlib>
#include <unordered_map>

#include "pbh_kernels.h"
#include "pbh_device.h"
#include "../../include/pbhip.h"

namespace pbh {

LaunchEvents &launch_events() {
  static thread_local LaunchEvents ev;
  return ev;
}

bool module_launch() {
  static const bool on = [] {
    const char *m = std::getenv("PBH_MODULE_LAUNCH");
    return !(m && m[0] == '0');
  }();
  return on;
}

// Keyed by (kernel, current device): a handle is resolved for the device
// that is current when it is looked up (engines on several devices in one
// process each get their own).  Null (the caller then takes
// hipLaunchKernelGGL) when the lookup fails.
hipFunction_t kernel_function(const void *kernel) {
  struct Key {
    const void *k;
    int dev;
    bool operator==(const Key &o) const { return k == o.k && dev == o.dev; }
  };
  struct Hash {
    size_t operator()(const Key &x) const {
      return std::hash<const void *>()(x.k) ^ ((size_t)x.dev * 0x9E3779B97F4A7C15ull);
    }
  };
  static thread_local std::unordered_map<Key, hipFunction_t, Hash> cache;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  const Key key{kernel, dev};
  auto it = cache.find(key);
  if (it != cache.end()) return it->second;
  hipFunction_t fn = nullptr;
  if (hipGetFuncBySymbol(&fn, kernel) != hipSuccess) fn = nullptr;
  cache.emplace(key, fn);
  return fn;
}


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

template <int D>
hipError_t launch_mh_server_d(const KArgs &a, hipStream_t st, int32_t *wgs, bool check);

hipError_t launch_mh_server(const KArgs &a, hipStream_t s, int32_t *wgs, bool check) {
  switch (a.d) {
#define PBH_CASE(D) \
  case D:           \
    return launch_mh_server_d<D>(a, s, wgs, check);
    PBH_DIMS(PBH_CASE)
#undef PBH_CASE
    default:
      return hipErrorNotSupported;
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

// Per-chain sums of a recorded trace [rec][d][n] over records [first, first +
// count): thread (k, c) walks its column; every wave reads 512 contiguous
// bytes per record.  Threads k == d count the accept bits of chain c.
__global__ void trace_stats_kernel(const double *tx, const uint64_t *tacc,
                                   int64_t n, int32_t d, int64_t W,
                                   int64_t first, int64_t count, double *sum,
                                   double *sumsq, int64_t *nacc) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t k = i / n, c = i % n;
  if (k > d) return;
  if (k < d) {
    double s = 0., q = 0.;
    const double *p = tx + (first * d + k) * n + c;
    for (int64_t r = 0; r < count; ++r, p += d * n) {
      const double v = *p;
      s += v;
      q = __builtin_fma(v, v, q);
    }
    sum[k * n + c] = s;
    sumsq[k * n + c] = q;
  } else {
    int64_t a = 0;
    const uint64_t *m = tacc + first * W + (c >> 6);
    for (int64_t r = 0; r < count; ++r, m += W) a += (*m >> (c & 63)) & 1u;
    nacc[c] = a;
  }
}

hipError_t launch_trace_stats(const double *tx, const uint64_t *tacc, int64_t n,
                              int32_t d, int64_t W, int64_t first,
                              int64_t count, double *sum, double *sumsq,
                              int64_t *nacc, hipStream_t s) {
  const int64_t m = (int64_t)(d + 1) * n;
  hipLaunchKernelGGL(trace_stats_kernel, dim3((unsigned)((m + 255) / 256)),
                     dim3(256), 0, s, tx, tacc, n, d, W, first, count, sum,
                     sumsq, nacc);
  return hipGetLastError();
}

// PD.expectation over trace records [first, first + count): thread (k, c)
// walks chain c's column of dim k and its log-probs in record order --
// NumPy's axis-0 sums are sequential per column, and prob * v is rounded
// before the add, as here (no contraction in this file's build).
__global__ void trace_expect_kernel(const double *tx, const double *tlp,
                                    int64_t n, int32_t d, int64_t first,
                                    int64_t count, double exponent, int32_t lin,
                                    double log_npi, double *out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t k = i / n, c = i % n;
  if (k >= d) return;
  const double *xv = tx + (first * d + k) * n + c;
  const double *lv = tlp + first * n + c;
  double sp = 0., spv = 0.;
  for (int64_t r = 0; r < count; ++r, xv += d * n, lv += n) {
    const double l = *lv;
    const double p = lin ? l : (l <= log_npi ? exp(l) : 1.7976931348623158e+308);
    double v = *xv;
    if (exponent == 2.0) v = v * v;                    // NumPy's square loop
    else if (exponent != 0.0 && exponent != 1.0) v = pow(v, exponent);
    sp = sp + p;
    spv = spv + p * v;
  }
  const double tiny = 2.2250738585072014e-308;       // NEARLY_POSITIVE_ZERO
  const double den = sp != sp ? sp : (sp > tiny ? sp : tiny);
  out[k * n + c] = spv / den;
}

hipError_t launch_trace_expectation(const double *tx, const double *tlp,
                                    int64_t n, int32_t d, int64_t first,
                                    int64_t count, double exponent, int32_t lin,
                                    double log_npi, double *out, hipStream_t s) {
  const int64_t m = (int64_t)d * n;
  hipLaunchKernelGGL(trace_expect_kernel, dim3((unsigned)((m + 255) / 256)),
                     dim3(256), 0, s, tx, tlp, n, d, first, count, exponent,
                     lin, log_npi, out);
  return hipGetLastError();
}

// Effective sample size of every (chain, dim) series of trace records
// [first, first + count): Geyer's initial positive sequence on the
// autocorrelations of the centred series, the estimator of
// scripts/bench_workloads.py ess_ips (rho_k = ac_k / ac_0 with ac_k =
// sum_t xc_t xc_{t+k}; pairs rho_{2j+1} + rho_{2j+2} summed up to the first
// non-positive one; ess = T / (1 + 2 sum)).
// Layout: a QUAD of lanes per series (16 series per wave, contiguous chains
// of one dim: each (lane j, t) load is a 128-byte row segment), lane j
// taking the j-th quarter of the records; the quad's partial sums combine by
// DPP (the same association in every lane, so the four lanes agree
// bitwise).  The mean is one pass over the quarter; then passes of 32 lags
// (K0 + 1 .. K0 + 32, lag 0 in the first): per record one load of x_t and
// one of the lagged x_{t-K0-1} into a 32-entry register ring indexed by
// t mod 32 (the record loop is unrolled by 32, so every ring index is
// static) and 32 fp64 FMAs.  A wave stops after the pass in which all its
// series reached a non-positive pair.
constexpr int kEssLags = 32;

template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
  const uint64_t u = __builtin_bit_cast(uint64_t, v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)u, CTRL, 0xF, 0xF, false);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)(u >> 32), CTRL, 0xF, 0xF, false);
  return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}
// sum over the quad, (a + b) + (c + d) in every lane
__device__ __forceinline__ double quad_sum(double v) {
  v = v + dpp_f64<0xB1>(v);   // quad_perm [1, 0, 3, 2]
  return v + dpp_f64<0x4E>(v);   // quad_perm [2, 3, 0, 1]
}

__global__ __launch_bounds__(256) void trace_ess_kernel(
    const double *tx, int64_t n, int32_t d, int64_t first, int64_t T, double *ess) {
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int j = threadIdx.x & 3;
  const int64_t sid = gid >> 2;              // series = k * n + c
  const bool valid = sid < (int64_t)d * n;
  const int64_t s0 = valid ? sid : 0;
  const int64_t k = s0 / n, c = s0 % n;
  const int64_t stride = (int64_t)d * n;
  const double *xs = tx + (first * d + k) * n + c;
  const int64_t seg = (T + 3) / 4;
  const int64_t t0 = j * seg < T ? j * seg : T;
  const int64_t t1 = t0 + seg < T ? t0 + seg : T;
  double sum = 0.;
  for (int64_t t = t0; t < t1; ++t) sum += xs[t * stride];
  const double mean = quad_sum(sum) / (double)T;
  const int64_t m = (T - 1) / 2;   // pairs (lags 2J+1, 2J+2), J < m
  double ac0 = 0., inv0 = 0., s = 0.;
  bool done = m <= 0 || !valid;
  for (int64_t K0 = 0; __ballot(!done); K0 += kEssLags) {
    // the ring R[(t - t0) mod 32] holds u_t = xc_{t-K0-1} (0 before record 0)
    double R[kEssLags], acc[kEssLags];
#pragma unroll
    for (int l = 0; l < kEssLags; ++l) {
      acc[l] = 0.;
      const int64_t tt = t0 - kEssLags + l - K0 - 1;   // u_{t0 - 32 + l}
      R[l] = (l > 0 && tt >= 0 && tt < T) ? xs[tt * stride] - mean : 0.;
    }
    double a0 = 0.;
    for (int64_t tb = t0; tb < t1; tb += kEssLags) {
#pragma unroll
      for (int i = 0; i < kEssLags; ++i) {
        const int64_t t = tb + i;
        const bool in = t < t1;
        const double xc = in ? xs[t * stride] - mean : 0.;
        const int64_t tu = t - K0 - 1;
        R[i] = (in && tu >= 0) ? xs[tu * stride] - mean : 0.;
        if (K0 == 0) a0 = __builtin_fma(xc, xc, a0);
#pragma unroll
        for (int l = 0; l < kEssLags; ++l)
          acc[l] = __builtin_fma(xc, R[(i - l + kEssLags) % kEssLags], acc[l]);
      }
    }
    if (K0 == 0) {
      ac0 = quad_sum(a0);
      inv0 = 1.0 / (ac0 > 1e-300 ? ac0 : 1e-300);
    }
#pragma unroll
    for (int l = 0; l < kEssLags; ++l) acc[l] = quad_sum(acc[l]);
    // pairs (K0 + 2q + 1, K0 + 2q + 2) = acc[2q], acc[2q + 1]
#pragma unroll
    for (int q = 0; q < kEssLags / 2; ++q) {
      if (!done) {
        if (K0 / 2 + q >= m) {
          done = true;
        } else {
          const double pr = acc[2 * q] * inv0 + acc[2 * q + 1] * inv0;
          if (pr <= 0.) done = true;
          else s += pr;
        }
      }
    }
  }
  if (valid && j == 0) {
    const double den = 1.0 + 2.0 * s;
    ess[s0] = (double)T / (den > 1e-12 ? den : 1e-12);
  }
}

// ---------------------------------------------------------------------------
// The same estimator through FFTs, the host's own method (ess_ips: rfft at
// length 2T, |F|^2, irfft): one workgroup per PAIR of series (a, b) --
// z_t = (a_t - mean a) + i (b_t - mean b) zero-padded to N = 4096 >= 2T, one
// complex FFT, the two power spectra unpacked (X_k = (Z_k + conj Z_{N-k}) / 2,
// Y_k = (Z_k - conj Z_{N-k}) / 2i) and packed again as P_k = |X_k|^2 + i
// |Y_k|^2, one inverse FFT: Re / Im of the result are N x the two series'
// autocovariance sums at every lag (no wrap: N >= 2T).  Then Geyer's pairs
// (rho_{2j+1} + rho_{2j+2}, rho = ac / ac_0) summed up to the first non-
// positive one, found by a block-wide min.  O(T log T) per series instead of
// O(T x lags): the GMM chains of cfg5 need a few hundred lags.
// FFT: Stockham autosort, radix 16 (4096 = 16^3, three passes, 256 threads
// x 16 points in registers, the 16-point DFT as 4 x 4).  Between passes the
// points are exchanged through ONE 32 KiB array of doubles, real parts then
// imaginary parts (four barriers per exchange instead of two, half the
// LDS): four workgroups of four waves fit a CU (a 64 KiB complex buffer
// held it to two, and two waves per SIMD left the fp64 pipe waiting on
// latency and barriers).  The array is XOR-swizzled within 16-entry rows
// (fsw): the stride-16 writes of the first pass and the contiguous reads are
// then conflict-free for ds_write_b64 / ds_read_b64.
// Twiddles: one sincospi per transform size and thread (the inverse's are
// conjugates), powers by a depth-4 product tree.  Series s (= k n + c) and
// s + 1 are adjacent doubles of every record, so a lane reads both with one
// 16-byte load; workgroups are mapped so that consecutive pairs share an XCD
// (and its L2) -- the reads of one record row by neighbouring pairs then hit
// the same L2 lines.
// ---------------------------------------------------------------------------
constexpr int kFftN = 4096, kFftT = 256;   // points, threads
struct cdbl { double re, im; };
__device__ __forceinline__ int fsw(int e) { return e + (e >> 4); }
__device__ __forceinline__ cdbl cadd(cdbl a, cdbl b) { return {a.re + b.re, a.im + b.im}; }
__device__ __forceinline__ cdbl csub(cdbl a, cdbl b) { return {a.re - b.re, a.im - b.im}; }
__device__ __forceinline__ cdbl cmul(cdbl a, cdbl b) {
  return {__builtin_fma(a.re, b.re, -(a.im * b.im)), __builtin_fma(a.re, b.im, a.im * b.re)};
}
__device__ __forceinline__ cdbl conj(cdbl a) { return {a.re, -a.im}; }
// times SIGN i
template <int SIGN>
__device__ __forceinline__ cdbl cmuli(cdbl a) {
  return SIGN > 0 ? cdbl{-a.im, a.re} : cdbl{a.im, -a.re};
}
template <int SIGN>
__device__ __forceinline__ void dft4(cdbl &a0, cdbl &a1, cdbl &a2, cdbl &a3) {
  const cdbl t0 = cadd(a0, a2), t1 = csub(a0, a2), t2 = cadd(a1, a3);
  const cdbl t3 = cmuli<SIGN>(csub(a1, a3));
  a0 = cadd(t0, t2);
  a2 = csub(t0, t2);
  a1 = cadd(t1, t3);
  a3 = csub(t1, t3);
}
// 16-point DFT (exponent sign SIGN) of v; X[k1 + 4 k2] lands in v[4 k1 + k2]
template <int SIGN>
__device__ __forceinline__ void dft16(cdbl (&v)[16]) {
  constexpr double C1 = 0.92387953251128675613, S1 = 0.38268343236508977173;
  constexpr double C2 = 0.70710678118654752440;
#pragma unroll
  for (int n2 = 0; n2 < 4; ++n2) dft4<SIGN>(v[n2], v[4 + n2], v[8 + n2], v[12 + n2]);
  // v[4 k1 + n2] *= W16^(SIGN n2 k1)
  const cdbl w1{C1, SIGN * S1}, w2{C2, SIGN * C2}, w3{S1, SIGN * C1};
  const cdbl w6{-C2, SIGN * C2}, w9{-C1, -SIGN * S1};
  v[5] = cmul(v[5], w1);
  v[6] = cmul(v[6], w2);
  v[7] = cmul(v[7], w3);
  v[9] = cmul(v[9], w2);
  v[10] = cmuli<SIGN>(v[10]);
  v[11] = cmul(v[11], w6);
  v[13] = cmul(v[13], w3);
  v[14] = cmul(v[14], w6);
  v[15] = cmul(v[15], w9);
#pragma unroll
  for (int k1 = 0; k1 < 4; ++k1) dft4<SIGN>(v[4 * k1], v[4 * k1 + 1], v[4 * k1 + 2], v[4 * k1 + 3]);
}
// The arithmetic of one Stockham pass (sub-transform size NS -> 16 NS) on
// the thread's points v[r] = x[j + 256 r]: twiddle, 16-point DFT.  w = exp(SIGN
// 2 pi i m / (16 NS)), m = j % NS.  IN_HALF:
// v[8..15] are zero (the padded series) and are not multiplied.
template <int SIGN, int NS, bool IN_HALF = false>
__device__ __forceinline__ void fft_compute(cdbl (&v)[16], cdbl w) {
  if constexpr (NS > 1) {
    // w^(4 a + b) = w^(4 a) w^b: six powers live, each other one formed
    // just before its product (14 complex products in all)
    const cdbl p1 = w, p2 = cmul(w, w), p3 = cmul(p2, w), p4 = cmul(p2, p2);
    const cdbl p8 = cmul(p4, p4), p12 = cmul(p8, p4);
    const cdbl pb[4] = {cdbl{1., 0.}, p1, p2, p3}, pa[4] = {cdbl{1., 0.}, p4, p8, p12};
#pragma unroll
    for (int r = 1; r < 16; ++r) {
      if (IN_HALF && r >= 8) continue;
      const int a = r >> 2, b = r & 3;
      v[r] = cmul(v[r], a == 0 ? pb[b] : b == 0 ? pa[a] : cmul(pa[a], pb[b]));
    }
  }
  dft16<SIGN>(v);
}
// where a pass leaves output v[i] (i = 4 k1 + k2): base + (k1 + 4 k2) NS
template <int NS>
__device__ __forceinline__ int fft_out(int i) {
  const int j = (int)threadIdx.x;
  return (j / NS) * NS * 16 + (j % NS) + ((i >> 2) + 4 * (i & 3)) * NS;
}
// Move the pass outputs (fft_out<NS>) to the next pass's inputs
// (x[j + 256 r] in v[r]) through sb, real parts then imaginary parts.
template <int NS>
__device__ __forceinline__ void fft_exchange(double *sb, cdbl (&v)[16]) {
  const int j = (int)threadIdx.x;
  double t[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) sb[fsw(fft_out<NS>(i))] = v[i].re;
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 16; ++r) t[r] = sb[fsw(j + r * kFftT)];
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 16; ++i) sb[fsw(fft_out<NS>(i))] = v[i].im;
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 16; ++r) v[r] = cdbl{t[r], sb[fsw(j + r * kFftT)]};
  __syncthreads();
}
// the twiddle bases of passes 2 and 3 (NS = 16, 256) for SIGN = -1; the
// inverse transform's are their conjugates
struct FftTw { cdbl w16, w256; };
__device__ __forceinline__ FftTw fft_twiddles() {
  const int j = (int)threadIdx.x;
  FftTw t;
  double sn, cs;
  sincospi(-(double)(2 * (j % 16)) / 256.0, &sn, &cs);
  t.w16 = cdbl{cs, sn};
  sincospi(-(double)(2 * (j % 256)) / 4096.0, &sn, &cs);
  t.w256 = cdbl{cs, sn};
  return t;
}

// block-wide sum / min over the 256 threads (red: 8 scratch entries)
__device__ __forceinline__ double block_sum(double v, double *red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  return (red[0] + red[1]) + (red[2] + red[3]);
}
__device__ __forceinline__ int block_min(int v, int *red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o));
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  return min(min(red[0], red[1]), min(red[2], red[3]));
}

// XCD-aware pair index: block b runs on XCD b % 8; give each XCD a
// contiguous range of pairs
__device__ __forceinline__ int64_t xcd_pair_index() {
  const int64_t nb = gridDim.x, b = blockIdx.x;
  const int64_t per = nb / 8, rem = nb % 8, xcd = b % 8, idx = b / 8;
  return xcd < rem ? xcd * (per + 1) + idx : rem * (per + 1) + (xcd - rem) * per + idx;
}

__device__ __forceinline__ void ess4k_pair(const double *tx, int64_t n, int32_t d,
                                           int64_t first, int32_t T, double *ess,
                                           int64_t P, double *sb, double *red, int *ired) {
  const int64_t S = (int64_t)d * n;
  const int64_t s0 = 2 * P;
  const bool has_b = s0 + 1 < S;
  const int j = (int)threadIdx.x;
  const int64_t row = (int64_t)d * n;
  const double *src = tx + first * row + s0;
  // ---- load (t = j + 256 q, q < 8: T <= 2048) and centre ----
  double xa[8], xb[8];
  double sa = 0., sb_ = 0.;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int t = j + q * kFftT;
    xa[q] = 0.;
    xb[q] = 0.;
    if (t < T) {
      if (has_b && !(row & 1)) {
        // series s0, s0 + 1: adjacent doubles, 16-byte aligned when the
        // record length d n is even (s0 is even, the trace base aligned)
        const double2 v = *reinterpret_cast<const double2 *>(src + (int64_t)t * row);
        xa[q] = v.x;
        xb[q] = v.y;
      } else if (has_b) {   // odd d n: every other record is 8-byte aligned
        xa[q] = src[(int64_t)t * row];
        xb[q] = src[(int64_t)t * row + 1];
      } else {
        xa[q] = src[(int64_t)t * row];
      }
    }
    sa += xa[q];
    sb_ += xb[q];
  }
  const double ma = block_sum(sa, red) / (double)T;
  const double mb = block_sum(sb_, red + 4) / (double)T;
  const FftTw tw = fft_twiddles();
  // ---- forward transform of a + i b (points 2048 .. 4095 zero): the
  // thread's points x[j + 256 r] are already in registers ----
  cdbl v[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int t = j + q * kFftT;
    v[q] = cdbl{0., 0.};
    if (q < 8 && t < T) v[q] = cdbl{xa[q] - ma, has_b ? xb[q] - mb : 0.};
  }
  fft_compute<-1, 1, true>(v, cdbl{1., 0.});
  fft_exchange<1>(sb, v);
  fft_compute<-1, 16>(v, tw.w16);
  fft_exchange<16>(sb, v);
  fft_compute<-1, 256>(v, tw.w256);
  // ---- unpack the two spectra (Z_k and Z_{N-k}), pack |X|^2 + i |Y|^2 at
  // k = j + 256 q: the inverse transform's first-pass points ----
  double xr[16], yi[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) sb[fsw(fft_out<256>(i))] = v[i].re;
  __syncthreads();
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int k = j + q * kFftT;
    const double zk = sb[fsw(k)], zm = sb[fsw((kFftN - k) & (kFftN - 1))];
    xr[q] = zk + zm;   // 2 Re X_k
    yi[q] = zm - zk;   // 2 Im Y_k
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 16; ++i) sb[fsw(fft_out<256>(i))] = v[i].im;
  __syncthreads();
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int k = j + q * kFftT;
    const double zk = sb[fsw(k)], zm = sb[fsw((kFftN - k) & (kFftN - 1))];
    const double xi = zk - zm, yr = zk + zm;   // 2 Im X_k, 2 Re Y_k
    v[q] = cdbl{__builtin_fma(xr[q], xr[q], xi * xi), __builtin_fma(yr, yr, yi[q] * yi[q])};
  }
  __syncthreads();
  // ---- inverse transform; only lags 0 .. 2047 are kept ----
  fft_compute<1, 1>(v, cdbl{1., 0.});
  fft_exchange<1>(sb, v);
  fft_compute<1, 16>(v, conj(tw.w16));
  fft_exchange<16>(sb, v);
  fft_compute<1, 256>(v, conj(tw.w256));
  // autocovariances of a in sb[0, 2048), of b in sb[2048, 4096)
#pragma unroll
  for (int i = 0; i < 16; ++i)
    if ((i & 3) < 2) {   // lag fft_out<256>(i) < 2048
      const int e = fsw(fft_out<256>(i));
      sb[e] = v[i].re;
      sb[kFftN / 2 + kFftN / 32 + e] = v[i].im;
    }
  __syncthreads();
  // ---- Geyer's initial positive sequence on both series ----
  const double a0 = sb[0], b0 = sb[kFftN / 2 + kFftN / 32];
  const double ia = 1.0 / (a0 > 1e-300 ? a0 : 1e-300);
  const double ib = 1.0 / (b0 > 1e-300 ? b0 : 1e-300);
  const int m = (T - 1) / 2;   // pairs (lags 2J + 1, 2J + 2), J < m
  double pa[4], pb[4];
  int fa = m, fb = m;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int J = j + q * kFftT;
    pa[q] = pb[q] = 0.;
    if (J < m) {
      const int e1 = fsw(2 * J + 1), e2 = fsw(2 * J + 2);
      pa[q] = sb[e1] * ia + sb[e2] * ia;
      pb[q] = sb[kFftN / 2 + kFftN / 32 + e1] * ib + sb[kFftN / 2 + kFftN / 32 + e2] * ib;
      if (pa[q] <= 0. && J < fa) fa = J;
      if (pb[q] <= 0. && J < fb) fb = J;
    }
  }
  fa = block_min(fa, ired);
  fb = block_min(fb, ired + 4);
  double qa = 0., qb = 0.;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int J = j + q * kFftT;
    if (J < fa) qa += pa[q];
    if (J < fb) qb += pb[q];
  }
  qa = block_sum(qa, red);
  qb = block_sum(qb, red + 4);
  if (j == 0) {
    const double da = 1.0 + 2.0 * qa, db = 1.0 + 2.0 * qb;
    ess[s0] = (double)T / (da > 1e-12 ? da : 1e-12);
    if (has_b) ess[s0 + 1] = (double)T / (db > 1e-12 ? db : 1e-12);
  }
}

__global__ __launch_bounds__(kFftT) __attribute__((amdgpu_waves_per_eu(3, 3)))
void trace_ess_fft_kernel(const double *tx, int64_t n, int32_t d, int64_t first,
                          int32_t T, double *ess) {
  __shared__ double sb[kFftN + kFftN / 16];
  __shared__ double red[8];
  __shared__ int ired[8];
  ess4k_pair(tx, n, d, first, T, ess, xcd_pair_index(), sb, red, ired);
}

// The 4 096-point form over a device list of pairs (the 2 048-point kernel's
// fallback: list[0] = count, pairs in list[1 ..]): one block per possible
// entry, the blocks past the count exit at once.  (A fixed grid striding over
// the list kept every block's registers live across iterations: 289 spilled
// VGPRs.)
__global__ __launch_bounds__(kFftT) __attribute__((amdgpu_waves_per_eu(3, 3)))
void trace_ess_fft_list_kernel(const double *tx, int64_t n, int32_t d, int64_t first,
                               int32_t T, double *ess, const int32_t *list) {
  __shared__ double sb[kFftN + kFftN / 16];
  __shared__ double red[8];
  __shared__ int ired[8];
  const int32_t cnt = __builtin_nontemporal_load(list);   // block-uniform
  if ((int32_t)blockIdx.x >= cnt) return;
  ess4k_pair(tx, n, d, first, T, ess, list[1 + blockIdx.x], sb, red, ired);
}

// ---------------------------------------------------------------------------
// The 2 048-point form (round 5): the same estimator with the pair's complex
// series zero-padded to N = 2 048 instead of 4 096.  The circular
// autocovariance at lag k is then a_k + a_{N-k}, and a_{N-k} = 0 while N - k
// >= T: lags k <= N - T are exact.  Geyer's scan needs lags up to its first
// non-positive pair, which for the cfg5 chains (T = 1 500, exact to lag 548)
// is at lag ~180 at the median and beyond 548 for ~1 % of the series (a
// NumPy simulation of the cfg5 target); a pair whose scan reaches the end of
// the exact range without a non-positive pair is appended to a device list
// and redone by the 4 096-point form (trace_ess_fft_list_kernel).  Half the
// points per transform (and one pass of radix 8 instead of 16): 128 threads
// x 16 points, radix 16, 16, 8.  The radix-8 pass leaves thread j holding
// X[j + 128 q] in natural order, so the spectrum's unpack and the inverse's
// first pass read and write the registers in place.
// ---------------------------------------------------------------------------
constexpr int kF2N = 2048, kF2T = 128;

template <int SIGN>
__device__ __forceinline__ void dft8(cdbl &a0, cdbl &a1, cdbl &a2, cdbl &a3, cdbl &a4,
                                     cdbl &a5, cdbl &a6, cdbl &a7) {
  // X[2k] = DFT4(a_n + a_{n+4})[k], X[2k+1] = DFT4((a_n - a_{n+4}) W8^n)[k]
  constexpr double C2 = 0.70710678118654752440;
  cdbl b0 = cadd(a0, a4), b1 = cadd(a1, a5), b2 = cadd(a2, a6), b3 = cadd(a3, a7);
  cdbl c0 = csub(a0, a4), c1 = csub(a1, a5), c2 = csub(a2, a6), c3 = csub(a3, a7);
  // W8 = (C2, SIGN C2): c1 W8, c2 (SIGN i), c3 W8^3 = (-C2, SIGN C2)
  c1 = cdbl{C2 * (c1.re - SIGN * c1.im), C2 * (c1.im + SIGN * c1.re)};
  c2 = cmuli<SIGN>(c2);
  c3 = cdbl{-C2 * (c3.re + SIGN * c3.im), C2 * (SIGN * c3.re - c3.im)};
  dft4<SIGN>(b0, b1, b2, b3);
  dft4<SIGN>(c0, c1, c2, c3);
  a0 = b0; a2 = b1; a4 = b2; a6 = b3;
  a1 = c0; a3 = c1; a5 = c2; a7 = c3;
}

// pass 3 (NS = 256, radix 8): thread j runs DFTs j and j + 128 over its
// even / odd points (x[m + 256 r] = v[2 r] or v[2 r + 1]), twiddles w^r with
// w = exp(SIGN 2 pi i m / 2048); outputs land in natural order, v[q] = X[j + 128 q]
template <int SIGN>
__device__ __forceinline__ void fft2_pass3(cdbl (&v)[16], cdbl wa) {
  constexpr double C1 = 0.92387953251128675613, S1 = 0.38268343236508977173;
  const cdbl wb = cmul(wa, cdbl{C1, SIGN * S1});   // m + 128: one more 1/16 turn
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const cdbl w = h ? wb : wa;
    const cdbl w2 = cmul(w, w), w3 = cmul(w2, w), w4 = cmul(w2, w2);
    v[2 + h] = cmul(v[2 + h], w);
    v[4 + h] = cmul(v[4 + h], w2);
    v[6 + h] = cmul(v[6 + h], w3);
    v[8 + h] = cmul(v[8 + h], w4);
    v[10 + h] = cmul(v[10 + h], cmul(w4, w));
    v[12 + h] = cmul(v[12 + h], cmul(w4, w2));
    v[14 + h] = cmul(v[14 + h], cmul(w4, w3));
    dft8<SIGN>(v[h], v[2 + h], v[4 + h], v[6 + h], v[8 + h], v[10 + h], v[12 + h], v[14 + h]);
  }
}

// pass outputs (fft_out<NS>, 128 threads) to the next pass's inputs
// x[j + 128 r] in v[r], through sb: real parts then imaginary parts
template <int NS>
__device__ __forceinline__ void fft2_exchange(double *sb, cdbl (&v)[16]) {
  const int j = (int)threadIdx.x;
  double t[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) sb[fsw(fft_out<NS>(i))] = v[i].re;
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 16; ++r) t[r] = sb[fsw(j + r * kF2T)];
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 16; ++i) sb[fsw(fft_out<NS>(i))] = v[i].im;
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 16; ++r) v[r] = cdbl{t[r], sb[fsw(j + r * kF2T)]};
  __syncthreads();
}

// the whole 2 048-point transform, natural order in and out (v[q] = x[j + 128 q])
template <int SIGN>
__device__ __forceinline__ void fft2k(double *sb, cdbl (&v)[16], cdbl w16, cdbl w2k) {
  fft_compute<SIGN, 1>(v, cdbl{1., 0.});
  fft2_exchange<1>(sb, v);
  fft_compute<SIGN, 16>(v, w16);
  fft2_exchange<16>(sb, v);
  fft2_pass3<SIGN>(v, w2k);
}

__device__ __forceinline__ double block2_sum(double v, double *red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  return red[0] + red[1];
}
__device__ __forceinline__ int block2_min(int v, int *red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o));
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  return min(red[0], red[1]);
}

// T <= kF2N - 2 records; list[0] counts the pairs handed to the 4 096-point
// form, list[1 ..] holds them (list[0] zeroed before the launch)
__global__ __launch_bounds__(kF2T) __attribute__((amdgpu_waves_per_eu(3, 3)))
void trace_ess_fft2k_kernel(const double *tx, int64_t n, int32_t d, int64_t first,
                            int32_t T, double *ess, int32_t *list) {
  __shared__ double sb[kF2N + kF2N / 16];
  __shared__ double red[4];
  __shared__ int ired[4];
  const int64_t P = xcd_pair_index();
  const int64_t S = (int64_t)d * n;
  const int64_t s0 = 2 * P;
  const bool has_b = s0 + 1 < S;
  const int j = (int)threadIdx.x;
  const int64_t row = S;
  const double *src = tx + first * row + s0;
  // ---- load (t = j + 128 q) and centre ----
  cdbl v[16];
  double sa = 0., sbb = 0.;
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int t = j + q * kF2T;
    v[q] = cdbl{0., 0.};
    if (t < T) {
      if (has_b && !(row & 1)) {
        const double2 x = *reinterpret_cast<const double2 *>(src + (int64_t)t * row);
        v[q] = cdbl{x.x, x.y};
      } else if (has_b) {   // odd d n: every other record is 8-byte aligned
        v[q] = cdbl{src[(int64_t)t * row], src[(int64_t)t * row + 1]};
      } else {
        v[q] = cdbl{src[(int64_t)t * row], 0.};
      }
    }
    sa += v[q].re;
    sbb += v[q].im;
  }
  const double ma = block2_sum(sa, red) / (double)T;
  const double mb = block2_sum(sbb, red + 2) / (double)T;
#pragma unroll
  for (int q = 0; q < 16; ++q)
    if (j + q * kF2T < T) v[q] = cdbl{v[q].re - ma, has_b ? v[q].im - mb : 0.};
  // twiddle bases: pass 2 exp(-2 pi i (j % 16) / 256), pass 3 exp(-2 pi i j / 2048)
  cdbl w16, w2k;
  {
    double sn, cs;
    sincospi(-(double)(2 * (j % 16)) / 256.0, &sn, &cs);
    w16 = cdbl{cs, sn};
    sincospi(-(double)(2 * j) / 2048.0, &sn, &cs);
    w2k = cdbl{cs, sn};
  }
  fft2k<-1>(sb, v, w16, w2k);
  // ---- unpack Z_k, Z_{N-k} (k = j + 128 q) and pack |X_k|^2 + i |Y_k|^2:
  // imaginary parts first, so that only their squares stay live (48 doubles
  // at the peak instead of 64) ----
  {
    double xi2[16], yr2[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) sb[fsw(j + q * kF2T)] = v[q].im;
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int k = j + q * kF2T;
      const double zk = v[q].im, zm = sb[fsw((kF2N - k) & (kF2N - 1))];
      const double xi = zk - zm, yr = zk + zm;   // 2 Im X_k, 2 Re Y_k
      xi2[q] = xi * xi;
      yr2[q] = yr * yr;
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 16; ++q) sb[fsw(j + q * kF2T)] = v[q].re;
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int k = j + q * kF2T;
      const double zk = v[q].re, zm = sb[fsw((kF2N - k) & (kF2N - 1))];
      const double xr = zk + zm, yi = zm - zk;   // 2 Re X_k, 2 Im Y_k
      v[q] = cdbl{__builtin_fma(xr, xr, xi2[q]), __builtin_fma(yi, yi, yr2[q])};
    }
    __syncthreads();
  }
  fft2k<1>(sb, v, conj(w16), conj(w2k));
  // ---- lags 0 .. 1023 of both series to LDS (a: [0, 1088), b: [1088, ...)) ----
  constexpr int kB = kF2N / 2 + kF2N / 32;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int e = fsw(j + q * kF2T);
    sb[e] = v[q].re;
    sb[kB + e] = v[q].im;
  }
  __syncthreads();
  // ---- Geyer's initial positive sequence over the exact pairs ----
  const double a0 = sb[0], b0 = sb[kB];
  const double ia = 1.0 / (a0 > 1e-300 ? a0 : 1e-300);
  const double ib = 1.0 / (b0 > 1e-300 ? b0 : 1e-300);
  const int m = (T - 1) / 2;          // pairs (lags 2J + 1, 2J + 2), J < m
  const int mx = (kF2N - T) / 2;      // pairs whose lags are all <= N - T
  const int lim = m < mx ? m : mx;    // <= 511: lags <= 1023
  double pa[4], pb[4];
  int fa = lim, fb = lim;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int J = j + q * kF2T;
    pa[q] = pb[q] = 0.;
    if (J < lim) {
      const int e1 = fsw(2 * J + 1), e2 = fsw(2 * J + 2);
      pa[q] = sb[e1] * ia + sb[e2] * ia;
      pb[q] = sb[kB + e1] * ib + sb[kB + e2] * ib;
      if (pa[q] <= 0. && J < fa) fa = J;
      if (pb[q] <= 0. && J < fb) fb = J;
    }
  }
  fa = block2_min(fa, ired);
  fb = block2_min(fb, ired + 2);
  // a scan that ran to the end of the exact range short of m: the 4 096-point
  // form decides this pair
  const bool redo = lim < m && (fa == lim || (has_b && fb == lim));
  if (redo) {
    if (j == 0) {
      const int32_t at = __hip_atomic_fetch_add(list, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      list[1 + at] = (int32_t)P;
    }
    return;   // block-uniform
  }
  double qa = 0., qb = 0.;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int J = j + q * kF2T;
    if (J < fa) qa += pa[q];
    if (J < fb) qb += pb[q];
  }
  qa = block2_sum(qa, red);
  qb = block2_sum(qb, red + 2);
  if (j == 0) {
    const double da = 1.0 + 2.0 * qa, db = 1.0 + 2.0 * qb;
    ess[s0] = (double)T / (da > 1e-12 ? da : 1e-12);
    if (has_b) ess[s0 + 1] = (double)T / (db > 1e-12 ? db : 1e-12);
  }
}

// ---------------------------------------------------------------------------
// The 2 048-point form on ONE wavefront per pair (the default): 64 lanes x 32
// points, the same radix 16, 16, 8 passes (two 16-point DFTs per lane in the
// first two, four 8-point DFTs in the third).  A one-wave workgroup has no
// barriers (the compiler drops them): its exchanges through LDS wait only on
// the wave's own accesses, and a SIMD's two waves never wait for each other
// (the two-wave form spent 41 % of its wave cycles parked at barriers and
// waits, r05a_ess).  The spectrum's unpack pairs lane j with lane 64 - j
// through ds_bpermute (Z_{N-k} for k = j + 64 r is lane 64 - j's point 31 -
// r; lane 0's is its own point 32 - r), in place, so no extra registers.
// ---------------------------------------------------------------------------
constexpr int kWL = 64;   // lanes

// exchange for the one-wave form: outputs (v[i] at lds index out(i)) to
// natural order x[j + 64 r] in v[r], real parts then imaginary parts
template <typename OUT>
__device__ __forceinline__ void fftw_exchange(double *sb, cdbl (&v)[32], OUT out) {
  // the real parts come back into the registers they left (in natural order,
  // while the imaginary parts still sit in pass order): no temporaries
  const int j = (int)threadIdx.x;
#pragma unroll
  for (int i = 0; i < 32; ++i) sb[fsw(out(i))] = v[i].re;
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 32; ++r) v[r].re = sb[fsw(j + r * kWL)];
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 32; ++i) sb[fsw(out(i))] = v[i].im;
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 32; ++r) v[r].im = sb[fsw(j + r * kWL)];
  __syncthreads();
}

// passes 1 and 2 (radix 16, NS = 1 / 16): DFTs m = j + 64 h, h = 0, 1, over
// x[m + 128 r'] = v[2 r' + h]; outputs k of DFT h land in v[2 i + h] with
// i = 4 k1 + k2 for k = k1 + 4 k2 (dft16's order)
template <int SIGN, int NS>
__device__ __forceinline__ void fftw_pass16(cdbl (&v)[32], cdbl w) {
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    cdbl u[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) u[r] = v[2 * r + h];
    fft_compute<SIGN, NS>(u, w);
#pragma unroll
    for (int i = 0; i < 16; ++i) v[2 * i + h] = u[i];
  }
}
template <int NS>
struct FftwOut {   // where v[2 i + h] of fftw_pass16<., NS> belongs
  int j;
  __device__ __forceinline__ int operator()(int e) const {
    const int h = e & 1, i = e >> 1;
    const int m = j + kWL * h, k = (i >> 2) + 4 * (i & 3);
    return (m / NS) * NS * 16 + (m % NS) + k * NS;
  }
};

// pass 3 (radix 8, NS = 256): DFTs m = j + 64 h, h < 4, over x[m + 256 r'] =
// v[h + 4 r']; twiddles w_m^r' with w_m = w_j exp(SIGN 2 pi i h / 32); outputs
// in place and natural: v[h + 4 k] = X[m + 256 k] = X[j + 64 (h + 4 k)]
template <int SIGN>
__device__ __forceinline__ void fftw_pass3(cdbl (&v)[32], cdbl wj) {
  // exp(SIGN 2 pi i h / 32), h = 1, 2, 3
  constexpr double c1 = 0.98078528040323044913, s1 = 0.19509032201612826785;
  constexpr double c2 = 0.92387953251128675613, s2 = 0.38268343236508977173;
  constexpr double c3 = 0.83146961230254523708, s3 = 0.55557023301960222474;
#pragma unroll
  for (int h = 0; h < 4; ++h) {
    const cdbl w = h == 0 ? wj
                 : cmul(wj, h == 1 ? cdbl{c1, SIGN * s1} : h == 2 ? cdbl{c2, SIGN * s2}
                                                          : cdbl{c3, SIGN * s3});
    const cdbl w2 = cmul(w, w), w3 = cmul(w2, w), w4 = cmul(w2, w2);
    v[4 + h] = cmul(v[4 + h], w);
    v[8 + h] = cmul(v[8 + h], w2);
    v[12 + h] = cmul(v[12 + h], w3);
    v[16 + h] = cmul(v[16 + h], w4);
    v[20 + h] = cmul(v[20 + h], cmul(w4, w));
    v[24 + h] = cmul(v[24 + h], cmul(w4, w2));
    v[28 + h] = cmul(v[28 + h], cmul(w4, w3));
    dft8<SIGN>(v[h], v[4 + h], v[8 + h], v[12 + h], v[16 + h], v[20 + h], v[24 + h], v[28 + h]);
  }
}

template <int SIGN>
__device__ __forceinline__ void fftw(double *sb, cdbl (&v)[32], cdbl w16, cdbl w2k) {
  const int j = (int)threadIdx.x;
  fftw_pass16<SIGN, 1>(v, cdbl{1., 0.});
  fftw_exchange(sb, v, FftwOut<1>{j});
  fftw_pass16<SIGN, 16>(v, w16);
  fftw_exchange(sb, v, FftwOut<16>{j});
  fftw_pass3<SIGN>(v, w2k);
}

__device__ __forceinline__ double bperm_f64(int addr, double x) {
  const uint64_t u = __builtin_bit_cast(uint64_t, x);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_ds_bpermute(addr, (int)(uint32_t)u);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_ds_bpermute(addr, (int)(uint32_t)(u >> 32));
  return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}
// 4 |X_k|^2 + 4 i |Y_k|^2 from z = Z_k and m = Z_{N-k} (X = (Z_k + conj
// Z_{N-k}) / 2, Y = (Z_k - conj Z_{N-k}) / 2i)
__device__ __forceinline__ cdbl ess_power(cdbl z, cdbl m) {
  const double xr = z.re + m.re, xi = z.im - m.im;   // 2 Re X, 2 Im X
  const double yr = z.im + m.im, yi = m.re - z.re;   // 2 Re Y, 2 Im Y
  return cdbl{__builtin_fma(xr, xr, xi * xi), __builtin_fma(yr, yr, yi * yi)};
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
__device__ __forceinline__ int wave_min(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o));
  return v;
}

// T <= 1 536 records (then v[24 ..] start at 0); list as trace_ess_fft2k_kernel
__global__ __launch_bounds__(kWL) __attribute__((amdgpu_waves_per_eu(2, 2)))
void trace_ess_fftw_kernel(const double *tx, int64_t n, int32_t d, int64_t first,
                           int32_t T, double *ess, int32_t *list) {
  __shared__ double sb[kF2N + kF2N / 16];
  const int64_t P = xcd_pair_index();
  const int64_t S = (int64_t)d * n;
  const int64_t s0 = 2 * P;
  const bool has_b = s0 + 1 < S;
  const int j = (int)threadIdx.x;
  const double *src = tx + first * S + s0;
  cdbl v[32];
  double sa = 0., sbb = 0.;
#pragma unroll
  for (int r = 0; r < 32; ++r) {
    const int t = j + r * kWL;
    v[r] = cdbl{0., 0.};
    if (r < 24 && t < T) {
      if (has_b && !(S & 1)) {
        const double2 x = *reinterpret_cast<const double2 *>(src + (int64_t)t * S);
        v[r] = cdbl{x.x, x.y};
      } else if (has_b) {   // odd d n: every other record is 8-byte aligned
        v[r] = cdbl{src[(int64_t)t * S], src[(int64_t)t * S + 1]};
      } else {
        v[r] = cdbl{src[(int64_t)t * S], 0.};
      }
    }
    sa += v[r].re;
    sbb += v[r].im;
  }
  const double ma = wave_sum(sa) / (double)T;
  const double mb = wave_sum(sbb) / (double)T;
#pragma unroll
  for (int r = 0; r < 24; ++r)
    if (j + r * kWL < T) v[r] = cdbl{v[r].re - ma, has_b ? v[r].im - mb : 0.};
  cdbl w16, w2k;
  {
    double sn, cs;
    sincospi(-(double)(2 * (j % 16)) / 256.0, &sn, &cs);
    w16 = cdbl{cs, sn};
    sincospi(-(double)(2 * j) / 2048.0, &sn, &cs);
    w2k = cdbl{cs, sn};
  }
  fftw<-1>(sb, v, w16, w2k);
  // ---- unpack in place: pairs (i, 31 - i) with lane 64 - j; lane 0 pairs
  // (i, 32 - i) within itself (and its point 16 alone) ----
  {
    const int addr = ((kWL - j) & (kWL - 1)) * 4;
    const bool l0 = j == 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const cdbl ra{bperm_f64(addr, v[31 - i].re), bperm_f64(addr, v[31 - i].im)};
      const cdbl rb{bperm_f64(addr, v[i].re), bperm_f64(addr, v[i].im)};
      const cdbl ma_ = l0 ? v[(32 - i) & 31] : ra;   // Z_{N-k} of point i
      const cdbl p1 = ess_power(v[i], ma_);
      const cdbl p2 = ess_power(v[31 - i], rb);
      // branch-free (a divergent branch per pair kept both paths' copies
      // of the points live: 99 spilled VGPRs)
      v[i] = p1;
      v[31 - i] = cdbl{l0 ? v[31 - i].re : p2.re, l0 ? v[31 - i].im : p2.im};
      if (i > 0)   // lane 0: P_{N-k} = P_k
        v[32 - i] = cdbl{l0 ? p1.re : v[32 - i].re, l0 ? p1.im : v[32 - i].im};
    }
    const cdbl p16 = ess_power(v[16], v[16]);
    v[16] = cdbl{l0 ? p16.re : v[16].re, l0 ? p16.im : v[16].im};
  }
  fftw<1>(sb, v, conj(w16), conj(w2k));
  // ---- lags 0 .. 1023 of both series to LDS (a: [0, 1088), b: [1088, ...)) ----
  constexpr int kB = kF2N / 2 + kF2N / 32;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int e = fsw(j + r * kWL);
    sb[e] = v[r].re;
    sb[kB + e] = v[r].im;
  }
  __syncthreads();
  const double a0 = sb[0], b0 = sb[kB];
  const double ia = 1.0 / (a0 > 1e-300 ? a0 : 1e-300);
  const double ib = 1.0 / (b0 > 1e-300 ? b0 : 1e-300);
  const int m = (T - 1) / 2;
  const int mx = (kF2N - T) / 2;
  const int lim = m < mx ? m : mx;   // <= 511
  double pa[8], pb[8];
  int fa = lim, fb = lim;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int J = j + q * kWL;
    pa[q] = pb[q] = 0.;
    if (J < lim) {
      const int e1 = fsw(2 * J + 1), e2 = fsw(2 * J + 2);
      pa[q] = sb[e1] * ia + sb[e2] * ia;
      pb[q] = sb[kB + e1] * ib + sb[kB + e2] * ib;
      if (pa[q] <= 0. && J < fa) fa = J;
      if (pb[q] <= 0. && J < fb) fb = J;
    }
  }
  fa = wave_min(fa);
  fb = wave_min(fb);
  if (lim < m && (fa == lim || (has_b && fb == lim))) {
    if (j == 0) {
      const int32_t at = __hip_atomic_fetch_add(list, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      list[1 + at] = (int32_t)P;
    }
    return;
  }
  double qa = 0., qb = 0.;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int J = j + q * kWL;
    if (J < fa) qa += pa[q];
    if (J < fb) qb += pb[q];
  }
  qa = wave_sum(qa);
  qb = wave_sum(qb);
  if (j == 0) {
    const double da = 1.0 + 2.0 * qa, db = 1.0 + 2.0 * qb;
    ess[s0] = (double)T / (da > 1e-12 ? da : 1e-12);
    if (has_b) ess[s0 + 1] = (double)T / (db > 1e-12 ? db : 1e-12);
  }
}

hipError_t launch_trace_ess(const double *tx, int64_t n, int32_t d,
                            int64_t first, int64_t count, double *ess,
                            hipStream_t st, int fft, int32_t *list) {
  const int64_t pairs = ((int64_t)d * n + 1) / 2;
  // the 2 048-point form while its exact range covers at least 512 lags
  // (2: one wave per pair, 3: two waves per pair)
  if ((fft == 2 || fft == 3) && list && count <= kF2N - 512) {
    hipError_t err = hipMemsetAsync(list, 0, sizeof(int32_t), st);
    if (err != hipSuccess) return err;
    if (fft == 2)
      hipLaunchKernelGGL(trace_ess_fftw_kernel, dim3((unsigned)pairs), dim3(kWL), 0, st,
                         tx, n, d, first, (int32_t)count, ess, list);
    else
      hipLaunchKernelGGL(trace_ess_fft2k_kernel, dim3((unsigned)pairs), dim3(kF2T), 0, st,
                         tx, n, d, first, (int32_t)count, ess, list);
    err = hipGetLastError();
    if (err != hipSuccess) return err;
    hipLaunchKernelGGL(trace_ess_fft_list_kernel, dim3((unsigned)pairs), dim3(kFftT), 0, st,
                       tx, n, d, first, (int32_t)count, ess, list);
    return hipGetLastError();
  }
  if (fft && count <= kFftN / 2) {
    hipLaunchKernelGGL(trace_ess_fft_kernel, dim3((unsigned)pairs), dim3(kFftT), 0, st,
                       tx, n, d, first, (int32_t)count, ess);
    return hipGetLastError();
  }
  const int64_t m = 4 * (int64_t)d * n;   // a quad of lanes per series
  hipLaunchKernelGGL(trace_ess_kernel, dim3((unsigned)((m + 255) / 256)),
                     dim3(256), 0, st, tx, n, d, first, count, ess);
  return hipGetLastError();
}

// The ESS total of one dim per workgroup: each of 1 024 threads sums the
// chains c = t, t + 1 024, ... in order, then a fixed tree over the threads
// (the same order every call: deterministic).
__global__ __launch_bounds__(1024) void ess_total_kernel(const double *ess, int64_t n,
                                                        double *total) {
  __shared__ double part[1024];
  const double *row = ess + (int64_t)blockIdx.x * n;
  double acc = 0.0;
  for (int64_t c = threadIdx.x; c < n; c += 1024) acc += row[c];
  part[threadIdx.x] = acc;
  __syncthreads();
  for (int w = 512; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) part[threadIdx.x] += part[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) total[blockIdx.x] = part[0];
}

hipError_t launch_ess_total(const double *ess, int64_t n, int32_t d, double *total,
                            hipStream_t st) {
  hipLaunchKernelGGL(ess_total_kernel, dim3((unsigned)d), dim3(1024), 0, st, ess, n, total);
  return hipGetLastError();
}

// The bm64 tables (pbh_device.h): sin(J 2 pi / 1024) and cos(J 2 pi / 1024),
// J = 0..1023 (the first quadrant evaluated, the others by exact symmetry)
// as four arrays of 32-bit words (sin lo, sin hi, cos lo, cos hi); then
// {-2 ln c_j, 1 / c_j} for c_j = (1024 + j) / 2048, j = 0..1024; then
// 2^(i/64), i = 0..63.  Evaluated in long double (64-bit significand) and
// rounded once to double.
void legacy_log_table(double *out) {
  for (int j = 0; j < kLegLogN; ++j) {
    const long double c = 0.5L + (long double)j / 256.0L;   // exact
    const long double t = logl(c);
    const double hi = (double)(roundl(t * 4294967296.0L) / 4294967296.0L);   // k 2^-32
    out[2 * j] = hi;
    out[2 * j + 1] = (double)(t - (long double)hi);
    out[kLegLogInv + j] = (double)(1.0L / c);
  }
  out[kLegLogDoubles - 1] = 0.0;
}

void bm64_tables(double *out) {
  double *lg = out + kBm64LogOff;
  for (int j = 0; j < kBm64LogN; ++j) {
    const double c = (1024 + j) / 2048.0;   // exact
    lg[2 * j] = (double)(-2.0L * logl((long double)c));
    lg[2 * j + 1] = 1.0 / c;
  }
  const long double pi = 3.141592653589793238462643383279502884L;
  uint32_t *sc = reinterpret_cast<uint32_t *>(out);
  constexpr int N = kBm64ScN, Q = kBm64ScN / 4;   // entries, per quadrant
  auto put = [&](int J, double s, double c) {
    uint64_t bs, bc;
    memcpy(&bs, &s, 8);
    memcpy(&bc, &c, 8);
    sc[J] = (uint32_t)bs;
    sc[N + J] = (uint32_t)(bs >> 32);
    sc[2 * N + J] = (uint32_t)bc;
    sc[3 * N + J] = (uint32_t)(bc >> 32);
  };
  for (int j = 0; j < Q; ++j) {
    const long double t = pi / 2.0L * (long double)j / (long double)Q;
    const double s = j == 0 ? 0.0 : (double)sinl(t);
    const double c = j == 0 ? 1.0 : (double)cosl(t);
    // angle J = j + k Q: (sin, cos) rotated by k quarter turns
    put(j, s, c);
    put(j + Q, c, -s);
    put(j + 2 * Q, -s, -c);
    put(j + 3 * Q, -c, s);
  }
  for (int i = 0; i < kExp2N; ++i) out[kBm64ExpOff + i] = (double)exp2l(i / 64.0L);
}

// Diagnostic: bm96_pair (one pair per 3 words) against the same
// construction through ocml's libm log / sqrt / sincos (u1 and the angle
// formed exactly as bm96_pair forms them).
__global__ void check_normals64_kernel(int64_t n, const uint32_t *words,
                                       const double *tab, double *fast,
                                       double *ref) {
  __shared__ double s_bmt[kBm64Doubles];
  bm64_load(s_bmt, tab);
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t a = words[3 * i], b = words[3 * i + 1], c = words[3 * i + 2];
  bm96_pair(a, b, c, s_bmt, fast[2 * i], fast[2 * i + 1]);
  const double u1 = from_words(0x3FF00000u | (b >> 12), a) - (1.0 - 0x1p-53);
  const double turn = ((double)((b >> 2) & 0x3FFu) + (double)c * 0x1p-32) * (1.0 / 1024.0);
  double sv, cv;
  sincospi(2.0 * turn, &sv, &cv);   // turn of 2 pi
  const double r = sqrt(-2.0 * log(u1));
  ref[2 * i] = r * cv;
  ref[2 * i + 1] = r * sv;
}

hipError_t launch_check_normals64(int64_t n, const uint32_t *words,
                                  const double *tab, double *fast, double *ref) {
  hipLaunchKernelGGL(check_normals64_kernel, dim3((unsigned)((n + 255) / 256)),
                     dim3(256), 0, 0, n, words, tab, fast, ref);
  return hipGetLastError();
}

}  // namespace pbh
