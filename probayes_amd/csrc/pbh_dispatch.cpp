// pbh_dispatch.cpp -- runtime dim -> compiled kernel instantiation.
// The kernels are instantiated per dimension in pbh_inst_*.hip so that the
// gfx950 code objects compile in parallel.
#include <cstring>
#include <cmath>

#include "pbh_kernels.h"
#include "pbh_device.h"
#include "../../include/pbhip.h"

namespace pbh {

LaunchEvents &launch_events() {
  static thread_local LaunchEvents ev;
  return ev;
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

hipError_t launch_trace_ess(const double *tx, int64_t n, int32_t d,
                            int64_t first, int64_t count, double *ess,
                            hipStream_t st) {
  const int64_t m = 4 * (int64_t)d * n;   // a quad of lanes per series
  hipLaunchKernelGGL(trace_ess_kernel, dim3((unsigned)((m + 255) / 256)),
                     dim3(256), 0, st, tx, n, d, first, count, ess);
  return hipGetLastError();
}

// The bm64 tables (pbh_device.h): sin(J 2 pi / 1024) and cos(J 2 pi / 1024),
// J = 0..1023 (the first quadrant evaluated, the others by exact symmetry)
// as four arrays of 32-bit words (sin lo, sin hi, cos lo, cos hi); then
// {-2 ln c_j, 1 / c_j} for c_j = (1024 + j) / 2048, j = 0..1024; then
// 2^(i/64), i = 0..63.  Evaluated in long double (64-bit significand) and
// rounded once to double.
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
