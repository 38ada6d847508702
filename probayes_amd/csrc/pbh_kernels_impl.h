// pbh_kernels_impl.h -- gfx950 kernels of the batched MH / CondCov-Gibbs engine.
//
// Layout and mapping: one chain per lane, 64 chains per
// wavefront, the chain state x[d] and running moments live in VGPRs for the
// whole fused step loop; every HBM access is chain-contiguous
// ([step][dim][chain]) so a wavefront moves 512 contiguous bytes per fp64
// load/store.  Model constants are read with wave-uniform addresses (scalar
// loads), NORM_IID observations are staged once per workgroup in LDS.
//
// One chain-step restates SP.next (sp.py:221-258):
//   draws -> delta (field.py:469-531 / variable.py:600-638 / callable Delta)
//   -> x' = x + delta or exp(log x + delta)   (variable.py:641-697)
//   -> joint density (rf.py:565-581, sd.py:148-161, rv_utils.py:8-47)
//   -> score (sp_utils.py:19-64) -> s >= t (sp_utils.py:34-37)
//   -> keep (x', p') on accept else (x, p)  (sp.py:253-256)
#pragma once
#include <utility>

#include "pbh_kernels.h"
#include "pbh_device.h"
#include "../../include/pbhip.h"

namespace pbh {

namespace {

constexpr int kBlock = 256;
constexpr int kPairFullBlock = 512;   // FULL pair kernel's largest workgroup

// Model constants are never written by a kernel: reading them through the
// constant address space lets the compiler use scalar loads (s_load) with
// wave-uniform addresses and hoist them, instead of per-step vector loads
// that it must assume alias the trace stores.
__device__ __forceinline__ double cld(const double *p, int64_t i) {
  return ((const __attribute__((address_space(4))) double *)p)[i];
}

// A wave-uniform value kept in SGPRs: a select between two such values
// cannot then be turned into a vector load from a selected address.
__device__ __forceinline__ double uni(double v) {
  const uint64_t u = __builtin_bit_cast(uint64_t, v);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)u);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(u >> 32));
  return __builtin_bit_cast(double, (uint64_t)lo | ((uint64_t)hi << 32));
}

// Covariance-matrix random walk (rf.py:340-354): delta' = tfun() . delta
// with the Cholesky factor RF.set_tran(ndarray) installs (rf.py:210-220).
// Row k sums tfun[k][j] * delta[j] in j order (the zero half of a triangular
// factor adds exact zeros); the factor is read with wave-uniform scalar
// loads.  d^2 FMAs per chain-step on the VALU: the per-chain (d x d)(d)
// product has no cross-chain reuse for the matrix cores at d <= 32.
template <int D>
__device__ __forceinline__ void apply_tfun(const double *tf, double (&dl)[D]) {
  double out[D];
#pragma unroll
  for (int k = 0; k < D; ++k) {
    double acc = cld(tf, k * D) * dl[0];
#pragma unroll
    for (int j = 1; j < D; ++j) acc = acc + cld(tf, k * D + j) * dl[j];
    out[k] = acc;
  }
#pragma unroll
  for (int k = 0; k < D; ++k) dl[k] = out[k];
}

// prob.py:354-357: the mvn density is evaluated at the values reversed and,
// for d > 2, rotated by one: [x_{d-2}, ..., x_0, x_{d-1}] (App. A-4).
template <int D>
__device__ __forceinline__ constexpr int mvn_perm(int i) {
  return D <= 1 ? 0 : (D == 2 ? 1 - i : (i < D - 1 ? D - 2 - i : D - 1));
}

// scipy norm.logpdf(x, loc, scale): _norm_logpdf((x - loc) / scale) -
// log(scale), _norm_logpdf(y) = -y**2 / 2.0 - _norm_pdf_logC.
__device__ __forceinline__ double norm_logpdf(double x, double loc,
                                              double scale, double logscale,
                                              double logC) {
  const double y = (x - loc) / scale;
  return ((-(y * y)) / 2.0 - logC) - logscale;
}

// scipy norm.pdf: np.exp(-y**2 / 2.0) / _norm_pdf_C / scale.
__device__ __forceinline__ double norm_pdf(double x, double loc, double scale,
                                           double C) {
  const double y = (x - loc) / scale;
  return (exp((-(y * y)) / 2.0) / C) / scale;
}

// scipy uniform.pdf: 1.0 / scale on the closed support [loc, loc + scale].
__device__ __forceinline__ double uniform_pdf(double x, double lo,
                                              double scale) {
  const double y = (x - lo) / scale;
  return (0.0 <= y && y <= 1.0) ? 1.0 / scale : 0.0;
}

__device__ __forceinline__ Xo xo_load(const KArgs &a, int h, int64_t c) {
  return Xo{a.xo[(0 * 2 + h) * a.n + c], a.xo[(1 * 2 + h) * a.n + c],
            a.xo[(2 * 2 + h) * a.n + c], a.xo[(3 * 2 + h) * a.n + c]};
}

__device__ __forceinline__ void xo_store(const KArgs &a, int h, int64_t c,
                                         const Xo &s) {
  a.xo[(0 * 2 + h) * a.n + c] = s.s0;
  a.xo[(1 * 2 + h) * a.n + c] = s.s1;
  a.xo[(2 * 2 + h) * a.n + c] = s.s2;
  a.xo[(3 * 2 + h) * a.n + c] = s.s3;
}

__device__ __forceinline__ u32x4 ctr(uint32_t j, int64_t g, int64_t chain) {
  return u32x4{j, (uint32_t)g, (uint32_t)chain,
               (uint32_t)((uint64_t)chain >> 32) ^
                   ((uint32_t)((uint64_t)g >> 32) << 16)};
}

// Production Gaussian draws of one chain-step (mh_kernel and the GMM
// lane-group / quad kernels draw this same stream): the words of Philox
// blocks ctr(q, g, chain), q = 0, 1, ..., in order (x, y, z, w); normal pair
// p takes words 3p .. 3p + 2 (bm96_pair), and the word after the last pair
// gives the threshold's leading kStepLead bits.  D <= 2: one block per step.
constexpr int kStepLead = 24;

template <int D>
__device__ __forceinline__ uint32_t step_draws(const KArgs &a, int64_t g,
                                               int64_t chain, const double *tab,
                                               double (&r)[D]) {
  constexpr int NP = (D + 1) / 2, NW = 3 * NP + 1, NB = (NW + 3) / 4;
  uint32_t w[4 * NB];
#pragma unroll
  for (int q = 0; q < NB; ++q) {
    const u32x4 b = philox4x32_10(ctr(q, g, chain), a.seed_lo, a.seed_hi);
    w[4 * q] = b.x;
    w[4 * q + 1] = b.y;
    w[4 * q + 2] = b.z;
    w[4 * q + 3] = b.w;
  }
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    double z0, z1;
    bm96_pair(w[3 * p], w[3 * p + 1], w[3 * p + 2], tab, z0, z1);
    r[2 * p] = z0;
    if (2 * p + 1 < D) r[2 * p + 1] = z1;
  }
  return w[3 * NP] >> (32 - kStepLead);
}

// ---------------------------------------------------------------------------
// Joint density of x' (in the pscale of the model)
// ---------------------------------------------------------------------------
template <int D>
__device__ __forceinline__ double mvn_density(const KArgs &a,
                                              const double (&x)[D]) {
  // scipy _PSD form: maha = sum(square(dev . prec_U)); logpdf =
  // -0.5 * (rank*log(2pi) + log_pdet + maha); pdf = exp(logpdf).
  double dev[D];
#pragma unroll
  for (int i = 0; i < D; ++i) dev[i] = x[mvn_perm<D>(i)] - cld(a.ta, i);
  double sq[D];
#pragma unroll
  for (int j = 0; j < D; ++j) {
    double y = dev[0] * cld(a.tb, j);
#pragma unroll
    for (int i = 1; i < D; ++i) y = y + dev[i] * cld(a.tb, i * D + j);
    sq[j] = y * y;
  }
  const double maha = np_sum_regs<D>(sq, D);
  const double logpdf = -0.5 * (cld(a.tc, 0) + maha);
  return a.pscale == PBH_PSCALE_LIN ? exp(logpdf) : logpdf;
}

// Production GMM log-density for a compile-time component count: the K
// independent exp chains interleave (ILP at one wavefront per SIMD).
template <int D, int K>
__device__ __forceinline__ double gmm_fast(const KArgs &a, const double (&x)[D]) {
  double v[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const double w = cld(a.tw, k);
    double acc = cld(a.tw, K + k);
#pragma unroll
    for (int i = 0; i < D; ++i) {
      const double u = (x[i] - cld(a.tb, k * D + i)) * w;
      acc = __builtin_fma(-u, u, acc);
    }
    v[k] = acc;
  }
  double m = v[0];
#pragma unroll
  for (int k = 1; k < K; ++k) m = __builtin_fmax(m, v[k]);
  double sum = 0.;
#pragma unroll
  for (int k = 0; k < K; ++k) sum += fast_exp(v[k] - m);
  return m + log(sum);
}

// lx (production, may be null): log of x for the dims with the (log, exp)
// ufun, as the proposal formed them (x' = exp(log x + delta)), so the
// density need not take the log of x' again.
template <int D, int TGT, bool FAST>
__device__ __forceinline__ double joint_density(const KArgs &a,
                                                const double (&x)[D],
                                                const double *obs_lds,
                                                bool use_lds,
                                                const double *lx = nullptr) {
  double out = 0.0;
  switch (TGT ? TGT : a.target) {
    case PBH_TARGET_DIAG_GAUSS: {
      // lp(**kw) = sum(norm.logpdf(kw[k], mu_k, sigma_k)): Python sum from 0
      if (FAST) {
        // production path: -sum_k (w_k (x_k - mu_k))^2 - ksum, w = sqrt(.5)/sigma
#pragma unroll
        for (int k = 0; k < D; ++k) {
          const double u = (x[k] - cld(a.ta, k)) * cld(a.tw, k);
          out = __builtin_fma(-u, u, out);
        }
        out = out - a.ksum;
      } else {
#pragma unroll
        for (int k = 0; k < D; ++k)
          out = out + norm_logpdf(x[k], cld(a.ta, k), cld(a.tb, k), cld(a.tc, k), a.norm_logC);
      }
      break;
    }
    case PBH_TARGET_NORM_IID: {
      double mu = 0., sg = 1.;
#pragma unroll
      for (int k = 0; k < D; ++k) {
        if (k == a.i0) mu = x[k];
        if (k == a.i1) sg = x[k];
      }
      double lsg = 0.;
      if (!FAST) {
        lsg = log(sg);
      } else {
        double l = 0.;
        bool have = false;
#pragma unroll
        for (int k = 0; k < D; ++k)
          if (k == a.i1 && lx && ((a.ufun >> k) & 1u)) { l = lx[k]; have = true; }
        lsg = have ? l : fast_log(sg);
      }
      const double logC = a.norm_logC;
      if (FAST) {
        // production path: sufficient statistics (obar, S2) of the data;
        // 1 / sigma^2 by the hardware reciprocal + two Newton steps
        const double n = (double)a.tn;
        const double dm = cld(a.tw, 0) - mu;
        const double ss = __builtin_fma(n * dm, dm, cld(a.tw, 1));
        const double s2 = sg * sg;
        double ri = __builtin_amdgcn_rcp(s2);
        ri = __builtin_fma(__builtin_fma(-s2, ri, 1.0), ri, ri);
        ri = __builtin_fma(__builtin_fma(-s2, ri, 1.0), ri, ri);
        out = -0.5 * ss * ri - n * (logC + lsg);
      } else if (use_lds) {
        out = np_pairwise(
            [&](int64_t j) { return norm_logpdf(obs_lds[j], mu, sg, lsg, logC); },
            a.tn);
      } else {
        const double *obs = a.ta;
        out = np_pairwise(
            [&](int64_t j) { return norm_logpdf(obs[j], mu, sg, lsg, logC); },
            a.tn);
      }
      break;
    }
    case PBH_TARGET_GMM: {
      // a_k = logw_k + sum_i logpdf(x_i, mu_ki, sd_k); m + log(sum exp(a - m))
      const int64_t K = a.tn;
      if (FAST) {
        // production path: a_k = c_k - sum_i ((x_i - mu_ki) w_k)^2 with
        // w_k = sqrt(.5) / sd_k, c_k = logw_k - d (logC + log sd_k) (host);
        // two passes (max, then sum of exp) recompute the cheap a_k rather
        // than keep K values in registers; K <= 4 unrolled at compile time
        if (K == 3) { out = gmm_fast<D, 3>(a, x); break; }
        if (K == 2) { out = gmm_fast<D, 2>(a, x); break; }
        if (K == 4) { out = gmm_fast<D, 4>(a, x); break; }
        auto comp = [&](int64_t k) {
          const double w = cld(a.tw, k);
          double v = cld(a.tw, K + k);
#pragma unroll
          for (int i = 0; i < D; ++i) {
            const double u = (x[i] - cld(a.tb, k * D + i)) * w;
            v = __builtin_fma(-u, u, v);
          }
          return v;
        };
        double m = comp(0);
        for (int64_t k = 1; k < K; ++k) m = __builtin_fmax(m, comp(k));
        double sum = 0.;
        for (int64_t k = 0; k < K; ++k) sum += fast_exp(comp(k) - m);
        out = m + log(sum);
        break;
      }
      auto comp = [&](int64_t k) {
        double v = cld(a.ta, k);
#pragma unroll
        for (int i = 0; i < D; ++i)
          v = v + norm_logpdf(x[i], cld(a.tb, k * D + i), cld(a.tc, k), cld(a.te, k),
                              a.norm_logC);
        return v;
      };
      double m = comp(0);
      for (int64_t k = 1; k < K; ++k) {
        const double v = comp(k);
        m = (m != m) ? m : ((v != v || v > m) ? v : m);  // np.max: NaN wins
      }
      const double s = np_pairwise([&](int64_t k) { return exp(comp(k) - m); }, K);
      out = m + log(s);
      break;
    }
    case PBH_TARGET_NORM_PDF: {
      out = norm_pdf(x[0], cld(a.ta, 0), cld(a.tb, 0), a.norm_C);
#pragma unroll
      for (int k = 1; k < D; ++k)
        out = out * norm_pdf(x[k], cld(a.ta, k), cld(a.tb, k), a.norm_C);
      break;
    }
    case PBH_TARGET_UNIFORM_PDF: {
      out = uniform_pdf(x[0], cld(a.ta, 0), cld(a.tb, 0));
#pragma unroll
      for (int k = 1; k < D; ++k) out = out * uniform_pdf(x[k], cld(a.ta, k), cld(a.tb, k));
      break;
    }
    case PBH_TARGET_MVN:
      out = mvn_density<D>(a, x);
      break;
    default:
      out = __builtin_nan("");
  }
  if (a.has_prior) {
    // rv_prod_rule of the roots' uniform_prob (rf_utils.py:10-42,
    // rv_utils.py:30-38), then product(cond, dist) (sd.py:158-161)
    bool inside = true;
#pragma unroll
    for (int k = 0; k < D; ++k) {
      const bool lo_ok = ((a.plo_incl >> k) & 1u) ? (x[k] >= cld(a.plo, k))
                                                   : (x[k] > cld(a.plo, k));
      const bool hi_ok = ((a.phi_incl >> k) & 1u) ? (x[k] <= cld(a.phi, k))
                                                   : (x[k] < cld(a.phi, k));
      inside = inside && lo_ok && hi_ok;
    }
    out = (inside ? a.prior_logp : kNearlyNegInf) + out;
  }
  return out;
}

// pscales.py:219-236 div_prob(a, b, pscale, pscale, pscale=1.)
__device__ __forceinline__ double div_prob(const KArgs &a, double num,
                                           double den) {
  const bool lin = a.pscale == PBH_PSCALE_LIN;
  const double A = lin ? num : exp_logp(num, a.log_npi);
  const double B = lin ? den : exp_logp(den, a.log_npi);
  return A / np_max_tiny(B);
}

// hastings_scores / metropolis_scores (sp_utils.py:19-64).  Returns false
// when the score is None (auto-accept), else writes s.
// eB = rescale(lp) of the current state (cached across steps, updated on
// accept by the caller with eA = rescale(lpp)); the division is the same
// IEEE operation as div_prob's, so caching changes no bits.
template <int D>
__device__ __forceinline__ bool score(const KArgs &a, const double (&x)[D],
                                      const double (&xp)[D], double lp,
                                      double lpp, double eA, double eB,
                                      double &s) {
  if (a.scores == PBH_SCORES_METROPOLIS) {
    const double q = eA / np_max_tiny(eB);
    s = q < 1. ? q : 1.;  // Python min(1., q)
    return true;
  }
  double q;
  if (a.tran_kind == PBH_TRAN_CONST) {
    q = a.tran_value;
  } else {
    // prod of norm.pdf(x'_k, x_k + off_k, scale) in the callable's order
    q = 1.0;
    bool first = true;
#pragma unroll
    for (int j = 0; j < D; ++j) {
      const int k = a.tran_rev ? (D - 1 - j) : j;
      double v = 0.;
#pragma unroll
      for (int kk = 0; kk < D; ++kk)
        if (kk == k) v = norm_pdf(xp[kk], x[kk] + cld(a.tran_off, kk), a.tran_scale, a.norm_C);
      q = first ? v : q * v;
      first = false;
    }
  }
  // rescale(q, pscale, 1.) (pscales.py:100-131)
  const double qt = a.pscale == PBH_PSCALE_LIN ? q : exp_logp(q, a.log_npi);
  if (qt <= 0.) return false;                      // sp_utils.py:53-54
  double r;
  if (a.tran_sym) {
    r = eA / np_max_tiny(eB);                      // :56
  } else {
    // reval_tran returns the forward value (rf.py:536): r~ == q~
    r = div_prob(a, lpp * qt, lp * qt);            // :62-64
  }
  s = r < 1. ? r : 1.;
  return true;
}

// ---------------------------------------------------------------------------
// Per-variable delta helpers (variable.py:618-739)
// ---------------------------------------------------------------------------
// np.minimum / np.maximum: a NaN operand propagates
__device__ __forceinline__ double np_minimum(double a, double b) {
  return (a != a || b != b) ? a + b : (a < b ? a : b);
}
__device__ __forceinline__ double np_maximum(double a, double b) {
  return (a != a || b != b) ? a + b : (a > b ? a : b);
}

// bound=True on one scalar value (variable.py:711-728): closed limits clamp;
// both exclusive: outside (lo, hi) returns the predecessor xo; one exclusive
// side: strictly beyond it returns xo, the other side clamps.
__device__ __forceinline__ double bound_value(double v, double xo, double lo,
                                              double hi, bool xl, bool xh) {
  if (!xl && !xh) return np_maximum(lo, np_minimum(hi, v));
  if (xl && xh) return (v > lo && v < hi) ? v : xo;
  if (xl) return v < lo ? xo : np_minimum(hi, v);
  return v > hi ? xo : np_maximum(lo, v);
}

// randint(-d0, d0) in the production modes from one 53-bit uniform: NumPy
// truncates both bounds toward zero; the value is lo + floor(u * span),
// uniform over [lo, hi) to within span * 2^-53.
__device__ __forceinline__ double randint_u(double u, double d0) {
  const double lo = trunc(-d0), span = trunc(d0) - lo;
  const double k = floor(u * span);
  return lo + (k < span - 1. ? k : span - 1.);
}

// ---------------------------------------------------------------------------
// MH kernel: n_steps fused chain-steps, one chain per lane
// ---------------------------------------------------------------------------
// REPLAY's draws of step s: row rep_row0 + s of the [T][R][N] stream (d
// draws in dim order, then the threshold).  The fused legacy kernel
// (pbh_legacy.hip legacy_mh_kernel) supplies another source that generates
// the same values in registers.
struct RowDraws {
  __device__ __forceinline__ void begin() {}
  template <int D>
  __device__ __forceinline__ void draws(const KArgs &a, int s, int64_t cc, double (&r)[D],
                                        double &thr) {
    const double *row = a.rep + (a.rep_row0 + s) * a.R * a.n + cc;
#pragma unroll
    for (int k = 0; k < D; ++k) r[k] = row[k * a.n];
    thr = row[(int64_t)D * a.n];
  }
};

// The kernel body; SRC supplies REPLAY's draws, s_obs is the workgroup's
// LDS for NORM_IID observations (lds_ok: the caller reserved a.tn doubles)
template <int D, int RNG, int TGT, int PROP, class SRC>
__device__ __forceinline__ void mh_body(const KArgs &a, SRC &src, double *s_obs,
                                        bool lds_ok) {
  // TGT / PROP != 0 compile the kernel for one target / proposal form;
  // 0 keeps the wave-uniform runtime switch (any model, one binary).
  // FAST = production Philox path (fp32 normals, FMA-corrected divisions);
  // REPLAY and PHILOX_F64 keep the reference's arithmetic exactly.
  constexpr bool FAST = RNG == PBH_RNG_PHILOX || RNG == PBH_RNG_XOSHIRO;
  // production Gaussian deltas draw bm64 fp64 normals from LDS tables; ufun
  // dims take their log / exp from the same tables
  constexpr bool TAB = FAST;
  const int prop = PROP ? PROP : a.prop;
  const bool lin = a.pscale == PBH_PSCALE_LIN;
  const bool mom = a.moments != 0;
  // production modes with the symmetric ratio form: the acceptance filter
  const bool simple = FAST && a.simple_acc && !a.debug;
  __shared__ double s_bmt[TAB ? kBm64Doubles : 2];
  if constexpr (TAB) bm64_load(s_bmt, a.bm64);
  const int64_t c = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const bool active = c < a.n;
  const int64_t cc = active ? c : 0;
  const int lane = threadIdx.x & 63;

  bool use_lds = false;
  if (!FAST && (TGT == 0 || TGT == PBH_TARGET_NORM_IID) && lds_ok &&
      a.target == PBH_TARGET_NORM_IID && a.tn <= 16384) {
    for (int64_t j = threadIdx.x; j < a.tn; j += kBlock) s_obs[j] = cld(a.ta, j);
    __syncthreads();
    use_lds = true;
  }

  double x[D], ms[D], mq[D];
#pragma unroll
  for (int k = 0; k < D; ++k) {
    x[k] = a.x[k * a.n + cc];
    ms[k] = 0.;
    mq[k] = 0.;
  }
  double lp = a.lp[cc];
  double eB = lin ? lp : (FAST ? exp_logp_fast(lp, a.log_npi)
                              : exp_logp(lp, a.log_npi));
  int64_t nacc = 0;
  const int64_t chain = a.off + cc;
  Xo xs{0u, 0u, 0u, 0u};
  if (RNG == PBH_RNG_XOSHIRO) xs = xo_load(a, 0, cc);
  // production: the carried logs of the ufun dims (KArgs.lx)
  double lx[D];
#pragma unroll
  for (int k = 0; k < D; ++k) {
    lx[k] = 0.;
    if (FAST && ((a.ufun >> k) & 1u))
      lx[k] = a.lx_init ? ln_ufun(x[k], s_bmt) : a.lx[k * a.n + cc];
  }

  // record phase / index of the trace, advanced per step (no 64-bit
  // division in the loop): step g records iff (g + 1) % thin == 0, at
  // record (g + 1) / thin - 1 - rec_base.
  int ph = (int)((a.g0 + 1) % a.thin);
  int64_t ri = (a.g0 + 1) / a.thin - 1 - a.rec_base;
  if (RNG == PBH_RNG_REPLAY) src.begin();
  for (int s = 0; s < a.n_steps; ++s) {
    const int64_t g = a.g0 + s;
    // ---- draws ----
    double r[D];
    double thr = 0.;
    uint32_t tw0 = 0, tw1 = 0;   // threshold words: thr = u01(tw0, tw1)
    // production Philox: t's leading lead_bits bits are `lead`, the rest come
    // from block lead_ctr (drawn on demand when the filter decides alone)
    uint32_t lead = 0, lead_ctr = 0;
    int lead_bits = 0;
    if (RNG == PBH_RNG_REPLAY) {
      src.template draws<D>(a, s, cc, r, thr);
    } else if (RNG == PBH_RNG_XOSHIRO) {
      // three words per normal pair, two per 53-bit uniform, in draw order
      if (prop == PBH_PROP_GAUSS) {
#pragma unroll
        for (int p = 0; p < (D + 1) / 2; ++p) {
          const uint32_t w0 = xo_next(xs), w1 = xo_next(xs), w2 = xo_next(xs);
          double z0, z1;
          bm96_pair(w0, w1, w2, s_bmt, z0, z1);
          r[2 * p] = z0;
          if (2 * p + 1 < D) r[2 * p + 1] = z1;
        }
      } else {
#pragma unroll
        for (int k = 0; k < D; ++k) {
          const uint32_t w0 = xo_next(xs);
          r[k] = u01(w0, xo_next(xs));
        }
      }
      tw0 = xo_next(xs);
      tw1 = xo_next(xs);
      thr = u01(tw0, tw1);
    } else if (TAB && prop == PBH_PROP_GAUSS) {
      // bm96 fp64 normal pairs (step_draws); t's leading 24 bits follow the
      // pairs' words, the rest come from block 0x40 -- the same t as the
      // multi-lane GMM kernels' (their lead + fallback block).  The filter
      // needs only the lead: block 0x40 is drawn when it cannot decide.
      lead = step_draws<D>(a, g, chain, s_bmt, r);
      lead_bits = kStepLead;
      lead_ctr = 0x40u;
      if (!simple) {
        const u32x4 w = philox4x32_10(ctr(lead_ctr, g, chain), a.seed_lo, a.seed_hi);
        tw0 = (lead << (32 - kStepLead)) | (w.x >> kStepLead);
        tw1 = w.y;
        thr = u01(tw0, tw1);
      }
    } else if (RNG == PBH_RNG_PHILOX && prop != PBH_PROP_GAUSS) {
      // production uniform draws: t's leading 22 bits are the spare low bits
      // of block 0's words (u01 keeps the top 27 + 26 bits of each pair; at
      // d = 1 the unused word z gives them), the rest come from block 0xFFFF,
      // drawn when the filter cannot decide (or every step without it)
#pragma unroll
      for (int p = 0; p < (D + 1) / 2; ++p) {
        const u32x4 w = philox4x32_10(ctr(p, g, chain), a.seed_lo, a.seed_hi);
        r[2 * p] = u01(w.x, w.y);
        if (2 * p + 1 < D) r[2 * p + 1] = u01(w.z, w.w);
        if (p == 0)
          lead = ((w.x & 31u) << 17) | ((w.y & 63u) << 11) |
                 (D >= 2 ? (((w.z & 31u) << 6) | (w.w & 63u)) : (w.z >> 21));
      }
      lead_bits = 22;
      lead_ctr = 0xFFFFu;
      if (!simple) {
        const u32x4 w = philox4x32_10(ctr(lead_ctr, g, chain), a.seed_lo, a.seed_hi);
        tw0 = (lead << 10) | (w.x >> 22);
        tw1 = w.y;
        thr = u01(tw0, tw1);
      }
    } else {
      if (prop == PBH_PROP_GAUSS) {
#pragma unroll
        for (int p = 0; p < (D + 1) / 2; ++p) {
          double z0, z1;
          box_muller(philox4x32_10(ctr(p, g, chain), a.seed_lo, a.seed_hi), z0, z1);
          r[2 * p] = z0;
          if (2 * p + 1 < D) r[2 * p + 1] = z1;
        }
      } else {
#pragma unroll
        for (int p = 0; p < (D + 1) / 2; ++p) {
          const u32x4 w = philox4x32_10(ctr(p, g, chain), a.seed_lo, a.seed_hi);
          r[2 * p] = u01(w.x, w.y);
          if (2 * p + 1 < D) r[2 * p + 1] = u01(w.z, w.w);
        }
      }
      const u32x4 w = philox4x32_10(ctr(0xFFFFu, g, chain), a.seed_lo, a.seed_hi);
      tw0 = w.x;
      tw1 = w.y;
      thr = u01(w.x, w.y);
    }
    // ---- proposal ----
    double xp[D], lxp[D];
#pragma unroll
    for (int k = 0; k < D; ++k) lxp[k] = 0.;
    {
      double dl[D];
      if (prop == PBH_PROP_GAUSS) {
        // scipy rv_generic.rvs: z * scale + loc
#pragma unroll
        for (int k = 0; k < D; ++k) dl[k] = r[k] * cld(a.pscl, k) + cld(a.ploc, k);
      } else if (prop == PBH_PROP_UNIFORM) {
        // np.random.uniform(-delta, delta) = low + (high - low) * u
#pragma unroll
        for (int k = 0; k < D; ++k) {
          const double d0 = cld(a.pdel, k);
          dl[k] = -d0 + (d0 - -d0) * r[k];
        }
      } else if (prop == PBH_PROP_VARDELTA) {
        // per-variable deltas (variable.py:618-640), modes 2 bits per dim
#pragma unroll
        for (int k = 0; k < D; ++k) {
          const double d0 = cld(a.pdel, k);
          const int md = (int)((a.vmode >> (2 * k)) & 3u);
          if (md == PBH_VAR_FIXED)
            dl[k] = d0;
          else if (md == PBH_VAR_POLARITY)
            dl[k] = r[k] > 0.5 ? d0 : -d0;
          else if (md == PBH_VAR_UNIFORM)
            dl[k] = -d0 + (d0 - -d0) * r[k];
          else   // replay streams carry the randint value itself
            dl[k] = RNG == PBH_RNG_REPLAY ? r[k] : randint_u(r[k], d0);
        }
      } else {
        // spherical tuple delta (field.py:509-531)
        const double d0 = a.sdelta;
        double sq[D];
#pragma unroll
        for (int k = 0; k < D; ++k) {
          dl[k] = -d0 + (d0 - -d0) * r[k];
          sq[k] = dl[k] * dl[k];
        }
        const double ss = np_sum_regs<D>(sq, D);
        if (FAST) {
          // production: the radius scale d0 / sqrt(ss) from one inverse
          // square root (no IEEE sqrt and division on the step's chain);
          // rsq of max(ss, tiny) and a select, so that no branch is made
          const double rq = rsq_nr(__builtin_fmax(ss, kNearlyPosZero));
          const double sc = ss >= kNearlyPosZero ? d0 * rq : __builtin_inf();
#pragma unroll
          for (int k = 0; k < D; ++k) dl[k] = (dl[k] * sc) * cld(a.plen, k);
        } else {
          const double rss = ss >= kNearlyPosZero ? sqrt(ss) : 0.;
#pragma unroll
          for (int k = 0; k < D; ++k) dl[k] = ((dl[k] * d0) / rss) * cld(a.plen, k);
        }
      }
      if (a.has_tfun) apply_tfun<D>(a.ptf, dl);   // wave-uniform
#pragma unroll
      for (int k = 0; k < D; ++k) {
        if ((a.ufun >> k) & 1u) {
          if (FAST) {
            lxp[k] = lx[k] + dl[k];
            xp[k] = exp_ufun(lxp[k], s_bmt);
          } else {
            xp[k] = exp(log(x[k]) + dl[k]);
          }
        } else {
          xp[k] = x[k] + dl[k];
        }
      }
      if (a.vint | a.bnd_on) {   // wave-uniform: int variables, bound=True
#pragma unroll
        for (int k = 0; k < D; ++k) {
          const double v0 = xp[k];
          if ((a.vint >> k) & 1u) xp[k] = trunc(xp[k]);
          if ((a.bnd_on >> k) & 1u)
            xp[k] = bound_value(xp[k], x[k], cld(a.blo, k), cld(a.bhi, k),
                                (a.bnd_xlo >> k) & 1u, (a.bnd_xhi >> k) & 1u);
          // a clamped / bounced ufun value: its log is taken afresh
          if (FAST && ((a.ufun >> k) & 1u) && !(xp[k] == v0))
            lxp[k] = ln_ufun(xp[k], s_bmt);
        }
      }
    }
    // ---- density, score, accept ----
    const double lpp = joint_density<D, TGT, FAST>(a, xp, s_obs, use_lds,
                                                   FAST ? lxp : nullptr);
    double eA = 0.;
    double sc = __builtin_nan("");
    bool acc;
    if (!a.has_pred && s == 0) {
      acc = true;                                  // s = None on step 1
      if (!simple) eA = lin ? lpp : (FAST ? exp_logp_fast(lpp, a.log_npi)
                                          : exp_logp(lpp, a.log_npi));
    } else if (simple) {
      // the ratio form's decision through the filter (see mh_pair_kernel);
      // a constant tuple tran scales both log-probs by q~ (App. A-1)
      const double bA = lpp * a.acc_beta, bB = lp * a.acc_beta;
      const Decision dc = lead_bits == kStepLead ? accept_filter_lead<kStepLead>(bA, bB, lead, lin)
                        : lead_bits == 22 ? accept_filter_lead<22>(bA, bB, lead, lin)
                                          : accept_filter(bA, bB, tw0, lin);
      acc = dc.acc;
      if (__ballot(dc.need)) {   // wave-uniform, rare
        if (dc.need) {
          if (lead_bits) {   // t's remaining bits
            const u32x4 w = philox4x32_10(ctr(lead_ctr, g, chain), a.seed_lo, a.seed_hi);
            tw0 = (lead << (32 - lead_bits)) | (w.x >> lead_bits);
            tw1 = w.y;
          }
          acc = ratio_accept(bA, bB, u01(tw0, tw1), lin, a.log_npi);
        }
      }
    } else {
      eA = lin ? lpp : (FAST ? exp_logp_fast(lpp, a.log_npi)
                             : exp_logp(lpp, a.log_npi));
      acc = !score<D>(a, x, xp, lp, lpp, eA, eB, sc) || (sc >= thr);
    }
    if (acc) {
#pragma unroll
      for (int k = 0; k < D; ++k) {
        x[k] = xp[k];
        if (FAST) lx[k] = lxp[k];
      }
      lp = lpp;
      eB = eA;
    }
    if (mom) {   // wave-uniform
      nacc += acc ? 1 : 0;
#pragma unroll
      for (int k = 0; k < D; ++k) {
        ms[k] += x[k];
        mq[k] += x[k] * x[k];
      }
    }
    // ---- trace (every thin-th step, wave-uniform condition) ----
    const bool rec_now = ph == 0;
    const int64_t rec = ri;
    ph = (ph + 1 == a.thin) ? 0 : ph + 1;   // next step's phase
    ri += (ph == 0) ? 1 : 0;
    if (rec_now) {
      if (rec >= 0 && rec < a.rec_cap) {
        if (active) {
#pragma unroll
          for (int k = 0; k < D; ++k) a.tx[(rec * D + k) * a.n + c] = x[k];
          a.tlp[rec * a.n + c] = lp;
          if (a.debug) {
#pragma unroll
            for (int k = 0; k < D; ++k) a.tpx[(rec * D + k) * a.n + c] = xp[k];
            a.tpp[rec * a.n + c] = lpp;
            a.ts[rec * a.n + c] = sc;
          }
        }
        const uint64_t mask = __ballot(active && acc);
        const int64_t wv = c >> 6;
        if (lane == 0 && wv < a.W) a.tacc[rec * a.W + wv] = mask;
      }
    }
  }

  if (active) {
#pragma unroll
    for (int k = 0; k < D; ++k) {
      a.x[k * a.n + c] = x[k];
      if (FAST && ((a.ufun >> k) & 1u)) a.lx[k * a.n + c] = lx[k];
    }
    a.lp[c] = lp;
    if (mom) {
#pragma unroll
      for (int k = 0; k < D; ++k) {
        a.msum[k * a.n + c] += ms[k];
        a.msq[k * a.n + c] += mq[k];
      }
      a.nacc[c] += nacc;
    }
    if (RNG == PBH_RNG_XOSHIRO) xo_store(a, 0, c, xs);
  }
}

template <int D, int RNG, int TGT, int PROP>
__global__ __launch_bounds__(kBlock) void mh_kernel(KArgs a) {
  extern __shared__ double s_obs[];
  RowDraws src;
  mh_body<D, RNG, TGT, PROP>(a, src, s_obs, true);
}

// ---------------------------------------------------------------------------
// cfg1's steady-state form (iid_full_form): the iid-Normal target (O(1)
// sufficient statistics), the spherical tuple delta, production Philox, the
// filtered ratio form, log pscale, thin 1, every record inside the trace,
// past step 1, no tfun / int / bound dims; the ufun mask UFM compile-time.
// mh_kernel's arithmetic and draws (the same joint_density, the same words),
// without its per-step wave-uniform switches: the loop is one basic block
// apart from the rare exact decision, the selects and stores take lane masks
// (padding lanes write nothing: the buffer range check), and the kernel keeps
// its uniform state in SGPRs without spilling them to VGPR lanes.  Identical
// chains (test_iid_steady_state_form_is_the_general_form).
// ---------------------------------------------------------------------------
template <int D, int UFM>
__global__ __launch_bounds__(kBlock) void mh_iid_full_kernel(KArgs a) {
  __shared__ double s_bmt[kBm64Doubles];
  const int64_t c = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const bool active = c < a.n;
  const int64_t cc = active ? c : 0;
  const int lane = threadIdx.x & 63;
  const int64_t chain = a.off + cc;
  double x[D];
#pragma unroll
  for (int k = 0; k < D; ++k) x[k] = a.x[k * a.n + cc];
  double lp = a.lp[cc];
  double plen[D];
#pragma unroll
  for (int k = 0; k < D; ++k) plen[k] = cld(a.plen, k);
  bm64_load(s_bmt, a.bm64);
  double lx[D];   // the carried logs of the ufun dims (KArgs.lx)
#pragma unroll
  for (int k = 0; k < D; ++k)
    lx[k] = ((UFM >> k) & 1) ? (a.lx_init ? ln_ufun(x[k], s_bmt) : a.lx[k * a.n + cc]) : 0.;
  __builtin_amdgcn_s_waitcnt(0);
  const double d0 = a.sdelta;
  const double beta = a.acc_beta;
  // the density's constants (the prior bounds in VGPRs: SGPR pressure)
  const int i0 = a.i0, i1 = a.i1;
  const double tw0 = cld(a.tw, 0), tw1 = cld(a.tw, 1), nobs = (double)a.tn;
  const double logC = a.norm_logC;
  const bool has_prior = a.has_prior != 0;
  const double prior_logp = a.prior_logp;
  // the prior box as closed limits (lo_closed / hi_closed: the same tests)
  double plo[D], phi[D];
#pragma unroll
  for (int k = 0; k < D; ++k) {
    plo[k] = has_prior ? in_vgpr_f64(lo_closed(cld(a.plo, k), (a.plo_incl >> k) & 1u)) : 0.;
    phi[k] = has_prior ? in_vgpr_f64(hi_closed(cld(a.phi, k), (a.phi_incl >> k) & 1u)) : 0.;
  }
  const uint32_t rowb = (uint32_t)(a.n * 8);
  // the launch's records through three loop-invariant resources spanning
  // them (iid_full_form: under kNoStore bytes), the record as the scalar
  // offset; padding lanes' voff kNoStore fails the range check
  const int64_t r0 = a.g0 - a.rec_base;
  double *const tx0 = wave_uniform(a.tx + r0 * D * a.n);
  double *const tl0 = wave_uniform(a.tlp + r0 * a.n);
  double *const ta0 = wave_uniform(reinterpret_cast<double *>(a.tacc + r0 * a.W));
  const uint32_t xspan = (uint32_t)(a.n_steps * D) * rowb;
  const uint32_t lspan = (uint32_t)a.n_steps * rowb;
  const uint32_t abytes = (uint32_t)(a.W * 8);
  const uint32_t aspan = (uint32_t)a.n_steps * abytes;
  uint32_t xoffk[D];
#pragma unroll
  for (int k = 0; k < D; ++k) xoffk[k] = active ? (uint32_t)(c * 8) + (uint32_t)k * rowb : kNoStore;
  const uint32_t xoff = active ? (uint32_t)(c * 8) : kNoStore;
  const uint32_t aoff = lane == 0 ? (uint32_t)((c >> 6) * 8) : kNoStore;
  const PhiloxKeys rk = philox_keys_v(a.seed_lo, a.seed_hi);   // SGPRs stay free
  for (int s = 0; s < a.n_steps; ++s) {
    const int64_t g = a.g0 + s;
    // ---- draws: mh_kernel's production uniform draws ----
    double r[D];
    uint32_t lead = 0;
#pragma unroll
    for (int p = 0; p < (D + 1) / 2; ++p) {
      const u32x4 w = philox4x32_10_rk(ctr(p, g, chain), rk);
      r[2 * p] = u01(w.x, w.y);
      if (2 * p + 1 < D) r[2 * p + 1] = u01(w.z, w.w);
      if (p == 0)
        lead = ((w.x & 31u) << 17) | ((w.y & 63u) << 11) |
               (D >= 2 ? (((w.z & 31u) << 6) | (w.w & 63u)) : (w.z >> 21));
    }
    // ---- proposal: the spherical tuple delta, then the ufun ----
    double dl[D], sq[D], xp[D], lxp[D];
#pragma unroll
    for (int k = 0; k < D; ++k) {
      dl[k] = -d0 + (d0 - -d0) * r[k];
      sq[k] = dl[k] * dl[k];
    }
    const double ss = np_sum_regs<D>(sq, D);
    const double rq = rsq_nr(__builtin_fmax(ss, kNearlyPosZero));
    const double sc = ss >= kNearlyPosZero ? d0 * rq : __builtin_inf();
#pragma unroll
    for (int k = 0; k < D; ++k) {
      dl[k] = (dl[k] * sc) * plen[k];
      lxp[k] = 0.;
      if (((UFM >> k) & 1) != 0) {   // folded per unrolled k
        lxp[k] = lx[k] + dl[k];
        xp[k] = exp_ufun(lxp[k], s_bmt);
      } else {
        xp[k] = x[k] + dl[k];
      }
    }
    // joint_density<D, NORM_IID, FAST> restated on the preloaded constants
    // (the same operations in the same order)
    double lpp;
    {
      double mu = 0., sg = 1., l = 0.;
      bool have = false;
#pragma unroll
      for (int k = 0; k < D; ++k) {
        if (k == i0) mu = xp[k];
        if (k == i1) sg = xp[k];
        if (k == i1 && ((UFM >> k) & 1)) { l = lxp[k]; have = true; }
      }
      const double lsg = have ? l : fast_log(sg);
      const double dm = tw0 - mu;
      const double ssd = __builtin_fma(nobs * dm, dm, tw1);
      const double s2 = sg * sg;
      double ri = __builtin_amdgcn_rcp(s2);
      ri = __builtin_fma(__builtin_fma(-s2, ri, 1.0), ri, ri);
      ri = __builtin_fma(__builtin_fma(-s2, ri, 1.0), ri, ri);
      double out = -0.5 * ssd * ri - nobs * (logC + lsg);
      if (has_prior) {   // wave-uniform
        // (x > lo) or (inclusive and x == lo): the reference's comparison
        uint64_t in = ~0ull;
#pragma unroll
        for (int k = 0; k < D; ++k) in &= __ballot(xp[k] >= plo[k]) & __ballot(xp[k] <= phi[k]);
        out = sel_f64(in, kNearlyNegInf, prior_logp) + out;
      }
      lpp = out;
    }
    // ---- the filtered ratio form of (beta lp', beta lp) ----
    const double bA = lpp * beta, bB = lp * beta;
    const DecisionMask dm = accept_filter_lead_mask<22>(bA, bB, lead, false);
    uint64_t accm = dm.acc;
    const uint64_t needm = dm.need & __ballot(true);
    if (needm) {   // wave-uniform, rare
      bool ex = false;
      if (__builtin_amdgcn_inverse_ballot_w64(needm)) {
        const u32x4 w = philox4x32_10(ctr(0xFFFFu, g, chain), a.seed_lo, a.seed_hi);
        ex = ratio_accept(bA, bB, u01((lead << 10) | (w.x >> 22), w.y), false, a.log_npi);
      }
      accm = (accm & ~needm) | (__ballot(ex) & needm);
    }
#pragma unroll
    for (int k = 0; k < D; ++k) {
      x[k] = sel_f64(accm, x[k], xp[k]);
      if ((UFM >> k) & 1) lx[k] = sel_f64(accm, lx[k], lxp[k]);
    }
    lp = sel_f64(accm, lp, lpp);
    // ---- trace: record g - rec_base = r0 + s ----
#pragma unroll
    for (int k = 0; k < D; ++k) st_buf_ns(tx0, xspan, xoffk[k], (uint32_t)s * (D * rowb), x[k]);
    st_buf_ns(tl0, lspan, xoff, (uint32_t)s * rowb, lp);
    const uint64_t am = accm & __ballot(active);
    st_buf_ns(ta0, aspan, aoff, (uint32_t)s * abytes, __builtin_bit_cast(double, am));
  }
  if (active) {
#pragma unroll
    for (int k = 0; k < D; ++k) {
      a.x[k * a.n + c] = x[k];
      if ((UFM >> k) & 1) a.lx[k * a.n + c] = lx[k];
    }
    a.lp[c] = lp;
  }
}

// ---------------------------------------------------------------------------
// Lane-pair MH kernel for the sum-of-terms diagonal Gaussian with the
// callable Gaussian delta (cfg2).  One chain per LANE PAIR (l, l + 32): lane
// half h owns dims [h*H, h*H + H), H = D/2, so 65 536 chains fill 2 048
// wavefronts = 2 per SIMD (one wave alone issues at most one VALU per ~6
// cycles, tools/ubench/isa_cost.hip; two interleaved waves reach the SIMD's
// rate).  Half 1 holds the threshold and makes the chain's decision; the
// accept bit returns to half 0 through a ballot (SALU mask ops, no VALU).
//
// Acceptance (all modes) is the reference's ratio form, sp_utils.py:40-64 +
// pscales.py:56-65,219-236: s = min(1, exp_logp(lp') / max(tiny,
// exp_logp(lp))), accept iff s >= t.  REPLAY evaluates it verbatim every
// step.  The production modes evaluate the SAME decision through a filter:
// e = 2^(fp32(log2e (lp' - lp))) on the hardware v_exp_f32 is within 2.7e-6
// relative of s whenever |lp|, |lp'| <= 700 (no exp clamp or underflow in
// the ratio form); t is known to 2^-24 from its leading word.  If t lies
// outside [e (1 - 4e-6) - 2^-24, e (1 + 4e-6)] the decision is certain;
// otherwise (about 1e-5 of chain-steps, and whenever the range test fails)
// the lane evaluates the ratio form exactly with the libm-accurate exp and
// an IEEE division, under a wave-uniform branch.  Decisions are therefore
// those of the fp64 ratio form, at ~8 VALU instead of ~30.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t swap_u32(uint32_t v, bool hi) {
  const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
  return hi ? r[0] : r[1];
}

__device__ __forceinline__ double swap_f64(double v, bool hi) {
  const uint64_t u = __builtin_bit_cast(uint64_t, v);
  const uint64_t lo = swap_u32((uint32_t)u, hi);
  const uint64_t up = swap_u32((uint32_t)(u >> 32), hi);
  return __builtin_bit_cast(double, lo | (up << 32));
}

// v_permlane32_swap with both operands = v: lo = the value of lane l & 31,
// hi = the value of lane l | 32, in every lane.
__device__ __forceinline__ void halves_f64(double v, double &lo, double &hi) {
  const uint64_t u = __builtin_bit_cast(uint64_t, v);
  const auto a = __builtin_amdgcn_permlane32_swap((uint32_t)u, (uint32_t)u, false, false);
  const auto b = __builtin_amdgcn_permlane32_swap((uint32_t)(u >> 32), (uint32_t)(u >> 32), false, false);
  lo = __builtin_bit_cast(double, (uint64_t)a[0] | ((uint64_t)b[0] << 32));
  hi = __builtin_bit_cast(double, (uint64_t)a[1] | ((uint64_t)b[1] << 32));
}

// v_permlane16_swap with both operands = v: ev / od = the value of this
// lane's position in the even / odd 16-lane row of its row pair.
__device__ __forceinline__ void rowpair_f64(double v, double &ev, double &od) {
  const uint64_t u = __builtin_bit_cast(uint64_t, v);
  const auto a = __builtin_amdgcn_permlane16_swap((uint32_t)u, (uint32_t)u, false, false);
  const auto b = __builtin_amdgcn_permlane16_swap((uint32_t)(u >> 32), (uint32_t)(u >> 32), false, false);
  ev = __builtin_bit_cast(double, (uint64_t)a[0] | ((uint64_t)b[0] << 32));
  od = __builtin_bit_cast(double, (uint64_t)a[1] | ((uint64_t)b[1] << 32));
}

// ---------------------------------------------------------------------------
// cfg1's steady-state form on lane PAIRS (mh_iid_pair_kernel, the default
// for iid_full_form).  One lane per chain leaves 65 536 chains at one
// wavefront per SIMD, and a lone wavefront issues at most one instruction
// per ~6 cycles: the step is issue- and latency-bound at half the SIMD's
// rate.  Here chain c sits in both lanes l and l + 32 of a wavefront of 32
// chains (2 048 wavefronts = 2 per SIMD).  The draws and the spherical delta
// depend on no state, so they are split: for the step pair (2P, 2P + 1)
// half h forms step 2P + h's Philox block, its uniforms, its 22-bit
// threshold lead and its scaled delta (the sphere's rsq included), and two
// v_permlane32_swap exchanges per double give both halves both steps'.
// Both halves then run the state update (ufun, density, filter, selects) on
// identical values, so every lane holds the chain's state.  The log of a
// ufun dim of the state is chain state (KArgs.lx, as in every production
// kernel): the accepted proposal's lx + delta.  Half 0 stores dim 0 and
// the lp row, half 1 dim 1 (D = 2: one store instruction for both dims), and
// each wavefront writes its 32-bit half of the record's 64-bit accept word.
// The draws and arithmetic are mh_iid_full_kernel's: identical chains
// (test_iid_pair_form_is_the_one_lane_form).
// ---------------------------------------------------------------------------
template <int D, int UFM>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(2)))
void mh_iid_pair_kernel(KArgs a) {
  static_assert(D >= 1 && D <= 2, "iid pair kernel: d <= 2");
  __shared__ double s_bmt[kBm64Doubles];
  const int64_t gt = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const int lane = threadIdx.x & 63;
  const int h = lane >> 5;
  const int64_t wave = gt >> 6;
  const int64_t c = wave * 32 + (lane & 31);
  const bool active = c < a.n;
  const int64_t cc = active ? c : 0;
  const int64_t chain = a.off + cc;
  double x[D];
#pragma unroll
  for (int k = 0; k < D; ++k) x[k] = a.x[k * a.n + cc];
  double lp = a.lp[cc];
  double plen[D];
#pragma unroll
  for (int k = 0; k < D; ++k) plen[k] = cld(a.plen, k);
  bm64_load(s_bmt, a.bm64);
  __builtin_amdgcn_s_waitcnt(0);
  const double d0 = a.sdelta;
  const double beta = a.acc_beta;
  const int i0 = a.i0, i1 = a.i1;
  const double tw0 = cld(a.tw, 0), tw1 = cld(a.tw, 1), nobs = (double)a.tn;
  const double logC = a.norm_logC;
  const bool has_prior = a.has_prior != 0;
  const double prior_logp = a.prior_logp;
  // the prior box as closed limits (lo_closed / hi_closed: the same tests)
  double plo[D], phi[D];
#pragma unroll
  for (int k = 0; k < D; ++k) {
    plo[k] = has_prior ? in_vgpr_f64(lo_closed(cld(a.plo, k), (a.plo_incl >> k) & 1u)) : 0.;
    phi[k] = has_prior ? in_vgpr_f64(hi_closed(cld(a.phi, k), (a.phi_incl >> k) & 1u)) : 0.;
  }
  double lx[D];   // ln x of the ufun dims of the state
#pragma unroll
  for (int k = 0; k < D; ++k)
    lx[k] = ((UFM >> k) & 1) ? (a.lx_init ? ln_ufun(x[k], s_bmt) : a.lx[k * a.n + cc]) : 0.;
  const uint32_t rowb = (uint32_t)(a.n * 8);
  // stores: half 0 dim 0 + lp, half 1 dim 1 (a D = 1 chain: half 0 only)
  const uint32_t xoff = active && (D == 2 || h == 0) ? (uint32_t)(h * a.n * 8 + c * 8) : kNoStore;
  const uint32_t loff = active && h == 0 ? (uint32_t)(c * 8) : kNoStore;
  const uint64_t hmask = 0xFFFFFFFF00000000ull;   // the lanes of half 1
  // the accept word: lane 0 writes this wavefront's 32 bits of chains
  // [64 w, 64 w + 64): the low or the high half of word w = c >> 6
  // (the last wavefront of an odd count also zeroes the high half: lane 1)
  const bool tail = (wave & 1) == 0 && 32 * (wave + 1) >= a.n;
  const uint32_t aoff = lane == 0 ? (uint32_t)(wave * 4)
                      : lane == 1 && tail ? (uint32_t)(wave * 4 + 4) : kNoStore;
  const uint32_t amsk = lane == 1 ? 0u : ~0u;
  const uint32_t abytes = (uint32_t)(a.W * 8);
  const PhiloxKeys rk = philox_keys_v(a.seed_lo, a.seed_hi);
  const int64_t gend = a.g0 + a.n_steps;
  const uint64_t actm = __ballot(active) & 0xFFFFFFFFull;
  for (int64_t P = a.g0 >> 1; 2 * P < gend; ++P) {
    // ---- this half's step of the pair: draws and the scaled delta ----
    const int64_t gh = 2 * P + h;
    double dl[D];
    uint32_t lead;
    {
      const u32x4 w = philox4x32_10_rk(ctr(0, gh, chain), rk);
      double r[D];
      r[0] = u01(w.x, w.y);
      if (D >= 2) r[D - 1] = u01(w.z, w.w);
      lead = ((w.x & 31u) << 17) | ((w.y & 63u) << 11) |
             (D >= 2 ? (((w.z & 31u) << 6) | (w.w & 63u)) : (w.z >> 21));
      double sq[D];
#pragma unroll
      for (int k = 0; k < D; ++k) {
        dl[k] = -d0 + (d0 - -d0) * r[k];
        sq[k] = dl[k] * dl[k];
      }
      const double ss = np_sum_regs<D>(sq, D);
      const double rq = rsq_nr(__builtin_fmax(ss, kNearlyPosZero));
      const double sc = ss >= kNearlyPosZero ? d0 * rq : __builtin_inf();
#pragma unroll
      for (int k = 0; k < D; ++k) dl[k] = (dl[k] * sc) * plen[k];
    }
    double dls[2][D];
    uint32_t leads[2];
#pragma unroll
    for (int k = 0; k < D; ++k) halves_f64(dl[k], dls[0][k], dls[1][k]);
    {
      const auto l2 = __builtin_amdgcn_permlane32_swap(lead, lead, false, false);
      leads[0] = l2[0];
      leads[1] = l2[1];
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int64_t g = 2 * P + j;
      if (g < a.g0 || g >= gend) continue;   // wave-uniform: a launch's ends
      double xp[D], lxp[D];
#pragma unroll
      for (int k = 0; k < D; ++k) {
        lxp[k] = 0.;
        if (((UFM >> k) & 1) != 0) {
          lxp[k] = lx[k] + dls[j][k];
          xp[k] = exp_ufun(lxp[k], s_bmt);
        } else {
          xp[k] = x[k] + dls[j][k];
        }
      }
      // the proposal's ln x' (the next state's, if accepted): beside the
      // density and the decision
      // joint_density<D, NORM_IID, FAST> (mh_iid_full_kernel's operations)
      double lpp;
      {
        double mu = 0., sg = 1., l = 0.;
        bool have = false;
#pragma unroll
        for (int k = 0; k < D; ++k) {
          if (k == i0) mu = xp[k];
          if (k == i1) sg = xp[k];
          if (k == i1 && ((UFM >> k) & 1)) { l = lxp[k]; have = true; }
        }
        const double lsg = have ? l : fast_log(sg);
        const double dm = tw0 - mu;
        const double ssd = __builtin_fma(nobs * dm, dm, tw1);
        const double s2 = sg * sg;
        double ri = __builtin_amdgcn_rcp(s2);
        ri = __builtin_fma(__builtin_fma(-s2, ri, 1.0), ri, ri);
        ri = __builtin_fma(__builtin_fma(-s2, ri, 1.0), ri, ri);
        double out = -0.5 * ssd * ri - nobs * (logC + lsg);
        if (has_prior) {
          uint64_t in = ~0ull;
#pragma unroll
          for (int k = 0; k < D; ++k) in &= __ballot(xp[k] >= plo[k]) & __ballot(xp[k] <= phi[k]);
          out = sel_f64(in, kNearlyNegInf, prior_logp) + out;
        }
        lpp = out;
      }
      const double bA = lpp * beta, bB = lp * beta;
      const DecisionMask dm = accept_filter_lead_mask<22>(bA, bB, leads[j], false);
      uint64_t accm = dm.acc;
      const uint64_t needm = dm.need & __ballot(true);
      if (needm) {   // wave-uniform, rare: both halves of a chain agree
        bool ex = false;
        if (__builtin_amdgcn_inverse_ballot_w64(needm)) {
          const u32x4 w = philox4x32_10(ctr(0xFFFFu, g, chain), a.seed_lo, a.seed_hi);
          ex = ratio_accept(bA, bB, u01((leads[j] << 10) | (w.x >> 22), w.y), false, a.log_npi);
        }
        accm = (accm & ~needm) | (__ballot(ex) & needm);
      }
#pragma unroll
      for (int k = 0; k < D; ++k) {
        x[k] = sel_f64(accm, x[k], xp[k]);
        if ((UFM >> k) & 1) lx[k] = sel_f64(accm, lx[k], lxp[k]);
      }
      lp = sel_f64(accm, lp, lpp);
      // ---- trace: record g - rec_base ----
      const int64_t rec = g - a.rec_base;
      double *row = a.tx + rec * D * a.n;   // wave-uniform
      st_buf_n(row, (uint32_t)D * rowb, xoff, D == 2 ? sel_f64(hmask, x[0], x[D - 1]) : x[0]);
      st_buf_n(a.tlp + rec * a.n, rowb, loff, lp);
      st_buf32_n(reinterpret_cast<uint32_t *>(a.tacc + rec * a.W), abytes, aoff,
                 (uint32_t)(accm & actm) & amsk);
    }
  }
  if (active && h == 0) {
#pragma unroll
    for (int k = 0; k < D; ++k) {
      a.x[k * a.n + c] = x[k];
      if ((UFM >> k) & 1) a.lx[k * a.n + c] = lx[k];
    }
    a.lp[c] = lp;
  }
}

template <int L>
__device__ __forceinline__ double part_sum(double v) {
  // sum of v over the L lanes of a group, identical (same order) in each
  if constexpr (L == 1) {
    return v;
  } else if constexpr (L == 2) {
    double lo, hi;
    halves_f64(v, lo, hi);
    return lo + hi;
  } else {
    double ev, od, lo, hi;
    rowpair_f64(v, ev, od);
    halves_f64(ev + od, lo, hi);
    return lo + hi;
  }
}

template <int L, int Q>
__device__ __forceinline__ double part_bcast(double v) {
  // the value of part Q's lane of the group, in every lane of it
  if constexpr (L == 1) {
    return v;
  } else if constexpr (L == 2) {
    double lo, hi;
    halves_f64(v, lo, hi);
    return Q ? hi : lo;
  } else {
    double ev, od, lo, hi;
    rowpair_f64(v, ev, od);
    halves_f64((Q & 1) ? od : ev, lo, hi);
    return (Q >> 1) ? hi : lo;
  }
}

template <int L>
__device__ __forceinline__ double part_max(double v) {
  // maximum of v over the L lanes of a group (fmax: NaN-ignoring)
  if constexpr (L == 1) {
    return v;
  } else if constexpr (L == 2) {
    double lo, hi;
    halves_f64(v, lo, hi);
    return __builtin_fmax(lo, hi);
  } else {
    double ev, od, lo, hi;
    rowpair_f64(v, ev, od);
    halves_f64(__builtin_fmax(ev, od), lo, hi);
    return __builtin_fmax(lo, hi);
  }
}



// Production draws of a PAIR of steps (2P, 2P + 1) for one lane half: H
// normals per step.  PHILOX: the words of Philox blocks q < NB (counter
// q + 16 h) in order; bm96 fp64 Box-Muller pair p takes words 3p .. 3p + 2
// (normals 0..H-1 feed step A, H..2H-1 step B) and word 3H holds the two
// steps' 16-bit threshold leads: 3H + 1 words, so at H = 5 (cfg2) the 10
// normals and both leads of the step pair fill exactly 4 blocks.
// PHILOX_FP32 (comparison mode): the round-1 fp32 draws, NP = H / 2 blocks
// of two fp32 pairs plus one block holding the odd normals and 14-bit leads.
template <int H, int RNG>
struct PairDraw {
  static constexpr bool F32 = RNG == PBH_RNG_PHILOX_FP32;
  static constexpr int LB = F32 ? ((H % 2 == 1) ? 14 : 24) : 16;

  __device__ __forceinline__ static void draw(const KArgs &a, const double *bmt,
                                              int h, int64_t P, int64_t chain,
                                              double (&ra)[H], double (&rb)[H],
                                              uint32_t &ta, uint32_t &tb) {
    if constexpr (F32) {
      constexpr int NP = H / 2;
#pragma unroll
      for (int q = 0; q < NP; ++q) {
        const u32x4 w = philox4x32_10(ctr(q + 16 * h, P, chain), a.seed_lo, a.seed_hi);
        double z0, z1, z2, z3;
        z0 = fast_normal_pair(w.x, w.z, z1);
        z2 = fast_normal_pair(w.y, w.w, z3);
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const int gp = 2 * q + e;
          const double u = e ? z2 : z0, v = e ? z3 : z1;
          if (gp < NP) { ra[2 * gp] = u; ra[2 * gp + 1] = v; }
          else { rb[2 * (gp - NP)] = u; rb[2 * (gp - NP) + 1] = v; }
        }
      }
      const u32x4 w = philox4x32_10(ctr(NP + 16 * h, P, chain), a.seed_lo, a.seed_hi);
      if constexpr (H % 2 == 1) {
        ra[H - 1] = fast_normal_single(w.x, w.y, ta);
        rb[H - 1] = fast_normal_single(w.z, w.w, tb);
      } else {
        ta = w.x >> 8;
        tb = w.y >> 8;
      }
    } else {
      constexpr int NW = 3 * H + 1, NB = (NW + 3) / 4;
      uint32_t w[4 * NB];
#pragma unroll
      for (int q = 0; q < NB; ++q) {
        const u32x4 b = philox4x32_10(ctr(q + 16 * h, P, chain), a.seed_lo, a.seed_hi);
        w[4 * q] = b.x;
        w[4 * q + 1] = b.y;
        w[4 * q + 2] = b.z;
        w[4 * q + 3] = b.w;
      }
#pragma unroll
      for (int q = 0; q < H; ++q) {
        double z0, z1;
        bm96_pair(w[3 * q], w[3 * q + 1], w[3 * q + 2], bmt, z0, z1);
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const int n = 2 * q + e;
          const double z = e ? z1 : z0;
          if (n < H) ra[n] = z;
          else rb[n - H] = z;
        }
      }
      ta = w[3 * H] >> 16;
      tb = w[3 * H] & 0xFFFFu;
    }
  }
};

// The steady-state pair kernel's rare undecided step (the lead could not
// decide): t's remaining 53 - 16 bits from a block of this step alone and
// the exact fp64 ratio form, out of line (the loop keeps neither its
// registers nor its code).
// The resident server's 16-byte command record, read and written whole with
// caches bypassed (sc0 sc1: host memory over PCIe, and the device mailbox at
// the coherence point, past the XCD's own L2).  The load waits for itself.
typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ u32x4v ld16_sys(const void *p) {
  u32x4v v;
  asm volatile("global_load_dwordx4 %0, %1, off sc0 sc1\n\ts_waitcnt vmcnt(0)"
               : "=v"(v) : "v"(p) : "memory");
  return v;
}
__device__ __forceinline__ void st16_sys(void *p, u32x4v v) {
  asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" : : "v"(p), "v"(v) : "memory");
}

__device__ __attribute__((noinline)) bool pair_exact(uint32_t seed_lo, uint32_t seed_hi,
                                                     double log_npi, int64_t g,
                                                     int64_t chain, int h,
                                                     uint32_t t0, double lpp,
                                                     double lp) {
  const u32x4 w = philox4x32_10(ctr(0x40u + 16u * h, g, chain), seed_lo, seed_hi);
  const double t = u01((t0 << 16) | (w.x >> 16), w.y);
  return ratio_accept(lpp, lp, t, false, log_npi);
}

// FULL (PHILOX only; pair_full_form): the steady-state launch -- thin 1,
// every record inside the trace, past step 1, log pscale, N a multiple of 32
// (no padding lanes).  Whole step pairs run branch-free apart from the rare
// exact decision, and the NEXT pair's Philox blocks and Box-Muller pairs are
// computed in the same basic blocks as the current pair's two dependent
// steps (software pipelining: the scheduler interleaves the independent
// integer/fp64 draw chains with each step's density -> decision -> select
// chain).  The same words and arithmetic as the general form: identical
// chains (tests/test_gpu_parity.py).
template <int D, int RNG, bool MOM, bool LOC0 = false, bool FULL = false, bool SRV = false>
__global__ __launch_bounds__(FULL ? kPairFullBlock : kBlock)
__attribute__((amdgpu_waves_per_eu(2)))
void mh_pair_kernel(KArgs a) {
  static_assert(!FULL || (RNG == PBH_RNG_PHILOX && !MOM), "FULL: production Philox");
  static_assert(!SRV || FULL, "the resident server runs the steady-state form");
  static_assert(D % 2 == 0, "lane-pair kernel needs even D");
  constexpr int H = D / 2;
  constexpr bool PHX = RNG == PBH_RNG_PHILOX || RNG == PBH_RNG_PHILOX_FP32;
  constexpr bool FAST = PHX || RNG == PBH_RNG_XOSHIRO;
  constexpr bool REPLAY = RNG == PBH_RNG_REPLAY;
  constexpr bool TAB = RNG == PBH_RNG_PHILOX || RNG == PBH_RNG_XOSHIRO;
  using PD = PairDraw<H, RNG>;
  __shared__ double s_bmt[TAB ? kBm64Doubles : 2];
  PBH_PHASE_DECL;
  PBH_PHASE(0);
  const bool lin = a.pscale == PBH_PSCALE_LIN;
  constexpr bool mom = MOM;   // running moments compiled in or out
  const int lane = threadIdx.x & 63;
  const bool hi = lane >= 32;
  const int h = hi ? 1 : 0;
  const int64_t wave =
      ((int64_t)blockIdx.x * (FULL ? (int)blockDim.x : kBlock) + threadIdx.x) >> 6;
  const int64_t c = wave * 32 + (lane & 31);
  const bool active = c < a.n;
  const int64_t cc = active ? c : 0;
  const int k0 = h * H;   // first dim of this half
  const uint64_t act_mask = __ballot(active);
  // byte offsets of this lane's trace elements inside a record (< 4 GB)
  const uint32_t boff = (uint32_t)(((int64_t)k0 * a.n + cc) * 8);
  const uint32_t bstride = (uint32_t)(a.n * 8);
  const uint32_t loff = (uint32_t)(cc * 8);

  // FULL: the LDS table's loads go first, so that the first pair's draws
  // (which need only the table) wait for them alone and run while the chain
  // state's loads below are still in flight
  Bm64Regs tabr;
  if constexpr (FULL) bm64_issue(a.bm64, tabr);

  // Per-lane model constants in VGPRs for the whole launch (the half's dims
  // differ between lanes, so these are vector values, loaded once).
  double psc[H], plc[H], ca[H], cb[H], cc2[H];
#pragma unroll
  for (int i = 0; i < H; ++i) {
    psc[i] = a.pscl[k0 + i];
    plc[i] = a.ploc[k0 + i];
    if (FAST) {
      // production density term u = x w - mu w, w = sqrt(0.5) / sigma
      cb[i] = a.tw[k0 + i];
      ca[i] = a.ta[k0 + i] * cb[i];
      cc2[i] = 0.;
    } else {
      ca[i] = a.ta[k0 + i];   // norm_logpdf loc, scale, log(scale)
      cb[i] = a.tb[k0 + i];
      cc2[i] = a.tc[k0 + i];
    }
  }

  double x[H], ms[H], mq[H];
#pragma unroll
  for (int i = 0; i < H; ++i) {
    x[i] = a.x[(k0 + i) * a.n + cc];
    ms[i] = 0.;
    mq[i] = 0.;
  }
  double lp = a.lp[cc];
  // REPLAY caches rescale(lp) (bit-identical to re-evaluating it)
  double eB = REPLAY ? (lin ? lp : exp_logp(lp, a.log_npi)) : 0.;
  int64_t nacc = 0;
  const int64_t chain = a.off + cc;
  Xo xs{0u, 0u, 0u, 0u};
  if (RNG == PBH_RNG_XOSHIRO) xs = xo_load(a, h, cc);

  // the LDS tables after the state's loads: all of them in flight at once
  if constexpr (FULL) bm64_commit(s_bmt, tabr);
  else if constexpr (TAB) bm64_load(s_bmt, a.bm64);

  // record phase / index of the trace, advanced per step (no 64-bit
  // division in the loop): step g records iff (g + 1) % thin == 0, at
  // record (g + 1) / thin - 1 - rec_base.
  int ph = (int)((a.g0 + 1) % a.thin);
  int64_t ri = (a.g0 + 1) / a.thin - 1 - a.rec_base;
  // Drain the entry loads here: a wait for them inside the loop would also
  // wait for every trace store issued before it.  (FULL drains after the
  // first pair's draws, before its first step.)
  if constexpr (!FULL) __builtin_amdgcn_s_waitcnt(0);
  PBH_PHASE(1);

  // One chain-step.  (r, t0, t1) are this step's draws (Philox: supplied by
  // the caller, t0 = the LB-bit threshold lead).
  auto step = [&](int s, double (&r)[H], uint32_t &t0, uint32_t &t1) {
    const int64_t g = a.g0 + s;
    double thr = 0.;
    if (REPLAY) {
      const double *row = a.rep + (a.rep_row0 + s) * a.R * a.n + cc;
#pragma unroll
      for (int i = 0; i < H; ++i) r[i] = row[(k0 + i) * a.n];
      thr = row[(int64_t)D * a.n];   // used by half 1
    } else if (RNG == PBH_RNG_XOSHIRO) {
      // this half's stream: three words per fp64 normal pair, then the
      // threshold (drawn by both halves so each stream advances the same)
#pragma unroll
      for (int p = 0; p < (H + 1) / 2; ++p) {
        const uint32_t w0 = xo_next(xs), w1 = xo_next(xs), w2 = xo_next(xs);
        double z0, z1;
        bm96_pair(w0, w1, w2, s_bmt, z0, z1);
        r[2 * p] = z0;
        if (2 * p + 1 < H) r[2 * p + 1] = z1;
      }
      t0 = xo_next(xs);
      t1 = xo_next(xs);
    } else if (PHX) {
      // drawn by the caller, a step pair ahead (PairDraw)
    } else {   // PHILOX_F64: libm fp64 Box-Muller
#pragma unroll
      for (int p = 0; p < (H + 1) / 2; ++p) {
        double z0, z1;
        box_muller(philox4x32_10(ctr(p + 16 * h, g, chain), a.seed_lo, a.seed_hi), z0, z1);
        r[2 * p] = z0;
        if (2 * p + 1 < H) r[2 * p + 1] = z1;
      }
      const u32x4 w = philox4x32_10(ctr(0xFFFFu, g, chain), a.seed_lo, a.seed_hi);
      t0 = w.x;
      t1 = w.y;
    }
    // proposal of this half's dims (scipy rvs: z * scale + loc)
    // (LOC0, production: every loc is 0, x' = fma(z, scale, x))
    double xp[H];
#pragma unroll
    for (int i = 0; i < H; ++i)
      xp[i] = LOC0 ? __builtin_fma(r[i], psc[i], x[i])
            : FAST ? x[i] + __builtin_fma(r[i], psc[i], plc[i])
                   : x[i] + (r[i] * psc[i] + plc[i]);
    // density: Python sum from 0, dims in order, split across the pair
    double lpp;
    if (FAST) {
      // production: -sum (x w - mu w)^2 - ksum; order of the sum is free
      double p0 = 0., p1 = 0.;
#pragma unroll
      for (int i = 0; i < H; ++i) {
        const double u = __builtin_fma(xp[i], cb[i], -ca[i]);
        if (i & 1) p1 = __builtin_fma(u, u, p1);
        else p0 = __builtin_fma(u, u, p0);
      }
      double lo, up;
      halves_f64(p0 + p1, lo, up);   // the two halves' sums, in every lane
      lpp = (-(lo + up)) - a.ksum;   // = -((lo + up) + ksum) exactly, one op
    } else {
      double tm[H];
#pragma unroll
      for (int i = 0; i < H; ++i)
        tm[i] = norm_logpdf(xp[i], ca[i], cb[i], cc2[i], a.norm_logC);
      double s0 = 0.0;
#pragma unroll
      for (int i = 0; i < H; ++i) s0 = s0 + (hi ? 0.0 : tm[i]);
      lpp = swap_f64(s0, hi);   // half 1 gets half 0's sum
#pragma unroll
      for (int i = 0; i < H; ++i) lpp = lpp + tm[i];
    }
    // half 1 holds the full density and the threshold: its decision is the
    // chain's (computed branch-free in both halves; half 0's is discarded)
    const bool first = !a.has_pred && s == 0;   // s = None on step 1
    constexpr uint64_t kHi = 0xFFFFFFFF00000000ull;
    uint64_t accm;   // lane mask of the decisions (half 1's bits count)
    double eA = 0.;
    if (REPLAY) {
      eA = lin ? lpp : exp_logp(lpp, a.log_npi);
      double q = eA / np_max_tiny(eB);
      q = q < 1. ? q : 1.;
      accm = __ballot(first || q >= thr);
    } else {
      // masks straight from the comparisons (no per-lane bool round trip)
      const DecisionMask dm = accept_filter_lead_mask<PHX ? PD::LB : 24>(
          lpp, lp, PHX ? t0 : t0 >> 8, lin);
      accm = first ? ~0ull : dm.acc;
      // half 1's undecided lanes (first is wave-uniform)
      const uint64_t needm = first ? 0ull : dm.need & kHi & __ballot(true);
      if (needm) {   // wave-uniform, rare
        bool ex = false;
        if (__builtin_amdgcn_inverse_ballot_w64(needm)) {
          double t;
          if (PHX) {
            // t's remaining 53 - LB bits from a block of this step alone
            const u32x4 w = philox4x32_10(ctr(0x40u + 16u * h, g, chain),
                                          a.seed_lo, a.seed_hi);
            t = u01((t0 << (32 - PD::LB)) | (w.x >> PD::LB), w.y);
          } else {
            t = u01(t0, t1);
          }
          ex = ratio_accept(lpp, lp, t, lin, a.log_npi);
        }
        accm = (accm & ~needm) | (__ballot(ex) & needm);
      }
    }
    // half 1's decision is the chain's: lanes l and l + 32 both take bit
    // l + 32 of the mask (SGPR mask ops; inverse_ballot feeds v_cndmask)
    const uint64_t mhi = accm & kHi;
    const uint64_t macc = mhi | (mhi >> 32);   // lane mask of the chain's decision
    const bool accl = __builtin_amdgcn_inverse_ballot_w64(macc);
#pragma unroll
    for (int i = 0; i < H; ++i) x[i] = sel_f64(macc, x[i], xp[i]);
    if (REPLAY) eB = sel_f64(macc, eB, eA);
    lp = sel_f64(macc, lp, lpp);
    if constexpr (mom) {
      nacc += accl ? 1 : 0;
#pragma unroll
      for (int i = 0; i < H; ++i) {
        ms[i] += x[i];
        mq[i] = __builtin_fma(x[i], x[i], mq[i]);
      }
    }
    const bool rec_now = ph == 0;
    const int64_t rec = ri;
    ph = (ph + 1 == a.thin) ? 0 : ph + 1;   // next step's phase
    ri += (ph == 0) ? 1 : 0;
    if (rec_now && rec >= 0 && rec < a.rec_cap) {
      double *row = a.tx + rec * D * a.n;   // wave-uniform
      if (active) {
#pragma unroll
        for (int i = 0; i < H; ++i) st_buf(row, boff, i * bstride, x[i]);
        if (hi) st_buf(a.tlp + rec * a.n, loff, 0, lp);
      }
      // 32 chains per wave: the upper half's ballot bits are the mask word
      if (lane == 32 && (c >> 5) < 2 * a.W)
        reinterpret_cast<uint32_t *>(a.tacc)[rec * 2 * a.W + (c >> 5)] =
            (uint32_t)((mhi & act_mask) >> 32);
    }
  };

  if constexpr (PHX) {
    // Draws come per step PAIR (2P, 2P + 1), P = absolute step / 2, so a run
    // split into launches at any step sees the same stream.  PHILOX_FP32
    // issues the next pair's blocks while the current pair's fp64 chain runs
    // (ping-pong over two draw sets); the fp64 normals hold too many live
    // registers for that at two waves per SIMD, so PHILOX draws each pair
    // just before its two steps and relies on the SIMD's other wave.
    double cA[H], cB[H];
    uint32_t ctA = 0, ctB = 0, t1 = 0;
    int s = 0;
    if constexpr (PD::F32) {
      double nA[H], nB[H];
      uint32_t ntA = 0, ntB = 0;
      PD::draw(a, s_bmt, h, a.g0 >> 1, chain, cA, cB, ctA, ctB);
      if ((a.g0 & 1) && s < a.n_steps) {   // launch starts on a pair's 2nd step
        step(s, cB, ctB, t1);
        ++s;
        if (s < a.n_steps)
          PD::draw(a, s_bmt, h, (a.g0 + s) >> 1, chain, cA, cB, ctA, ctB);
      }
      for (; s + 3 < a.n_steps; s += 4) {
        PD::draw(a, s_bmt, h, ((a.g0 + s) >> 1) + 1, chain, nA, nB, ntA, ntB);
        step(s, cA, ctA, t1);
        step(s + 1, cB, ctB, t1);
        PD::draw(a, s_bmt, h, ((a.g0 + s) >> 1) + 2, chain, cA, cB, ctA, ctB);
        step(s + 2, nA, ntA, t1);
        step(s + 3, nB, ntB, t1);
      }
      if (s + 1 < a.n_steps) {
        step(s, cA, ctA, t1);
        step(s + 1, cB, ctB, t1);
        s += 2;
        if (s < a.n_steps)
          PD::draw(a, s_bmt, h, (a.g0 + s) >> 1, chain, cA, cB, ctA, ctB);
      }
      if (s < a.n_steps) step(s, cA, ctA, t1);
    } else if constexpr (FULL) {
        // the launch's (or, SRV, the current command's) first step, step
        // count and wave-slot alternation
        int64_t g0v = a.g0;
        int32_t nsv = a.n_steps, fairv = a.fair, fair_relv = a.fair_rel;
        // ---- steady state: whole pairs (see FULL above the kernel) ----
        constexpr int NW = 3 * H + 1, NB = (NW + 3) / 4, QA = (H + 1) / 2;
        constexpr uint64_t kHi = 0xFFFFFFFF00000000ull;
        // the state's range bit (|lp| <= 700) as a lane mask, carried by the
        // selects (one compare per step instead of two)
        uint64_t inl = __ballot(__builtin_fabs(lp) <= 700.);
        // lp rows: the lower half's lanes write nothing (range check)
        const uint32_t lpoff = hi ? loff : kNoStore;
        const uint32_t lpbytes = (uint32_t)(a.n * 8);
        const uint32_t aoff = lane == 32 ? (uint32_t)((c >> 5) * 4) : kNoStore;
        const uint32_t abytes = (uint32_t)(a.W * 8);
        int64_t rec = g0v + s - a.rec_base;   // thin 1: record = step
        const PhiloxKeys rk = philox_keys_v(a.seed_lo, a.seed_hi);
        // blocks Q0 .. NB-1 of pair P (the words before block Q0 unused)
        auto philox_from = [&](int64_t P, uint32_t (&w)[4 * NB], auto Q0) {
#pragma unroll
          for (int q = 0; q < 4 * decltype(Q0)::value; ++q) w[q] = 0u;
#pragma unroll
          for (int q = decltype(Q0)::value; q < NB; ++q) {
            const u32x4 b = philox4x32_10_rk(ctr(q + 16 * h, P, chain), rk);
            w[4 * q] = b.x;
            w[4 * q + 1] = b.y;
            w[4 * q + 2] = b.z;
            w[4 * q + 3] = b.w;
          }
        };
        auto philox = [&](int64_t P, uint32_t (&w)[4 * NB]) {
#pragma unroll
          for (int q = 0; q < NB; ++q) {
            const u32x4 b = philox4x32_10_rk(ctr(q + 16 * h, P, chain), rk);
            w[4 * q] = b.x;
            w[4 * q + 1] = b.y;
            w[4 * q + 2] = b.z;
            w[4 * q + 3] = b.w;
          }
        };
        // Box-Muller pairs q0 <= q < q1 of a pair's words into the two steps'
        // normals (PairDraw's layout)
        auto normals = [&](const uint32_t (&w)[4 * NB], auto Q0, auto Q1,
                           double (&ra)[H], double (&rb)[H]) {
          constexpr int q0 = decltype(Q0)::value, q1 = decltype(Q1)::value;
#pragma unroll
          for (int q = q0; q < q1; ++q) {
            double z0, z1;
            bm96_pair(w[3 * q], w[3 * q + 1], w[3 * q + 2], s_bmt, z0, z1);
#pragma unroll
            for (int e = 0; e < 2; ++e) {
              const int n = 2 * q + e;
              const double z = e ? z1 : z0;
              if (n < H) ra[n] = z;
              else rb[n - H] = z;
            }
          }
        };
        auto step_full = [&](int si, const double (&r)[H], uint32_t t0) {
          double xp[H];
#pragma unroll
          for (int i = 0; i < H; ++i)
            xp[i] = LOC0 ? __builtin_fma(r[i], psc[i], x[i])
                         : x[i] + __builtin_fma(r[i], psc[i], plc[i]);
          double p0 = 0., p1 = 0.;
#pragma unroll
          for (int i = 0; i < H; ++i) {
            const double u = __builtin_fma(xp[i], cb[i], -ca[i]);
            if (i & 1) p1 = __builtin_fma(u, u, p1);
            else p0 = __builtin_fma(u, u, p0);
          }
          double lo, up;
          halves_f64(p0 + p1, lo, up);
          const double lpp = (-(lo + up)) - a.ksum;
          // accept_filter_lead_mask<16>, log pscale, the state's range bit
          // carried in inl
          const float eL = __builtin_amdgcn_exp2f(
              (float)__builtin_fma(lpp - lp, 1.4426950408889634, 16.0));
          const float fl = (float)t0;
          const uint64_t inp = __ballot(__builtin_fabs(lpp) <= 700.);
          const uint64_t inr = inp & inl;
          const uint64_t af = __ballot(fl <= __builtin_fmaf(eL, 0.999996f, -1.0f));
          const uint64_t rf = __ballot(fl > eL * 1.000004f);
          uint64_t accm = inr & af;
          const uint64_t needm = ~(inr & (af | rf)) & kHi;
          if (needm) {   // wave-uniform, rare
            bool ex = false;
            if (__builtin_amdgcn_inverse_ballot_w64(needm))
              ex = pair_exact(a.seed_lo, a.seed_hi, a.log_npi, g0v + si, chain, h,
                              t0, lpp, lp);
            accm = (accm & ~needm) | (__ballot(ex) & needm);
          }
          const uint64_t mhi = accm & kHi;
          const uint64_t macc = mhi | (mhi >> 32);
#pragma unroll
          for (int i = 0; i < H; ++i) x[i] = sel_f64(macc, x[i], xp[i]);
          lp = sel_f64(macc, lp, lpp);
          inl = (inl & ~macc) | (inp & macc);
          double *row = a.tx + rec * D * a.n;   // wave-uniform
#pragma unroll
          for (int i = 0; i < H; ++i) st_buf(row, boff, i * bstride, x[i]);
          st_buf_n(a.tlp + rec * a.n, lpbytes, lpoff, lp);
          st_buf32_n(reinterpret_cast<uint32_t *>(a.tacc + rec * a.W), abytes, aoff,
                     (uint32_t)(mhi >> 32));
          ++rec;
        };
        using I0 = std::integral_constant<int, 0>;
        using IA = std::integral_constant<int, QA>;
        using IH = std::integral_constant<int, H>;
        // one launch's (one command's) steps [g0v, g0v + nsv)
        auto run_block = [&]() {
          if (g0v & 1) {   // launch starts on a pair's 2nd step
            // only step B's normals: Box-Muller pairs H/2 .. H-1 and the lead
            // word, i.e. the blocks from the one holding word 3 (H / 2) on
            constexpr int QB = 3 * (H / 2) / 4;
            uint32_t w[4 * NB];
            philox_from(g0v >> 1, w, std::integral_constant<int, QB>{});
            normals(w, std::integral_constant<int, H / 2>{}, IH{}, cA, cB);
            __builtin_amdgcn_s_waitcnt(0);   // the entry loads, before the first step
            step_full(0, cB, w[3 * H] & 0xFFFFu);
            s = 1;
          }
          if (s + 1 < nsv) {
            uint32_t w[4 * NB];
            philox((g0v + s) >> 1, w);
            normals(w, I0{}, IH{}, cA, cB);
            ctA = w[3 * H] >> 16;
            ctB = w[3 * H] & 0xFFFFu;
            if (s == 0) __builtin_amdgcn_s_waitcnt(0);   // no stores in flight yet
            PBH_PHASE(2);
            const uint32_t slot = fairv ? simd_wave_slot() : 0u;
            // fair_relv: the alternation's clock starts at this wave's loop
            // entry (the waves of a launch start within ~0.4 us of each other),
            // so the hand-overs of a short launch fall at the same points of
            // every launch instead of wherever the free-running clock is
            const uint64_t tfair0 =
                fair_relv ? __builtin_amdgcn_s_memrealtime() : 0ull;
            for (; s + 3 < nsv; s += 2) {
              if (fairv) {
                const int64_t el = (int64_t)(__builtin_amdgcn_s_memrealtime() - tfair0);
                fair_prio((uint32_t)((el > 0 ? (uint64_t)el : 0ull) >> fairv) + slot);
              }
              PBH_PHASE_Q(s >> 1, nsv >> 1);
              uint32_t nw[4 * NB];
              double nA[H], nB[H];
              philox(((g0v + s) >> 1) + 1, nw);
              step_full(s, cA, ctA);
              normals(nw, I0{}, IA{}, nA, nB);
              step_full(s + 1, cB, ctB);
              normals(nw, IA{}, IH{}, nA, nB);
  #pragma unroll
              for (int i = 0; i < H; ++i) {
                cA[i] = nA[i];
                cB[i] = nB[i];
              }
              ctA = nw[3 * H] >> 16;
              ctB = nw[3 * H] & 0xFFFFu;
            }
            step_full(s, cA, ctA);
            step_full(s + 1, cB, ctB);
            s += 2;
          }
          if (s < nsv) {   // launch ends on a pair's 1st step
            uint32_t w[4 * NB];
            philox((g0v + s) >> 1, w);
            normals(w, I0{}, IA{}, cA, cB);
            if (s == 0) __builtin_amdgcn_s_waitcnt(0);   // a one-step launch
            step_full(s, cA, w[3 * H] >> 16);
          }
        };
        if constexpr (SRV) {
          // ---- resident sampling server (engine pbh_server_*): the chain
          // state stays in registers and the tables in LDS across commands.
          // Thread 0 of each workgroup polls the host command block (pinned,
          // fine-grained memory, uncached system-scope loads); the other
          // waves wait at the barrier.  After a command, every wave's stores
          // have left (vmcnt 0), and thread 0 writes the workgroup's
          // completion word with (seq, start, end) real-time stamps through
          // vector system-scope stores.  No command for srv_idle ticks (or
          // an exit command) ends the loop: the epilogue stores x and lp.
          // (wave 0 of the workgroup polls as a whole wave -- the same
          // address in every lane, one request -- and writes the same values
          // from every lane: no divergent branch around the step code, whose
          // lane masks must stay in SGPRs)
          __shared__ int64_t s_cmd[6];
          SrvCmd *const hcmd = reinterpret_cast<SrvCmd *>(a.srv_cmd);
          SrvCmd *const mail = reinterpret_cast<SrvCmd *>(a.srv_mail);
          SrvDone *const donep = reinterpret_cast<SrvDone *>(a.srv_done) + blockIdx.x;
          const bool poller = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)) == 0;
          const bool direct = (a.srv_mode & 1) != 0;
          // the one host poller (direct: none -- the host writes the mailbox)
          const bool relay = blockIdx.x == 0 && !direct;
          uint32_t seen = 0u;
          for (;;) {
            if (poller) {
              const uint64_t tw = __builtin_amdgcn_s_memrealtime();
              // workgroup 0 reads the host block, the others the device
              // mailbox: one 16-byte volatile load (caches bypassed) per poll
              const SrvCmd *src = relay ? hcmd : mail;
              uint32_t q;
              u32x4v v;
              for (;;) {
                v = ld16_sys(src);
                q = (uint32_t)__builtin_amdgcn_readfirstlane((int)v.x);
                const uint32_t chk = (uint32_t)__builtin_amdgcn_readfirstlane((int)v.w) >> 24;
                if (q != seen && chk == (q & 0xFFu)) break;   // new and whole
                if (__builtin_amdgcn_s_memrealtime() - tw > (uint64_t)a.srv_idle) {
                  q = 0u;   // idle: exit (seq 0 is never issued)
                  break;
                }
                __builtin_amdgcn_s_sleep(1);
              }
              const uint64_t tsee = __builtin_amdgcn_s_memrealtime();
              if (relay && q) st16_sys(mail, v);   // relay, whole
              const uint32_t n = (uint32_t)__builtin_amdgcn_readfirstlane((int)v.y);
              const uint64_t arg =
                  (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)v.z) |
                  ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)v.w) << 32);
              const int64_t g0 = (int64_t)(arg & 0xFFFFFFFFFFFFull);
              const uint32_t fr = (uint32_t)(arg >> 48) & 31u, frel = (uint32_t)(arg >> 53) & 1u;
              const uint32_t op = (uint32_t)(arg >> 54) & 1u;
              s_cmd[0] = q;
              s_cmd[1] = op;
              s_cmd[2] = g0;
              s_cmd[3] = n;
              s_cmd[4] = ((int64_t)frel << 32) | fr;
              s_cmd[5] = (int64_t)tsee;
            }
            __syncthreads();
            const uint32_t q = (uint32_t)__builtin_amdgcn_readfirstlane((int)s_cmd[0]);
            const uint32_t op = (uint32_t)__builtin_amdgcn_readfirstlane((int)s_cmd[1]);
            if (q == 0u || op == kSrvExit) {
              if (poller && q != 0u)
                __hip_atomic_store(&donep->seq, q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
              break;
            }
            const int64_t c2 = s_cmd[2], c4 = s_cmd[4];
            g0v = (int64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)c2) |
                  ((int64_t)__builtin_amdgcn_readfirstlane((int)(c2 >> 32)) << 32);
            nsv = __builtin_amdgcn_readfirstlane((int)s_cmd[3]);
            fairv = __builtin_amdgcn_readfirstlane((int)(uint32_t)c4);
            fair_relv = __builtin_amdgcn_readfirstlane((int)(c4 >> 32));
            const uint64_t tseen = (uint64_t)s_cmd[5];
            // (the poller writes s_cmd again only after the command's closing
            // barrier: every wave has read it by then)
            s = 0;
            rec = g0v - a.rec_base;
            run_block();
            __builtin_amdgcn_s_waitcnt(0);   // this wave's stores have left
            __syncthreads();
            if (poller) {
              __hip_atomic_store(&donep->t0, tseen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
              __hip_atomic_store(&donep->t1, (uint64_t)__builtin_amdgcn_s_memrealtime(),
                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
              __builtin_amdgcn_s_waitcnt(0);   // the stamps before the seq
              __hip_atomic_store(&donep->seq, q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
            seen = q;
          }
        } else {
          run_block();
        }
        PBH_PHASE(3);
    } else {
      if (a.g0 & 1) {   // launch starts on a pair's 2nd step
        PD::draw(a, s_bmt, h, a.g0 >> 1, chain, cA, cB, ctA, ctB);
        step(s, cB, ctB, t1);
        ++s;
      }
      for (; s + 1 < a.n_steps; s += 2) {
        PD::draw(a, s_bmt, h, (a.g0 + s) >> 1, chain, cA, cB, ctA, ctB);
        step(s, cA, ctA, t1);
        step(s + 1, cB, ctB, t1);
      }
      if (s < a.n_steps) {
        PD::draw(a, s_bmt, h, (a.g0 + s) >> 1, chain, cA, cB, ctA, ctB);
        step(s, cA, ctA, t1);
      }
    }
  } else {
    double r[H];
    uint32_t t0 = 0, t1 = 0;
    for (int s = 0; s < a.n_steps; ++s) step(s, r, t0, t1);
  }

  if (active) {
#pragma unroll
    for (int i = 0; i < H; ++i) a.x[(k0 + i) * a.n + c] = x[i];
    if (hi) a.lp[c] = lp;
    if constexpr (mom) {
#pragma unroll
      for (int i = 0; i < H; ++i) {
        a.msum[(k0 + i) * a.n + c] += ms[i];
        a.msq[(k0 + i) * a.n + c] += mq[i];
      }
      if (hi) a.nacc[c] += nacc;
    }
    if (RNG == PBH_RNG_XOSHIRO) xo_store(a, h, c, xs);
  }
  if constexpr (FULL) {   // probe build only (a.rep is the phase buffer)
    PBH_PHASE(4);
    PBH_PHASE_STORE(a.rep, wave, lane);
  }
}
// ---------------------------------------------------------------------------
// Multi-lane MH kernel for the Gaussian-mixture target with the callable
// Gaussian delta (cfg5, production RNG).  At d = 2 a chain per lane leaves
// SIMDs idle at 32 768 chains; here one chain is a group of L lanes (rows of
// 64 / L lanes) holding the whole state.
//  * Draws: steps come in aligned groups of L (absolute step / L), and part
//    p of a group draws step L G + p alone (step_draws: bm96 fp64 normals +
//    a 24-bit threshold lead); one all-gather over the
//    group's lanes (v_permlane16/32_swap) hands every lane the L steps'
//    draws, so each lane runs 1/L of the Philox and Box-Muller work.
//  * Density: the K components are dealt over the parts (k = p + L kk);
//    each part forms its partial log-sum-exp and the group combines them,
//    lse = M + log S, S = sum_p sum_k exp(v_k - M), M = max_k v_k.
//  * Acceptance never waits for that log: the state's density is carried as
//    (M, S) besides lp = M + log S, and the filter's ratio is
//    exp(M' - M) S' / S -- the log of S' (the recorded v.prob) runs off the
//    step-to-step dependency chain.  Undecided steps (about 1e-4) evaluate the
//    exact ratio form of (lp', lp) under a wave-uniform branch, as everywhere.
// ---------------------------------------------------------------------------
template <int L>
__device__ __forceinline__ void gather_f64(double v, double (&all)[L]) {
  if constexpr (L == 2) {
    halves_f64(v, all[0], all[1]);
  } else {
    static_assert(L == 4, "lanes per chain: 2 or 4");
    double ev, od;
    rowpair_f64(v, ev, od);
    halves_f64(ev, all[0], all[2]);
    halves_f64(od, all[1], all[3]);
  }
}

template <int L>
__device__ __forceinline__ void gather_u32(uint32_t v, uint32_t (&all)[L]) {
  if constexpr (L == 2) {
    const auto a = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    all[0] = a[0];
    all[1] = a[1];
  } else {
    const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    const auto e = __builtin_amdgcn_permlane32_swap(r[0], r[0], false, false);
    const auto o = __builtin_amdgcn_permlane32_swap(r[1], r[1], false, false);
    all[0] = e[0];
    all[2] = e[1];
    all[1] = o[0];
    all[3] = o[1];
  }
}

// filter of the ratio form for a state carried as (M, S): e = exp(M' - M)
// S' / S in fp32 (v_exp_f32 1 ulp, argument rounding 4.2e-8 |y| as in
// accept_filter_lead, S' rcp(S) 3 roundings of 2^-24: within 3e-6 of the
// ratio wherever |M|, |M'| <= 698, K <= 7)
template <int LB>
__device__ __forceinline__ Decision accept_filter_ms(double Mp, double Sp,
                                                     double M, double S,
                                                     uint32_t lead) {
  constexpr float w = 1.0f / (float)(1u << LB);
  const float e = __builtin_amdgcn_exp2f((float)((Mp - M) * 1.4426950408889634)) *
                  ((float)Sp * __builtin_amdgcn_rcpf((float)S));
  const float tlo = (float)lead * w;
  const float thi = tlo + w;
  // bitwise & / |: evaluated branch-free (no exec-masked region around e)
  const bool inr = (__builtin_fabs(Mp) <= 698.) & (__builtin_fabs(M) <= 698.);
  const bool af = thi <= e * 0.999996f;
  const bool rf = tlo > e * 1.000004f;
  return Decision{(bool)(inr & af), !(inr & (af | rf))};
}

template <int D, int K, int L>
__global__ __launch_bounds__(kBlock) void mh_gmm_lanes_kernel(KArgs a) {
  constexpr int KL = (K + L - 1) / L;    // component slots per part
  constexpr int CW = 64 / L;             // chains per wavefront
  constexpr int LB = kStepLead;          // threshold lead bits (step_draws)
  constexpr double kNegInf = -__builtin_inf();
  __shared__ double s_bmt[kBm64Doubles];
  bm64_load(s_bmt, a.bm64);
  const bool mom = a.moments != 0;
  const int lane = threadIdx.x & 63;
  const int p = lane / CW;
  const int64_t wave = ((int64_t)blockIdx.x * kBlock + threadIdx.x) >> 6;
  const int64_t c = wave * CW + (lane % CW);
  const bool active = c < a.n;
  const int64_t cc = active ? c : 0;
  const uint64_t act_mask = __ballot(active);
  const int64_t chain = a.off + cc;

  // this part's components k = p + L kk (a missing one contributes 0)
  double cw[KL], c0[KL], cmu[KL][D];
  bool any = false;
#pragma unroll
  for (int kk = 0; kk < KL; ++kk) {
    const int k = p + L * kk;
    const bool ok = k < K;
    any = any || ok;
    cw[kk] = ok ? a.tw[k] : 0.;
    c0[kk] = ok ? a.tw[K + k] : kNegInf;
#pragma unroll
    for (int i = 0; i < D; ++i) cmu[kk][i] = ok ? a.tb[k * D + i] : 0.;
  }
  double psc[D], plc[D];
#pragma unroll
  for (int i = 0; i < D; ++i) {
    psc[i] = cld(a.pscl, i);
    plc[i] = cld(a.ploc, i);
  }
  double x[D], ms[D], mq[D];
#pragma unroll
  for (int i = 0; i < D; ++i) {
    x[i] = a.x[i * a.n + cc];
    ms[i] = 0.;
    mq[i] = 0.;
  }
  double lp = a.lp[cc];
  double lm = lp, ls = 1.0;   // the state's density as (M, S): lp = M + log S
  int64_t nacc = 0;
  int ph = (int)((a.g0 + 1) % a.thin);
  int64_t ri = (a.g0 + 1) / a.thin - 1 - a.rec_base;
  const uint32_t boff = (uint32_t)(cc * 8), bstride = (uint32_t)(a.n * 8);
  __builtin_amdgcn_s_waitcnt(0);   // entry loads drained before the loop

  const int64_t gend = a.g0 + a.n_steps;
  for (int64_t G = a.g0 / L; G * L < gend; ++G) {
    // ---- this part's draws for step L G + p, then the group's all-gather
    double rown[D];
    const uint32_t lown = step_draws<D>(a, G * L + p, chain, s_bmt, rown);
    double rall[D][L];
    uint32_t lall[L];
#pragma unroll
    for (int i = 0; i < D; ++i) gather_f64<L>(rown[i], rall[i]);
    gather_u32<L>(lown, lall);
#pragma unroll
    for (int j = 0; j < L; ++j) {
      const int64_t g = G * L + j;
      if (g < a.g0 || g >= gend) continue;   // wave-uniform
      const int s = (int)(g - a.g0);
      double xp[D];
#pragma unroll
      for (int i = 0; i < D; ++i) xp[i] = x[i] + __builtin_fma(rall[i][j], psc[i], plc[i]);
      // ---- partial log-sum-exp over this part's components, then the group's
      double v[KL];
#pragma unroll
      for (int kk = 0; kk < KL; ++kk) {
        double acc = c0[kk];
#pragma unroll
        for (int i = 0; i < D; ++i) {
          const double u = (xp[i] - cmu[kk][i]) * cw[kk];
          acc = __builtin_fma(-u, u, acc);
        }
        v[kk] = acc;
      }
      double m = v[0];
#pragma unroll
      for (int kk = 1; kk < KL; ++kk) m = __builtin_fmax(m, v[kk]);
      const double M = part_max<L>(m);
      double e = 0.;
#pragma unroll
      for (int kk = 0; kk < KL; ++kk) e += exp_tab(v[kk] - M, s_bmt);
      const double S = part_sum<L>(any ? e : 0.);   // in [1, K]
      // the recorded v.prob: the table log of S in [1, K] (off the
      // acceptance's dependency chain)
      const double lpp = M + ln_tab(S, s_bmt);
      // ---- acceptance (identical in every lane of the group) ----
      bool acc;
      if (!a.has_pred && s == 0) {
        acc = true;                                  // s = None on step 1
      } else if (a.acc_beta == 1.0) {
        const Decision dc = accept_filter_ms<LB>(M, S, lm, ls, lall[j]);
        acc = dc.acc;
        if (__ballot(dc.need)) {   // wave-uniform, rare
          if (dc.need) {
            const u32x4 w = philox4x32_10(ctr(0x40u, g, chain), a.seed_lo, a.seed_hi);
            const double t = u01((lall[j] << (32 - LB)) | (w.x >> LB), w.y);
            acc = ratio_accept(lpp, lp, t, false, a.log_npi);
          }
        }
      } else {
        // e-tempered ratio form (App. A-1): the filter on (beta lp', beta lp)
        const double bA = lpp * a.acc_beta, bB = lp * a.acc_beta;
        const Decision dc = accept_filter_lead<LB>(bA, bB, lall[j], false);
        acc = dc.acc;
        if (__ballot(dc.need)) {
          if (dc.need) {
            const u32x4 w = philox4x32_10(ctr(0x40u, g, chain), a.seed_lo, a.seed_hi);
            const double t = u01((lall[j] << (32 - LB)) | (w.x >> LB), w.y);
            acc = ratio_accept(bA, bB, t, false, a.log_npi);
          }
        }
      }
#pragma unroll
      for (int i = 0; i < D; ++i) x[i] = acc ? xp[i] : x[i];
      lp = acc ? lpp : lp;
      lm = acc ? M : lm;
      ls = acc ? S : ls;
      if (mom) {
        nacc += acc ? 1 : 0;
#pragma unroll
        for (int i = 0; i < D; ++i) {
          if (i % L == p) {
            ms[i] += x[i];
            mq[i] = __builtin_fma(x[i], x[i], mq[i]);
          }
        }
      }
      const bool rec_now = ph == 0;
      const int64_t rec = ri;
      ph = (ph + 1 == a.thin) ? 0 : ph + 1;
      ri += (ph == 0) ? 1 : 0;
      if (rec_now && rec >= 0 && rec < a.rec_cap) {
        if (active) {
          double *row = a.tx + rec * D * a.n;   // wave-uniform
#pragma unroll
          for (int i = 0; i < D; ++i)
            if (i % L == p) st_buf(row, boff, i * bstride, x[i]);
          if (p == (D % L)) st_buf(a.tlp + rec * a.n, boff, 0, lp);
        }
        // the parts agree: part 0's lanes (bits [0, CW)) carry the chains
        const uint64_t am = __ballot(acc) & act_mask;
        if (lane == 0 && wave < (64 / CW) * a.W) {   // stay inside the record
          const int64_t wi = rec * (64 / CW) * a.W + wave;
          if constexpr (CW == 32) reinterpret_cast<uint32_t *>(a.tacc)[wi] = (uint32_t)am;
          else reinterpret_cast<uint16_t *>(a.tacc)[wi] = (uint16_t)am;
        }
      }
    }
  }
  if (active) {
#pragma unroll
    for (int i = 0; i < D; ++i) {
      if (i % L == p) {
        a.x[i * a.n + c] = x[i];
        if (mom) {
          a.msum[i * a.n + c] += ms[i];
          a.msq[i * a.n + c] += mq[i];
        }
      }
    }
    if (p == 0) {
      a.lp[c] = lp;
      if (mom) a.nacc[c] += nacc;
    }
  }
}
// ---------------------------------------------------------------------------
// Quad MH kernel for the Gaussian-mixture target (cfg5, production RNG,
// K <= 4 components, D <= 4): one chain per QUAD of adjacent lanes (lane
// 4 c + p), 16 chains per wavefront, so 32 768 chains fill 2 048 wavefronts
// (2 per SIMD).  Every exchange inside a chain is a DPP quad_perm move (one
// VALU per 32-bit word), not a cross-row permlane.
//  * Draws: aligned groups of 4 steps; lane p draws step 4 G + p alone
//    (step_draws: bm96 fp64 normals, a 24-bit threshold lead) and
//    the quad broadcasts the group's draws to every lane.
//  * Density: lane p owns component p; M = max and S = sum of exp(v_k - M)
//    over the quad (two xor rounds each, the same association in every
//    lane); log-sum-exp = M + ln S.
//  * Acceptance on (M, S) -- no log on the step-to-step chain (see
//    accept_filter_ms); the recorded v.prob M + ln S of a group's 4 states
//    is evaluated after the group, one state per lane, so each lane pays one
//    table log per 4 steps.  Undecided steps (~1e-4) take the exact ratio
//    form of (lp', lp) with both logs evaluated on the spot (the same
//    function of the same (M, S) as the recorded values).
// The draws, counters and decisions are those of mh_kernel's production
// Gaussian path; densities differ from it by rounding only.
// ---------------------------------------------------------------------------
constexpr int kQuadXor1 = 0xB1, kQuadXor2 = 0x4E;   // quad_perm [1,0,3,2], [2,3,0,1]

template <int CTRL>
__device__ __forceinline__ uint32_t qperm_u32(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, false);
}
template <int CTRL>
__device__ __forceinline__ double qperm_f64(double v) {
  return from_words(qperm_u32<CTRL>(hi32(v)), qperm_u32<CTRL>(lo32(v)));
}
// quad_perm [q, q, q, q]: lane q's value in every lane of the quad
template <int Q>
__device__ __forceinline__ double qbcast_f64(double v) {
  return qperm_f64<Q * 85>(v);
}

// The quad kernel's decision path in fp32: e = exp(M' - M) S32' / S32 with
// S32 = sum_k exp2f(fp32((v_k - M) log2 e)).  Error where a decision can
// hinge on it (e in [2^-15, 1], i.e. |M' - M| log2 e <= 15): the argument
// rounding 4.2e-8 x 15 = 6.3e-7, each S32 within 5.1e-7 (K <= 4 terms: a
// term 2^y errs by at most 4.1e-8 |y| 2^y + 1 ulp <= 8.2e-8, plus three
// fp32 additions), rcp / products 1.8e-7: about 2.3e-6 < the 4e-6 margin.
// Outside that range the decision is certain (thi <= 1 < e, or tlo >= 2^-14
// > e) or the lead is 0 and the exact form decides.
template <int LB>
__device__ __forceinline__ Decision accept_filter_ms32(double Mp, float Sp,
                                                       double M, float S,
                                                       uint32_t lead) {
  constexpr float w = 1.0f / (float)(1u << LB);
  const float e = __builtin_amdgcn_exp2f((float)((Mp - M) * 1.4426950408889634)) *
                  (Sp * __builtin_amdgcn_rcpf(S));
  const float tlo = (float)lead * w;
  const float thi = tlo + w;
  const bool inr = __builtin_fabs(Mp) <= 698. && __builtin_fabs(M) <= 698.;
  const bool af = thi <= e * 0.999996f;
  const bool rf = tlo > e * 1.000004f;
  return Decision{inr && af, !(inr && (af || rf))};
}

// The same decision with the proposal's terms taken relative to the STATE's
// max lm instead of its own: e = sum_k exp2f(fp32((v'_k - lm) log2 e)) x
// rcp(fp32(S)), S the state's sum relative to lm.  The proposal's max M' (two
// DPP rounds) is then off the decision's dependency chain.  Where a decision
// can hinge on e (e <= 1: every term 2^y <= K, y <= 2; terms below 2^-15 do
// not matter at the 4e-6 margin) |y| <= 17: argument rounding 4.2e-8 x 17 =
// 7.1e-7 + 1 ulp per term, the sum within 1.1e-6, rcp and the conversion of S
// 1.8e-7: about 1.4e-6 < 4e-6.  e = inf (a far better proposal) accepts;
// e = 0 with lead 0 is undecided.  inr: |M'|, |lm| <= 698 as before.
// Form used by the quad kernel: the state's fp32 sum ls32 scales the
// threshold instead of dividing the proposal's sum (e = sp / ls32, t < e
// <=> t ls32 < sp; ls32 > 0): no reciprocal per step; the two products add
// an ulp each, inside the same 4e-6 margin.
template <int LB>
__device__ __forceinline__ Decision accept_filter_rel32(float sp, float ls32, bool inr,
                                                        uint32_t lead) {
  constexpr float w = 1.0f / (float)(1u << LB);
  const float tlo = (float)lead * w;
  const float thi = tlo + w;
  const bool af = thi * ls32 <= sp * 0.999996f;
  const bool rf = tlo * ls32 > sp * 1.000004f;
  return Decision{(bool)(inr & af), !(inr & (af | rf))};
}

// The same as lane masks (accept_filter_lead_mask): inrm is the ballot of
// the range condition.
template <int LB>
__device__ __forceinline__ DecisionMask accept_filter_rel32_mask(float sp, float ls32,
                                                                 uint64_t inrm,
                                                                 uint32_t lead) {
  constexpr float w = 1.0f / (float)(1u << LB);
  const float tlo = (float)lead * w;
  const float thi = tlo + w;
  const uint64_t af = __ballot(thi * ls32 <= sp * 0.999996f);
  const uint64_t rf = __ballot(tlo * ls32 > sp * 1.000004f);
  return DecisionMask{inrm & af, ~(inrm & (af | rf))};
}

__device__ __forceinline__ double max_f64_raw(double a, double b) {
  double r;
  asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

template <int CTRL>
__device__ __forceinline__ float qperm_f32(float v) {
  return __builtin_bit_cast(float, (uint32_t)__builtin_amdgcn_mov_dpp(
                                       __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}

// the same permutation for a summand: old = 0.0f and bound_ctrl set, the
// form GCNDPPCombine folds into the consuming v_add_f32 (quad_perm reads a
// valid lane everywhere, so the result is qperm_f32's)
template <int CTRL>
__device__ __forceinline__ float qperm_add_f32(float v) {
  return __builtin_bit_cast(float, (uint32_t)__builtin_amdgcn_update_dpp(
                                       0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, true));
}

// The rare undecided step of the quad kernel (accept_filter_ms32's need):
// the exact ratio form of (lp', lp) on t's full 53 bits, out of line so that
// the steady-state loop keeps neither its registers nor its code.
// (Scalars, not the KArgs: a reference to the kernel arguments would make
// the kernel copy all of them to its private stack at entry.)
__device__ __attribute__((noinline)) bool gmm_quad_exact(
    uint32_t seed_lo, uint32_t seed_hi, double acc_beta, double log_npi,
    const double *tab, int64_t g, int64_t chain, uint32_t lead,
    double M, double S, double lm, double ls, double lp0) {
  constexpr int LB = kStepLead;
  const u32x4 w = philox4x32_10(ctr(0x40u, g, chain), seed_lo, seed_hi);
  const double t = u01((lead << (32 - LB)) | (w.x >> LB), w.y);
  const double lpp = M + ln_tab(S, tab);
  const double lpc = lm == lp0 && ls == 1.0 ? lp0 : lm + ln_tab(ls, tab);
  return ratio_accept(lpp * acc_beta, lpc * acc_beta, t, false, log_npi);
}

// FULL: the steady-state launch (gmm_quad_full): whole groups of GS = 8
// steps where the launch's start and length are multiples of 8, else of 4,
// every step recorded (thin 1, inside the trace), the chains past step 1 and
// the plain ratio form (acc_beta = 1) -- no per-step range, record or
// first-step tests, and branch-free stores: a lane with nothing of its own
// to write (a part p >= D, or a padding chain, which runs chain 0's exact
// trajectory) rewrites the identical value of a lane that has.  Its steps
// run only the fp32 decision path; the fp64 record path (the state's M and
// S, i.e. v.prob) is evaluated once per group per lane (round 4: ~100 -> ~65
// VALU per wave-step), bit-identical to the general form's per-step records
// (test_gmm_quad_steady_state_form_is_the_general_form).
// LOC0: every proposal loc is 0 (the examples' norm.rvs(scale=...)): x' =
// fma(r, scale, x), one rounding, instead of x + fma(r, scale, loc).
template <int D, int K, bool MOM, bool FULL, bool LOC0 = false, int GS = 4>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(2)))
void mh_gmm_quad_kernel(KArgs a) {
  static_assert(GS == 4 || GS == 8, "quad kernel: groups of 4 or 8 steps");
  static_assert(GS == 4 || FULL, "the general form runs groups of 4");
  static_assert(K >= 1 && K <= 4 && D >= 1 && D <= 4, "quad kernel: K, D <= 4");
  constexpr int LB = kStepLead;          // threshold lead bits (step_draws)
  __shared__ double s_bmt[kBm64Doubles];
  PBH_PHASE_DECL;
  PBH_PHASE(0);
  const int lane = threadIdx.x & 63;
  const int p = lane & 3;
  const int64_t gt = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const int64_t wave = gt >> 6;
  const int64_t c = gt >> 2;
  const bool active = c < a.n;
  const int64_t cc = active ? c : 0;
  const int64_t chain = a.off + cc;
  const uint64_t act_bits = __ballot(active && p == 0);

  // this lane's component (a lane p >= K contributes exp(-inf) = 0)
  const bool own = p < K;
  const double cw = own ? a.tw[p] : 0.;
  const double c0 = own ? a.tw[K + p] : -__builtin_inf();
  // component term u = x w - mu w (mu w precomputed: one fma per dim)
  double cmw[D], psc[D], plc[D];
#pragma unroll
  for (int i = 0; i < D; ++i) {
    cmw[i] = own ? a.tb[p * D + i] * cw : 0.;
    psc[i] = cld(a.pscl, i);
    plc[i] = cld(a.ploc, i);
  }
  double x[D], ms = 0., mq = 0.;   // moments of dim p (p < D)
#pragma unroll
  for (int i = 0; i < D; ++i) x[i] = a.x[i * a.n + cc];
  const double lp0 = a.lp[cc];
  double lm = lp0, ls = 1.0;   // the state's density as (M, S): lp = M + ln S
  float ls32 = 1.0f;           // fp32(S) of the state (the decision path)
  int64_t nacc = 0;
  int ph = (int)((a.g0 + 1) % a.thin);
  int64_t ri = (a.g0 + 1) / a.thin - 1 - a.rec_base;
  const uint32_t xoff = (uint32_t)(((int64_t)(p % D) * a.n + cc) * 8);
  const uint32_t lpoff = (uint32_t)(((int64_t)p * a.n + cc) * 8);   // FULL
  double *txrow = a.tx + ri * D * a.n;   // record ri's rows (wave-uniform)
  const int64_t rstride = (int64_t)D * a.n;
  bm64_load(s_bmt, a.bm64);        // after the state's loads: all in flight
  __builtin_amdgcn_s_waitcnt(0);   // entry loads drained before the loop
  PBH_PHASE(1);

  const int64_t gend = a.g0 + a.n_steps;
  // FULL: lane p writes the group's record row 4 G + p, every dim (the
  // states staged in LDS for the records), one store per dim per group
  uint32_t xoffd[D];
#pragma unroll
  for (int i = 0; i < D; ++i) xoffd[i] = (uint32_t)(((int64_t)i * a.n + cc) * 8);
  const uint32_t rbytes = (uint32_t)(rstride * 8);
  // FULL: the draws are software-pipelined by group -- group G + 1's Philox
  // block(s) are computed beside group G's first step and its Box-Muller
  // pair(s) beside the second (step_draws' words and arithmetic, split)
  constexpr int NP = (D + 1) / 2, NW = 3 * NP + 1, NB = (NW + 3) / 4;
  constexpr int NG = GS / 4;   // draw sets per lane per group (FULL)
  double rnext[NG][D];
  uint32_t lnext[NG] = {};
  // FULL: the step's two filter thresholds, margins folded in, as one packed
  // pair (thi x 1.000008, tlo x 0.999992): af = thi' ls32 <= E32, rf = tlo'
  // ls32 > E32 -- one v_pk_mul_f32 per step for the four products of
  // thi ls32 <= E32 x 0.999992 and tlo ls32 > E32 x 1.000008 (the margin
  // moves by one fp32 rounding, 7.99e-6 -> 7.87e-6, against the 2.3e-6 error
  // budget of accept_filter_ms32)
  typedef float f32x2 __attribute__((ext_vector_type(2)));
  auto thr_pair = [](uint32_t lead) {
    constexpr float w = 1.0f / (float)(1u << LB);
    const float tlo = (float)lead * w;   // exact: lead < 2^24
    return f32x2{(tlo + w) * 1.000008f, tlo * 0.999992f};
  };
  f32x2 thnext[NG];
  if constexpr (FULL) {
#pragma unroll
    for (int h = 0; h < NG; ++h) {
      lnext[h] = step_draws<D>(a, a.g0 + 4 * h + p, chain, s_bmt, rnext[h]);   // g0 % GS == 0
      thnext[h] = thr_pair(lnext[h]);
    }
  }
  PBH_PHASE(2);
  const uint32_t slot = FULL && a.fair ? simd_wave_slot() : 0u;
  if constexpr (FULL) {
    // ---- steady state with the record path deferred to the group's end ----
    // Per step only the decision path runs: this lane's component term of the
    // proposal, its fp32 weight relative to the group's reference R (the
    // state's max at the group start) and the quad's fp32 sum E32, against
    // the state's sum ls32 (relative to the same R; on accept ls32 = E32).
    // The recorded v.prob of step 4 G + p is lane p's after the group: the
    // state after that step (its x staged in LDS) re-evaluated -- every
    // component's term, M = max, S = (e0 + e1) + (e2 + e3), M + ln S: the same
    // operations on the same values as the general form's per-step (M, S),
    // so the same bits -- or lp0 while no step of this launch has accepted.
    // Decisions are the fp64 ratio form's (filter with a 7.9e-6 margin, the
    // exact form for the rest): |y| <= 40 (log2) on every fp32 weight used.
    // Measured and not kept: the draws handed to the quad through
    // LDS instead of DPP broadcasts (+12 %: the reads' latency lands on the
    // decision chain), and a reference moved by whole powers of two with the
    // records one group behind, interleaved with the next group's steps (+6 %:
    // SGPR spills, no gain in issue).
    // GS = 8: groups of eight steps, lane p drawing steps GS G + p and GS G +
    // 4 + p and recording the states after them: the per-group work (the
    // reference's re-anchoring, the accept words' assembly and store, the
    // loop and priority bookkeeping) is paid once per eight steps
    __shared__ double s_xs[GS * D * kBlock];   // the state after each step
    // every component's constants (uniform; held in VGPRs -- in SGPRs they
    // pushed ~30 SGPR spill reloads per group into the loop)
    double kcw[4], kc0[4], kcmw[4][D];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const bool ok = k < K;
      kcw[k] = ok ? in_vgpr_f64(cld(a.tw, k)) : 0.;
      kc0[k] = ok ? in_vgpr_f64(cld(a.tw, K + k)) : -__builtin_inf();
#pragma unroll
      for (int i = 0; i < D; ++i) kcmw[k][i] = ok ? in_vgpr_f64(cld(a.tb, k * D + i) * kcw[k]) : 0.;
    }
    const double e_absent = exp_tab(-__builtin_inf(), s_bmt);   // exp of a -inf term
    // the decision's weight 2^y, y = (v' - R) log2 e, with log2 e folded into
    // this lane's component constants: y = c0l - sum_i (x'_i cwl - cmwl_i)^2,
    // cwl = cw sqrt(log2 e), cmwl = cmw sqrt(log2 e), c0l = (c0 - R) log2 e
    // (per group); two fp64 operations fewer per step.  The fp64 rounding of
    // the rescaled constants (~1e-16 relative) is far below the argument's
    // fp32 rounding (4.2e-8 |y|) that the filter's margin covers.
    constexpr double kSqrtLog2e = 1.2011224087864498;
    const double cwl = cw * kSqrtLog2e;
    double cmwl[D];
#pragma unroll
    for (int i = 0; i < D; ++i) cmwl[i] = cmw[i] * kSqrtLog2e;
    constexpr uint64_t kQ0 = 0x1111111111111111ull;
    double R = lp0;          // the decision's reference (group start)
    uint64_t initm = ~0ull;  // lanes whose chain has not accepted in this launch
    uint64_t rinm = __ballot(__builtin_fabs(R) <= 650.);
    uint64_t sinm = ~0ull;   // ls32 within [2^-40, 2^40]
    const uint64_t allm = __ballot(true);
    // accept words: lane c < 16 reads lane 4 c (chain c of the wave); act16 =
    // the wave's active chains as the word's bits
    const int bperm4 = (lane & 15) * 16;
    const uint32_t woff = (uint32_t)(wave * 2 + (int64_t)(lane & (GS - 1)) * a.W * 8);   // step lane's word
    const PhiloxKeys rk = philox_keys_v(a.seed_lo, a.seed_hi);   // SGPRs stay free
    const uint64_t act16 = __ballot(lane < 16 && wave * 16 + lane < a.n);
    for (int64_t G = a.g0 / GS; G * GS < gend; ++G) {
      if (a.fair) fair_prio((uint32_t)(__builtin_amdgcn_s_memrealtime() >> a.fair) + slot);
      PBH_PHASE_Q(G - a.g0 / GS, (gend + GS - 1) / GS - a.g0 / GS);
      uint32_t lown[NG];
      double rown[NG][D];
      f32x2 thown[NG];
#pragma unroll
      for (int h = 0; h < NG; ++h) {
        lown[h] = lnext[h];
        thown[h] = thnext[h];
#pragma unroll
        for (int i = 0; i < D; ++i) rown[h][i] = rnext[h][i];
      }
      const double c0l = (c0 - R) * 1.4426950408889634;
      uint32_t wn[NG][4 * NB];   // group G + 1's words
      auto next_blocks = [&](auto H_) {
        constexpr int h = decltype(H_)::value;
#pragma unroll
        for (int q = 0; q < NB; ++q) {
          const u32x4 b = philox4x32_10_rk(ctr(q, GS * (G + 1) + 4 * h + p, chain), rk);
          wn[h][4 * q] = b.x;
          wn[h][4 * q + 1] = b.y;
          wn[h][4 * q + 2] = b.z;
          wn[h][4 * q + 3] = b.w;
        }
      };
      auto next_normals = [&](auto H_) {
        constexpr int h = decltype(H_)::value;
#pragma unroll
        for (int q = 0; q < NP; ++q) {
          double z0, z1;
          bm96_pair(wn[h][3 * q], wn[h][3 * q + 1], wn[h][3 * q + 2], s_bmt, z0, z1);
          rnext[h][2 * q] = z0;
          if (2 * q + 1 < D) rnext[h][2 * q + 1] = z1;
        }
        lnext[h] = wn[h][3 * NP] >> (32 - kStepLead);
        thnext[h] = thr_pair(lnext[h]);
      };
      double *const gtx = wave_uniform(txrow);
      uint16_t *const gacc = wave_uniform(reinterpret_cast<uint16_t *>(a.tacc + ri * a.W));
      uint64_t ginit[GS], gacm[GS];
      // the quad's (M, S) of a term v (the general form's record arithmetic)
      auto quad_ms = [&](double v, double &M, double &S) {
        M = max_f64_raw(v, qperm_f64<kQuadXor1>(v));
        M = max_f64_raw(M, qperm_f64<kQuadXor2>(M));
        double e = exp_tab(v - M, s_bmt);
        e = e + qperm_f64<kQuadXor1>(e);
        S = e + qperm_f64<kQuadXor2>(e);
      };
      auto term = [&](const double (&xv)[D], double cwv, double c0v, const double (&cm)[D]) {
        double v = c0v;
#pragma unroll
        for (int i = 0; i < D; ++i) {
          const double u = __builtin_fma(xv[i], cwv, -cm[i]);
          v = __builtin_fma(-u, u, v);
        }
        return v;
      };
      auto step = [&](auto J) {
        constexpr int j = decltype(J)::value, h = j / 4, jq = j % 4;   // set h, lane jq's draws
        double r[D];
#pragma unroll
        for (int i = 0; i < D; ++i) r[i] = qperm_f64<jq * 85>(rown[h][i]);
        const f32x2 th = {qperm_f32<jq * 85>(thown[h].x), qperm_f32<jq * 85>(thown[h].y)};
        const int64_t g = GS * G + j;
        double xp[D];
#pragma unroll
        for (int i = 0; i < D; ++i)
          xp[i] = LOC0 ? __builtin_fma(r[i], psc[i], x[i]) : x[i] + __builtin_fma(r[i], psc[i], plc[i]);
        float e32 = __builtin_amdgcn_exp2f((float)term(xp, cwl, c0l, cmwl));
        e32 = e32 + qperm_add_f32<kQuadXor1>(e32);
        const float E32 = e32 + qperm_add_f32<kQuadXor2>(e32);
        const f32x2 tl = th * ls32;   // (thi' ls32, tlo' ls32)
        // two compares straight into masks (a ballot of their AND would
        // materialise the bool in a VGPR first)
        const uint64_t pinm = __ballot(E32 >= 0x1p-40f) & __ballot(E32 <= 0x1p40f);
        const uint64_t inrm = rinm & sinm & pinm;
        const uint64_t af = __ballot(tl.x <= E32);
        const uint64_t rf = __ballot(tl.y > E32);
        uint64_t accm = inrm & af;
        const uint64_t needm = ~(inrm & (af | rf)) & allm;
        if (needm) {   // wave-uniform, rare: the exact ratio form in fp64
          double M, S, ms_, ss_;
          quad_ms(term(xp, cw, c0, cmw), M, S);        // the proposal
          quad_ms(term(x, cw, c0, cmw), ms_, ss_);     // the state
          const bool st0 = __builtin_amdgcn_inverse_ballot_w64(initm);
          const double lm_ = st0 ? lp0 : ms_, ls_ = st0 ? 1.0 : ss_;
          const uint32_t ld = qperm_u32<jq * 85>(lown[h]);
          bool ex = false;
          if (__builtin_amdgcn_inverse_ballot_w64(needm))
            ex = gmm_quad_exact(a.seed_lo, a.seed_hi, a.acc_beta, a.log_npi, s_bmt,
                                g, chain, ld, M, S, lm_, ls_, lp0);
          accm = (accm & ~needm) | (__ballot(ex) & needm);
        }
#pragma unroll
        for (int i = 0; i < D; ++i) x[i] = sel_f64(accm, x[i], xp[i]);
        ls32 = __builtin_amdgcn_inverse_ballot_w64(accm) ? E32 : ls32;
        sinm = (sinm & ~accm) | (pinm & accm);
        initm &= ~accm;
        ginit[j] = initm;
        if constexpr (MOM) {
          nacc += __builtin_amdgcn_inverse_ballot_w64(accm) ? 1 : 0;
          double xo = x[0];
#pragma unroll
          for (int i = 1; i < D; ++i) xo = p == i ? x[i] : xo;
          ms += xo;
          mq = __builtin_fma(xo, xo, mq);
        }
#pragma unroll
        for (int i = 0; i < D; ++i) s_xs[(j * D + i) * kBlock + threadIdx.x] = x[i];
        gacm[j] = accm;
      };
      using I0 = std::integral_constant<int, 0>;
      using I1 = std::integral_constant<int, 1>;
      next_blocks(I0{});
      step(std::integral_constant<int, 0>{});
      next_normals(I0{});
      step(std::integral_constant<int, 1>{});
      if constexpr (NG == 2) next_blocks(I1{});
      step(std::integral_constant<int, 2>{});
      if constexpr (NG == 2) next_normals(I1{});
      step(std::integral_constant<int, 3>{});
      if constexpr (GS == 8) {
        step(std::integral_constant<int, 4>{});
        step(std::integral_constant<int, 5>{});
        step(std::integral_constant<int, 6>{});
        step(std::integral_constant<int, 7>{});
      }
      {
        // the group's accept words: lane c < 16 takes chain c's GS decision
        // bits from its quad (lane 4 c, ds_bpermute) and each step's word is
        // one ballot -- instead of compressing every step's 64-bit mask on
        // the SALU
        uint32_t vf = 0u;
#pragma unroll
        for (int j = 0; j < GS; ++j)
          vf |= __builtin_amdgcn_inverse_ballot_w64(gacm[j]) ? (1u << j) : 0u;
        const uint32_t fl = (uint32_t)__builtin_amdgcn_ds_bpermute(bperm4, (int)vf);
        // lane j < GS holds step j's word (v_writelane) and one store writes
        // the group's words (a store instruction costs more than its few
        // VALU: one per group instead of one per step)
        uint32_t wv = 0u;
#pragma unroll
        for (int j = 0; j < GS; ++j) {
          const uint32_t w16 = (uint32_t)(__ballot((fl >> j) & 1u) & act16);
          asm volatile("v_writelane_b32 %0, %1, %2" : "+v"(wv) : "s"(w16), "n"(j));
        }
        if (lane < GS) st_buf16(gacc, woff, (uint16_t)wv);
      }
      // ---- the group's records: lane p, the states after steps GS G + 4 h
      // + p; their x rows too (one store per dim and state per group instead
      // of one per dim per step) ----
      double pm = lp0, pss = 1.0;
#pragma unroll
      for (int h = 0; h < NG; ++h) {
        double xs[D];
#pragma unroll
        for (int i = 0; i < D; ++i) {
          xs[i] = s_xs[((4 * h + p) * D + i) * kBlock + threadIdx.x];
          st_buf_n(gtx, GS * rbytes, (uint32_t)(4 * h + p) * rbytes + xoffd[i], xs[i]);   // row GS G + 4 h + p
        }
        const uint64_t pinit = (ginit[4 * h] & kQ0) | (ginit[4 * h + 1] & (kQ0 << 1)) |
                               (ginit[4 * h + 2] & (kQ0 << 2)) | (ginit[4 * h + 3] & (kQ0 << 3));
        double vk[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) vk[k] = k < K ? term(xs, kcw[k], kc0[k], kcmw[k]) : -__builtin_inf();
        const double M = max_f64_raw(max_f64_raw(vk[0], vk[1]), max_f64_raw(vk[2], vk[3]));
        ExpPre ep[4];
#pragma unroll
        for (int k = 0; k < K; ++k) ep[k] = exp_tab_pre(vk[k] - M, s_bmt);   // the K table reads first
        double ek[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) ek[k] = k < K ? exp_tab_fin(ep[k]) : e_absent;
        const double S = (ek[0] + ek[1]) + (ek[2] + ek[3]);
        const bool pi0 = __builtin_amdgcn_inverse_ballot_w64(pinit);
        pm = pi0 ? lp0 : M;
        pss = pi0 ? 1.0 : S;
        const double lpr = pm == lp0 && pss == 1.0 ? lp0 : pm + ln_tab(pss, s_bmt);
        st_buf(wave_uniform(a.tlp + (ri + 4 * h) * a.n), lpoff, 0, lpr);
      }
      // the next group's reference: the state after step GS G + GS - 1 (lane 3)
      R = qbcast_f64<3>(pm);
      lm = R;
      ls = qbcast_f64<3>(pss);
      ls32 = (float)ls;
      rinm = __ballot(__builtin_fabs(R) <= 650.);
      sinm = allm;   // ls in [1, K] (or 1)
      ri += GS;
      txrow += GS * rstride;
    }
  } else {
  // ---- the general form: any launch (partial groups, thinning, step 1,
  // tempered ratio forms), the state carried as (M, S) step by step
  for (int64_t G = a.g0 >> 2; G * 4 < gend; ++G) {
    // ---- lane p draws step 4 G + p; the quad shares the group's draws
    double rown[D];
    const uint32_t lown = step_draws<D>(a, 4 * G + p, chain, s_bmt, rown);
    double gm[4], gs[4];     // the group's states (M, S), for the records
    int64_t grec[4];
    // one step of the group; j is a compile-time constant (DPP controls)
    auto step = [&](auto J) {
      constexpr int j = decltype(J)::value;
      double r[D];
#pragma unroll
      for (int i = 0; i < D; ++i) r[i] = qperm_f64<j * 85>(rown[i]);
      const uint32_t lead = qperm_u32<j * 85>(lown);
      const int64_t g = 4 * G + j;
      grec[j] = -1;
      gm[j] = lm;
      gs[j] = ls;
      if (g < a.g0 || g >= gend) return;   // wave-uniform
      const int s = (int)(g - a.g0);
      double xp[D];
#pragma unroll
      for (int i = 0; i < D; ++i)
        xp[i] = LOC0 ? __builtin_fma(r[i], psc[i], x[i]) : x[i] + __builtin_fma(r[i], psc[i], plc[i]);
      double v = c0;
#pragma unroll
      for (int i = 0; i < D; ++i) {
        const double u = __builtin_fma(xp[i], cw, -cmw[i]);
        v = __builtin_fma(-u, u, v);
      }
      // decision path: the terms relative to the state's max lm
      // (accept_filter_rel32).  A lane p >= K holds v = -inf: its terms are
      // exp(-inf) = 0 in both paths without a select (exp_tab clamps at -746:
      // 0 to within 2^-1074)
      float e32 = __builtin_amdgcn_exp2f((float)((v - lm) * 1.4426950408889634));
      // (update_dpp with old = 0 and bound_ctrl: the DPP combiner folds
      // each move into the add, v_add_f32_dpp, one VALU per round)
      e32 = e32 + qperm_add_f32<kQuadXor1>(e32);
      const float E32 = e32 + qperm_add_f32<kQuadXor2>(e32);   // the proposal's sum
      // record path (off the decision's chain): M' and S in fp64
      // v_max_f64 without the compiler's canonicalising max of the DPP'd
      // operand (the values are never NaN: finite or -inf)
      double M = max_f64_raw(v, qperm_f64<kQuadXor1>(v));
      M = max_f64_raw(M, qperm_f64<kQuadXor2>(M));
      const double dv = v - M;
      const bool inr = (__builtin_fabs(M) <= 698.) & (__builtin_fabs(lm) <= 698.);
      double e = exp_tab(dv, s_bmt);
      e = e + qperm_f64<kQuadXor1>(e);
      const double S = e + qperm_f64<kQuadXor2>(e);   // in [1, K]
      bool acc;
      if (!a.has_pred && s == 0) {
        acc = true;                                  // s = None on step 1
      } else {
        const Decision dc = a.acc_beta == 1.0
            ? accept_filter_rel32<LB>(E32, ls32, inr, lead)
            : accept_filter_lead<LB>((M + ln_tab(S, s_bmt)) * a.acc_beta,
                                     (lm + ln_tab(ls, s_bmt)) * a.acc_beta,
                                     lead, false);
        acc = dc.acc;
        if (__ballot(dc.need)) {   // wave-uniform, rare
          if (dc.need) {
            const u32x4 w = philox4x32_10(ctr(0x40u, g, chain), a.seed_lo, a.seed_hi);
            const double t = u01((lead << (32 - LB)) | (w.x >> LB), w.y);
            const double lpp = M + ln_tab(S, s_bmt);
            const double lpc = lm == lp0 && ls == 1.0 ? lp0 : lm + ln_tab(ls, s_bmt);
            acc = ratio_accept(lpp * a.acc_beta, lpc * a.acc_beta, t, false, a.log_npi);
          }
        }
      }
#pragma unroll
        for (int i = 0; i < D; ++i) x[i] = acc ? xp[i] : x[i];
        lm = acc ? M : lm;
        ls = acc ? S : ls;
        ls32 = (float)ls;
      gm[j] = lm;
      gs[j] = ls;
      if constexpr (MOM) {
        nacc += acc ? 1 : 0;
        double xo = x[0];
#pragma unroll
        for (int i = 1; i < D; ++i) xo = p == i ? x[i] : xo;
        ms += xo;
        mq = __builtin_fma(xo, xo, mq);
      }
      const bool rec_now = ph == 0;
      const int64_t rec = ri;
      double *row = txrow;
      ph = (ph + 1 == a.thin) ? 0 : ph + 1;
      if (ph == 0) {
        ++ri;
        txrow += rstride;
      }
      if (rec_now && rec >= 0 && rec < a.rec_cap) {
        grec[j] = rec;
        if (active && p < D) {
          double xo = x[0];
#pragma unroll
          for (int i = 1; i < D; ++i) xo = p == i ? x[i] : xo;
          st_buf(row, xoff, 0, xo);   // wave-uniform base
        }
        // the quad agrees: bit 4 c of the ballot is chain c's; compress the
        // 16 chain bits of this wave (SALU)
        uint64_t m = __ballot(acc) & 0x1111111111111111ull & act_bits;
        m = (m | (m >> 3)) & 0x0303030303030303ull;
        m = (m | (m >> 6)) & 0x000F000F000F000Full;
        m = (m | (m >> 12)) & 0x000000FF000000FFull;
        m = (m | (m >> 24)) & 0xFFFFull;
        if (lane == 0 && wave < 4 * a.W)   // stay inside the record
          reinterpret_cast<uint16_t *>(a.tacc)[rec * 4 * a.W + wave] = (uint16_t)m;
      }
    };
    step(std::integral_constant<int, 0>{});
    step(std::integral_constant<int, 1>{});
    step(std::integral_constant<int, 2>{});
    step(std::integral_constant<int, 3>{});
    // ---- the group's recorded v.prob: lane p evaluates step 4 G + p's
    double pm = gm[0], pss = gs[0];
    int64_t prec = grec[0];
#pragma unroll
    for (int j = 1; j < 4; ++j) {
      pm = p == j ? gm[j] : pm;
      pss = p == j ? gs[j] : pss;
      prec = p == j ? grec[j] : prec;
    }
    if (prec >= 0 && active) {
      const double lpr = pm == lp0 && pss == 1.0 ? lp0 : pm + ln_tab(pss, s_bmt);
      __builtin_nontemporal_store(lpr, &a.tlp[prec * a.n + cc]);
    }
  }
  }
  PBH_PHASE(3);
  if (active) {
    if (p < D) {
      double xo = x[0];
#pragma unroll
      for (int i = 1; i < D; ++i) xo = p == i ? x[i] : xo;
      a.x[p * a.n + c] = xo;
      if constexpr (MOM) {
        a.msum[p * a.n + c] += ms;
        a.msq[p * a.n + c] += mq;
      }
    }
    if (p == 0) {
      a.lp[c] = lm == lp0 && ls == 1.0 ? lp0 : lm + ln_tab(ls, s_bmt);
      if constexpr (MOM) a.nacc[c] += nacc;
    }
  }
  if constexpr (FULL) {   // probe build only (a.rep is the phase buffer)
    PBH_PHASE(4);
    PBH_PHASE_STORE(a.rep, wave, lane);
  }
}
// ---------------------------------------------------------------------------
// MFMA form of the mvn quadratic form for a wavefront of 64 chains:
//   Y^T (16 x 16 chains) = U^T (16 x 4) . DEV^T (4 x 16 chains), K-chunks of 4
// with v_mfma_f64_16x16x4_f64 (A = U^T, constant, in VGPRs; B = the chains'
// deviations, re-read from a per-wave LDS tile [chain][dim] so that lane l
// holds chain l & 15's dim 4kc + (l >> 4)); then maha = sum_o y_o^2: four
// squares per lane plus a two-step butterfly over the 16-lane groups leaves
// every lane of group g holding its own chain's value -- no transposes back.
// ---------------------------------------------------------------------------
typedef double f64x4 __attribute__((ext_vector_type(4)));

template <int D>
struct MvnMfma {
  static constexpr int KC = (D + 3) / 4;     // K-chunks of 4 dims
  static constexpr int S = KC * 4 + 1;       // LDS row stride (doubles), odd
  double ua[KC];                              // A operand: U[4kc + l>>4][l&15]

  __device__ __forceinline__ void init(const KArgs &a, double *tile) {
    const int lane = threadIdx.x & 63;
    const int o = lane & 15, k = lane >> 4;
#pragma unroll
    for (int kc = 0; kc < KC; ++kc) {
      const int i = 4 * kc + k;
      ua[kc] = (i < D && o < D) ? cld(a.tb, i * D + o) : 0.0;
    }
    double *row = tile + lane * S;
#pragma unroll
    for (int i = D; i < KC * 4; ++i) row[i] = 0.0;   // zero K padding
  }

  __device__ __forceinline__ double density(const KArgs &a, const double (&x)[D],
                                            double *tile) const {
    const int lane = threadIdx.x & 63;
    double *row = tile + lane * S;
#pragma unroll
    for (int i = 0; i < D; ++i) row[i] = x[mvn_perm<D>(i)] - cld(a.ta, i);
    double maha = 0.0;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      f64x4 acc = {0.0, 0.0, 0.0, 0.0};
      const double *col = tile + (16 * g + (lane & 15)) * S + (lane >> 4);
#pragma unroll
      for (int kc = 0; kc < KC; ++kc)
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(ua[kc], col[4 * kc], acc, 0,
                                                   0, 0);
      double p = acc[0] * acc[0];
      p = p + acc[1] * acc[1];
      p = p + acc[2] * acc[2];
      p = p + acc[3] * acc[3];
      p = p + __shfl_xor(p, 16);
      p = p + __shfl_xor(p, 32);
      if ((lane >> 4) == g) maha = p;
    }
    const double logpdf = -0.5 * (cld(a.tc, 0) + maha);
    return a.pscale == PBH_PSCALE_LIN ? exp(logpdf) : logpdf;
  }
};

// ---------------------------------------------------------------------------
// CondCov Gibbs kernel (cond_cov.py:42-65 per coordinate; rf.py:446-458
// cycling).  One SP step updates tsteps coordinates; u is always True.
// ---------------------------------------------------------------------------
template <int D, int RNG, bool MF>
__global__ __launch_bounds__(kBlock) void gibbs_kernel(KArgs a) {
  extern __shared__ double s_tile[];
  const int64_t c = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const bool active = c < a.n;
  const int64_t cc = active ? c : 0;
  const int lane = threadIdx.x & 63;
  // MF: the density's quadratic form on the matrix cores (MvnMfma)
  double *tile = s_tile + (threadIdx.x >> 6) * 64 * MvnMfma<D>::S;
  MvnMfma<D> mf;
  if (MF) mf.init(a, tile);
  double x[D], ms[D], mq[D];
#pragma unroll
  for (int k = 0; k < D; ++k) {
    x[k] = a.x[k * a.n + cc];
    ms[k] = 0.;
    mq[k] = 0.;
  }
  double lp = a.lp[cc];
  const int64_t chain = a.off + cc;
  Xo xs{0u, 0u, 0u, 0u};
  if (RNG == PBH_RNG_XOSHIRO) xs = xo_load(a, 0, cc);
  const int ts = a.tsteps;
  const int nblk = (D + ts - 1) / ts;

  // record phase / index of the trace, advanced per step (no 64-bit
  // division in the loop): step g records iff (g + 1) % thin == 0, at
  // record (g + 1) / thin - 1 - rec_base.
  int ph = (int)((a.g0 + 1) % a.thin);
  int64_t ri = (a.g0 + 1) / a.thin - 1 - a.rec_base;

  for (int s = 0; s < a.n_steps; ++s) {
    const int64_t g = a.g0 + s;
    const int cm = (int)(g % nblk) * ts;
    int j = 0;
#pragma unroll
    for (int k = 0; k < D; ++k) {
      if (k >= cm && k < cm + ts) {
        double u;
        if (RNG == PBH_RNG_REPLAY) {
          u = a.rep[((a.rep_row0 + s) * a.R + j) * a.n + cc];
        } else if (RNG == PBH_RNG_XOSHIRO) {
          const uint32_t w0 = xo_next(xs);
          u = u01(w0, xo_next(xs));
        } else {
          const u32x4 w = philox4x32_10(ctr(j, g, chain), a.seed_lo, a.seed_hi);
          u = u01(w.x, w.y);
        }
        ++j;
        // mean + coef_k . (x_{-k} - mu_{-k})
        double dot = 0.;
        bool first = true;
#pragma unroll
        for (int i = 0; i < D; ++i) {
          if (i == k) continue;
          const int jj = i < k ? i : i - 1;
          const double t = cld(a.gcoef, k * (D - 1) + jj) * (x[i] - cld(a.gmean, i));
          dot = first ? t : dot + t;
          first = false;
        }
        const double lo = cld(a.gcdf, 2 * k), hi = cld(a.gcdf, 2 * k + 1);
        const double cdf = lo + (hi - lo) * u;     // np.random.uniform(lo, hi)
        const double m = cld(a.gmean, k) + dot;
        x[k] = ndtri(cdf) * cld(a.gstdv, k) + m;        // norm.ppf(cdf, m, sd)
      }
    }
    lp = MF ? mf.density(a, x, tile) : mvn_density<D>(a, x);
    if (a.moments) {   // wave-uniform
#pragma unroll
      for (int k = 0; k < D; ++k) {
        ms[k] += x[k];
        mq[k] += x[k] * x[k];
      }
    }
    const bool rec_now = ph == 0;
    const int64_t rec = ri;
    ph = (ph + 1 == a.thin) ? 0 : ph + 1;   // next step's phase
    ri += (ph == 0) ? 1 : 0;
    if (rec_now) {
      if (rec >= 0 && rec < a.rec_cap) {
        if (active) {
#pragma unroll
          for (int k = 0; k < D; ++k) a.tx[(rec * D + k) * a.n + c] = x[k];
          a.tlp[rec * a.n + c] = lp;
          if (a.debug) {
#pragma unroll
            for (int k = 0; k < D; ++k) a.tpx[(rec * D + k) * a.n + c] = x[k];
            a.tpp[rec * a.n + c] = lp;
            a.ts[rec * a.n + c] = __builtin_nan("");
          }
        }
        const uint64_t mask = __ballot(active);
        const int64_t wv = c >> 6;
        if (lane == 0 && wv < a.W) a.tacc[rec * a.W + wv] = mask;
      }
    }
  }
  if (active) {
#pragma unroll
    for (int k = 0; k < D; ++k) a.x[k * a.n + c] = x[k];
    a.lp[c] = lp;
    if (a.moments) {
#pragma unroll
      for (int k = 0; k < D; ++k) {
        a.msum[k * a.n + c] += ms[k];
        a.msq[k * a.n + c] += mq[k];
      }
      a.nacc[c] += a.n_steps;
    }
    if (RNG == PBH_RNG_XOSHIRO) xo_store(a, 0, c, xs);
  }
}

// ---------------------------------------------------------------------------
// Production CondCov Gibbs kernel (PBH_RNG_PHILOX).  The replay kernel above
// restates cond_cov.py:42-65 operation by operation; this one samples the
// same conditional law at a fraction of the cost:
//
//  * one chain per group of L lanes (rows of 64/L lanes, L = 4 at d % 4 == 0),
//    so 32 768 chains fill 2 048 wavefronts (2 per SIMD) instead of 512.
//    Every lane of a group holds the chain's full state; the groups' lanes
//    split the normal draws, the running moments and the trace stores.
//  * x_k ~ N(m_k, sd_k) truncated to the reference's cdf limits
//    (cond_cov.py:57-62: ppf(U(cdf_lo, cdf_hi)) is exactly the standard
//    normal truncated to [ndtri(cdf_lo), ndtri(cdf_hi)]): an fp64 Box-Muller
//    normal, replaced -- under a wave-uniform branch, for the lanes that need
//    it -- by the reference's inversion draw when it falls outside those
//    limits.  That mixture is exactly the truncated normal.  Each lane makes
//    one Box-Muller pair per coordinate cycle and the group all-gathers the
//    cycle's d normals through v_permlane16/32_swap.
//  * v.prob: the quadratic form Q = (x[perm] - mu)^T Sigma^-1 (x[perm] - mu)
//    (prob.py:349-358, App. A-4) is kept up to date in O(d) per coordinate
//    update: with g = P'(x - mu') (P', mu' the precision and mean re-indexed
//    to x order), a change D of x_k gives Q += D (g_k + g'_k), g += D P'_k.
//    g and Q are recomputed exactly every kRefreshCycles coordinate cycles
//    (absolute cycle index) and persisted between launches, so results do not depend on how
//    a run is split into launches.  An fp64 GEMV per coordinate step -- the
//    VALU or MFMA form -- costs d^2 instead of d: on gfx950 the fp64 matrix
//    rate equals the fp64 vector rate, so the matrix cores buy nothing here
//    (DESIGN.md §4).
// ---------------------------------------------------------------------------
constexpr int kRefreshCycles = 32;   // g, Q refreshed every 32 coordinate cycles

// all[q * M + i] = own[i] of the group's lane in part q (part = row index).
template <int L, int M>
__device__ __forceinline__ void gather_parts(const double (&own)[M],
                                             double (&all)[L * M]) {
  if constexpr (L == 1) {
#pragma unroll
    for (int i = 0; i < M; ++i) all[i] = own[i];
  } else if constexpr (L == 2) {
#pragma unroll
    for (int i = 0; i < M; ++i) halves_f64(own[i], all[i], all[M + i]);
  } else {
    static_assert(L == 4, "lanes per chain: 1, 2 or 4");
    double blk[2 * M];
#pragma unroll
    for (int i = 0; i < M; ++i) rowpair_f64(own[i], blk[i], blk[M + i]);
#pragma unroll
    for (int j = 0; j < 2 * M; ++j) halves_f64(blk[j], all[j], all[2 * M + j]);
  }
}

template <int D, int L>
struct GibbsFast {
  static constexpr int M = D / L;     // dims owned per lane
  static constexpr int CW = 64 / L;   // chains per wavefront
  // Per-lane constants of the owned dims i = p M + ii.  For every coordinate
  // K: cf[K][ii] = coef_K at dim i (0 for i == K), pp[K][ii] = P'[K][i];
  // for the owned coordinates: ako[ii] = a_i, sdo[ii] = sd_i.
  double cf[D][M], pp[D][M];
  double ako[M], sdo[M];
  double zlo[M], zhi[M];   // truncation limits of the owned coordinates' z
  double xo[M];     // owned dims of x (the state)
  double zo[M];     // this cycle's normals of the owned coordinates
  double zn[M];     // the next cycle's, drawn during this one (full cycles)
  double go[M];     // owned dims of g = P'(x - mu')
  double ms[M], mq[M];   // running moments of the owned dims
  double Q;         // (x - mu')^T g (identical in the group)
  double lp;        // v.prob of the state
  int p;            // part = lane / CW

  __device__ __forceinline__ void load_consts(const KArgs &a) {
#pragma unroll
    for (int ii = 0; ii < M; ++ii) {
      const int i = p * M + ii;
#pragma unroll
      for (int K = 0; K < D; ++K) {
        cf[K][ii] = i == K ? 0. : a.gcoef[K * (D - 1) + (i < K ? i : i - 1)];
        pp[K][ii] = a.gpp[K * D + i];
      }
      ako[ii] = a.gak[i];
      sdo[ii] = a.gstdv[i];
      zlo[ii] = a.gzlo[i];
      zhi[ii] = a.gzhi[i];
    }
  }

  // g = P'(x - mu') on the owned dims, Q = (x - mu')^T g  (exact refresh)
  __device__ __forceinline__ void refresh(const KArgs &a) {
    // No vector loads inside the step loop: a load's s_waitcnt vmcnt would
    // also wait for every trace store issued before it.  mu' by scalar
    // loads, selected per part.
    double dpo[M], dp[D];
#pragma unroll
    for (int ii = 0; ii < M; ++ii) {
      double mu = uni(cld(a.gmup, ii));
#pragma unroll
      for (int q = 1; q < L; ++q) mu = p == q ? uni(cld(a.gmup, q * M + ii)) : mu;
      dpo[ii] = xo[ii] - mu;
    }
    gather_parts<L, M>(dpo, dp);
    double q = 0.;
#pragma unroll
    for (int ii = 0; ii < M; ++ii) {
      double s = 0.;
#pragma unroll
      for (int j = 0; j < D; ++j) s = __builtin_fma(pp[j][ii], dp[j], s);  // P' symmetric
      go[ii] = s;
      q = __builtin_fma(dpo[ii], s, q);
    }
    Q = part_sum<L>(q);
  }

  // The normals of this lane's coordinates [p M, p M + M) for the coordinate
  // cycle starting at step gc, from Philox blocks 0x100 + 16 p + b.
  const BMTables *bmt;   // LDS tables of the normals' log and sin / cos

  // the cycle's Box-Muller normals (branch-free)
  __device__ __forceinline__ void draw_raw(const KArgs &a, int64_t gc, int64_t chain,
                                           double (&z)[M]) {
#pragma unroll
    for (int b = 0; b < (M + 1) / 2; ++b) {
      double z0, z1;
      box_muller_tab(philox4x32_10(ctr(0x100u + 16u * p + b, gc, chain),
                                   a.seed_lo, a.seed_hi), bmt, z0, z1);
      z[2 * b] = z0;
      if (2 * b + 1 < M) z[2 * b + 1] = z1;
    }
  }

  __device__ __forceinline__ void draw_cycle(const KArgs &a, int64_t gc,
                                             int64_t chain) {
    draw_raw(a, gc, chain, zo);
    fix_trunc(a, gc, chain);
  }

  __device__ __forceinline__ void fix_trunc(const KArgs &a, int64_t gc,
                                            int64_t chain) {
    // Truncation (cond_cov.py:57-62): a normal outside coordinate k's limits
    // is replaced by the reference's inversion draw ppf(U(cdf_lo, cdf_hi)).
    // Rare; one wave-uniform loop keeps a single copy of ndtri in the code.
    uint32_t badm = 0;
#pragma unroll
    for (int ii = 0; ii < M; ++ii)
      badm |= (zo[ii] >= zlo[ii] && zo[ii] <= zhi[ii]) ? 0u : (1u << ii);
    while (__ballot(badm != 0)) {
      const int ii = badm ? __builtin_ctz(badm) : 0;
      const int k = p * M + ii;
      double lo = 0., hi = 1.;   // scalar loads (see refresh)
#pragma unroll
      for (int kk = 0; kk < D; ++kk)
        if (kk == k) { lo = uni(cld(a.gcdf, 2 * kk)); hi = uni(cld(a.gcdf, 2 * kk + 1)); }
      const u32x4 w = philox4x32_10(ctr(0x200u + k, gc, chain), a.seed_lo, a.seed_hi);
      const double zr = ndtri(lo + (hi - lo) * u01(w.x, w.y));
#pragma unroll
      for (int jj = 0; jj < M; ++jj)
        if (badm != 0 && jj == ii) zo[jj] = zr;
      badm &= badm - 1;
    }
  }

  // One coordinate update of coordinate K (cond_cov.py:42-65):
  // x_K = mean_K + coef_K . (x_-K - mean_-K) + sd_K z_K
  //     = a_K + coef_K . x_-K + sd_K z_K,  a_K = mean_K - coef_K . mean_-K.
  // Every part forms its share of the dot product; the owning part OQ makes
  // x_K, its change D and the change of Q, D (g_K + g'_K), and broadcasts
  // D and the Q change; every part then updates its own dims of g += D P'_K.
  // The state is x itself, so a run split into launches reloads exactly the
  // values it stored.
  template <int K>
  __device__ __forceinline__ void update() {
    constexpr int OQ = K / M, OI = K % M;   // owning part, its local index
    double d0 = 0., d1 = 0.;
#pragma unroll
    for (int ii = 0; ii < M; ++ii) {
      if (ii & 1) d1 = __builtin_fma(cf[K][ii], xo[ii], d1);
      else d0 = __builtin_fma(cf[K][ii], xo[ii], d0);
    }
    const double dot = part_sum<L>(d0 + d1);
    // meaningful in the owning part only
    const double xn = __builtin_fma(zo[OI], sdo[OI], dot + ako[OI]);
    const double del = part_bcast<L, OQ>(xn - xo[OI]);
    const double gk = go[OI];
#pragma unroll
    for (int ii = 0; ii < M; ++ii) go[ii] = __builtin_fma(pp[K][ii], del, go[ii]);
    Q += part_bcast<L, OQ>(del * (gk + go[OI]));
    if (p == OQ) xo[OI] = xn;
  }
};

// Per-launch state and step epilogue of gibbs_fast_kernel.  Everything the
// step loop touches is a member (no lambdas capturing by reference), so the
// whole state is promoted to registers.
template <int D, int L>
struct GibbsFastRun : GibbsFast<D, L> {
  using B = GibbsFast<D, L>;
  static constexpr int M = B::M, CW = B::CW;
  int64_t c, wave, ri;
  int lane, ph;
  bool active, lin;
  uint64_t act;

  __device__ __forceinline__ double vprob(const KArgs &a, double q) const {
    const double lq = -0.5 * (a.gconst + q);
    return lin ? fast_exp(lq) : lq;
  }

  // after a step: moments, trace record of x and u; returns the step's
  // record index, or -1 when the step is not recorded
  __device__ __forceinline__ int64_t post_x(const KArgs &a) {
    if (a.moments) {   // wave-uniform
#pragma unroll
      for (int ii = 0; ii < M; ++ii) {
        this->ms[ii] += this->xo[ii];
        this->mq[ii] = __builtin_fma(this->xo[ii], this->xo[ii], this->mq[ii]);
      }
    }
    const bool rec_now = ph == 0;
    const int64_t rec = ri;
    ph = (ph + 1 == a.thin) ? 0 : ph + 1;
    ri += (ph == 0) ? 1 : 0;
    const bool r = rec_now && rec >= 0 && rec < a.rec_cap;
    if (r) {
      if (active) {
#pragma unroll
        for (int ii = 0; ii < M; ++ii)
          __builtin_nontemporal_store(this->xo[ii], &a.tx[(rec * D + this->p * M + ii) * a.n + c]);
      }
      // u is always True for Gibbs (sp_utils.py:75-84): the active chains
      if (lane == 0 && wave < (64 / CW) * a.W) {   // stay inside the record
        const int64_t wi = rec * (64 / CW) * a.W + wave;
        if constexpr (CW == 64) a.tacc[wi] = act;
        else if constexpr (CW == 32) reinterpret_cast<uint32_t *>(a.tacc)[wi] = (uint32_t)act;
        else reinterpret_cast<uint16_t *>(a.tacc)[wi] = (uint16_t)act;
      }
    }
    return r ? rec : -1;
  }

  // after a step: v.prob of the state (every lane), then post_x
  __device__ __forceinline__ void post(const KArgs &a) {
    this->lp = vprob(a, this->Q);
    const int64_t rec = post_x(a);
    if (rec >= 0 && active && this->p == 0)
      __builtin_nontemporal_store(this->lp, &a.tlp[rec * a.n + c]);
  }

  // Steps K - 1, K (K odd) of a paired cycle: parts with p odd evaluate
  // step K's v.prob, parts with p even step K - 1's, so each lane runs one
  // exp per two steps; parts 0 and 1 store the two records.
  template <int K>
  __device__ __forceinline__ void post_pair(const KArgs &a, double &qprev,
                                            int64_t &rprev) {
    const int64_t r = post_x(a);
    if constexpr (K % 2 == 0) {
      qprev = this->Q;
      rprev = r;
    } else {
      const bool odd = this->p & 1;
      const double v = vprob(a, odd ? this->Q : qprev);
      const int64_t rr = odd ? r : rprev;
      if (rr >= 0 && active && this->p < 2)
        __builtin_nontemporal_store(v, &a.tlp[rr * a.n + c]);
    }
  }

  // Coordinates [kb, ke) of a cycle, unrolled at compile time (a runtime
  // coordinate index would make the compiler merge the per-coordinate code
  // and index the constant arrays dynamically, i.e. through scratch).  A
  // step ends after coordinate K when bit K of post_mask is set.  FULL: the
  // whole cycle of single-coordinate steps, with no predicates at all.
  template <bool FULL, int... K>
  __device__ __forceinline__ void cycle(const KArgs &a, int kb, int ke,
                                        uint32_t post_mask,
                                        std::integer_sequence<int, K...>) {
    if constexpr (FULL) {
      if constexpr (L >= 2 && D % 2 == 0) {
        double qprev = 0.;
        int64_t rprev = -1;
        ((this->template update<K>(), post_pair<K>(a, qprev, rprev)), ...);
      } else {
        ((this->template update<K>(), post(a)), ...);
      }
    } else {
      ((K >= kb && K < ke
            ? (this->template update<K>(),
               ((post_mask >> K) & 1u) ? post(a) : void())
            : void()),
       ...);
    }
  }
};

template <int D, int L>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(L == 4 && D <= 8 ? 2 : 1)))
void gibbs_fast_kernel(KArgs a) {
  using S = GibbsFastRun<D, L>;
  constexpr int M = S::M, CW = S::CW;
  __shared__ BMTables s_bmt;
  bm_tables_init(&s_bmt);
  S st;
  st.bmt = &s_bmt;
  st.lane = threadIdx.x & 63;
  st.wave = ((int64_t)blockIdx.x * kBlock + threadIdx.x) >> 6;
  st.c = st.wave * CW + (st.lane % CW);
  st.active = st.c < a.n;
  const int64_t cc = st.active ? st.c : 0;
  const int64_t chain = a.off + cc;
  st.lin = a.pscale == PBH_PSCALE_LIN;
  st.p = st.lane / CW;
  const int p = st.p;
  st.load_consts(a);
#pragma unroll
  for (int ii = 0; ii < M; ++ii) {
    st.xo[ii] = a.x[(p * M + ii) * a.n + cc];
    st.ms[ii] = st.mq[ii] = 0.;
  }
  if (a.gq_init) {
    st.refresh(a);
  } else {
#pragma unroll
    for (int ii = 0; ii < M; ++ii) st.go[ii] = a.gq[(p * M + ii) * a.n + cc];
    st.Q = a.gq[D * a.n + cc];
  }
  st.lp = a.lp[cc];
  const int ts = a.tsteps;
  const int nblk = (D + ts - 1) / ts;
  int cm = (int)(a.g0 % nblk) * ts;    // first coordinate of the next step
  st.draw_cycle(a, a.g0 - a.g0 % nblk, chain);
  st.act = __ballot(st.active && p == 0);
  st.ph = (int)((a.g0 + 1) % a.thin);
  st.ri = (a.g0 + 1) / a.thin - 1 - a.rec_base;
  int64_t cyc = (a.g0 + nblk - 1) / nblk;   // index of the next cycle start

  // steps end after coordinates ts - 1, 2 ts - 1, ..., and d - 1
  uint32_t post_mask = 1u << (D - 1);
  for (int k = ts - 1; k < D; k += ts) post_mask |= 1u << k;
  // Drain the entry loads here: otherwise the waits for them land inside the
  // loop, where each s_waitcnt vmcnt would also wait for the trace stores.
  __builtin_amdgcn_s_waitcnt(0);
  int s = 0;
  bool entry = true;   // the entry drew the current cycle already
  bool have_next = false;   // zn holds this cycle's normals (wave-uniform)
  while (s < a.n_steps) {
    if (cm == 0) {     // a coordinate cycle starts
      if (!entry) {
        if (have_next) {
#pragma unroll
          for (int ii = 0; ii < M; ++ii) st.zo[ii] = st.zn[ii];
          st.fix_trunc(a, a.g0 + s, chain);
        } else {
          st.draw_cycle(a, a.g0 + s, chain);
        }
      }
      if ((cyc & (kRefreshCycles - 1)) == 0) st.refresh(a);
      ++cyc;
    }
    entry = false;
    have_next = false;
    const int nst = min(nblk - cm / ts, a.n_steps - s);   // steps in this cycle
    const int ke = min(D, cm + nst * ts);
    if (ts == 1 && cm == 0 && ke == D) {
      // software pipelining: the next cycle's Philox blocks and Box-Muller
      // pairs (state-independent) beside this cycle's dependent updates
      st.draw_raw(a, a.g0 + s + D, chain, st.zn);
      have_next = true;
      st.template cycle<true>(a, 0, D, post_mask, std::make_integer_sequence<int, D>{});
    } else
      st.template cycle<false>(a, cm, ke, post_mask, std::make_integer_sequence<int, D>{});
    s += nst;
    cm = ke == D ? 0 : ke;
  }
  st.lp = st.vprob(a, st.Q);   // (paired cycles leave it unset)
  if (st.active) {
    const int64_t c = st.c;
#pragma unroll
    for (int ii = 0; ii < M; ++ii) {
      a.x[(p * M + ii) * a.n + c] = st.xo[ii];
      if (a.moments) {
        a.msum[(p * M + ii) * a.n + c] += st.ms[ii];
        a.msq[(p * M + ii) * a.n + c] += st.mq[ii];
      }
      a.gq[(p * M + ii) * a.n + c] = st.go[ii];
    }
    if (p == 0) {
      a.lp[c] = st.lp;
      if (a.moments) a.nacc[c] += a.n_steps;
      a.gq[D * a.n + c] = st.Q;
    }
  }
}

}  // namespace

template <int D, int TGT, int PROP>
void launch_mh_spec(const KArgs &a, hipStream_t st, size_t lds) {
  const dim3 grid((unsigned)((a.n + kBlock - 1) / kBlock)), block(kBlock);
  if (a.rng == PBH_RNG_REPLAY)
    pbh_launch((mh_kernel<D, PBH_RNG_REPLAY, TGT, PROP>), grid, block,
                       lds, st, a);
  else if (a.rng == PBH_RNG_PHILOX)
    pbh_launch((mh_kernel<D, PBH_RNG_PHILOX, TGT, PROP>), grid, block,
                       lds, st, a);
  else if (a.rng == PBH_RNG_XOSHIRO)
    pbh_launch((mh_kernel<D, PBH_RNG_XOSHIRO, TGT, PROP>), grid, block,
                       lds, st, a);
  else
    pbh_launch((mh_kernel<D, PBH_RNG_PHILOX_F64, TGT, PROP>), grid,
                       block, lds, st, a);
}

// The lane-pair kernel's steady-state form applies (see mh_pair_kernel
// FULL): production Philox, thin 1, every record of the launch inside the
// trace, past step 1, log pscale, no padding lanes.  PBH_PAIR_FULL=0
// (engine: pair_full) keeps the general form.
inline bool pair_full_form(const KArgs &a) {
  return a.pair_full && a.rng == PBH_RNG_PHILOX && a.has_pred && a.thin == 1 &&
         a.pscale != PBH_PSCALE_LIN && a.tx != nullptr && a.n % 32 == 0 &&
         a.n * 8 <= (int64_t)kNoStore &&   // masked stores: kNoStore out of range
         a.g0 - a.rec_base >= 0 && a.g0 + a.n_steps - a.rec_base <= a.rec_cap;
}

// cfg1's steady-state form applies (see mh_iid_full_kernel): production
// Philox, the filtered ratio form, log pscale, thin 1, every record of the
// launch inside the trace, past step 1, no tfun / int / bound dims, no
// moments, a ufun mask of the kernel's d.  PBH_IID_FULL=0 (engine:
// iid_full) keeps the general form.
inline bool iid_full_form(const KArgs &a) {
  return a.iid_full && a.rng == PBH_RNG_PHILOX && a.simple_acc && !a.debug &&
         a.has_pred && a.thin == 1 && a.pscale != PBH_PSCALE_LIN && a.tx != nullptr &&
         !a.has_tfun && a.vint == 0 && a.bnd_on == 0 && !a.moments &&
         a.ufun < (1u << a.d) && a.n * 8 <= (int64_t)kNoStore &&   // masked stores
         (int64_t)a.n_steps * a.d * a.n * 8 <= (int64_t)kNoStore &&   // the launch's span
         a.g0 - a.rec_base >= 0 && a.g0 + a.n_steps - a.rec_base <= a.rec_cap;
}

template <int D, bool MOM>
void launch_mh_pair_m(const KArgs &a, hipStream_t st, dim3 grid, dim3 block) {
  if constexpr (!MOM) {
    if (pair_full_form(a)) {
      if (a.ploc_zero)
        pbh_launch((mh_pair_kernel<D, PBH_RNG_PHILOX, false, true, true>), grid, block, 0, st, a);
      else
        pbh_launch((mh_pair_kernel<D, PBH_RNG_PHILOX, false, false, true>), grid, block, 0, st, a);
      return;
    }
  }
  if (a.rng == PBH_RNG_REPLAY)
    pbh_launch((mh_pair_kernel<D, PBH_RNG_REPLAY, MOM>), grid, block, 0, st, a);
  else if (a.rng == PBH_RNG_PHILOX && a.ploc_zero)
    pbh_launch((mh_pair_kernel<D, PBH_RNG_PHILOX, MOM, true>), grid, block, 0, st, a);
  else if (a.rng == PBH_RNG_PHILOX)
    pbh_launch((mh_pair_kernel<D, PBH_RNG_PHILOX, MOM>), grid, block, 0, st, a);
  else if (a.rng == PBH_RNG_XOSHIRO)
    pbh_launch((mh_pair_kernel<D, PBH_RNG_XOSHIRO, MOM>), grid, block, 0, st, a);
  else if (a.rng == PBH_RNG_PHILOX_FP32)
    pbh_launch((mh_pair_kernel<D, PBH_RNG_PHILOX_FP32, MOM>), grid, block, 0, st, a);
  else
    pbh_launch((mh_pair_kernel<D, PBH_RNG_PHILOX_F64, MOM>), grid, block, 0, st, a);
}

template <int D>
void launch_mh_pair(const KArgs &a, hipStream_t st) {
  const int64_t waves = (a.n + 31) / 32;
  if (!a.moments && pair_full_form(a)) {   // FULL: 4- or 8-wave workgroups
    const int wg = a.pair_wg == kPairFullBlock ? kPairFullBlock : kBlock;
    const dim3 grid((unsigned)((waves * 64 + wg - 1) / wg)), block(wg);
    launch_mh_pair_m<D, false>(a, st, grid, block);
    return;
  }
  const dim3 grid((unsigned)((waves * 64 + kBlock - 1) / kBlock)), block(kBlock);
  if (a.moments) launch_mh_pair_m<D, true>(a, st, grid, block);
  else launch_mh_pair_m<D, false>(a, st, grid, block);
}

// The resident server (engine pbh_server_*) runs the FULL lane-pair kernel
// in 8-wave workgroups; each command must itself be a FULL launch.  check:
// report whether `a` (with the command's g0 / n_steps) qualifies and whether
// the whole grid fits the device at once (every workgroup resident: the
// server's waves never wait for one another, but a workgroup that is not
// resident would see no command until the others exit); otherwise launch.
inline bool pair_form(const KArgs &a);
template <int D>
hipError_t launch_mh_server_d(const KArgs &a, hipStream_t st, int32_t *wgs, bool check) {
  if constexpr (D % 2 == 0 && D >= 4) {
    if (!(pair_form(a) && a.pair_ok && !a.moments && pair_full_form(a) &&
          a.pair_wg == kPairFullBlock && a.srv_cmd && a.srv_done && a.srv_mail))
      return hipErrorNotSupported;
    const int64_t waves = a.n / 32;
    const int64_t grid = (waves * 64 + kPairFullBlock - 1) / kPairFullBlock;
    const void *kern = a.ploc_zero
        ? reinterpret_cast<const void *>(mh_pair_kernel<D, PBH_RNG_PHILOX, false, true, true, true>)
        : reinterpret_cast<const void *>(mh_pair_kernel<D, PBH_RNG_PHILOX, false, false, true, true>);
    int dev = 0, cus = 0, per = 0;
    hipError_t err = hipGetDevice(&dev);
    if (err == hipSuccess) err = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (err == hipSuccess)
      err = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kern, kPairFullBlock, 0);
    if (err != hipSuccess) return err;
    if ((int64_t)per * cus < grid) return hipErrorNotSupported;
    if (wgs) *wgs = (int32_t)grid;
    if (check) return hipSuccess;
    if (a.ploc_zero)
      hipLaunchKernelGGL((mh_pair_kernel<D, PBH_RNG_PHILOX, false, true, true, true>),
                         dim3((unsigned)grid), dim3(kPairFullBlock), 0, st, a);
    else
      hipLaunchKernelGGL((mh_pair_kernel<D, PBH_RNG_PHILOX, false, false, true, true>),
                         dim3((unsigned)grid), dim3(kPairFullBlock), 0, st, a);
    return hipGetLastError();
  } else {
    (void)a; (void)st; (void)wgs; (void)check;
    return hipErrorNotSupported;
  }
}

// The lane-pair kernel covers the cfg2 form: diagonal Gaussian, callable
// Gaussian delta, no ufun / prior, symmetric tran or metropolis, debug off.
inline bool pair_form(const KArgs &a) {
  return a.target == PBH_TARGET_DIAG_GAUSS && a.prop == PBH_PROP_GAUSS &&
         a.ufun == 0 && a.vint == 0 && a.bnd_on == 0 && !a.has_prior && !a.debug && !a.has_tfun &&
         a.d * a.n * 8 < (int64_t(1) << 32) &&   // 32-bit trace byte offsets
         (a.scores == PBH_SCORES_METROPOLIS ||
          (a.scores == PBH_SCORES_HASTINGS && a.tran_sym &&
           a.tran_kind == PBH_TRAN_CONST));
}

// The GMM lane-pair kernel: production Philox, the filtered ratio form, no
// ufun / prior / debug records.
inline bool gmm_pair_form(const KArgs &a) {
  return a.rng == PBH_RNG_PHILOX && a.simple_acc && a.pair_ok && a.ufun == 0 &&
         a.vint == 0 && a.bnd_on == 0 && !a.has_prior && !a.debug && !a.has_tfun &&
         (a.d > 4 ? a.d : 4) * a.n * 8 < (int64_t(1) << 32);   // 32-bit trace byte
                                                               // offsets (quad: 4 rows)
}

// The quad kernel's steady-state form applies (see mh_gmm_quad_kernel FULL):
// whole 4-step groups (8-step ones where gmm_quad_full8), thin 1, every record inside the trace, past step 1,
// acc_beta = 1.  PBH_GMM_FULL=0 (engine: gmm_full) keeps the general form.
inline bool gmm_quad_full(const KArgs &a) {
  return a.gmm_full && a.has_pred && a.acc_beta == 1.0 && a.thin == 1 &&
         (int64_t)4 * a.d * a.n * 8 < (int64_t(1) << 32) &&   // group row offsets
         (int64_t)a.d * a.n * 8 <= (int64_t)kNoStore &&      // masked stores
         a.tx != nullptr && a.g0 % 4 == 0 && a.n_steps % 4 == 0 &&
         a.g0 - a.rec_base >= 0 && a.g0 + a.n_steps - a.rec_base <= a.rec_cap;
}

// FULL groups of eight steps where the launch allows (g0 and n_steps
// multiples of 8, eight record rows addressable), else of four
inline bool gmm_quad_full8(const KArgs &a) {
  return a.g0 % 8 == 0 && a.n_steps % 8 == 0 &&
         (int64_t)8 * a.d * a.n * 8 < (int64_t(1) << 32);
}

template <int D, int K, bool MOM, bool FULL, bool LOC0>
void launch_gmm_quad_k(const KArgs &a, const dim3 &grid, const dim3 &block, hipStream_t st) {
  if constexpr (FULL) {
    if (gmm_quad_full8(a)) {
      pbh_launch((mh_gmm_quad_kernel<D, K, MOM, true, LOC0, 8>), grid, block, 0, st, a);
      return;
    }
  }
  pbh_launch((mh_gmm_quad_kernel<D, K, MOM, FULL, LOC0>), grid, block, 0, st, a);
}

template <int D, bool MOM, bool FULL>
void launch_gmm_quad(const KArgs &a, const dim3 &grid, const dim3 &block,
                     hipStream_t st) {
  if constexpr (D == 2) {   // cfg5's d: the zero-loc form
    if (a.ploc_zero) {
      if (a.tn == 2)
        launch_gmm_quad_k<D, 2, MOM, FULL, true>(a, grid, block, st);
      else if (a.tn == 3)
        launch_gmm_quad_k<D, 3, MOM, FULL, true>(a, grid, block, st);
      else
        launch_gmm_quad_k<D, 4, MOM, FULL, true>(a, grid, block, st);
      return;
    }
  }
  if (a.tn == 2)
    launch_gmm_quad_k<D, 2, MOM, FULL, false>(a, grid, block, st);
  else if (a.tn == 3)
    launch_gmm_quad_k<D, 3, MOM, FULL, false>(a, grid, block, st);
  else
    launch_gmm_quad_k<D, 4, MOM, FULL, false>(a, grid, block, st);
}

template <int D>
hipError_t launch_mh_d(const KArgs &a, hipStream_t st, size_t lds) {
  if constexpr (D % 2 == 0 && D >= 4) {
    if (pair_form(a) && a.pair_ok) {
      launch_mh_pair<D>(a, st);
      return hipGetLastError();
    }
  }
  if (a.rng == PBH_RNG_PHILOX_FP32) return hipErrorInvalidValue;   // pair kernel only
  // Specialised forms: the cfg2 diagonal Gaussian with the callable Gaussian
  // delta at every d; the other example forms at the small d they use.
  if (a.target == PBH_TARGET_DIAG_GAUSS && a.prop == PBH_PROP_GAUSS) {
    launch_mh_spec<D, PBH_TARGET_DIAG_GAUSS, PBH_PROP_GAUSS>(a, st, lds);
    return hipGetLastError();
  }
  if constexpr (D <= 4) {
    if (a.target == PBH_TARGET_GMM && a.prop == PBH_PROP_GAUSS) {
      if (gmm_pair_form(a) && a.tn >= 2 && a.tn <= 4) {
        // lanes per chain: PBH_GMM_LANES = 4 (default: the quad kernel) or
        // 2 (the lane-pair kernel, rows of 32 lanes)
        const int L = a.gmm_lanes == 2 ? 2 : 4;
        const int64_t waves = (a.n + 64 / L - 1) / (64 / L);
        const dim3 grid((unsigned)((waves * 64 + kBlock - 1) / kBlock)), block(kBlock);
        if (L == 2) {
          if (a.tn == 2)
            pbh_launch((mh_gmm_lanes_kernel<D, 2, 2>), grid, block, 0, st, a);
          else if (a.tn == 3)
            pbh_launch((mh_gmm_lanes_kernel<D, 3, 2>), grid, block, 0, st, a);
          else
            pbh_launch((mh_gmm_lanes_kernel<D, 4, 2>), grid, block, 0, st, a);
        } else if (gmm_quad_full(a)) {
          if (a.moments)
            launch_gmm_quad<D, true, true>(a, grid, block, st);
          else
            launch_gmm_quad<D, false, true>(a, grid, block, st);
        } else if (a.moments) {
          launch_gmm_quad<D, true, false>(a, grid, block, st);
        } else {
          launch_gmm_quad<D, false, false>(a, grid, block, st);
        }
        return hipGetLastError();
      }
      launch_mh_spec<D, PBH_TARGET_GMM, PBH_PROP_GAUSS>(a, st, lds);
      return hipGetLastError();
    }
    if (a.target == PBH_TARGET_NORM_IID && a.prop == PBH_PROP_SPHERE) {
      if constexpr (D <= 2) {
        if (iid_full_form(a) && a.iid_pair && 2 * a.n * 8 <= (int64_t)kNoStore) {
          // lane pairs: 32 chains per wavefront
          const int64_t waves = (a.n + 31) / 32;
          const dim3 grid((unsigned)((waves * 64 + kBlock - 1) / kBlock)), block(kBlock);
          switch (a.ufun) {
            case 0: pbh_launch((mh_iid_pair_kernel<D, 0>), grid, block, 0, st, a); break;
            case 1: pbh_launch((mh_iid_pair_kernel<D, 1>), grid, block, 0, st, a); break;
            case 2: pbh_launch((mh_iid_pair_kernel<D, 2>), grid, block, 0, st, a); break;
            default: pbh_launch((mh_iid_pair_kernel<D, 3>), grid, block, 0, st, a); break;
          }
          return hipGetLastError();
        }
        if (iid_full_form(a)) {
          const dim3 grid((unsigned)((a.n + kBlock - 1) / kBlock)), block(kBlock);
          switch (a.ufun) {
            case 0: pbh_launch((mh_iid_full_kernel<D, 0>), grid, block, 0, st, a); break;
            case 1: pbh_launch((mh_iid_full_kernel<D, 1>), grid, block, 0, st, a); break;
            case 2: pbh_launch((mh_iid_full_kernel<D, 2>), grid, block, 0, st, a); break;
            default: pbh_launch((mh_iid_full_kernel<D, 3>), grid, block, 0, st, a); break;
          }
          return hipGetLastError();
        }
      }
      launch_mh_spec<D, PBH_TARGET_NORM_IID, PBH_PROP_SPHERE>(a, st, lds);
      return hipGetLastError();
    }
  }
  launch_mh_spec<D, 0, 0>(a, st, lds);
  return hipGetLastError();
}

template <int D>
hipError_t launch_gibbs_d(const KArgs &a, hipStream_t st) {
  if (gibbs_fast_form(a)) {
    // lanes per chain: PBH_GIBBS_LANES if it divides d, else the default
    // (2 for even d <= 12, measured fastest at d = 8; 4 for d = 16, whose
    // per-lane constant block 2 d^2 / L would not fit the VGPRs at L = 2)
    constexpr int LD = D % 2 ? 1 : (D <= 12 ? 2 : (D % 4 == 0 ? 4 : 2));
    const int L = (a.gibbs_lanes > 0 && D % a.gibbs_lanes == 0 &&
                   (a.gibbs_lanes == 1 || a.gibbs_lanes == 2 || a.gibbs_lanes == 4))
                      ? a.gibbs_lanes : LD;
    const int64_t waves = (a.n + 64 / L - 1) / (64 / L);
    const dim3 grid((unsigned)((waves * 64 + kBlock - 1) / kBlock)), block(kBlock);
    if constexpr (D % 4 == 0) {
      if (L == 4) {
        pbh_launch((gibbs_fast_kernel<D, 4>), grid, block, 0, st, a);
        return hipGetLastError();
      }
    }
    if constexpr (D % 2 == 0) {
      if (L == 2) {
        pbh_launch((gibbs_fast_kernel<D, 2>), grid, block, 0, st, a);
        return hipGetLastError();
      }
    }
    pbh_launch((gibbs_fast_kernel<D, 1>), grid, block, 0, st, a);
    return hipGetLastError();
  }
  const dim3 grid((unsigned)((a.n + kBlock - 1) / kBlock)), block(kBlock);
  if constexpr (D <= 16) {
    if (a.gibbs_mfma) {
      const size_t lds = (kBlock / 64) * 64 * MvnMfma<D>::S * sizeof(double);
      if (a.rng == PBH_RNG_REPLAY)
        pbh_launch((gibbs_kernel<D, PBH_RNG_REPLAY, true>), grid, block,
                           lds, st, a);
      else if (a.rng == PBH_RNG_XOSHIRO)
        pbh_launch((gibbs_kernel<D, PBH_RNG_XOSHIRO, true>), grid, block,
                           lds, st, a);
      else
        pbh_launch((gibbs_kernel<D, PBH_RNG_PHILOX, true>), grid, block,
                           lds, st, a);
      return hipGetLastError();
    }
  }
  if (a.rng == PBH_RNG_REPLAY)
    pbh_launch((gibbs_kernel<D, PBH_RNG_REPLAY, false>), grid, block, 0,
                       st, a);
  else if (a.rng == PBH_RNG_XOSHIRO)
    pbh_launch((gibbs_kernel<D, PBH_RNG_XOSHIRO, false>), grid, block, 0,
                       st, a);
  else
    pbh_launch((gibbs_kernel<D, PBH_RNG_PHILOX, false>), grid, block, 0,
                       st, a);
  return hipGetLastError();
}

#define PBH_INSTANTIATE(D)                                                  \
  template hipError_t launch_mh_d<D>(const KArgs &, hipStream_t, size_t); \
  template hipError_t launch_gibbs_d<D>(const KArgs &, hipStream_t);      \
  template hipError_t launch_mh_server_d<D>(const KArgs &, hipStream_t, int32_t *, bool);

}  // namespace pbh
