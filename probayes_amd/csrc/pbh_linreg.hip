// pbh_linreg.hip -- user-conditional (tfun) Gibbs for the conjugate linear
// regression of examples/mcmc/gibbs_linreg.py on gfx950.
//
// Reference path: SP.next -> RF.eval_tfun (rf.py:413-462) calls the user
// conditional cond_reg (gibbs_linreg.py:34-62) for ONE parameter per step,
// cycling beta_0, beta_1, y_sigma through the RF's __cond_mod (rf.py:446-452);
// gibbs scores accept every step (sp_utils.py:75-84); v.prob is the iid sum
// of norm.logpdf(y, b0 + b1 x, y_sigma) over the observations (rf.py:541-562)
// plus the joint uniform root priors (rv_utils.py:30-38).
//
// One chain per lane; the observations (x, y) are staged once per workgroup in
// LDS and read with wave-uniform addresses (LDS broadcast, no bank conflicts).
// Two arithmetic forms:
//   EXACT (REPLAY, PHILOX_F64): the reference's operations -- numpy's pairwise
//     sums over the observations, true IEEE divisions, scipy's logpdf -- so a
//     REPLAY run reproduces the reference chain from its standard draws;
//   FAST (PHILOX): the sums come from CENTRED sufficient statistics (O(1) per
//     step instead of O(n)); same conditional law.  With xbar, ybar and the
//     centred Cxx, Cxy, Cyy (host, long double, two passes):
//       sum (y - b0 - b1 x)^2 = Cyy + b1 (b1 Cxx - 2 Cxy) + n (ybar - b0 - b1 xbar)^2,
//       sum (y - b1 x) = n (ybar - b1 xbar),  sum x (y - b0) = Cxy + n xbar (ybar - b0),
//     free of the cancellation of raw moments when x or y carry a large offset.
// Draws: REPLAY reads the standard gauss / standard_gamma(a + n/2) of each step
// from rand[T][N]; PHILOX modes draw fp64 Box-Muller normals (libm in
// PHILOX_F64, LDS tables in PHILOX) and Marsaglia-Tsang gammas from
// Philox-4x32-10 keyed by (seed, global chain), counter (3-step cycle,
// attempt), so traces do not depend on sharding or launch splits.
// Trace: x [T][3][N] (chain fastest), lp [T][N]; every step is accepted.
#include <hip/hip_runtime.h>
#include <cstdint>
#include "../../include/pbhip.h"
#include "pbh_device.h"
#include "pbh_kernels.h"

namespace pbh {
namespace {

constexpr int kBlock = 256;

// scipy norm.logpdf(x, loc, scale) = _norm_logpdf((x - loc) / scale) -
// log(scale), _norm_logpdf(y) = -y**2 / 2.0 - _norm_pdf_logC.
__device__ __forceinline__ double lr_norm_logpdf(double x, double loc,
                                                 double scale, double logscale,
                                                 double logC) {
  const double y = (x - loc) / scale;
  return ((-(y * y)) / 2.0 - logC) - logscale;
}

struct LinregK {
  const double *x_obs, *y_obs;
  int64_t n_obs;
  // hyper: p0, m0, p1, m1 (prior precisions and means), alpha_post, beta0,
  // sxx = np.sum(x**2) (host), prior[3], logC, and the sufficient statistics
  // Sx, Sy, Sxy, Syy (FAST only)
  double p0, m0, p1, m1, alpha, beta, sxx, pri0, pri1, pri2, logC;
  double xbar, ybar, cxx, cxy, cyy;     // centred statistics (FAST only)
  double lo0, hi0, lo1, hi1, lo2, hi2;  // closed vsets of the root priors
  double *state;          // [3][n] beta_0, beta_1, y_sigma (in/out)
  double *lp_state;       // [n] (out)
  const double *rand;     // REPLAY [T][n]
  double *tx, *tp;        // trace [T][3][n], [T][n]
  int64_t n, chain_offset, n_steps, step0;
  uint64_t seed;
  int32_t mode;           // PBH_RNG_REPLAY / PHILOX / PHILOX_F64
};

__device__ __forceinline__ u32x4 draw_block(const LinregK &a, int64_t gc,
                                            int64_t step, uint32_t attempt) {
  return philox4x32_10(u32x4{(uint32_t)step, (uint32_t)(step >> 32), attempt,
                             0x4c524547u /* "LREG" */},
                       (uint32_t)(a.seed ^ (uint64_t)gc * 0x9E3779B97F4A7C15ull),
                       (uint32_t)((a.seed >> 32) ^ (uint64_t)(gc >> 32)) + (uint32_t)gc);
}

// Standard normal pair from one Philox block: libm Box-Muller in the
// reference-arithmetic modes, the LDS-table form (pbh_device.h) in PHILOX.
template <bool EXACT>
__device__ __forceinline__ void normal_pair(u32x4 w, const BMTables *t,
                                            double &z0, double &z1) {
  if (EXACT) box_muller(w, z0, z1);
  else box_muller_tab(w, t, z0, z1);
}

// Marsaglia & Tsang (2000) for shape a >= 1: d = a - 1/3, c = 1/sqrt(9d);
// z ~ N(0,1), v = (1 + c z)^3; accept d v when v > 0 and u < 1 - 0.0331 z^4
// (the squeeze, ~98 % of proposals at a = 31, no log) or
// log u < z^2/2 + d - d v + d log v.  Attempt k of the step's cycle uses the
// blocks (cycle, k) for z and (cycle, k + 2^16) for u, so the loop ends with
// probability 1 (capped at 64 attempts, beyond which the last proposal is
// returned).
template <bool EXACT>
__device__ __forceinline__ double mt_gamma(const LinregK &a, const BMTables *tb,
                                           int64_t gc, int64_t cycle) {
  const double d = a.alpha - 1.0 / 3.0;
  const double c = 1.0 / sqrt(9.0 * d);
  double out = d;
  for (uint32_t att = 1; att <= 64; ++att) {
    double z, z1;
    normal_pair<EXACT>(draw_block(a, gc, cycle, att), tb, z, z1);
    const double t = 1.0 + c * z;
    if (t <= 0.0) continue;
    const double v = t * t * t;
    out = d * v;
    const u32x4 w2 = draw_block(a, gc, cycle, att + 0x10000u);
    const double u = 1.0 - u01(w2.x, w2.y);  // (0, 1]
    const double z2 = z * z;
    if (u < 1.0 - 0.0331 * (z2 * z2)) break;
    const double lu = EXACT ? log(u) : fast_log(u);
    const double lv = EXACT ? log(v) : fast_log(v);
    if (lu < 0.5 * z2 + d - d * v + d * lv) break;
  }
  return out;
}

// sum_j (y_j - b0 - b1 x_j)^2 from the centred statistics
__device__ __forceinline__ double fast_ss(const LinregK &a, double nd, double b0,
                                          double b1) {
  const double r = a.ybar - b0 - b1 * a.xbar;
  return __builtin_fma(nd * r, r, __builtin_fma(b1, __builtin_fma(b1, a.cxx, -2.0 * a.cxy), a.cyy));
}

template <bool EXACT>
__global__ void __launch_bounds__(kBlock)
linreg_gibbs_kernel(LinregK a) {
  extern __shared__ double lds[];
  double *xs = lds, *ys_obs = lds + a.n_obs;
  __shared__ BMTables s_bmt;
  if (!EXACT) bm_tables_init(&s_bmt);
  if (EXACT) {
    for (int64_t j = threadIdx.x; j < a.n_obs; j += blockDim.x) {
      xs[j] = a.x_obs[j];
      ys_obs[j] = a.y_obs[j];
    }
    __syncthreads();
  }
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= a.n) return;
  const int64_t gc = a.chain_offset + c;
  const int64_t n = a.n;
  double b0 = a.state[c], b1 = a.state[n + c], sg = a.state[2 * n + c];
  const double nd = (double)a.n_obs;
  double lp = 0., z_next = 0.;
  // FAST: 1 / sg^2 and log sg change only on y_sigma steps (same values as
  // recomputing them every step)
  double yp_c = 1.0 / (sg * sg), lsg_c = EXACT ? 0. : fast_log(sg);
  for (int64_t t = 0; t < a.n_steps; ++t) {
    const int64_t step = a.step0 + t;
    const int key = (int)(step % 3);
    // Philox draws per 3-step cycle: block (cycle, 0) gives the normals of
    // the beta_0 and beta_1 steps (z0, z1); the gamma's attempts use their
    // own blocks.  A launch starting on a beta_1 step recomputes the pair.
    double z;
    const int64_t cycle = step / 3;
    if (a.mode == PBH_RNG_REPLAY) {
      z = a.rand[t * n + c];
    } else if (key == 2) {
      z = mt_gamma<EXACT>(a, &s_bmt, gc, cycle);
    } else if (key == 0 || t == 0) {
      double z0, z1;
      normal_pair<EXACT>(draw_block(a, gc, cycle, 0), &s_bmt, z0, z1);
      z = key == 0 ? z0 : z1;
      z_next = z1;
    } else {
      z = z_next;
    }
    if (key == 2) {
      // cond_beta = b + 0.5 * sum((y - b0 - b1 x)**2); 1/sqrt(gamma(a, 1/cb))
      double ss;
      if (EXACT) {
        ss = np_pairwise([&](int64_t j) {
          const double r = (ys_obs[j] - b0) - b1 * xs[j];
          return r * r;
        }, a.n_obs);
      } else {
        ss = fast_ss(a, nd, b0, b1);
      }
      const double cb = a.beta + 0.5 * ss;
      sg = 1.0 / sqrt((1.0 / cb) * z);
      if (!EXACT) {
        yp_c = 1.0 / (sg * sg);
        lsg_c = fast_log(sg);
      }
    } else {
      const double yp = EXACT ? 1.0 / (sg * sg) : yp_c;
      if (key == 0) {
        const double v = 1.0 / (a.p0 + nd * yp);
        const double s = EXACT ? np_pairwise([&](int64_t j) {
          return ys_obs[j] - b1 * xs[j]; }, a.n_obs) : nd * (a.ybar - b1 * a.xbar);
        const double m = (a.p0 * a.m0 + yp * s) * v;
        b0 = m + sqrt(v) * z;
      } else {
        const double v = 1.0 / (a.p1 + yp * a.sxx);
        const double s = EXACT ? np_pairwise([&](int64_t j) {
          return xs[j] * (ys_obs[j] - b0); }, a.n_obs)
                               : __builtin_fma(nd * a.xbar, a.ybar - b0, a.cxy);
        const double m = (a.p1 * a.m1 + yp * s) * v;
        b1 = m + sqrt(v) * z;
      }
    }
    // v.prob: sum_j norm.logpdf(y_j, b0 + b1 x_j, sg) + the root priors
    const double lsg = EXACT ? log(sg) : lsg_c;
    if (EXACT) {
      lp = np_pairwise([&](int64_t j) {
        return lr_norm_logpdf(ys_obs[j], b0 + b1 * xs[j], sg, lsg, a.logC);
      }, a.n_obs);
    } else {
      lp = -0.5 * fast_ss(a, nd, b0, b1) / (sg * sg) - nd * (a.logC + lsg);
    }
    // uniform_prob (rv_utils.py:30-38): -log L inside the vset, else
    // NEARLY_NEGATIVE_INF; added one parameter at a time
    const double q0 = (b0 >= a.lo0 && b0 <= a.hi0) ? a.pri0 : kNearlyNegInf;
    const double q1 = (b1 >= a.lo1 && b1 <= a.hi1) ? a.pri1 : kNearlyNegInf;
    const double q2 = (sg >= a.lo2 && sg <= a.hi2) ? a.pri2 : kNearlyNegInf;
    lp = ((lp + q0) + q1) + q2;
    if (a.tx) {   // uniform: the trace buffers are optional
      double *tx = a.tx + t * 3 * n;
      __builtin_nontemporal_store(b0, tx + c);
      __builtin_nontemporal_store(b1, tx + n + c);
      __builtin_nontemporal_store(sg, tx + 2 * n + c);
    }
    if (a.tp) __builtin_nontemporal_store(lp, a.tp + t * n + c);
  }
  a.state[c] = b0;
  a.state[n + c] = b1;
  a.state[2 * n + c] = sg;
  a.lp_state[c] = lp;
}

// FAST arithmetic (PHILOX): no IEEE divisions or square roots on the step's
// dependency chain -- reciprocals and inverse square roots from v_rcp_f64 /
// v_rsq_f64 with two Newton steps (within an ulp or two of the IEEE forms; the
// FAST chain is a production form, checked against the reference arithmetic
// to 1e-9 in tests/test_linreg.py):
//   beta_k:  P = p_k + yp S_k,  r = P^-1/2,  b_k = (p_k m_k + yp s) r^2 + r z
//            (v = 1/P and sqrt(v) = r of cond_reg);
//   y_sigma: w = z / cb,  sg = w^-1/2  (1/sqrt((1/cb) z));
//   v.prob:  -ss yp / 2 - n (logC + log sg),  yp = 1/sg^2.
// yp and log sg are pure functions of sg (cached between y_sigma steps and
// recomputed at launch entry), so launch splits give identical chains.

struct FastState {
  double b0, b1, sg, yp, lsg, lp;
  __device__ __forceinline__ void set_sg(double s) {
    sg = s;
    yp = rcp_nr(s * s);
    lsg = fast_log(s);
  }
};

__device__ __forceinline__ void fast_step(const LinregK &a, int key, double z,
                                          double nd, FastState &f) {
  if (key == 2) {
    const double cb = a.beta + 0.5 * fast_ss(a, nd, f.b0, f.b1);
    f.set_sg(rsq_nr(z * rcp_nr(cb)));
  } else if (key == 0) {
    const double r = rsq_nr(__builtin_fma(nd, f.yp, a.p0));
    const double s = nd * (a.ybar - f.b1 * a.xbar);
    f.b0 = __builtin_fma(r, z, (a.p0 * a.m0 + f.yp * s) * (r * r));
  } else {
    const double r = rsq_nr(__builtin_fma(f.yp, a.sxx, a.p1));
    const double s = __builtin_fma(nd * a.xbar, a.ybar - f.b0, a.cxy);
    f.b1 = __builtin_fma(r, z, (a.p1 * a.m1 + f.yp * s) * (r * r));
  }
  double lp = __builtin_fma(-0.5 * fast_ss(a, nd, f.b0, f.b1), f.yp, -nd * (a.logC + f.lsg));
  const double q0 = (f.b0 >= a.lo0 && f.b0 <= a.hi0) ? a.pri0 : kNearlyNegInf;
  const double q1 = (f.b1 >= a.lo1 && f.b1 <= a.hi1) ? a.pri1 : kNearlyNegInf;
  const double q2 = (f.sg >= a.lo2 && f.sg <= a.hi2) ? a.pri2 : kNearlyNegInf;
  f.lp = ((lp + q0) + q1) + q2;
}

// Marsaglia-Tsang attempts 2.. of a cycle (attempt 1 is drawn up front with
// the cycle's normal pair); the same blocks and tests as mt_gamma<false>.
__device__ __attribute__((noinline)) double mt_gamma_tail(const LinregK &a, const BMTables *tb,
                                                          int64_t gc, int64_t cycle,
                                                          double out) {
  const double d = a.alpha - 1.0 / 3.0;
  const double c = 1.0 / sqrt(9.0 * d);
  for (uint32_t att = 2; att <= 64; ++att) {
    double z, z1;
    normal_pair<false>(draw_block(a, gc, cycle, att), tb, z, z1);
    const double t = 1.0 + c * z;
    if (t <= 0.0) continue;
    const double v = t * t * t;
    out = d * v;
    const u32x4 w2 = draw_block(a, gc, cycle, att + 0x10000u);
    const double u = 1.0 - u01(w2.x, w2.y);
    const double z2 = z * z;
    if (u < 1.0 - 0.0331 * (z2 * z2)) break;
    if (fast_log(u) < 0.5 * z2 + d - d * v + d * fast_log(v)) break;
  }
  return out;
}

// A cycle's draws: the beta normals (block (cycle, 0)) and the y_sigma gamma,
// whose first Marsaglia-Tsang attempt (blocks (cycle, 1), (cycle, 1 + 2^16))
// is computed beside the normals (three independent Philox blocks, two
// Box-Muller pairs); a rejected first attempt continues out of line.
// A cycle's draws in two parts.  cycle_head: the beta normals (block
// (cycle, 0)) and the y_sigma gamma's first Marsaglia-Tsang proposal (blocks
// (cycle, 1), (cycle, 1 + 2^16)) -- three independent Philox blocks and two
// Box-Muller pairs, branch-free.  cycle_gamma: the attempt's squeeze / log
// tests and, when it is rejected, the remaining attempts out of line.
struct CycleHead {
  double z0, z1, t, v, u, z2;
};

__device__ __forceinline__ CycleHead cycle_head(const LinregK &a, const BMTables *tb,
                                                int64_t gc, int64_t cycle, double cm) {
  const u32x4 wn = draw_block(a, gc, cycle, 0u);
  const u32x4 wg = draw_block(a, gc, cycle, 1u);
  const u32x4 wu = draw_block(a, gc, cycle, 1u + 0x10000u);
  CycleHead h;
  double zg, zg1;
  normal_pair<false>(wn, tb, h.z0, h.z1);
  normal_pair<false>(wg, tb, zg, zg1);
  h.t = 1.0 + cm * zg;
  h.v = h.t * h.t * h.t;
  h.u = 1.0 - u01(wu.x, wu.y);
  h.z2 = zg * zg;
  return h;
}

__device__ __forceinline__ double cycle_gamma(const LinregK &a, const BMTables *tb,
                                              int64_t gc, int64_t cycle, double dg,
                                              const CycleHead &h) {
  bool done = h.t > 0.0 && h.u < 1.0 - 0.0331 * (h.z2 * h.z2);
  if (!done && h.t > 0.0)
    done = fast_log(h.u) < 0.5 * h.z2 + dg - dg * h.v + dg * fast_log(h.v);
  double g = dg * h.v;
  if (!done) g = mt_gamma_tail(a, tb, gc, cycle, h.t > 0.0 ? dg * h.v : dg);
  return g;
}

// PHILOX production kernel, one chain per lane, software-pipelined by cycle:
// while a 3-step cycle's O(1) updates run (a dependent chain), the NEXT
// cycle's Philox blocks and Box-Muller pairs are computed beside them in the
// same basic block; its gamma tests follow the updates.  Partial cycles at a
// launch's ends take the same draws one step at a time.
__global__ void __launch_bounds__(kBlock)
linreg_fast_kernel(LinregK a) {
  __shared__ BMTables s_bmt;
  bm_tables_init(&s_bmt);
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= a.n) return;
  const int64_t gc = a.chain_offset + c;
  const int64_t n = a.n;
  FastState f;
  f.b0 = a.state[c];
  f.b1 = a.state[n + c];
  f.set_sg(a.state[2 * n + c]);
  f.lp = 0.;
  const double nd = (double)a.n_obs;
  const double dg = a.alpha - 1.0 / 3.0;
  const double cm = 1.0 / sqrt(9.0 * dg);
  auto record = [&](int64_t t) {
    if (a.tx) {
      double *tx = a.tx + t * 3 * n;
      __builtin_nontemporal_store(f.b0, tx + c);
      __builtin_nontemporal_store(f.b1, tx + n + c);
      __builtin_nontemporal_store(f.sg, tx + 2 * n + c);
    }
    if (a.tp) __builtin_nontemporal_store(f.lp, a.tp + t * n + c);
  };
  int64_t t = 0;
  int64_t cycle = a.step0 / 3;
  CycleHead h = cycle_head(a, &s_bmt, gc, cycle, cm);
  double g = cycle_gamma(a, &s_bmt, gc, cycle, dg, h);
  // a launch starting inside a cycle: its remaining steps
  for (int key = (int)(a.step0 % 3); key != 0 && key < 3 && t < a.n_steps; ++key, ++t) {
    fast_step(a, key, key == 1 ? h.z1 : g, nd, f);
    record(t);
  }
  if (a.step0 % 3 != 0 && t < a.n_steps) {   // on to the next whole cycle
    ++cycle;
    h = cycle_head(a, &s_bmt, gc, cycle, cm);
    g = cycle_gamma(a, &s_bmt, gc, cycle, dg, h);
  }
  for (; t + 3 <= a.n_steps; t += 3) {
    const CycleHead hn = cycle_head(a, &s_bmt, gc, cycle + 1, cm);
    fast_step(a, 0, h.z0, nd, f);
    record(t);
    fast_step(a, 1, h.z1, nd, f);
    record(t + 1);
    fast_step(a, 2, g, nd, f);
    record(t + 2);
    ++cycle;
    h = hn;
    g = cycle_gamma(a, &s_bmt, gc, cycle, dg, h);
  }
  for (int key = 0; t < a.n_steps; ++key, ++t) {   // a trailing partial cycle
    fast_step(a, key, key == 0 ? h.z0 : h.z1, nd, f);
    record(t);
  }
  a.state[c] = f.b0;
  a.state[n + c] = f.b1;
  a.state[2 * n + c] = f.sg;
  a.lp_state[c] = f.lp;
}

__device__ __forceinline__ void lr_halves(double v, double &lo, double &hi) {
  const uint64_t u = __builtin_bit_cast(uint64_t, v);
  const auto x = __builtin_amdgcn_permlane32_swap((uint32_t)u, (uint32_t)u, false, false);
  const auto y = __builtin_amdgcn_permlane32_swap((uint32_t)(u >> 32), (uint32_t)(u >> 32), false, false);
  lo = __builtin_bit_cast(double, (uint64_t)x[0] | ((uint64_t)y[0] << 32));
  hi = __builtin_bit_cast(double, (uint64_t)x[1] | ((uint64_t)y[1] << 32));
}

// PHILOX production kernel with one chain per lane PAIR (l, l + 32): 65 536
// chains fill 2 048 wavefronts (2 per SIMD) instead of 1 024.  The draws of
// a 3-step cycle are split over the halves with one instruction stream: each
// half forms one Philox block and one Box-Muller pair -- half 0 the beta
// normals (block (cycle, 0)), half 1 the first Marsaglia-Tsang attempt
// (blocks (cycle, 1) and (cycle, 1 + 2^16)); the rare rejected attempts
// continue in mt_gamma.  Two v_permlane32_swap exchanges give every lane the
// cycle's three draws; both halves then carry the O(1) state update and split
// the stores (half 0: beta_0, beta_1; half 1: y_sigma, lp).  Draws and
// arithmetic equal linreg_fast_kernel's, so the chains are identical.
// Measured slower (1.60 vs 1.22 ms at 65 536 chains x 1 000 steps): the
// gamma half diverges from the normal half and both halves repeat the fp64
// update, which outweighs the second wavefront per SIMD.  Off by default
// (PBH_LINREG_PAIR=1).
__global__ void __launch_bounds__(kBlock)
linreg_pair_kernel(LinregK a) {
  __shared__ BMTables s_bmt;
  bm_tables_init(&s_bmt);
  const int lane = threadIdx.x & 63;
  const bool hi = lane >= 32;
  const int64_t c = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x - lane) / 2 +
                    (lane & 31);
  const bool live = c < a.n;            // dead lanes still join the swaps
  const int64_t cc = live ? c : 0;
  const int64_t gc = a.chain_offset + cc;
  const int64_t n = a.n;
  FastState f;
  f.b0 = a.state[cc];
  f.b1 = a.state[n + cc];
  f.set_sg(a.state[2 * n + cc]);
  f.lp = 0.;
  const double nd = (double)a.n_obs;
  const double d = a.alpha - 1.0 / 3.0;
  const double cm = 1.0 / sqrt(9.0 * d);
  double z0 = 0., z1 = 0., g = 0.;
  for (int64_t t = 0; t < a.n_steps; ++t) {
    const int64_t step = a.step0 + t;
    const int key = (int)(step % 3);
    const int64_t cycle = step / 3;
    if (key == 0 || t == 0) {
      double p0, p1;
      normal_pair<false>(draw_block(a, gc, cycle, hi ? 1u : 0u), &s_bmt, p0, p1);
      double gv = p0;
      if (hi) {
        // attempt 1 of mt_gamma, then the rest of its loop if rejected
        const double tt = 1.0 + cm * p0;
        bool done = false;
        if (tt > 0.0) {
          const double v = tt * tt * tt;
          gv = d * v;
          const u32x4 w2 = draw_block(a, gc, cycle, 1u + 0x10000u);
          const double u = 1.0 - u01(w2.x, w2.y);
          const double z2 = p0 * p0;
          done = u < 1.0 - 0.0331 * (z2 * z2) ||
                 fast_log(u) < 0.5 * z2 + d - d * v + d * fast_log(v);
        }
        if (!done) {
          double out = tt > 0.0 ? gv : d;
          for (uint32_t att = 2; att <= 64; ++att) {
            double z, zz;
            normal_pair<false>(draw_block(a, gc, cycle, att), &s_bmt, z, zz);
            const double t2 = 1.0 + cm * z;
            if (t2 <= 0.0) continue;
            const double v = t2 * t2 * t2;
            out = d * v;
            const u32x4 w3 = draw_block(a, gc, cycle, att + 0x10000u);
            const double u = 1.0 - u01(w3.x, w3.y);
            const double z2 = z * z;
            if (u < 1.0 - 0.0331 * (z2 * z2)) break;
            if (fast_log(u) < 0.5 * z2 + d - d * v + d * fast_log(v)) break;
          }
          gv = out;
        }
      }
      double lo_v, hi_v, lo_w, hi_w;
      lr_halves(gv, lo_v, hi_v);
      lr_halves(p1, lo_w, hi_w);
      z0 = lo_v; g = hi_v; z1 = lo_w;
      (void)hi_w;
    }
    const double z = key == 0 ? z0 : (key == 1 ? z1 : g);
    fast_step(a, key, z, nd, f);
    if (live) {
      if (!hi && a.tx) {
        double *tx = a.tx + t * 3 * n;
        __builtin_nontemporal_store(f.b0, tx + c);
        __builtin_nontemporal_store(f.b1, tx + n + c);
      } else if (hi) {
        if (a.tx) __builtin_nontemporal_store(f.sg, a.tx + t * 3 * n + 2 * n + c);
        if (a.tp) __builtin_nontemporal_store(f.lp, a.tp + t * n + c);
      }
    }
  }
  if (live) {
    if (!hi) {
      a.state[c] = f.b0;
      a.state[n + c] = f.b1;
    } else {
      a.state[2 * n + c] = f.sg;
      a.lp_state[c] = f.lp;
    }
  }
}

}  // namespace

int64_t linreg_max_obs() { return 8192; }  // 2 x 8192 x 8 B = 128 KB of LDS

hipError_t launch_linreg_gibbs(const LinregArgs &h, hipStream_t s) {
  LinregK a;
  a.x_obs = h.x_obs; a.y_obs = h.y_obs; a.n_obs = h.n_obs;
  a.p0 = h.hyper[0]; a.m0 = h.hyper[1]; a.p1 = h.hyper[2]; a.m1 = h.hyper[3];
  a.alpha = h.hyper[4]; a.beta = h.hyper[5]; a.sxx = h.hyper[6];
  a.pri0 = h.hyper[7]; a.pri1 = h.hyper[8]; a.pri2 = h.hyper[9];
  a.logC = h.hyper[10];
  a.lo0 = h.bounds[0]; a.hi0 = h.bounds[1]; a.lo1 = h.bounds[2];
  a.hi1 = h.bounds[3]; a.lo2 = h.bounds[4]; a.hi2 = h.bounds[5];
  a.xbar = h.stats[0]; a.ybar = h.stats[1]; a.cxx = h.stats[2];
  a.cxy = h.stats[3]; a.cyy = h.stats[4];
  a.state = h.state; a.lp_state = h.lp_state; a.rand = h.rand;
  a.tx = h.tx; a.tp = h.tp;
  a.n = h.n; a.chain_offset = h.chain_offset; a.n_steps = h.n_steps;
  a.step0 = h.step0; a.seed = h.seed; a.mode = h.mode;
  const dim3 grid((unsigned)((h.n + kBlock - 1) / kBlock)), block(kBlock);
  if (h.mode == PBH_RNG_PHILOX && h.pair) {
    const dim3 grid2((unsigned)((2 * h.n + kBlock - 1) / kBlock));
    hipLaunchKernelGGL(linreg_pair_kernel, grid2, block, 0, s, a);
  } else if (h.mode == PBH_RNG_PHILOX) {
    hipLaunchKernelGGL(linreg_fast_kernel, grid, block, 0, s, a);
  } else {
    const size_t lds = (size_t)(2 * h.n_obs) * sizeof(double);
    if (lds > 65536) {
      const hipError_t e = hipFuncSetAttribute(
          (const void *)linreg_gibbs_kernel<true>,
          hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(linreg_gibbs_kernel<true>, grid, block, lds, s, a);
  }
  return hipGetLastError();
}

}  // namespace pbh
