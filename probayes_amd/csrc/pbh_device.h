// pbh_device.h -- device arithmetic for the gfx950 MH / Gibbs kernels.
//
// Everything here is IEEE fp64 and is compiled with -ffp-contract=off so that
// each expression rounds exactly like the NumPy/SciPy expression it restates
// (replay-mode parity with the reference, SURVEY.md §7 "hard parts").
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pbh {

// constants.py:9-35 (64-bit precision)
constexpr double kNearlyPosZero = 2.2250738585072014e-308;
constexpr double kNearlyPosInf = 1.7976931348623158e+308;
constexpr double kNearlyNegInf = -1.7976931348623158e+308;
// np.log(NEARLY_POSITIVE_INF), passed in from the host (bit-identical to the
// reference's LOG_NEARLY_POSITIVE_INF) via KArgs::log_npi.

// scipy.stats._continuous_distns: _norm_pdf_C = sqrt(2 pi), _norm_pdf_logC
// = log(_norm_pdf_C); both evaluated by NumPy on the host, passed as doubles.

// ---------------------------------------------------------------------------
// Philox-4x32-10 (Salmon et al., SC'11), the production RNG.  Counter-based:
// the stream of chain c at step g is a pure function of (seed, c, g), so
// traces are identical for any sharding of chains over GPUs.
// ---------------------------------------------------------------------------
struct u32x4 { uint32_t x, y, z, w; };

__device__ __forceinline__ u32x4 philox4x32_10(u32x4 c, uint32_t k0,
                                                uint32_t k1) {
  constexpr uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
  constexpr uint32_t W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const uint64_t p0 = (uint64_t)M0 * c.x;
    const uint64_t p1 = (uint64_t)M1 * c.z;
    const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    // three-input XORs as one v_bitop3_b32 each (truth table 0x96)
    c = u32x4{(uint32_t)__builtin_amdgcn_bitop3_b32(hi1, c.y, k0, 0x96), lo1,
              (uint32_t)__builtin_amdgcn_bitop3_b32(hi0, c.w, k1, 0x96), lo0};
    k0 += W0;
    k1 += W1;
  }
  return c;
}

// The ten round keys in VGPRs (uniform values kept out of the SGPR file:
// the steady-state loops run short of SGPRs, and a uniform value the
// compiler demotes on its own costs a readfirstlane loop per buffer store).
// The v_mov is an asm so that the result counts as divergent.
struct PhiloxKeys { uint32_t k0[10], k1[10]; };
__device__ __forceinline__ uint32_t in_vgpr(uint32_t v) {
  uint32_t r;
  asm("v_mov_b32 %0, %1" : "=v"(r) : "s"(v));
  return r;
}
__device__ __forceinline__ double in_vgpr_f64(double v) {
  const uint64_t b = __builtin_bit_cast(uint64_t, v);
  return __builtin_bit_cast(double, ((uint64_t)in_vgpr((uint32_t)(b >> 32)) << 32) |
                                        in_vgpr((uint32_t)b));
}
__device__ __forceinline__ PhiloxKeys philox_keys_v(uint32_t k0, uint32_t k1) {
  PhiloxKeys k;
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    k.k0[i] = in_vgpr(k0 + (uint32_t)i * 0x9E3779B9u);
    k.k1[i] = in_vgpr(k1 + (uint32_t)i * 0xBB67AE85u);
  }
  return k;
}
// philox4x32_10 on precomputed round keys (the same bijection)
__device__ __forceinline__ u32x4 philox4x32_10_rk(u32x4 c, const PhiloxKeys &k) {
  constexpr uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const uint64_t p0 = (uint64_t)M0 * c.x;
    const uint64_t p1 = (uint64_t)M1 * c.z;
    const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    c = u32x4{(uint32_t)__builtin_amdgcn_bitop3_b32(hi1, c.y, k.k0[i], 0x96), lo1,
              (uint32_t)__builtin_amdgcn_bitop3_b32(hi0, c.w, k.k1[i], 0x96), lo0};
  }
  return c;
}

// xoshiro128** (Blackman & Vigna 2018): 128-bit state, 32-bit outputs,
// passes BigCrush; ~10 full-rate integer ops per word against ~55 mixed-rate
// ops per 4 words of Philox-4x32-10 (20 of them v_mad_u64_u32).  One
// independent stream per chain (per lane half), seeded by SplitMix64.
struct Xo { uint32_t s0, s1, s2, s3; };

__device__ __forceinline__ uint32_t rotl32(uint32_t x, int k) {
  return (x << k) | (x >> (32 - k));
}

__device__ __forceinline__ uint32_t xo_next(Xo &s) {
  const uint32_t r = rotl32(s.s1 * 5u, 7) * 9u;
  const uint32_t t = s.s1 << 9;
  s.s2 ^= s.s0;
  s.s3 ^= s.s1;
  s.s1 ^= s.s2;
  s.s0 ^= s.s3;
  s.s2 ^= t;
  s.s3 = rotl32(s.s3, 11);
  return r;
}

__host__ __device__ __forceinline__ uint64_t splitmix64(uint64_t &z) {
  uint64_t x = (z += 0x9E3779B97F4A7C15ull);
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

// 53-bit double in [0, 1) from two words, the same construction as NumPy's
// legacy random_sample: ((a >> 5) * 2^26 + (b >> 6)) / 2^53.
__device__ __forceinline__ double u01(uint32_t a, uint32_t b) {
  return ((double)(a >> 5) * 67108864.0 + (double)(b >> 6)) *
         (1.0 / 9007199254740992.0);
}

// Two standard normals from one Philox block (Box-Muller, sincospi form).
__device__ __forceinline__ void box_muller(u32x4 w, double &z0, double &z1) {
  const double u1 = 1.0 - u01(w.x, w.y);  // (0, 1]
  const double u2 = u01(w.z, w.w);
  const double r = sqrt(-2.0 * log(u1));
  double s, c;
  sincospi(2.0 * u2, &s, &c);
  z0 = r * c;
  z1 = r * s;
}

// fp64 log of a positive normal double (the Box-Muller magnitude takes u in
// [2^-53, 1]): u = 2^e m with m in [sqrt(1/2), sqrt(2)), log m = 2 atanh(t),
// t = (m - 1) / (m + 1), |t| <= 0.1716, 12 series terms (truncation
// < 1e-17); ~35 VALU against ~100 for the general libm log (special cases,
// denormals).  Within 2 ulp.
__device__ __forceinline__ double log_unit(double u) {
  const uint64_t b = __builtin_bit_cast(uint64_t, u);
  int e = (int)((b >> 52) & 0x7FF) - 1023;
  double m = __builtin_bit_cast(double, (b & 0x000FFFFFFFFFFFFFull) |
                                            0x3FF0000000000000ull);
  const bool big = m > 1.4142135623730951;
  m = big ? m * 0.5 : m;
  e += big ? 1 : 0;
  const double t = (m - 1.0) / (m + 1.0);
  const double s = t * t;
  double p = 1.0 / 23.0;
  p = __builtin_fma(p, s, 1.0 / 21.0);
  p = __builtin_fma(p, s, 1.0 / 19.0);
  p = __builtin_fma(p, s, 1.0 / 17.0);
  p = __builtin_fma(p, s, 1.0 / 15.0);
  p = __builtin_fma(p, s, 1.0 / 13.0);
  p = __builtin_fma(p, s, 1.0 / 11.0);
  p = __builtin_fma(p, s, 1.0 / 9.0);
  p = __builtin_fma(p, s, 1.0 / 7.0);
  p = __builtin_fma(p, s, 1.0 / 5.0);
  p = __builtin_fma(p, s, 1.0 / 3.0);
  p = __builtin_fma(p, s, 1.0);
  const double lm = 2.0 * t * p;
  const double de = (double)e;
  return __builtin_fma(de, 6.93147180369123816490e-01,
                       __builtin_fma(de, 1.90821492927058770002e-10, lm));
}

// fp64 log of any double for the production paths: log_unit's series on
// positive normal numbers; zero, negatives, denormals, inf and NaN take the
// libm log (a divergent branch that is never entered for model values).
__device__ __forceinline__ double fast_log(double x) {
  const bool normal = x >= 2.2250738585072014e-308 && x <= 1.7976931348623157e308;
  double r = log_unit(normal ? x : 1.0);
  if (!normal) r = log(x);
  return r;
}

// Table-driven fp64 Box-Muller for the Gibbs production kernel: log and
// (sin, cos)(2 pi u) from small LDS tables plus short polynomials.
//   log u = e ln2 + log c_j + log1p(r), c_j = 1 + j/128 (top 7 mantissa
//           bits), r = m / c_j - 1 in [0, 1/128): degree 7 (truncation 2e-18);
//           in [1/2, 1) the table holds log(c_j / 2) itself (no cancellation
//           against ln 2), and above 1 - 1/128 the series takes r = u - 1
//           (exact) so that log u keeps its relative accuracy as u -> 1;
//   (sin, cos)(2 pi u) = rotation of the table angle j / 256 turn by
//           theta = 2 pi (u - j/256) < 0.0246: degrees 7 / 8.
// Values within a few ulp of the libm form (tests/test_gpu_normals.py).
struct BMTables {
  double logc[128], logh[128], invc[128], sn[256], cs[256];
};

__device__ __forceinline__ void bm_tables_init(BMTables *t) {
  for (int i = threadIdx.x; i < 256; i += blockDim.x) {
    if (i < 128) {
      const double c = 1.0 + i / 128.0;
      t->logc[i] = log(c);
      t->logh[i] = log(0.5 * c);
      t->invc[i] = 1.0 / c;
    }
    double sv, cv;
    sincospi(i / 128.0, &sv, &cv);
    t->sn[i] = sv;
    t->cs[i] = cv;
  }
  __syncthreads();
}

__device__ __forceinline__ double log_tab(double u, const BMTables *t) {
  const uint64_t b = __builtin_bit_cast(uint64_t, u);
  const int e = (int)((b >> 52) & 0x7FF) - 1023;
  const uint64_t mb = b & 0x000FFFFFFFFFFFFFull;
  const int j = (int)(mb >> 45);
  const double m = __builtin_bit_cast(double, mb | 0x3FF0000000000000ull);
  const bool near1 = u > 0.9921875;   // 1 - 1/128
  const double r = near1 ? u - 1.0 : __builtin_fma(m, t->invc[j], -1.0);
  double p = 1.0 / 7.0;
  p = __builtin_fma(p, r, -1.0 / 6.0);
  p = __builtin_fma(p, r, 1.0 / 5.0);
  p = __builtin_fma(p, r, -1.0 / 4.0);
  p = __builtin_fma(p, r, 1.0 / 3.0);
  p = __builtin_fma(p, r, -0.5);
  const double l1p = __builtin_fma(p * r, r, r);
  const double de = (double)e;
  const double base = e == -1 ? t->logh[j]
                              : __builtin_fma(de, 6.93147180369123816490e-01,
                                              __builtin_fma(de, 1.90821492927058770002e-10,
                                                            t->logc[j]));
  return near1 ? l1p : base + l1p;
}

__device__ __forceinline__ void sincos_tab(double u, const BMTables *t,
                                           double &sn, double &cs) {
  const int j = (int)(u * 256.0);
  const double th = (u - j * (1.0 / 256.0)) * 6.283185307179586;
  const double f = th * th;
  double ps = -1.9841269841269841270e-04;               // -1/7!
  ps = __builtin_fma(ps, f, 8.3333333333333333333e-03);  //  1/5!
  ps = __builtin_fma(ps, f, -1.6666666666666666667e-01); // -1/3!
  const double st = __builtin_fma(ps * f, th, th);
  double pc = 2.4801587301587301587e-05;                 //  1/8!
  pc = __builtin_fma(pc, f, -1.3888888888888888889e-03); // -1/6!
  pc = __builtin_fma(pc, f, 4.1666666666666666667e-02);  //  1/4!
  pc = __builtin_fma(pc, f, -0.5);                       // -1/2!
  const double ct = __builtin_fma(pc, f, 1.0);
  const double sj = t->sn[j], cj = t->cs[j];
  sn = __builtin_fma(sj, ct, cj * st);
  cs = __builtin_fma(cj, ct, -(sj * st));
}

__device__ __forceinline__ void box_muller_tab(u32x4 w, const BMTables *t,
                                               double &z0, double &z1) {
  const double u1 = 1.0 - u01(w.x, w.y);  // (0, 1]
  const double u2 = u01(w.z, w.w);
  const double r = sqrt(-2.0 * log_tab(u1, t));
  double s, c;
  sincos_tab(u2, t, s, c);
  z0 = r * c;
  z1 = r * s;
}

// ---------------------------------------------------------------------------
// Production fp64 normals (PBH_RNG_PHILOX, PBH_RNG_XOSHIRO): Box-Muller on
// 96 random bits per pair (the reference draws fp64 normals: NumPy's legacy
// polar gauss on 53-bit uniforms behind scipy norm.rvs,
// examples/mcmc/mcmc_prob2.py:31).  Three 32-bit words (a, b, c) give
//   u1 = (k1 + 1/2) 2^-52 in (0, 1), k1 = b[31:12]:a    (never 0 or 1;
//        the largest radius is sqrt(2 ln 2^53) = 8.57),
//   alpha = (J + c 2^-32) 2 pi / 1024,  J = b[11:2]      (a full turn, 42
//        bits of angle; b[1:0] unused),
//   z0 = r cos(alpha), z1 = r sin(alpha), r = sqrt(-2 ln u1).
//   E = -2 ln u1 = e (-2 ln 2) + T_j + r q(r): u1 = m 2^e with m in [1/2, 1)
//             (v_frexp_mant / v_frexp_exp), c_j = m rounded to 10 fraction
//             bits (c_j = (1024 + j) / 2048, j in [0, 1024]), T_j = -2 ln c_j,
//             r = (m - c_j) / c_j with one rounding (m - c_j is exact),
//             |r| <= 2^-11, q(r) = -2 log1p(r) / r to degree 4 (truncation
//             r^5 / 6 < 2^-58 relative); u1 -> 1 takes c = 1 and T = 0, so E
//             keeps its relative accuracy there;
//   sqrt    = v_rsq_f64 + one third-order (Goldschmidt) correction;
//   (sin, cos)(alpha) = table angle J rotated by theta < pi/512: sin degree
//             5, cos degree 4 (truncations 2e-19 relative, 1e-18 absolute).
// The bit positions make every index one VALU op: the hi word of 1 + k1
// 2^-52 is v_alignbit(0x3FF, b, 12), the sin/cos row's byte offset 4 J is
// b & 0xFFC (the table is four arrays of 32-bit words: sin lo, sin hi, cos
// lo, cos hi), the log row's byte offset is a v_bfe of c_j's hi word.
// Tables (host-computed in long double, pbh_dispatch.cpp bm64_tables) live
// in LDS: 1024 {sin, cos} values (the full turn, exact quadrant symmetry) at
// offset 0 -- so the two ds_read2st64_b32 take the row offset b & 0xFFC as
// is -- then 1025 {-2 ln c_j, 1/c_j} pairs (their base is the ds_read_b128's
// immediate offset) and the exp2 table, 33 KB.  About 35 VALU per pair.  A 128-bit Philox block carries one pair and a 32-bit word
// (the threshold lead of the one-lane and lane-group kernels); the lane-pair
// kernel packs 5 pairs and two 16-bit leads into 4 blocks.  Accuracy:
// tests/test_gpu_normals.py (libm form, NumPy).
// ---------------------------------------------------------------------------
// Two waves share each SIMD in the steady-state kernels, and the SIMD's
// arbiter issues the OLDER wave first among equal priorities: left alone, the
// first workgroup generation finishes a 250-step cfg2 launch at 175 us and the
// second runs on by itself, at one wave per SIMD, until 264 us
// (profiles/r03_phase_*, scripts/phase_probe.py).  Alternating the priority
// between the SIMD's two wave slots on a shared clock (the 100 MHz real-time
// counter; a wave's own step count would drift out of phase with the other
// wave's) every ~20 us (PBH_FAIR=11, the engine's default) hands the lead
// back and forth, so both end together: cfg2 250-step launches 0.59 -> 0.63
// of HBM, cfg5's quad kernel 1 071 -> 956 us.  Short periods (1.3 us) and
// workgroup barriers keep the waves in phase and lose the leader / filler
// interleave (r03_phase_quarters.txt).
__device__ __forceinline__ uint32_t simd_wave_slot() {
  return __builtin_amdgcn_s_getreg(4 | (0 << 6) | (3 << 11));   // HW_ID.WAVE_ID
}
__device__ __forceinline__ uint32_t simd_id() {
  return __builtin_amdgcn_s_getreg(4 | (4 << 6) | (1 << 11));    // HW_ID.SIMD_ID
}
__device__ __forceinline__ void fair_prio(uint32_t phase) {
  if (phase & 1u) __builtin_amdgcn_s_setprio(1);
  else __builtin_amdgcn_s_setprio(0);
}

// Probe build only (-DPBH_PHASES, scripts/phase_probe.sh): per-wave
// real-time stamps (100 MHz) at the FULL pair kernel's phase boundaries.
#ifdef PBH_PHASES
#define PBH_PHASE_DECL uint64_t pbh_tph[8] = {0, 0, 0, 0, 0, 0, 0, 0}
#define PBH_PHASE(k) (pbh_tph[k] = __builtin_amdgcn_s_memrealtime())
// the loop's quarter points (i of n iterations) into words 5, 6, 7
// word 4's bits 40..63: a 24-bit tag of the kernel's choosing
#define PBH_PHASE_TAG(v) (pbh_tph[4] = (uint64_t)(v))
#define PBH_PHASE_Q(i, n)                                                     \
  do {                                                                        \
    if ((i) == (n) / 4) PBH_PHASE(5);                                         \
    if ((i) == (n) / 2) PBH_PHASE(6);                                         \
    if ((i) == 3 * (n) / 4) PBH_PHASE(7);                                     \
  } while (0)
// lane 0 of each wave writes its stamps, HW_ID and XCC_ID (8 words per wave)
#define PBH_PHASE_STORE(buf, wave, lane)                                      \
  do {                                                                        \
    if ((lane) == 0 && (buf)) {                                               \
      uint64_t *pb_ = reinterpret_cast<uint64_t *>(const_cast<double *>(buf)) \
                      + (wave) * 8;                                           \
      for (int k_ = 0; k_ < 8; ++k_) pb_[k_] = pbh_tph[k_];                   \
      pb_[4] = (uint64_t)__builtin_amdgcn_s_getreg(4 | (0 << 6) | (31 << 11)) \
               | ((uint64_t)__builtin_amdgcn_s_getreg(20 | (0 << 6) | (3 << 11)) << 32) \
               | ((pbh_tph[4] & 0xFFFFFFull) << 40);                           \
    }                                                                         \
  } while (0)
#else
#define PBH_PHASE_DECL
#define PBH_PHASE(k) ((void)0)
#define PBH_PHASE_Q(i, n) ((void)0)
#define PBH_PHASE_TAG(v) ((void)0)
#define PBH_PHASE_STORE(buf, wave, lane) ((void)0)
#endif

constexpr int kBm64LogN = 1025, kBm64ScN = 1024, kExp2N = 64;
// layout in doubles: sin/cos words [0, 2048), log rows [2048, 4098), exp2
constexpr int kBm64LogOff = 2 * kBm64ScN;                  // {-2 ln c, 1/c} rows
constexpr int kBm64ExpOff = kBm64LogOff + 2 * kBm64LogN;   // 2^(i/64) table
constexpr int kBm64Doubles = kBm64ExpOff + kExp2N;         // 4162 doubles

__device__ __forceinline__ uint32_t hi32(double v) {
  return (uint32_t)(__builtin_bit_cast(uint64_t, v) >> 32);
}
__device__ __forceinline__ uint32_t lo32(double v) {
  return (uint32_t)__builtin_bit_cast(uint64_t, v);
}
__device__ __forceinline__ double from_words(uint32_t hi, uint32_t lo) {
  return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}

// Copies the global table block (pbh_engine's bm64_tables) into LDS; every
// thread of the workgroup takes part, then one barrier.
// All of a thread's loads are issued before the first LDS write (one
// global-memory round trip per launch instead of one per 4 KB slice: the
// rolled loop waited for each load in turn, several microseconds of every
// short launch).  Complete for blocks of >= 256 threads (all kernels here
// run 256).
// The same in two halves: bm64_issue puts this thread's global loads in
// flight (registers), bm64_commit writes them to LDS and syncs.  Loads the
// caller issues in between (the chain state) are waited for only when used:
// the ds_writes wait for the table's loads alone (vmcnt counts in order).
struct Bm64Regs {
  static constexpr int N2 = kBm64Doubles / 2, T = 256, R = N2 / T;   // 8 full rounds
  static_assert(N2 - R * T <= T, "one partial round");
  double2 v[R], w;
};
__device__ __forceinline__ void bm64_issue(const double *g, Bm64Regs &r) {
  constexpr int N2 = Bm64Regs::N2, T = Bm64Regs::T, R = Bm64Regs::R;
  const int t = (int)(threadIdx.x & (T - 1));   // >= 256 threads: duplicates
  const double2 *src = reinterpret_cast<const double2 *>(g);
#pragma unroll
  for (int k = 0; k < R; ++k) r.v[k] = src[t + k * T];
  r.w = t < N2 - R * T ? src[t + R * T] : double2{0., 0.};
}
__device__ __forceinline__ void bm64_commit(double *lds, const Bm64Regs &r) {
  constexpr int N2 = Bm64Regs::N2, T = Bm64Regs::T, R = Bm64Regs::R;
  const int t = (int)(threadIdx.x & (T - 1));
  double2 *dst = reinterpret_cast<double2 *>(lds);
#pragma unroll
  for (int k = 0; k < R; ++k) dst[t + k * T] = r.v[k];
  if (t < N2 - R * T) dst[t + R * T] = r.w;
  __syncthreads();
}
__device__ __forceinline__ void bm64_load(double *lds, const double *g) {
  Bm64Regs r;
  bm64_issue(g, r);
  bm64_commit(lds, r);
}

// -2 ln(m 2^e) + offsets for the log table: x = m 2^e (frexp, m in [1/2, 1)),
// c = m rounded to 10 fraction bits, returns r = (m - c) / c and the table
// row {-2 ln c, 1/c}; q4 is -2 log1p(r) / r to degree 4.
struct LogTerm { double r, T; int e; };

// Timing-only A/B build (never shipped, wrong numbers):
// -DPBH_LDS_AB replaces every table lookup's LDS offset by a lane-based one
// (lane x the entry size: consecutive entries, no two lanes of a lookup in
// the same bank) that still depends on the original offset (v_and with 0,
// v_add: one VALU more per lookup, so the loads stay in place).  The values
// read are wrong but valid table entries, so the chains keep their ranges and
// the filters their rare exact paths.  (A wave-uniform offset through
// v_readfirstlane serialised every lookup on an SGPR round trip: 0.27 ->
// 0.39 ms per 250-step launch, not a conflict measurement.)
#ifdef PBH_LDS_AB
template <int ENTRY>
__device__ __forceinline__ uint32_t lds_ab(uint32_t off) {
  uint32_t r;
  asm volatile("v_and_b32 %0, 0, %1\n\tv_add_u32 %0, %0, %2"
               : "=&v"(r) : "v"(off), "v"((uint32_t)(threadIdx.x & 63u) * ENTRY));
  return r;
}
#else
template <int ENTRY>
__device__ __forceinline__ uint32_t lds_ab(uint32_t off) { return off; }
#endif

__device__ __forceinline__ uint32_t bfe_6_15(uint32_t v) {
  // v_bfe_u32 v, 6, 15 as written (LLVM turns a bfe of a masked value into a
  // shift and a second mask, one VALU more)
  uint32_t r;
  asm("v_bfe_u32 %0, %1, 6, 15" : "=v"(r) : "v"(v));
  return r;
}

__device__ __forceinline__ LogTerm log_term(double x, const double *tab) {
  const double m = __builtin_amdgcn_frexp_mant(x);                 // [1/2, 1)
  const int e = __builtin_amdgcn_frexp_exp(x);
  const uint32_t ch = (hi32(m) + 0x200u) & 0xFFFFFC00u;            // c (hi word)
  // row j = (ch - 0x3FE00000) >> 10: byte offset 16 j = bits [20:6] of ch
  const double2 lt = *reinterpret_cast<const double2 *>(
      reinterpret_cast<const char *>(tab + kBm64LogOff) + lds_ab<16>(bfe_6_15(ch)));
  return LogTerm{(m - from_words(ch, 0u)) * lt.y, lt.x, e};
}

__device__ __forceinline__ double q4(double r) {
  double q = __builtin_fma(r, -0.4, 0.5);
  q = __builtin_fma(q, r, -2.0 / 3.0);
  q = __builtin_fma(q, r, 1.0);
  return __builtin_fma(q, r, -2.0);
}

__device__ __forceinline__ void bm96_pair(uint32_t a, uint32_t b, uint32_t c,
                                          const double *tab, double &z0,
                                          double &z1) {
  // ---- E = -2 ln u1 ----
  const double d1 = from_words(__builtin_amdgcn_alignbit(0x3FFu, b, 12), a);   // [1, 2)
  const double u1 = d1 - (1.0 - 0x1p-53);                          // exact (Sterbenz)
  const LogTerm lt = log_term(u1, tab);
  const double de = (double)lt.e;
  const double base = __builtin_fma(de, -2.0 * 6.93147180369123816490e-01,
                                    __builtin_fma(de, -2.0 * 1.90821492927058770002e-10, lt.T));
  const double E = __builtin_fma(lt.r, q4(lt.r), base);             // > 0
  // ---- sqrt(E) = t (1 + e/2 + 3e^2/8 + ...), t = E y, e = 1 - E y^2, y =
  // v_rsq_f64(E) (|e| < 2^-21): the truncation 5e^3/16 < 2^-64, the rounding
  // of t enters e and cancels to first order: within an ulp, 5 VALU + rsq ----
  const double yr = __builtin_amdgcn_rsq(E);
  const double tt = E * yr;
  const double ee = __builtin_fma(-tt, yr, 1.0);
  const double rr = __builtin_fma(tt * ee, __builtin_fma(ee, 0.375, 0.5), tt);
  // ---- (sin, cos) of the full-turn angle ----
  const char *sct = reinterpret_cast<const char *>(tab) + lds_ab<4>(b & 0xFFCu);
  const uint32_t *scw = reinterpret_cast<const uint32_t *>(sct);
  const double2 sc{from_words(scw[kBm64ScN], scw[0]),
                   from_words(scw[3 * kBm64ScN], scw[2 * kBm64ScN])};
  constexpr double kTh = 3.14159265358979323846 * 0x1p-41;   // 2 pi 2^-10 2^-32
  const double th = (double)c * kTh;                          // [0, pi/512)
  const double f = th * th;
  const double ps = __builtin_fma(f, 8.3333333333333333333e-03, -1.6666666666666666667e-01);
  const double st = __builtin_fma(th * f, ps, th);
  const double ct = __builtin_fma(f, __builtin_fma(f, 4.1666666666666666667e-02, -0.5), 1.0);
  const double sn = __builtin_fma(sc.x, ct, sc.y * st);
  const double cs = __builtin_fma(sc.y, ct, -(sc.x * st));
  z0 = rr * cs;
  z1 = rr * sn;
}

// ln S of a positive normal double from the same LDS log table: S = m 2^e,
// ln S = e ln 2 - (T_j + r q(r)) / 2 (log_term).  About 18 VALU; absolute
// error ~1e-16 (relative near S = 1 is not kept: used for log-sum-exp sums
// S in [1, K], added to the max).
__device__ __forceinline__ double ln_tab(double S, const double *tab) {
  const LogTerm lt = log_term(S, tab);
  const double de = (double)lt.e;
  const double h = -0.5 * __builtin_fma(lt.r, q4(lt.r), lt.T);
  return __builtin_fma(de, 6.93147180369123816490e-01,
                       __builtin_fma(de, 1.90821492927058770002e-10, h));
}

// exp(y) for y <= 0 (log-sum-exp terms): y = (n + i/64) ln 2 + r, |r| <=
// ln2 / 128, exp(y) = 2^n 2^(i/64) poly5(r) from the 64-entry LDS table.
// About 16 VALU, within 2 ulp; y < -745 gives 0.
// (in two halves, exp_tab_pre / exp_tab_fin, so that a caller with several
// independent terms can issue every table read before the first is used)
struct ExpPre {
  double p, t;
  int ki;
};
__device__ __forceinline__ ExpPre exp_tab_pre(double y, const double *tab) {
  y = __builtin_fmax(y, -746.0);                             // -inf -> 0
  const double k = __builtin_rint(y * 92.332482616893656);   // 64 / ln 2
  // ln2/64 = hi + lo, hi with 36 significant bits: k hi exact for |k| < 2^17
  double r = __builtin_fma(-k, 0.010830424696223417, y);
  r = __builtin_fma(-k, 2.572804622327669e-14, r);
  double p = __builtin_fma(r, 1.0 / 120.0, 1.0 / 24.0);
  p = __builtin_fma(p, r, 1.0 / 6.0);
  p = __builtin_fma(p, r, 0.5);
  p = __builtin_fma(p, r, 1.0);
  p = __builtin_fma(p, r, 1.0);
  const int ki = (int)k;
  return ExpPre{p, tab[kBm64ExpOff + lds_ab<1>((uint32_t)ki & 63u)], ki};
}
__device__ __forceinline__ double exp_tab_fin(const ExpPre &e) {
  return __builtin_ldexp(e.t * e.p, e.ki >> 6);
}
__device__ __forceinline__ double exp_tab(double y, const double *tab) {
  return exp_tab_fin(exp_tab_pre(y, tab));
}

// Production log / exp of a ufun dimension (x' = exp(log x + delta)) from the
// same LDS tables: ln_tab's ~18 VALU against fast_log's ~35, exp_tab's ~16
// against fast_exp's ~20.  Only the absolute accuracy of log x matters here
// (it is exponentiated again): ~1e-16.  log: positive normal x through the
// table, anything else through libm (a divergent branch no model value
// takes); exp: any y, NaN propagated, +inf above 709.78, 0 below -746.
__device__ __forceinline__ double ln_ufun(double x, const double *tab) {
  const bool normal = x >= 2.2250738585072014e-308 && x <= 1.7976931348623157e308;
  double r = ln_tab(normal ? x : 1.0, tab);
  if (!normal) r = log(x);
  return r;
}
__device__ __forceinline__ double exp_ufun(double y, const double *tab) {
  const double e = exp_tab(__builtin_fmin(y, 710.0), tab);
  return y != y ? y : (y > 709.782712893384 ? __builtin_inf() : e);
}

// Trace store through a buffer resource: base = a wave-uniform (SGPR)
// pointer, voff = a loop-invariant per-lane byte offset, soff = a
// wave-uniform byte offset: no per-store VALU address arithmetic.  nt: the
// trace is write-once (aux bit 1 = nt on gfx950).
__device__ __forceinline__ void st_buf(double *base, uint32_t voff,
                                       uint32_t soff, double v) {
  typedef unsigned int u32x2_t __attribute__((__vector_size__(8)));
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc(base, 0, -1, 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2_t, v), rs,
                                        (int)voff, (int)soff, 2);
}

// The same through a resource of exactly nbytes: a lane whose voff is at or
// past nbytes writes nothing (the raw buffer range check), so a loop-
// invariant offset of kNoStore masks a lane's store without a branch.
// Callers keep nbytes <= kNoStore (the launch conditions check it).
constexpr uint32_t kNoStore = 0x80000000u;
__device__ __forceinline__ void st_buf_n(double *base, uint32_t nbytes,
                                         uint32_t voff, double v) {
  typedef unsigned int u32x2_t __attribute__((__vector_size__(8)));
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc(base, 0, (int)nbytes, 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2_t, v), rs,
                                        (int)voff, 0, 2);
}
// The same with a wave-uniform byte offset soff: the range check covers
// voff + soff (measured on gfx950, tools/ubench/soffset_range.hip), so a
// loop-invariant resource over a launch's whole span of rows takes the row
// as soff (one scalar add per step instead of a new resource per store).
__device__ __forceinline__ void st_buf_ns(double *base, uint32_t nbytes, uint32_t voff,
                                          uint32_t soff, double v) {
  typedef unsigned int u32x2_t __attribute__((__vector_size__(8)));
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc(base, 0, (int)nbytes, 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2_t, v), rs,
                                        (int)voff, (int)soff, 2);
}
__device__ __forceinline__ void st_buf32_n(uint32_t *base, uint32_t nbytes,
                                           uint32_t voff, uint32_t v) {
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc(base, 0, (int)nbytes, 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b32(v, rs, (int)voff, 0, 0);
}

// Lane selects in the VOP3 (e64) encoding.  On gfx950 the VOP2 form
// v_cndmask_b32_e32 (mask implicitly in VCC), which the compiler picks
// whenever the condition sits in VCC, issues at ~23 cycles per wave
// instruction at any occupancy, against ~5 for the e64 form reading the same
// mask -- VCC included (tools/ubench/isa_cost.hip, profiles/r02y_isa_cnd.txt).
// These helpers pin the e64 form: m is the lane mask (a ballot of the
// condition; inactive lanes' bits do not matter).
__device__ __forceinline__ uint32_t sel_u32(uint64_t m, uint32_t if0, uint32_t if1) {
  uint32_t r;
  asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(if0), "v"(if1), "s"(m));
  return r;
}
__device__ __forceinline__ double sel_f64(uint64_t m, double if0, double if1) {
  const uint64_t a = __builtin_bit_cast(uint64_t, if0), b = __builtin_bit_cast(uint64_t, if1);
  const uint32_t lo = sel_u32(m, (uint32_t)a, (uint32_t)b);
  const uint32_t hi = sel_u32(m, (uint32_t)(a >> 32), (uint32_t)(b >> 32));
  return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ float sel_f32(uint64_t m, float if0, float if1) {
  return __builtin_bit_cast(float, sel_u32(m, __builtin_bit_cast(uint32_t, if0),
                                           __builtin_bit_cast(uint32_t, if1)));
}

// A uniform prior's limits as closed ones: for every double x, x > lo is
// x >= lo_closed(lo, false) and x >= lo is x >= lo_closed(lo, true) (a NaN
// limit compares false both ways); likewise x < hi is x <= hi_closed(hi,
// false).  One compare per limit and dim in the steady-state kernels instead
// of a compare, an equality test and a wave-uniform branch on the flag.
__device__ __forceinline__ double lo_closed(double lo, bool incl) {
  if (incl || lo != lo) return lo;
  if (lo == __builtin_inf()) return __builtin_nan("");   // x > +inf: never
  if (lo == 0.) return 0x1p-1074;                        // x > 0: x >= the least denormal
  const int64_t b = __builtin_bit_cast(int64_t, lo);
  return __builtin_bit_cast(double, lo > 0. ? b + 1 : b - 1);   // the next double up
}
__device__ __forceinline__ double hi_closed(double hi, bool incl) {
  if (incl || hi != hi) return hi;
  if (hi == -__builtin_inf()) return __builtin_nan("");
  if (hi == 0.) return -0x1p-1074;
  const int64_t b = __builtin_bit_cast(int64_t, hi);
  return __builtin_bit_cast(double, hi > 0. ? b - 1 : b + 1);   // the next double down
}

// 1/x and 1/sqrt(x) for positive normal x: the hardware v_rcp_f64 /
// v_rsq_f64 estimate and two Newton steps (within an ulp or two of the IEEE
// forms), for the production (non-replay) arithmetic.
__device__ __forceinline__ double rcp_nr(double x) {
  double r = __builtin_amdgcn_rcp(x);
  r = __builtin_fma(__builtin_fma(-x, r, 1.0), r, r);
  return __builtin_fma(__builtin_fma(-x, r, 1.0), r, r);
}
__device__ __forceinline__ double rsq_nr(double x) {
  double y = __builtin_amdgcn_rsq(x);
  const double hx = 0.5 * x;
  y = y * __builtin_fma(-hx * y, y, 1.5);
  return y * __builtin_fma(-hx * y, y, 1.5);
}

// 16-bit store through a buffer resource (accept words of the 16-chain
// kernels); base wave-uniform as in st_buf.
__device__ __forceinline__ void st_buf16(void *base, uint32_t voff, uint16_t v) {
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc(base, 0, -1, 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b16(v, rs, (int)voff, 0, 0);
}
__device__ __forceinline__ void st_buf16(void *base, uint32_t voff, uint32_t soff,
                                         uint16_t v) {
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc(base, 0, -1, 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b16(v, rs, (int)voff, (int)soff, 0);
}

// A pointer the compiler cannot prove wave-uniform but that is: its
// first lane's value in SGPRs, so that a buffer resource built from it is
// scalar (no waterfall loop around the store).
template <typename T>
__device__ __forceinline__ T *wave_uniform(T *p) {
  const uint64_t v = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32));
  return reinterpret_cast<T *>(((uint64_t)hi << 32) | lo);
}

// Legacy fp32 normals (PBH_RNG_PHILOX_FP32, the round-1 production form, kept
// as a labelled comparison): two standard-normal pairs per Philox
// block from the hardware fp32 transcendentals (v_log_f32, v_sin_f32,
// v_cos_f32), widened to fp64.  The magnitude r = sqrt(-2 ln u1) uses 24-bit
// u1 in (0, 1] (|z| <= 5.77) and the angle lives in one quadrant; each
// coordinate's sign is an independent Philox bit, so the proposal density is
// EXACTLY symmetric, f(delta) = f(-delta) -- the only property the random-walk
// MH acceptance relies on (sp_utils.py:56 drops q).  Its precision (~2^-22
// relative) affects only proposal shape, never the fp64 chain arithmetic.
__device__ __forceinline__ double fast_normal_pair(uint32_t wu, uint32_t wa,
                                                   double &z1) {
  const float u1 = (float)((wu >> 8) + 1u) * 5.9604644775390625e-08f;  // 2^-24
  const float rev = (float)(wa >> 8) * 1.4901161193847656e-08f;      // [0, 1/4)
  const float r = __builtin_amdgcn_sqrtf(-1.3862943611198906f *    // -2 ln 2
                                         __builtin_amdgcn_logf(u1)); // log2
  const float c = r * __builtin_amdgcn_cosf(rev);   // cos(2 pi rev)
  const float s = r * __builtin_amdgcn_sinf(rev);
  const uint64_t s0 = (uint64_t)(wa & 1u) << 63, s1 = (uint64_t)(wa & 2u) << 62;
  z1 = __builtin_bit_cast(double, __builtin_bit_cast(uint64_t, (double)s) ^ s1);
  return __builtin_bit_cast(double, __builtin_bit_cast(uint64_t, (double)c) ^ s0);
}

// One production normal from two words (the cosine half of fast_normal_pair),
// for odd per-lane draw counts.  Bits used: wu[31:8], wa[31:8], wa[0]; the
// 14 bits wu[7:0], wa[6:1] are returned in spare (independent of the normal).
__device__ __forceinline__ double fast_normal_single(uint32_t wu, uint32_t wa,
                                                     uint32_t &spare) {
  const float u1 = (float)((wu >> 8) + 1u) * 5.9604644775390625e-08f;  // 2^-24
  const float rev = (float)(wa >> 8) * 1.4901161193847656e-08f;      // [0, 1/4)
  const float r = __builtin_amdgcn_sqrtf(-1.3862943611198906f *
                                         __builtin_amdgcn_logf(u1));
  const float c = r * __builtin_amdgcn_cosf(rev);
  spare = ((wu & 0xFFu) << 6) | ((wa >> 1) & 0x3Fu);
  const uint64_t s0 = (uint64_t)(wa & 1u) << 63;
  return __builtin_bit_cast(double, __builtin_bit_cast(uint64_t, (double)c) ^ s0);
}

// a / b for a loop-invariant b with its reciprocal rb = 1/b: one FMA
// correction of a*rb (Markstein) -- the correctly rounded quotient in all but
// rare ties; used only on the production path (parity paths divide).
__device__ __forceinline__ double div_by(double a, double b, double rb) {
  const double q = a * rb;
  const double e = __builtin_fma(-q, b, a);
  return __builtin_fma(e, rb, q);
}

// ---------------------------------------------------------------------------
// NumPy pairwise summation (numpy/_core/src/umath/loops_utils.h.src
// pairwise_sum, numpy 2.2): < 8 terms sequential from 0, <= 128 terms with
// eight interleaved accumulators, larger blocks split at n2 = n/2 - (n/2)%8.
// np.sum == this for contiguous float64 (checked in tests on the host).
// ---------------------------------------------------------------------------
template <int N>
__device__ __forceinline__ double np_sum_regs(const double (&a)[N], int n) {
  // n <= N <= 128, compile-time unrolled with wave-uniform predicates.
  if (n < 8) {
    double res = 0.;
#pragma unroll
    for (int i = 0; i < N; ++i)
      if (i < n) res += a[i];
    return res;
  }
  double r[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (j < N) ? a[j < N ? j : 0] : 0.;
  const int full = n - (n % 8);
#pragma unroll
  for (int i = 8; i < N; i += 8) {
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (i + j < N && i < full) r[j] += a[(i + j) < N ? (i + j) : 0];
  }
  double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
#pragma unroll
  for (int i = 0; i < N; ++i)
    if (i >= full && i < n) res += a[i];
  return res;
}

// Pairwise sum of f(j) for j in [0, n) with f evaluated on the fly (the iid
// observation reduction PD.prod, pd.py:368).  Leaves of <= 128 terms use the
// 8-accumulator block; the split tree is walked with an explicit stack.
template <class F>
__device__ __forceinline__ double np_leaf(F f, int64_t s, int64_t n) {
  if (n < 8) {
    double res = 0.;
    for (int64_t i = 0; i < n; ++i) res += f(s + i);
    return res;
  }
  double r0 = f(s), r1 = f(s + 1), r2 = f(s + 2), r3 = f(s + 3);
  double r4 = f(s + 4), r5 = f(s + 5), r6 = f(s + 6), r7 = f(s + 7);
  int64_t i = 8;
  for (; i < n - (n % 8); i += 8) {
    r0 += f(s + i);
    r1 += f(s + i + 1);
    r2 += f(s + i + 2);
    r3 += f(s + i + 3);
    r4 += f(s + i + 4);
    r5 += f(s + i + 5);
    r6 += f(s + i + 6);
    r7 += f(s + i + 7);
  }
  double res = ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7));
  for (; i < n; ++i) res += f(s + i);
  return res;
}

template <class F>
__device__ double np_pairwise(F f, int64_t n) {
  if (n <= 128) return np_leaf(f, 0, n);
  // Post-order walk of numpy's recursion.  Depth <= 48 for any int64 n.
  int64_t st_s[48], st_n[48];
  double st_v[48];
  int st_state[48];
  int sp = 0;
  st_s[0] = 0; st_n[0] = n; st_state[0] = 0;
  double ret = 0.;
  while (sp >= 0) {
    const int64_t s = st_s[sp], m = st_n[sp];
    if (m <= 128) {
      ret = np_leaf(f, s, m);
      --sp;
      continue;
    }
    int64_t m2 = m / 2;
    m2 -= m2 % 8;
    if (st_state[sp] == 0) {           // descend left
      st_state[sp] = 1;
      ++sp;
      st_s[sp] = s; st_n[sp] = m2; st_state[sp] = 0;
    } else if (st_state[sp] == 1) {    // left done -> descend right
      st_v[sp] = ret;
      st_state[sp] = 2;
      ++sp;
      st_s[sp] = s + m2; st_n[sp] = m - m2; st_state[sp] = 0;
    } else {                           // both done
      ret = st_v[sp] + ret;
      --sp;
    }
  }
  return ret;
}

// ---------------------------------------------------------------------------
// scipy.special.ndtri: Cephes ndtri.c (S. L. Moshier), the algorithm scipy
// 1.15 ships; the coefficients below reproduce scipy's ndtri bit-for-bit on
// the host (tests/test_device_math.py) -- on the device up to log/sqrt ulps.
// ---------------------------------------------------------------------------
__host__ __device__ inline double ndtri(double y0) {
  constexpr double s2pi = 2.50662827463100050242E0;
  constexpr double P0[5] = {-5.99633501014107895267E1, 9.80010754185999661536E1,
                            -5.66762857469070293439E1, 1.39312609387279679503E1,
                            -1.23916583867381258016E0};
  constexpr double Q0[8] = {1.95448858338141759834E0, 4.67627912898881538453E0,
                            8.63602421390890590575E1, -2.25462687854119370527E2,
                            2.00260212380060660359E2, -8.20372256168333339912E1,
                            1.59056225126211695515E1, -1.18331621121330003142E0};
  constexpr double P1[9] = {4.05544892305962419923E0, 3.15251094599893866154E1,
                            5.71628192246421288162E1, 4.40805073893200834700E1,
                            1.46849561928858024014E1, 2.18663306850790267539E0,
                            -1.40256079171354495875E-1, -3.50424626827848203418E-2,
                            -8.57456785154685413611E-4};
  constexpr double Q1[8] = {1.57799883256466749731E1, 4.53907635128879210584E1,
                            4.13172038254672030440E1, 1.50425385692907503408E1,
                            2.50464946208309415979E0, -1.42182922854787788574E-1,
                            -3.80806407691578277194E-2, -9.33259480895457427372E-4};
  constexpr double P2[9] = {3.23774891776946035970E0, 6.91522889068984211695E0,
                            3.93881025292474443415E0, 1.33303460815807542389E0,
                            2.01485389549179081538E-1, 1.23716634817820021358E-2,
                            3.01581553508235416007E-4, 2.65806974686737550832E-6,
                            6.23974539184983293730E-9};
  constexpr double Q2[8] = {6.02427039364742014255E0, 3.67983563856160859403E0,
                            1.37702099489081330271E0, 2.16236993594496635890E-1,
                            1.34204006088543189037E-2, 3.28014464682127739104E-4,
                            2.89247864745380683936E-6, 6.79019408009981274425E-9};
  if (y0 == 0.0) return -__builtin_inf();
  if (y0 == 1.0) return __builtin_inf();
  if (y0 < 0.0 || y0 > 1.0) return __builtin_nan("");
  bool negate = true;
  double y = y0;
  if (y > (1.0 - 0.13533528323661269189)) {
    y = 1.0 - y;
    negate = false;
  }
  if (y > 0.13533528323661269189) {
    y = y - 0.5;
    const double y2 = y * y;
    double p = P0[0];
#pragma unroll
    for (int i = 1; i < 5; ++i) p = p * y2 + P0[i];
    double q = y2 + Q0[0];
#pragma unroll
    for (int i = 1; i < 8; ++i) q = q * y2 + Q0[i];
    double x = y + y * (y2 * p / q);
    return x * s2pi;
  }
  const double x = sqrt(-2.0 * log(y));
  const double x0 = x - log(x) / x;
  const double z = 1.0 / x;
  double p, q;
  if (x < 8.0) {
    p = P1[0];
#pragma unroll
    for (int i = 1; i < 9; ++i) p = p * z + P1[i];
    q = z + Q1[0];
#pragma unroll
    for (int i = 1; i < 8; ++i) q = q * z + Q1[i];
  } else {
    p = P2[0];
#pragma unroll
    for (int i = 1; i < 9; ++i) p = p * z + P2[i];
    q = z + Q2[0];
#pragma unroll
    for (int i = 1; i < 8; ++i) q = q * z + Q2[i];
  }
  const double x1 = z * p / q;
  const double r = x0 - x1;
  return negate ? -r : r;
}

// exp(x) for the production path: Cody-Waite reduction x = k ln2 + r,
// |r| <= ln2/2, a degree-12 Taylor polynomial (truncation 2.1e-16 relative)
// and v_ldexp_f64: about 20 VALU ops against ~40 for the libm-accurate ocml
// exp, within 2 ulp, same overflow / underflow / NaN behaviour.
__device__ __forceinline__ double fast_exp(double x) {
  const double k = __builtin_rint(x * 1.4426950408889634);
  double r = __builtin_fma(-k, 6.93147180369123816490e-01, x);
  r = __builtin_fma(-k, 1.90821492927058770002e-10, r);
  double p = 2.08767569878680989792e-09;                  // 1/12!
  p = __builtin_fma(p, r, 2.50521083854417187751e-08);    // 1/11!
  p = __builtin_fma(p, r, 2.75573192239858906526e-07);    // 1/10!
  p = __builtin_fma(p, r, 2.75573192239858906526e-06);    // 1/9!
  p = __builtin_fma(p, r, 2.48015873015873015873e-05);    // 1/8!
  p = __builtin_fma(p, r, 1.98412698412698412698e-04);    // 1/7!
  p = __builtin_fma(p, r, 1.38888888888888888889e-03);    // 1/6!
  p = __builtin_fma(p, r, 8.33333333333333333333e-03);    // 1/5!
  p = __builtin_fma(p, r, 4.16666666666666666667e-02);    // 1/4!
  p = __builtin_fma(p, r, 1.66666666666666666667e-01);    // 1/3!
  p = __builtin_fma(p, r, 0.5);
  p = __builtin_fma(p, r, 1.0);
  p = __builtin_fma(p, r, 1.0);
  const int ki = (int)__builtin_fmax(__builtin_fmin(k, 2100.0), -2100.0);
  const double y = __builtin_ldexp(p, ki);
  return x > 709.782712893384 ? __builtin_inf()
         : (x < -745.2 ? 0.0 : (x != x ? x : y));
}

// pscales.py:56-65 exp_logp (scalar branch).
__device__ __forceinline__ double exp_logp(double lp, double log_npi) {
  return (lp <= log_npi) ? exp(lp) : kNearlyPosInf;
}

__device__ __forceinline__ double exp_logp_fast(double lp, double log_npi) {
  return (lp <= log_npi) ? fast_exp(lp) : kNearlyPosInf;
}

// np.maximum(NEARLY_POSITIVE_ZERO, b): NaN propagates.
__device__ __forceinline__ double np_max_tiny(double b) {
  return (b != b) ? b : (b >= kNearlyPosZero ? b : kNearlyPosZero);
}

// ---------------------------------------------------------------------------
// MH acceptance (sp_utils.py:40-64, pscales.py:56-65,219-236): the
// reference's ratio form s = min(1, exp_logp(lp') / max(tiny, exp_logp(lp))),
// accept iff s >= t.
// ---------------------------------------------------------------------------
__device__ __forceinline__ bool ratio_accept(double lpp, double lp, double t,
                                            bool lin, double log_npi) {
  const double eA = lin ? lpp : exp_logp(lpp, log_npi);
  const double eB = lin ? lp : exp_logp(lp, log_npi);
  double q = eA / np_max_tiny(eB);
  q = q < 1. ? q : 1.;
  return q >= t;
}

// The same decision through a cheap filter (production RNG modes).  With
// t = u01(t0, t1), t lies in [tlo, tlo + 2^-24), tlo = (t0 >> 8) 2^-24.
// e = 2^(fp32(log2e (lp' - lp))) on v_exp_f32 is within 2.7e-6 relative of
// s whenever |lp|, |lp'| <= 700 (then no exp clamp, overflow or underflow
// occurs in the ratio form): fp32 rounding of the argument (|y| <= 60 where
// it matters) costs 4.2e-8 |y|, v_exp_f32 1 ulp.  So t < e (1 - 4e-6)
// proves accept and t > e (1 + 4e-6) proves reject; otherwise `need` is set
// and the caller must evaluate ratio_accept (about 1e-5 of chain-steps).
struct Decision { bool acc, need; };

// LB = number of leading bits of t known to the filter: t lies in
// [lead 2^-LB, (lead + 1) 2^-LB).  The lane-pair kernel's Philox path packs a
// 14-bit lead beside its normals (its fallback draws the remaining bits).
// The comparison runs in units of 2^-LB: eL = e 2^LB = 2^(fp32(log2e (lp' -
// lp) + LB)), so t < e (1 - 4e-6) is proven by lead + 1 <= eL (1 - 4e-6)
// (one fp32 fma: lead <= eL (1 - 4e-6) - 1, rounding 2^-24 eL) and t > e (1 +
// 4e-6) by lead > eL (1 + 4e-6).  Where a decision can hinge on e (e in
// [2^-LB, 1]) the argument is in [0, LB]: its fp32 rounding costs at most
// 4.2e-8 LB relative, as before.
template <int LB>
__device__ __forceinline__ Decision accept_filter_lead(double lpp, double lp,
                                                       uint32_t lead, bool lin) {
  const float eL = __builtin_amdgcn_exp2f(
      (float)__builtin_fma(lpp - lp, 1.4426950408889634, (double)LB));
  const float fl = (float)lead;
  const bool inr = !lin && __builtin_fabs(lpp) <= 700. &&
                   __builtin_fabs(lp) <= 700.;
  const bool af = fl <= __builtin_fmaf(eL, 0.999996f, -1.0f);
  const bool rf = fl > eL * 1.000004f;
  return Decision{inr && af, !(inr && (af || rf))};
}

// The same decision as lane masks (bit l = lane l; inactive lanes' bits are
// meaningless): each comparison's ballot is the compare's own scalar result,
// so acc / need combine in SALU instead of being turned into per-lane bools
// and back (v_cndmask + v_cmp per ballot).  lin is wave-uniform.
struct DecisionMask { uint64_t acc, need; };

template <int LB>
__device__ __forceinline__ DecisionMask accept_filter_lead_mask(double lpp, double lp,
                                                                uint32_t lead, bool lin) {
  const float eL = __builtin_amdgcn_exp2f(
      (float)__builtin_fma(lpp - lp, 1.4426950408889634, (double)LB));
  const float fl = (float)lead;
  const uint64_t inr = lin ? 0ull : __ballot(__builtin_fabs(lpp) <= 700.) &
                                        __ballot(__builtin_fabs(lp) <= 700.);
  const uint64_t af = __ballot(fl <= __builtin_fmaf(eL, 0.999996f, -1.0f));
  const uint64_t rf = __ballot(fl > eL * 1.000004f);
  return DecisionMask{inr & af, ~(inr & (af | rf))};
}

// t = u01(t0, t1): the lead is t0's top 24 bits.
__device__ __forceinline__ Decision accept_filter(double lpp, double lp,
                                                  uint32_t t0, bool lin) {
  return accept_filter_lead<24>(lpp, lp, t0 >> 8, lin);
}

}  // namespace pbh
