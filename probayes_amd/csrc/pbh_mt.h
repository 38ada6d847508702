// pbh_mt.h -- MT19937 / NumPy legacy-stream helpers shared by the device
// generators (pbh_legacy.hip: the chain-per-lane generators and the fused
// REPLAY kernel; pbh_legacy_wp.hip: the word-parallel generator).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pbh_kernels.h"

namespace pbh {
namespace {

constexpr int kN = 624, kM = 397;
constexpr uint32_t kMatrixA = 0x9908b0dfu, kUpper = 0x80000000u, kLower = 0x7fffffffu;
constexpr int kQ = kN / 4;   // 156 quads per block
__device__ __forceinline__ uint32_t mt_f(uint32_t a, uint32_t b) {
  const uint32_t y = (a & kUpper) | (b & kLower);
  return (y >> 1) ^ ((0u - (y & 1u)) & kMatrixA);
}
typedef uint32_t w4 __attribute__((ext_vector_type(4)));
// Mt4's buffers per chain (a power of two: the current block and up to
// kK4 - 1 twisted ahead; legacy_ahead_kernel fills them before a fused
// REPLAY launch) and 8-quad chunks per (padded) block
constexpr int kK4 = 16, kCh = 20;
constexpr int kBufMask = kK4 - 1;
__device__ __forceinline__ w4 &k4q(w4 *key, int64_t n, int64_t c, int b, int i) {
  return key[((int64_t)(b * kCh + (i >> 3)) * n + c) * 8 + (i & 7)];
}
__device__ __forceinline__ uint32_t mt_temper(uint32_t y) {
  y ^= y >> 11;
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= y >> 18;
  return y;
}
// random_sample of two raw words (tempered here)
__device__ __forceinline__ double mt_dbl(uint32_t wa, uint32_t wb) {
  const int32_t a = (int32_t)(mt_temper(wa) >> 5), b = (int32_t)(mt_temper(wb) >> 6);
  return (a * 67108864.0 + b) / 9007199254740992.0;
}
// log(x) of the polar method's r2 in (0, 1) (a normal double) for Mt4
// (Tang's table method): x = m 2^e, m in [1/2, 1), c = m rounded to 1/256,
// r = (m - c) / c (|r| <= 2^-8; m - c exact), log x = (e ln2_hi + T_hi) +
// (r + (r^2 q(r) + (e ln2_lo + T_lo))) with ln c = T_hi + T_lo, T_hi and
// ln2_hi multiples of 2^-32 so that their sum is exact, q the log1p series
// to r^8 (truncation < 2^-70 relative).  About 20 VALU and two LDS reads
// against ~75 VALU for OCML's log; within ~0.5 ulp, so the normals stay
// within the last ulp of NumPy's (tests/test_gpu_legacy.py).
__device__ __forceinline__ double log_leg(double x, const double *tab) {
  const double m = __builtin_amdgcn_frexp_mant(x);
  const int e = __builtin_amdgcn_frexp_exp(x);
  const uint32_t ch = ((uint32_t)(__builtin_bit_cast(uint64_t, m) >> 32) + 0x1000u) & 0xFFFFE000u;
  const uint32_t off = (ch >> 9) & 0xFFFu;   // 16 j
  const char *tb = reinterpret_cast<const char *>(tab);
  const double2 t = *reinterpret_cast<const double2 *>(tb + off);
  const double ic = *reinterpret_cast<const double *>(tb + kLegLogInv * 8 + (off >> 1));
  const double r = (m - __builtin_bit_cast(double, (uint64_t)ch << 32)) * ic;
  double q = __builtin_fma(r, -1.0 / 8.0, 1.0 / 7.0);
  q = __builtin_fma(q, r, -1.0 / 6.0);
  q = __builtin_fma(q, r, 1.0 / 5.0);
  q = __builtin_fma(q, r, -1.0 / 4.0);
  q = __builtin_fma(q, r, 1.0 / 3.0);
  q = __builtin_fma(q, r, -0.5);
  const double de = (double)e;
  const double lo = __builtin_fma(de, 1.90821492927058770002e-10, t.y);
  const double shi = __builtin_fma(de, 6.93147180369123816490e-01, t.x);   // exact
  const double p = __builtin_fma(r * r, q, lo);
  return shi + (r + p);
}

}  // namespace
}  // namespace pbh
