// pbh_legacy.hip -- the reference's random streams generated on the GPU.
//
// The reference draws every random number from NumPy's legacy RandomState
// (SURVEY.md App. A-7): MT19937 seeded by init_genrand (RandomState(int)),
// random_sample = (a >> 5, b >> 6) 53-bit doubles, and the polar-method
// legacy gauss with its cached second deviate.  These kernels restate that
// generator (numpy 2.2.6 random/src/mt19937 + legacy-distributions.c, the
// version pinned in SURVEY.md §8c) per chain, one chain per lane, and write
// the draws in the replay layout [T][R][N] the REPLAY kernels read -- so a
// full-width reference-identical run needs no host stream generation.
//
// State per chain: key[624] in [624][N] (word-major, so lanes of a wave
// touch neighbouring words while their positions agree), pos, the cached
// gauss and its flag.  Lanes drift apart (the polar rejection consumes a
// variable number of words); correctness does not depend on it.
// Per step the order is the reference's: MH draws d normals (callable
// Gaussian Delta) or d raw doubles (tuple / list delta), then one double for
// the threshold; CondCov Gibbs draws one double per updated coordinate of
// the rf.py:446-452 cycle and pads the row with NaN.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pbh_kernels.h"
#include "pbhip.h"

namespace pbh {
namespace {

constexpr int kN = 624, kM = 397;
constexpr uint32_t kMatrixA = 0x9908b0dfu, kUpper = 0x80000000u, kLower = 0x7fffffffu;

__global__ __launch_bounds__(256) void mt_seed_kernel(uint32_t *key, int32_t *pos,
                                                      double *gauss, int32_t *has_gauss,
                                                      const uint32_t *seeds, int64_t n) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= n) return;
  uint32_t s = seeds[c];
  // mt19937_seed (init_genrand)
  for (int i = 0; i < kN; ++i) {
    key[(int64_t)i * n + c] = s;
    s = 1812433253u * (s ^ (s >> 30)) + (uint32_t)(i + 1);
  }
  pos[c] = kN;
  gauss[c] = 0.0;
  has_gauss[c] = 0;
}

struct Mt {
  static constexpr bool kLockstep = false;
  uint32_t *key;
  int64_t n, c;
  int pos;

  __device__ __forceinline__ uint32_t &k(int i) { return key[(int64_t)i * n + c]; }

  // mt19937_gen in the reference order (later words read updated ones),
  // in chunks of kB words whose loads are all issued before the chunk's
  // stores: a chunk reads k[i+1 .. i+kB] (old values, read before they are
  // overwritten, as in the sequential loop) and k[j] with j = i + 397 (not yet
  // written) or j = i - 227 (written by an earlier chunk since kB <= 227), so
  // the result is the sequential one while kB loads are in flight instead of
  // one.  The chunk grid splits at 227 = N - M (where j wraps) and at 623.
  // 98 -> 29 ms for the cfg2-width 250-step streams (kB = 16).
  static constexpr int kB = 16;
  __device__ __forceinline__ void twist_chunk(int i0, int cnt) {
    uint32_t nx[kB + 1], src[kB];
#pragma unroll
    for (int u = 0; u <= kB; ++u)
      if (u <= cnt) nx[u] = k(i0 + u);
#pragma unroll
    for (int u = 0; u < kB; ++u)
      if (u < cnt) {
        const int i = i0 + u;
        src[u] = k(i < kN - kM ? i + kM : i + kM - kN);
      }
#pragma unroll
    for (int u = 0; u < kB; ++u)
      if (u < cnt) {
        const uint32_t y = (nx[u] & kUpper) | (nx[u + 1] & kLower);
        k(i0 + u) = src[u] ^ (y >> 1) ^ ((0u - (y & 1u)) & kMatrixA);
      }
  }

  __device__ void twist() {
    for (int i = 0; i < kN - kM; i += kB)          // [0, 227)
      twist_chunk(i, (kN - kM) - i < kB ? (kN - kM) - i : kB);
    for (int i = kN - kM; i < kN - 1; i += kB)     // [227, 623)
      twist_chunk(i, (kN - 1) - i < kB ? (kN - 1) - i : kB);
    const uint32_t y = (k(kN - 1) & kUpper) | (k(0) & kLower);
    k(kN - 1) = k(kM - 1) ^ (y >> 1) ^ ((0u - (y & 1u)) & kMatrixA);
    pos = 0;
  }

  __device__ __forceinline__ uint32_t next32() {
    if (pos == kN) twist();
    uint32_t y = k(pos++);
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
  }

  // legacy_double / random_sample
  __device__ __forceinline__ double next_double() {
    const int32_t a = (int32_t)(next32() >> 5), b = (int32_t)(next32() >> 6);
    return (a * 67108864.0 + b) / 9007199254740992.0;
  }
};

// The same generator with a DOUBLE-BUFFERED state [2][624][N] and a
// wave-synchronous refill.  A lane consumes block b from buffer `buf`; the
// other buffer already holds block b + 1, so reaching word 624 only flips
// `buf` and marks the lane pending (the buffer it left is free).  A pending
// lane's free buffer is refilled with block b + 2 by an OUT-OF-PLACE twist of
// its current block -- the sequential twist's result: dst[i] = src[i + 397]
// (i < 227) or dst[i - 227] (i >= 227) ^ f(src[i], src[i + 1]), dst[623] =
// dst[396] ^ f(src[623], dst[0]) -- and every pending lane of the wave twists
// together, as soon as any of them is kRefill words into its block.  Lanes
// drift apart by a few dozen words per block (polar rejections), so a wave
// twists about once per 624 words instead of once per distinct lane position,
// and every twist load / store is coalesced over the wave's pending lanes.
// A lane always passes kRefill < 624 before its block ends, so the next
// block is ready whenever it is needed, whatever the drift.
// Per-lane state word: pos | buf << 16 | pending << 17.
struct Mt2 {
  static constexpr bool kLockstep = true;
  uint32_t *key;
  int64_t n, c;
  int pos, buf, pend;
  static constexpr int kRefill = 312;
  static constexpr int kB = 16;

  __device__ __forceinline__ uint32_t &k(int b, int i) {
    return key[((int64_t)b * kN + i) * n + c];
  }

  __device__ __forceinline__ void twist_chunk(int s, int i0, int cnt) {
    const int d = s ^ 1;
    uint32_t nx[kB + 1], src[kB];
#pragma unroll
    for (int u = 0; u <= kB; ++u)
      if (u <= cnt) nx[u] = k(s, i0 + u);
#pragma unroll
    for (int u = 0; u < kB; ++u)
      if (u < cnt) {
        const int i = i0 + u;
        src[u] = i < kN - kM ? k(s, i + kM) : k(d, i + kM - kN);
      }
#pragma unroll
    for (int u = 0; u < kB; ++u)
      if (u < cnt) {
        const uint32_t y = (nx[u] & kUpper) | (nx[u + 1] & kLower);
        k(d, i0 + u) = src[u] ^ (y >> 1) ^ ((0u - (y & 1u)) & kMatrixA);
      }
  }

  // block in buffer s -> next block in buffer s ^ 1
  __device__ void twist_from(int s) {
    const int d = s ^ 1;
    for (int i = 0; i < kN - kM; i += kB)          // [0, 227): old words
      twist_chunk(s, i, (kN - kM) - i < kB ? (kN - kM) - i : kB);
    for (int i = kN - kM; i < kN - 1; i += kB)     // [227, 623): new words
      twist_chunk(s, i, (kN - 1) - i < kB ? (kN - 1) - i : kB);
    const uint32_t y = (k(s, kN - 1) & kUpper) | (k(d, 0) & kLower);
    k(d, kN - 1) = k(d, kM - 1) ^ (y >> 1) ^ ((0u - (y & 1u)) & kMatrixA);
  }

  __device__ __forceinline__ uint32_t next32() {
    if (__builtin_amdgcn_ballot_w64(pend && pos >= kRefill)) {   // wave-uniform
      if (pend) {
        twist_from(buf);
        pend = 0;
      }
    }
    if (pos == kN) {
      buf ^= 1;
      pos = 0;
      pend = 1;
    }
    uint32_t y = k(buf, pos++);
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
  }

  __device__ __forceinline__ double next_double() {
    const int32_t a = (int32_t)(next32() >> 5), b = (int32_t)(next32() >> 6);
    return (a * 67108864.0 + b) / 9007199254740992.0;
  }

  __device__ __forceinline__ int packed() const {
    return pos | (buf << 16) | (pend << 17);
  }
};

// legacy_gauss: polar method, second deviate cached across calls
template <class M>
__device__ __forceinline__ double legacy_gauss(M &m, double &gauss, int &has) {
  if (has) {
    const double t = gauss;
    has = 0;
    gauss = 0.0;
    return t;
  }
  double x1, x2, r2;
  do {
    x1 = 2.0 * m.next_double() - 1.0;
    x2 = 2.0 * m.next_double() - 1.0;
    r2 = x1 * x1 + x2 * x2;
  } while (r2 >= 1.0 || r2 == 0.0);
  const double f = sqrt(-2.0 * log(r2) / r2);
  gauss = f * x1;
  has = 1;
  return f * x2;
}

// RandomState.randint(-d0, d0) (mtrand.pyx randint -> _rand_int64 with
// use_masked=True): bounds truncated toward zero, rng = hi - 1 - lo, then
// words & mask (the smallest all-ones >= rng) until <= rng
// (distributions.c buffered_bounded_masked_uint32).
template <class M>
__device__ __forceinline__ double legacy_randint(M &m, double d0) {
  const int64_t lo = (int64_t)trunc(-d0), hi = (int64_t)trunc(d0);
  const uint32_t rng = (uint32_t)(hi - 1 - lo);
  if (rng == 0) return (double)lo;
  uint32_t mask = rng;
  mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4;
  mask |= mask >> 8; mask |= mask >> 16;
  uint32_t v;
  while ((v = (m.next32() & mask)) > rng) {
  }
  return (double)(lo + (int64_t)v);
}

// Seeding for the double-buffered state: init_genrand into buffer 0, then
// the first twist (which the reference makes at its first draw) into buffer 1:
// the lane starts at word 0 of buffer 1 with buffer 0 free (pending).
__global__ __launch_bounds__(256) void mt_seed_db_kernel(uint32_t *key, int32_t *pos,
                                                         double *gauss, int32_t *has_gauss,
                                                         const uint32_t *seeds, int64_t n) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= n) return;
  uint32_t s = seeds[c];
  for (int i = 0; i < kN; ++i) {
    key[(int64_t)i * n + c] = s;
    s = 1812433253u * (s ^ (s >> 30)) + (uint32_t)(i + 1);
  }
  Mt2 m{key, n, c, 0, 0, 0};
  m.twist_from(0);
  m.buf = 1;
  m.pos = 0;
  m.pend = 1;
  pos[c] = m.packed();
  gauss[c] = 0.0;
  has_gauss[c] = 0;
}

template <class M>
__device__ __forceinline__ void legacy_gen_body(const LegacyArgs &a, int64_t c, M &m) {
  double gauss = a.gauss[c];
  int has = a.has_gauss[c];
  const int64_t rowlen = (int64_t)a.R * a.n;
  for (int64_t t = 0; t < a.n_steps; ++t) {
    double *row = a.out + t * rowlen + c;
    if (a.gibbs) {
      // rf.py:446-452: block (step0 + t) mod ceil(d / tsteps) of the cycle
      const int64_t nblk = (a.d + a.R - 1) / a.R;
      const int cm = (int)(((a.step0 + t) % nblk) * a.R);
      const int cnt = (cm + a.R < a.d ? cm + a.R : a.d) - cm;
      for (int j = 0; j < a.R; ++j)
        row[(int64_t)j * a.n] = j < cnt ? m.next_double() : __builtin_nan("");
      continue;
    }
    if (a.vardelta) {
      // Field.eval_delta draws per variable in key order (variable.py:618-633)
      for (int j = 0; j < a.d; ++j) {
        const int md = (int)((a.vmode >> (2 * j)) & 3u);
        double v = __builtin_nan("");
        if (md == PBH_VAR_RANDINT)
          v = legacy_randint(m, a.vdelta[j]);
        else if (md != PBH_VAR_FIXED)
          v = m.next_double();
        row[(int64_t)j * a.n] = v;
      }
      row[(int64_t)a.d * a.n] = m.next_double();   // the MH threshold
      continue;
    }
    if (M::kLockstep && a.normal) {
      // the step's d polar-method normals, lanes in lockstep over ATTEMPTS:
      // each lane makes one attempt per iteration until it holds its pairs,
      // so a wave loops ~max over lanes of the step's attempts (about 9.5
      // for 5 pairs) instead of the sum over pairs of the per-pair maxima
      // (about 18).  The draws, their order and the cached deviate are
      // legacy_gauss's exactly.
      int j = 0;
      if (has) {
        row[(int64_t)a.order[0] * a.n] = gauss;
        has = 0;
        gauss = 0.0;
        j = 1;
      }
      while (__builtin_amdgcn_ballot_w64(j < a.d)) {   // wave-uniform
        if (j < a.d) {
          const double x1 = 2.0 * m.next_double() - 1.0;
          const double x2 = 2.0 * m.next_double() - 1.0;
          const double r2 = x1 * x1 + x2 * x2;
          if (r2 < 1.0 && r2 != 0.0) {
            const double f = sqrt(-2.0 * log(r2) / r2);
            row[(int64_t)a.order[j] * a.n] = f * x2;
            if (++j < a.d) {
              row[(int64_t)a.order[j] * a.n] = f * x1;
              ++j;
            } else {
              gauss = f * x1;   // cached for the next draw (odd d)
              has = 1;
            }
          }
        }
      }
      row[(int64_t)a.d * a.n] = m.next_double();   // the MH threshold
      continue;
    }
    for (int j = 0; j < a.d; ++j) {
      const double v = a.normal ? legacy_gauss(m, gauss, has) : m.next_double();
      row[(int64_t)a.order[j] * a.n] = v;    // draw j feeds dim order[j]
    }
    row[(int64_t)a.d * a.n] = m.next_double();   // the MH threshold
  }
  a.gauss[c] = gauss;
  a.has_gauss[c] = has;
}

__global__ __launch_bounds__(256) void legacy_gen_kernel(LegacyArgs a) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= a.n) return;
  Mt m{a.key, a.n, c, a.pos[c]};
  legacy_gen_body(a, c, m);
  a.pos[c] = m.pos;
}

// Lanes past the last chain leave at once; the refill ballot counts the
// active lanes only.
__global__ __launch_bounds__(256) void legacy_gen_db_kernel(LegacyArgs a) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= a.n) return;
  const int st = a.pos[c];
  Mt2 m{a.key, a.n, c, st & 0xFFFF, (st >> 16) & 1, (st >> 17) & 1};
  legacy_gen_body(a, c, m);
  a.pos[c] = m.packed();
}

}  // namespace

hipError_t launch_legacy_seed(uint32_t *key, int32_t *pos, double *gauss,
                              int32_t *has_gauss, const uint32_t *seeds,
                              int64_t n, int32_t db, hipStream_t s) {
  const dim3 grid((unsigned)((n + 255) / 256)), block(256);
  if (db)
    hipLaunchKernelGGL(mt_seed_db_kernel, grid, block, 0, s, key, pos, gauss,
                       has_gauss, seeds, n);
  else
    hipLaunchKernelGGL(mt_seed_kernel, grid, block, 0, s, key, pos, gauss,
                       has_gauss, seeds, n);
  return hipGetLastError();
}

hipError_t launch_legacy_gen(const LegacyArgs &a, hipStream_t s) {
  const dim3 grid((unsigned)((a.n + 255) / 256)), block(256);
  if (a.db)
    hipLaunchKernelGGL(legacy_gen_db_kernel, grid, block, 0, s, a);
  else
    hipLaunchKernelGGL(legacy_gen_kernel, grid, block, 0, s, a);
  return hipGetLastError();
}

}  // namespace pbh
