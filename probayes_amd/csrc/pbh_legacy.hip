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
#include <cstdlib>

#include "pbh_kernels.h"
#include "pbh_kernels_impl.h"   // mh_body: the fused REPLAY kernel
#include "pbhip.h"
#include "pbh_mt.h"

namespace pbh {
namespace {

constexpr int kBlockLegacy = 256;   // threads per workgroup of the generators

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
  static constexpr bool kPeek = false;
  static constexpr bool kPeek4 = false;
  static constexpr bool kLogTab = false;
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
  __device__ __forceinline__ void maintain() {}
};

// The same generator with a DOUBLE-BUFFERED state and a wave-synchronous
// refill.  A lane consumes block b from buffer `buf`; the other buffer
// already holds block b + 1, so reaching word 624 only flips `buf` and marks
// the lane pending (the buffer it left is free).  A pending lane's free
// buffer is refilled with block b + 2 by an OUT-OF-PLACE twist of its current
// block -- the sequential twist's result: dst[i] = src[i + 397] (i < 227) or
// dst[i - 227] (i >= 227) ^ f(src[i], src[i + 1]), dst[623] = dst[396] ^
// f(src[623], dst[0]) -- and every pending lane of the wave twists together,
// as soon as any of them is kRefill words into its block.  Lanes drift apart
// by a few dozen words per block (polar rejections), so a wave twists about
// once per 624 words instead of once per distinct lane position.  A lane
// always passes kRefill < 624 before its block ends, so the next block is
// ready whenever it is needed, whatever the drift.
//
// Layout [2][156][N] of uint4: a lane's words 4q .. 4q + 3 are one 16-byte
// quad, so the drifting lanes read their words 16 bytes at a time (a
// register quad, reloaded every fourth word) and the twist moves whole
// quads: each quad of dst needs the quad q of src and the first word of quad
// q + 1, words 4q + 397 .. + 400 (quads q + 99, q + 100, at offset 1) or
// dst words 4q - 227 .. - 224 (quads q - 57, q - 56, at offset 1).
// Per-lane state word: pos | buf << 16 | pending << 17.


struct Mt2 {
  static constexpr bool kLockstep = true;
  static constexpr bool kPeek = false;
  static constexpr bool kPeek4 = false;
  static constexpr bool kLogTab = false;
  static constexpr int kRefill = 312;
  uint4 *key;
  int64_t n, c;
  int pos, buf, pend;
  uint4 cur;   // the quad holding word pos (valid when pos % 4 != 0)

  __device__ __forceinline__ uint4 &q(int b, int i) {
    return key[((int64_t)b * kQ + i) * n + c];
  }

  // block in buffer s -> next block in buffer s ^ 1
  __device__ void twist_from(int s) {
    const int d = s ^ 1;
    uint4 a = q(s, 0);          // src quad i
    uint4 hi0 = q(s, 99), hi1 = q(s, 100);   // src quads i + 99, i + 100
    for (int i = 0; i < 56; ++i) {            // words 0 .. 223: src[w + 397]
      const uint4 nx = q(s, i + 1);
      uint4 o;
      o.x = hi0.y ^ mt_f(a.x, a.y);
      o.y = hi0.z ^ mt_f(a.y, a.z);
      o.z = hi0.w ^ mt_f(a.z, a.w);
      o.w = hi1.x ^ mt_f(a.w, nx.x);
      q(d, i) = o;
      a = nx;
      hi0 = hi1;
      if (i + 101 < kQ) hi1 = q(s, i + 101);   // (quad 156 is past the block)
    }
    {                                          // quad 56: words 224 .. 227
      const uint4 nx = q(s, 57);
      const uint4 d0 = q(d, 0);
      uint4 o;
      o.x = hi0.y ^ mt_f(a.x, a.y);            // src[621]
      o.y = hi0.z ^ mt_f(a.y, a.z);            // src[622]
      o.z = hi0.w ^ mt_f(a.z, a.w);            // src[623]
      o.w = d0.x ^ mt_f(a.w, nx.x);            // dst[0]
      q(d, 56) = o;
      a = nx;
    }
    uint4 lo0 = q(d, 0), lo1 = q(d, 1);       // dst quads i - 57, i - 56
    for (int i = 57; i < kQ - 1; ++i) {       // words 228 .. 619
      const uint4 nx = q(s, i + 1);
      uint4 o;
      o.x = lo0.y ^ mt_f(a.x, a.y);
      o.y = lo0.z ^ mt_f(a.y, a.z);
      o.z = lo0.w ^ mt_f(a.z, a.w);
      o.w = lo1.x ^ mt_f(a.w, nx.x);
      q(d, i) = o;
      a = nx;
      lo0 = lo1;
      lo1 = q(d, i - 55);
    }
    {                                          // quad 155: words 620 .. 623
      const uint4 d0 = q(d, 0);
      const uint4 d99 = q(d, 99);
      uint4 o;
      o.x = lo0.y ^ mt_f(a.x, a.y);            // dst[393]
      o.y = lo0.z ^ mt_f(a.y, a.z);            // dst[394]
      o.z = lo0.w ^ mt_f(a.z, a.w);            // dst[395]
      o.w = d99.x ^ mt_f(a.w, d0.x);           // dst[396], with the new dst[0]
      q(d, kQ - 1) = o;
    }
  }

  __device__ __forceinline__ void load_cur() {
    if (pos & 3) cur = q(buf, pos >> 2);
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
    const int u = pos & 3;
    if (u == 0) cur = q(buf, pos >> 2);
    ++pos;
    uint32_t y = u == 0 ? cur.x : (u == 1 ? cur.y : (u == 2 ? cur.z : cur.w));
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
  __device__ __forceinline__ void maintain() {}
};

// The double-buffered state consumed through an LDS WINDOW (the default).
// Mt2's lanes read their next quad from HBM when they reach it: in the
// polar-method loop that is one dependent global load per attempt, and at one
// wavefront per SIMD nothing hides it.  Here each lane's upcoming words are
// staged in LDS ahead of use: a ring of 2H quads per lane ([slot][256
// threads] of uint4, conflict-free whatever the lanes' positions), refilled H
// quads at a time (H loads in flight) at the top of a step whenever a lane
// has H or fewer quads left -- the ballot makes the refills wave-wide.  The
// head (next quad to load) runs at most 2H quads ahead of the consumption
// position, so it is inside the current block or the next one; the next
// block must be twisted before the head enters it (forced here if the step-top
// trigger at word 312 has not yet run).  A twist overwrites only the block
// BEFORE the consumption position's, whose words are consumed, so the state
// in HBM (pos, buf, pend: Mt2's packed word) stays valid when a launch ends
// with words still in the window.
//
// The twist itself runs in batches of 14 quads: part 1 (dst quads 0 .. 55)
// reads src quads i .. i + 14 and i + 99 .. i + 113, part 2 (quads 57 ..
// 154) src quads i .. i + 14 and dst quads i - 57 .. i - 43 (written by part
// 1 or an earlier batch), so ~30 loads are in flight instead of two.
// a quad as a plain vector (SROA splits arrays of it into registers; arrays
// of HIP's uint4 struct stayed in scratch)

// a block -> the next block: ld(0, i) / ld(1, i) read quad i of the source /
// destination block, st(i, v) writes quad i of the destination
template <class L, class S>
__device__ __forceinline__ void twist_ls(L ld, S st) {
  constexpr int kTB = 14;   // twist batch (56 = 4 x 14, 98 = 7 x 14)
#pragma unroll
  for (int i0 = 0; i0 < 56; i0 += kTB) {
    w4 a[kTB + 1], h[kTB + 1];
#pragma unroll
    for (int u = 0; u <= kTB; ++u) {
      a[u] = ld(0, i0 + u);
      h[u] = ld(0, i0 + 99 + u);
    }
#pragma unroll
    for (int u = 0; u < kTB; ++u) {
      w4 o;
      o.x = h[u].y ^ mt_f(a[u].x, a[u].y);
      o.y = h[u].z ^ mt_f(a[u].y, a[u].z);
      o.z = h[u].w ^ mt_f(a[u].z, a[u].w);
      o.w = h[u + 1].x ^ mt_f(a[u].w, a[u + 1].x);
      st(i0 + u, o);
    }
  }
  {                                          // quad 56: words 224 .. 227
    const w4 a = ld(0, 56), nx = ld(0, 57), h = ld(0, 155), d0 = ld(1, 0);
    w4 o;
    o.x = h.y ^ mt_f(a.x, a.y);              // src[621]
    o.y = h.z ^ mt_f(a.y, a.z);              // src[622]
    o.z = h.w ^ mt_f(a.z, a.w);              // src[623]
    o.w = d0.x ^ mt_f(a.w, nx.x);            // dst[0]
    st(56, o);
  }
#pragma unroll
  for (int i0 = 57; i0 < kQ - 1; i0 += kTB) {
    w4 a[kTB + 1], l[kTB + 1];
#pragma unroll
    for (int u = 0; u <= kTB; ++u) {
      a[u] = ld(0, i0 + u);
      l[u] = ld(1, i0 - 57 + u);
    }
#pragma unroll
    for (int u = 0; u < kTB; ++u) {
      w4 o;
      o.x = l[u].y ^ mt_f(a[u].x, a[u].y);
      o.y = l[u].z ^ mt_f(a[u].y, a[u].z);
      o.z = l[u].w ^ mt_f(a[u].z, a[u].w);
      o.w = l[u + 1].x ^ mt_f(a[u].w, a[u + 1].x);
      st(i0 + u, o);
    }
  }
  {                                          // quad 155: words 620 .. 623
    const w4 a = ld(0, kQ - 1), d0 = ld(1, 0), d98 = ld(1, 98), d99 = ld(1, 99);
    w4 o;
    o.x = d98.y ^ mt_f(a.x, a.y);            // dst[393]
    o.y = d98.z ^ mt_f(a.y, a.z);            // dst[394]
    o.z = d98.w ^ mt_f(a.z, a.w);            // dst[395]
    o.w = d99.x ^ mt_f(a.w, d0.x);           // dst[396], with the new dst[0]
    st(kQ - 1, o);
  }
}

// block in buffer s -> the next block in buffer d, quads addressed by q(b, i)
template <class Q>
__device__ __forceinline__ void twist_q(Q q, int s, int d) {
  constexpr int kTB = 14;   // twist batch (56 = 4 x 14, 98 = 7 x 14)
  for (int i0 = 0; i0 < 56; i0 += kTB) {
    w4 a[kTB + 1], h[kTB + 1];
#pragma unroll
    for (int u = 0; u <= kTB; ++u) {
      a[u] = q(s, i0 + u);
      h[u] = q(s, i0 + 99 + u);
    }
#pragma unroll
    for (int u = 0; u < kTB; ++u) {
      w4 o;
      o.x = h[u].y ^ mt_f(a[u].x, a[u].y);
      o.y = h[u].z ^ mt_f(a[u].y, a[u].z);
      o.z = h[u].w ^ mt_f(a[u].z, a[u].w);
      o.w = h[u + 1].x ^ mt_f(a[u].w, a[u + 1].x);
      q(d, i0 + u) = o;
    }
  }
  {                                          // quad 56: words 224 .. 227
    const w4 a = q(s, 56), nx = q(s, 57), h = q(s, 155), d0 = q(d, 0);
    w4 o;
    o.x = h.y ^ mt_f(a.x, a.y);              // src[621]
    o.y = h.z ^ mt_f(a.y, a.z);              // src[622]
    o.z = h.w ^ mt_f(a.z, a.w);              // src[623]
    o.w = d0.x ^ mt_f(a.w, nx.x);            // dst[0]
    q(d, 56) = o;
  }
  for (int i0 = 57; i0 < kQ - 1; i0 += kTB) {
    w4 a[kTB + 1], l[kTB + 1];
#pragma unroll
    for (int u = 0; u <= kTB; ++u) {
      a[u] = q(s, i0 + u);
      l[u] = q(d, i0 - 57 + u);
    }
#pragma unroll
    for (int u = 0; u < kTB; ++u) {
      w4 o;
      o.x = l[u].y ^ mt_f(a[u].x, a[u].y);
      o.y = l[u].z ^ mt_f(a[u].y, a[u].z);
      o.z = l[u].w ^ mt_f(a[u].z, a[u].w);
      o.w = l[u + 1].x ^ mt_f(a[u].w, a[u + 1].x);
      q(d, i0 + u) = o;
    }
  }
  {                                          // quad 155: words 620 .. 623
    const w4 a = q(s, kQ - 1), d0 = q(d, 0), d98 = q(d, 98), d99 = q(d, 99);
    w4 o;
    o.x = d98.y ^ mt_f(a.x, a.y);            // dst[393]
    o.y = d98.z ^ mt_f(a.y, a.z);            // dst[394]
    o.z = d98.w ^ mt_f(a.z, a.w);            // dst[395]
    o.w = d99.x ^ mt_f(a.w, d0.x);           // dst[396], with the new dst[0]
    q(d, kQ - 1) = o;
  }
}

__device__ __forceinline__ void mt3_twist(w4 *key, int64_t n, int64_t c, int s) {
  twist_q([&](int b, int i) -> w4 & { return key[((int64_t)b * kQ + i) * n + c]; }, s, s ^ 1);
}

// Mt3's rare refills (a launch's first two, and a step longer than the
// window) out of line, with plain values in and out so that the generator's
// state never has to live in memory; the step-top refill stays inline.
template <int H>
__device__ __attribute__((noinline)) int mt3_refill_cold(w4 *key, int64_t n, int64_t c,
                                                         w4 *win, int hq, int blk,
                                                         int buf, int pend) {
  const int nb = (blk + 1) * kQ;
  if (pend && hq + H > nb) {   // the head enters the next block
    mt3_twist(key, n, c, buf);
    pend = 0;
  }
  w4 v[H];
#pragma unroll
  for (int u = 0; u < H; ++u) {
    const int k = hq + u;
    const bool nx = k >= nb;
    v[u] = key[((int64_t)(buf ^ (nx ? 1 : 0)) * kQ + (nx ? k - nb : k - blk * kQ)) * n + c];
  }
#pragma unroll
  for (int u = 0; u < H; ++u) win[((hq + u) & (2 * H - 1)) * kBlockLegacy] = v[u];
  return pend;
}

template <int H>
struct Mt3 {
  static constexpr bool kLockstep = true;
  static constexpr bool kPeek = true;   // attempts2 / advance
  static constexpr bool kPeek4 = false;
  static constexpr bool kLogTab = false;
  static constexpr int kRefill = 312;
  static constexpr int kW = 2 * H;   // window quads per lane (a power of two)
  static constexpr int kTB = 14;     // twist batch (56 = 4 x 14, 98 = 7 x 14)
  w4 *key;
  int64_t n, c;
  int pos, buf, pend;
  int blk;      // launch-relative block of pos
  int hq;       // launch-relative index of the next quad to load
  w4 cur;
  w4 *win;   // this lane's slot 0 (slot stride blockDim.x)

  __device__ __forceinline__ w4 &q(int b, int i) {
    return key[((int64_t)b * kQ + i) * n + c];
  }
  __device__ __forceinline__ w4 &slot(int k) {
    return win[(k & (kW - 1)) * kBlockLegacy];
  }
  __device__ __forceinline__ int aq() const { return blk * kQ + (pos >> 2); }

  __device__ __forceinline__ void twist_from(int s) { mt3_twist(key, n, c, s); }

  // quads hq .. hq + H - 1 into the ring (their slots' quads are consumed)
  // the step-top refill: maintain() has twisted the next block already
  __device__ __forceinline__ void refill() {
    const int nb = (blk + 1) * kQ;   // first quad of the next block
    w4 v[H];
#pragma unroll
    for (int u = 0; u < H; ++u) {
      const int k = hq + u;
      const bool nx = k >= nb;
      v[u] = q(buf ^ (nx ? 1 : 0), nx ? k - nb : k - blk * kQ);
    }
#pragma unroll
    for (int u = 0; u < H; ++u) slot(hq + u) = v[u];
    hq += H;
  }

  __device__ __forceinline__ void refill_cold() {
    pend = mt3_refill_cold<H>(key, n, c, win, hq, blk, buf, pend);
    hq += H;
  }

  __device__ __forceinline__ void init(int st, w4 *w) {
    pos = st & 0xFFFF;
    buf = (st >> 16) & 1;
    pend = (st >> 17) & 1;
    blk = 0;
    win = w;
    if (pend && pos >= kRefill) {
      twist_from(buf);
      pend = 0;
    }
    hq = pos >> 2;
    refill_cold();
    refill_cold();
    if (pos & 3) cur = slot(aq());
  }

  // wave-uniform point (top of a step): the refill twist, then the window
  __device__ __forceinline__ void maintain() {
    // the refill twist: at word 312, or earlier when the head's next refill
    // enters the next block
    const bool due = pend && (pos >= kRefill || hq + H > (blk + 1) * kQ);
    if (__builtin_amdgcn_ballot_w64(due)) {
      if (pend) {   // every pending lane: its free buffer holds a consumed block
        twist_from(buf);
        pend = 0;
      }
    }
    if (__builtin_amdgcn_ballot_w64(hq - aq() <= H)) {
      if (hq - aq() <= H) refill();
    }
  }

  __device__ __forceinline__ uint32_t next32() {
    if (pos == kN) {
      buf ^= 1;
      pos = 0;
      pend = 1;
      ++blk;
    }
    const int u = pos & 3;
    if (u == 0) {
      const int k = aq();
      if (k >= hq) refill_cold();   // a step longer than the window (rare)
      cur = slot(k);
    }
    ++pos;
    uint32_t y = u == 0 ? cur.x : (u == 1 ? cur.y : (u == 2 ? cur.z : cur.w));
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
  }

  __device__ __forceinline__ static uint32_t temper(uint32_t y) {
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
  }

  // random_sample's two words at once: at an even position both words lie in
  // one quad (words 0-1 or 2-3) and in one block (624 is even).  Only
  // randint's single words make the position odd.
  __device__ __forceinline__ double next_double() {
    uint32_t wa, wb;
    if (pos & 1) {
      wa = next32();
      wb = next32();
    } else {
      if (pos == kN) {
        buf ^= 1;
        pos = 0;
        pend = 1;
        ++blk;
      }
      const bool lo = (pos & 3) == 0;
      if (lo) {
        const int k = aq();
        if (k >= hq) refill_cold();   // a step longer than the window (rare)
        cur = slot(k);
      }
      pos += 2;
      wa = temper(lo ? cur.x : cur.z);
      wb = temper(lo ? cur.y : cur.w);
    }
    const int32_t a = (int32_t)(wa >> 5), b = (int32_t)(wb >> 6);
    return (a * 67108864.0 + b) / 9007199254740992.0;
  }

  // Two polar attempts read ahead without consuming: the four doubles
  // (x1, x2 of attempt a, x1, x2 of attempt b) at words pos .. pos + 7
  // (pos even: two quads, or three when pos is 2 mod 4), as 2 d - 1.
  __device__ __forceinline__ void attempts2(double &x1a, double &x2a, double &x1b,
                                            double &x2b) {
    if (pos == kN) {
      buf ^= 1;
      pos = 0;
      pend = 1;
      ++blk;
    }
    const int k = aq();
    if (k + 2 >= hq) refill_cold();   // fewer than 3 quads staged (rare)
    const w4 A = slot(k), B = slot(k + 1), C = slot(k + 2);
    const bool lo = (pos & 3) == 0;
    const uint32_t w0 = temper(lo ? A.x : A.z), w1 = temper(lo ? A.y : A.w);
    const uint32_t w2 = temper(lo ? A.z : B.x), w3 = temper(lo ? A.w : B.y);
    const uint32_t w4_ = temper(lo ? B.x : B.z), w5 = temper(lo ? B.y : B.w);
    const uint32_t w6 = temper(lo ? B.z : C.x), w7 = temper(lo ? B.w : C.y);
    auto dbl = [](uint32_t a, uint32_t b) {
      const int32_t ai = (int32_t)(a >> 5), bi = (int32_t)(b >> 6);
      return (ai * 67108864.0 + bi) / 9007199254740992.0;
    };
    x1a = 2.0 * dbl(w0, w1) - 1.0;
    x2a = 2.0 * dbl(w2, w3) - 1.0;
    x1b = 2.0 * dbl(w4_, w5) - 1.0;
    x2b = 2.0 * dbl(w6, w7) - 1.0;
  }

  // consume nw (4 or 8) words read by attempts2
  __device__ __forceinline__ void advance(int nw) {
    pos += nw;
    if (pos > kN) {   // (pos == kN flips lazily, as in next_double)
      pos -= kN;
      buf ^= 1;
      pend = 1;
      ++blk;
    }
    if (pos & 3) cur = slot(aq());
  }

  __device__ __forceinline__ int packed() const {
    return pos | (buf << 16) | (pend << 17);
  }
};

// ---------------------------------------------------------------------------
// Mt4 (the default since round 4): FOUR blocks per chain in a chunked
// layout, consumed through Mt3's LDS window.
// Why: the lanes of a wave drift apart in the stream (the polar rejection
// consumes a variable number of words: after 1 000 cfg2 steps the spread is
// several hundred words), and with two buffers a lane can twist only between
// flipping into a block and reaching its middle -- so the twist ran as
// several partial-wave rounds per block, and the [quad][chain] layout made a
// drifted lane's 16-byte reads and writes share 128-byte lines with lanes that
// needed them at other times (profiles/r04p_leg: 2 487 VALU per wave-step,
// 14.4 GB of HBM traffic per 250 cfg2-width steps against ~7 GB of data, the
// time growing call after call with the drift).
// Here each chain keeps its current block and up to three twisted blocks
// after it (`ready`).  A twist round runs for the whole wave when any lane
// has nothing ahead and is half-way through its block (or its window head is
// about to enter the next block); every lane that is not full twists one
// block further, so the leader sets the pace and the laggards bank blocks
// (correct for any drift: a lane that reaches a block end with nothing ahead
// twists alone, out of line).  Layout [4][20 chunks][n][8 quads] of uint4: a
// block of 156 quads padded to 160, and a chunk is one 128-byte line per lane,
// so the window's refills (whole chunks) and the twists move whole lines
// whatever the other lanes' positions.
// Packed state: pos | cb << 16 | ready << 20 (4-bit fields: kK4 = 16 buffers) (cb = the current block's buffer).
// ---------------------------------------------------------------------------
// The twist through a raw buffer resource over the whole state (the engine
// takes this layout only while it spans < 2^32 bytes): each lane's source and
// destination buffers are one per-lane byte offset each, and every quad's
// chunk and position a uniform offset -- no per-load 64-bit address
// arithmetic (with plain pointers the compiler spent ~8 VALU per load on
// (b 20 + chunk) n + c).
__device__ __forceinline__ void mt4_twist(w4 *key, int64_t n, int64_t c, int s, int d) {
  typedef uint32_t v4u __attribute__((ext_vector_type(4)));
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(key, 0, -1, 0x00020000);
  const uint32_t plane = (uint32_t)n * 128u;   // one chunk of every chain
  const uint32_t vs = (uint32_t)c * 128u + (uint32_t)(s * kCh) * plane;
  const uint32_t vd = (uint32_t)c * 128u + (uint32_t)(d * kCh) * plane;
  auto off = [&](int i) { return (uint32_t)(i >> 3) * plane + (uint32_t)(i & 7) * 16u; };
  twist_ls(
      [&](int b, int i) -> w4 {
        const v4u v = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(b ? vd : vs), (int)off(i), 0);
        return w4{v.x, v.y, v.z, v.w};
      },
      [&](int i, w4 v) {
        __builtin_amdgcn_raw_buffer_store_b128(v4u{v.x, v.y, v.z, v.w}, rs, (int)vd, (int)off(i), 0);
      });
}
// a lane that needs a block nobody twisted for it (out of line, rare)
__device__ __attribute__((noinline)) void mt4_twist_cold(w4 *key, int64_t n, int64_t c,
                                                         int s, int d) {
  mt4_twist(key, n, c, s, d);
}
// stage the chunk at stream quad hq (launch-relative; block hq / 156) into
// the ring; returns the number of quads staged (8, or 4 for a block's last)
__device__ __forceinline__ void mt4_load(w4 *key, int64_t n, int64_t c, int b, int hc,
                                         w4 (&v)[8]) {
  typedef uint32_t v4u __attribute__((ext_vector_type(4)));
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(key, 0, -1, 0x00020000);
  const uint32_t vo = ((uint32_t)(b * kCh + hc) * (uint32_t)n + (uint32_t)c) * 128u;
#pragma unroll
  for (int u = 0; u < 8; ++u) {   // one line
    const v4u t = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)vo, u * 16, 0);
    v[u] = w4{t.x, t.y, t.z, t.w};
  }
}
// DBL: the ring holds each quad as the two random_sample doubles of its
// word pairs (every draw of the Normal / Raw / Gibbs streams is a double at
// an even position), tempered and converted once per word as the quad is
// staged instead of at every read-ahead of the lockstep attempts
template <bool DBL>
__device__ __forceinline__ int mt4_put(w4 *win, int kw, int hc, int hq, const w4 (&v)[8]) {
  const int nq = hc == kCh - 1 ? 4 : 8;
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    if (u < nq) {
      if constexpr (DBL) {
        const double2 d{mt_dbl(v[u].x, v[u].y), mt_dbl(v[u].z, v[u].w)};
        reinterpret_cast<double2 *>(win)[((hq + u) & (kw - 1)) * kBlockLegacy] = d;
      } else {
        win[((hq + u) & (kw - 1)) * kBlockLegacy] = v[u];
      }
    }
  }
  return nq;
}
template <bool DBL>
__device__ __forceinline__ int mt4_stage(w4 *key, int64_t n, int64_t c, w4 *win, int kw,
                                         int b, int hc, int hq) {
  w4 v[8];
  mt4_load(key, n, c, b, hc, v);
  return mt4_put<DBL>(win, kw, hc, hq, v);
}
// the rare refills (a launch's first, a step longer than the window) out of
// line; the head's block is twisted first if nothing has (values in and out:
// returns (ready << 32) | hq, each a full 32-bit field: hq counts the launch's
// quads per chain and grows past 2^24 in a launch of a few million steps)
// (NC chunks: H / 8 when the window is nearly empty, the regular refill's
// kRC at a step top)
template <int H, bool DBL, int NC = H / 8>
__device__ __attribute__((noinline)) uint64_t mt4_refill_cold(w4 *key, int64_t n, int64_t c,
                                                         w4 *win, int hq, int blk, int cb,
                                                         int ready) {
#pragma unroll 1
  for (int k = 0; k < NC; ++k) {
    const int hb = hq / kQ, hc = (hq - hb * kQ) >> 3;
    if (hb - blk > ready) {   // the head's block is not twisted yet
      mt4_twist_cold(key, n, c, (cb + ready) & kBufMask, (cb + ready + 1) & kBufMask);
      ++ready;
    }
    hq += mt4_stage<DBL>(key, n, c, win, 2 * H, (cb + hb - blk) & kBufMask, hc, hq);
  }
  return ((uint64_t)(uint32_t)ready << 32) | (uint32_t)hq;
}

// Window refills of kRC chunks (PBH_LEGACY_RC, default 1): a lane stages
// its next chunk whenever the ring has room for it.  The lanes of a wave
// reach their refills at different steps (they drift apart in the stream),
// so a refill's code runs for the wave at nearly every step whoever needs it:
// with two-chunk refills (16 quads, the round-4 form, PBH_LEGACY_RC=2) the
// wave converted 16 quads' worth of doubles per step for ~7 quads consumed
// per lane-step; with one-chunk refills it converts 8.
#ifndef PBH_LEGACY_RC
#define PBH_LEGACY_RC 1
#endif
template <int H, bool DBL = false>
struct Mt4 {
  static constexpr bool kLockstep = true;
  static constexpr bool kPeek = true;   // attempts2 / advance
  static constexpr bool kPeek4 = DBL;   // attempts4 (four attempts per iteration)
  static constexpr bool kLogTab = true;  // the polar log from log_leg's table
  static constexpr int kRefill = 312;
  static constexpr int kW = 2 * H;      // window quads per lane (a power of two)
  static_assert(H % 8 == 0, "whole chunks per refill");
  // chunks per regular refill (the cold path stages H / 8); a refill when
  // the ring has room for them
  static constexpr int kRC = PBH_LEGACY_RC < H / 8 ? PBH_LEGACY_RC : H / 8;
  static constexpr int kRoom = kW - 8 * kRC;
  w4 *key;
  int64_t n, c;
  int pos, cb, ready;
  int blk;      // launch-relative block of pos
  int hq;       // launch-relative stream quad (blk * 156 + quad) the head stages next
  int hb, hc;   // the head's launch-relative block and chunk
  w4 cur;
  w4 *win;      // this lane's slot 0 (slot stride blockDim.x)
  // the next refill's chunks, loaded one refill ahead (pf): their loads
  // complete during the steps in between instead of stalling the step top
  w4 pfv[kRC][8];
  bool pf;

  __device__ __forceinline__ w4 &slot(int k) {
    return win[(k & (kW - 1)) * kBlockLegacy];
  }
  __device__ __forceinline__ int aq() const { return blk * kQ + (pos >> 2); }

  template <int NC = H / 8>
  __device__ __forceinline__ void refill_cold() {
    const uint64_t r = mt4_refill_cold<H, DBL, NC>(key, n, c, win, hq, blk, cb, ready);
    hq = (int)(uint32_t)r;
    ready = (int)(uint32_t)(r >> 32);
    hb = hq / kQ;
    hc = (hq - hb * kQ) >> 3;
    pf = false;   // the head moved: a prefetched refill is stale
  }

  // the next refill's blocks are twisted
  __device__ __forceinline__ bool ahead_ok() const {
    return (hb - blk) + (hc + kRC > kCh ? 1 : 0) <= ready;
  }
  __device__ __forceinline__ void prefetch() {
    int b = hb, ch = hc;
#pragma unroll
    for (int k = 0; k < kRC; ++k) {
      mt4_load(key, n, c, (cb + b - blk) & kBufMask, ch, pfv[k]);
      if (++ch == kCh) {
        ch = 0;
        ++b;
      }
    }
    pf = true;
  }
  __device__ __forceinline__ void commit() {
#pragma unroll
    for (int k = 0; k < kRC; ++k) {
      hq += mt4_put<DBL>(win, kW, hc, hq, pfv[k]);
      if (++hc == kCh) {
        hc = 0;
        ++hb;
      }
    }
    pf = false;
  }

  __device__ __forceinline__ void init(int st, w4 *w) {
    pos = st & 0xFFFF;
    cb = (st >> 16) & kBufMask;
    ready = (st >> 20) & kBufMask;
    blk = 0;
    win = w;
    hb = 0;
    pf = false;
    hc = (pos >> 2) >> 3;   // the chunk holding pos (pos = 624: the last one)
    hq = hc * 8;
    refill_cold();
    refill_cold();
    if (pos & 3) cur = slot(aq());
  }

  // wave-uniform point (top of a step): a twist round, then the window
  __device__ __forceinline__ void maintain() {
    const bool due = ready == 0 && (pos >= kRefill || hb > blk || hc + kRC > kCh);
    if (__builtin_amdgcn_ballot_w64(due)) {
      if (ready < kK4 - 1) {   // every lane with a free buffer: one block further
        mt4_twist(key, n, c, (cb + ready) & kBufMask, (cb + ready + 1) & kBufMask);
        ++ready;
      }
    }
    if (__builtin_amdgcn_ballot_w64(hq - aq() <= kRoom)) {
      if (hq - aq() <= kRoom) {
        // loaded ahead (complete since the last step's mid-step wait), or not
        // (its block was not twisted then): the same chunks staged out of
        // line, so that the common path's code carries no wait for loads
        // just issued (one shared commit waited vmcnt down to 0 -- i.e. for
        // the last step's trace stores -- on both paths)
        if (pf) commit();
        else refill_cold<kRC>();   // (the ring has room for kRC chunks only)
      }
    }
    // the next refill, ahead (whenever its blocks are twisted)
    if (__builtin_amdgcn_ballot_w64(!pf && ahead_ok())) {
      if (!pf && ahead_ok()) prefetch();
    }
  }

  __device__ __forceinline__ void flip() {   // into the next block (pos = kN)
    if (ready == 0) {   // nothing twisted ahead (a step longer than half a block)
      mt4_twist_cold(key, n, c, cb, (cb + 1) & kBufMask);
      ready = 1;
    }
    cb = (cb + 1) & kBufMask;
    --ready;
    pos = 0;
    ++blk;
  }

  __device__ __forceinline__ static uint32_t temper(uint32_t y) {
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
  }

  __device__ __forceinline__ uint32_t next32() {
    static_assert(!DBL, "the staged-double ring holds no raw words");
    if (pos == kN) flip();
    const int u = pos & 3;
    if (u == 0) {
      const int k = aq();
      if (k >= hq) refill_cold();   // a step longer than the window (rare)
      cur = slot(k);
    }
    ++pos;
    return temper(u == 0 ? cur.x : (u == 1 ? cur.y : (u == 2 ? cur.z : cur.w)));
  }

  __device__ __forceinline__ const double2 &dslot(int k) {
    return reinterpret_cast<const double2 *>(win)[(k & (kW - 1)) * kBlockLegacy];
  }

  // random_sample's two words at once (as Mt3); DBL: the staged double
  __device__ __forceinline__ double next_double() {
    if constexpr (DBL) {   // positions are even
      if (pos == kN) flip();
      const int k = aq();
      if (k >= hq) refill_cold();
      const double2 d = dslot(k);
      const double r = (pos & 2) ? d.y : d.x;
      pos += 2;
      return r;
    } else {
      uint32_t wa, wb;
      if (pos & 1) {
        wa = next32();
        wb = next32();
      } else {
        if (pos == kN) flip();
        const bool lo = (pos & 3) == 0;
        if (lo) {
          const int k = aq();
          if (k >= hq) refill_cold();
          cur = slot(k);
        }
        pos += 2;
        wa = temper(lo ? cur.x : cur.z);
        wb = temper(lo ? cur.y : cur.w);
      }
      const int32_t a = (int32_t)(wa >> 5), b = (int32_t)(wb >> 6);
      return (a * 67108864.0 + b) / 9007199254740992.0;
    }
  }

  // two polar attempts read ahead without consuming (as Mt3): the stream's
  // quads are contiguous in the ring across a block end
  __device__ __forceinline__ void attempts2(double &x1a, double &x2a, double &x1b,
                                            double &x2b) {
    if (pos == kN) flip();
    const int k = aq();
    if (k + 2 >= hq) refill_cold();   // fewer than 3 quads staged (rare)
    const w4 A = slot(k), B = slot(k + 1), C = slot(k + 2);
    const bool lo = (pos & 3) == 0;
    const uint32_t w0 = temper(lo ? A.x : A.z), w1 = temper(lo ? A.y : A.w);
    const uint32_t w2 = temper(lo ? A.z : B.x), w3 = temper(lo ? A.w : B.y);
    const uint32_t w4_ = temper(lo ? B.x : B.z), w5 = temper(lo ? B.y : B.w);
    const uint32_t w6 = temper(lo ? B.z : C.x), w7 = temper(lo ? B.w : C.y);
    auto dbl = [](uint32_t a, uint32_t b) {
      const int32_t ai = (int32_t)(a >> 5), bi = (int32_t)(b >> 6);
      return (ai * 67108864.0 + bi) / 9007199254740992.0;
    };
    x1a = 2.0 * dbl(w0, w1) - 1.0;
    x2a = 2.0 * dbl(w2, w3) - 1.0;
    x1b = 2.0 * dbl(w4_, w5) - 1.0;
    x2b = 2.0 * dbl(w6, w7) - 1.0;
  }

  // DBL: four polar attempts read ahead without consuming (words pos ..
  // pos + 15, pos even: four slots, or five when pos is 2 mod 4), as 2 d - 1
  __device__ __forceinline__ void attempts4(double (&x1)[4], double (&x2)[4]) {
    if (pos == kN) flip();
    const int k = aq();
    if (k + 4 >= hq) refill_cold();   // fewer than 5 quads staged (rare)
    const double2 A = dslot(k), B = dslot(k + 1), C = dslot(k + 2), D = dslot(k + 3),
                  E = dslot(k + 4);
    const bool lo = (pos & 3) == 0;
    const double d[8] = {lo ? A.x : A.y, lo ? A.y : B.x, lo ? B.x : B.y, lo ? B.y : C.x,
                         lo ? C.x : C.y, lo ? C.y : D.x, lo ? D.x : D.y, lo ? D.y : E.x};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      x1[i] = 2.0 * d[2 * i] - 1.0;
      x2[i] = 2.0 * d[2 * i + 1] - 1.0;
    }
  }

  // consume nw (a multiple of 4, <= 16) words read by attempts2 / attempts4
  __device__ __forceinline__ void advance(int nw) {
    pos += nw;
    if (pos > kN) {   // (pos == kN flips lazily)
      const int rest = pos - kN;
      pos = kN;
      flip();
      pos = rest;
    }
    if constexpr (!DBL)
      if (pos & 3) cur = slot(aq());
  }

  __device__ __forceinline__ int packed() const { return pos | (cb << 16) | (ready << 20); }
};

// Seeding for Mt4: init_genrand into buffer 0, the first twist into buffer 1;
// the lane starts at word 0 of buffer 1 with nothing twisted ahead.
__global__ __launch_bounds__(256) void mt_seed_k4_kernel(uint32_t *key, int32_t *pos,
                                                         double *gauss, int32_t *has_gauss,
                                                         const uint32_t *seeds, int64_t n) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= n) return;
  w4 *qk = reinterpret_cast<w4 *>(key);
  uint32_t s = seeds[c];
  for (int i = 0; i < kQ; ++i) {
    w4 w;
    w.x = s; s = 1812433253u * (s ^ (s >> 30)) + (uint32_t)(4 * i + 1);
    w.y = s; s = 1812433253u * (s ^ (s >> 30)) + (uint32_t)(4 * i + 2);
    w.z = s; s = 1812433253u * (s ^ (s >> 30)) + (uint32_t)(4 * i + 3);
    w.w = s; s = 1812433253u * (s ^ (s >> 30)) + (uint32_t)(4 * i + 4);
    k4q(qk, n, c, 0, i) = w;
  }
  mt4_twist(qk, n, c, 0, 1);
  pos[c] = 0 | (1 << 16) | (0 << 20);
  gauss[c] = 0.0;
  has_gauss[c] = 0;
}

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
  uint4 *qk = reinterpret_cast<uint4 *>(key);
  uint32_t s = seeds[c];
  for (int i = 0; i < kQ; ++i) {
    uint32_t w[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      w[u] = s;
      s = 1812433253u * (s ^ (s >> 30)) + (uint32_t)(4 * i + u + 1);
    }
    qk[(int64_t)i * n + c] = make_uint4(w[0], w[1], w[2], w[3]);
  }
  Mt2 m{qk, n, c, 0, 0, 0, make_uint4(0u, 0u, 0u, 0u)};
  m.twist_from(0);
  m.buf = 1;
  m.pos = 0;
  m.pend = 1;
  pos[c] = m.packed();
  gauss[c] = 0.0;
  has_gauss[c] = 0;
}

// MODE: -1 any (runtime flags), else the one path a kernel compiles
// (kModeGibbs, kModeVardelta, kModeNormal, kModeRaw) -- one path per kernel
// keeps each function small (isa_e64.py rewrites only functions < 128 KB).
constexpr int kModeAny = -1, kModeGibbs = 0, kModeVardelta = 1, kModeNormal = 2,
              kModeRaw = 3;


// The polar method's attempts of one step (legacy_gauss's draws): lanes run
// the ATTEMPTS in lockstep (one per iteration until each holds its `need`
// pairs: a wave loops ~max over lanes of the step's attempts, about 9.5 for 5
// pairs, not the sum over pairs of per-pair maxima, about 18), keeping only
// the accepted (x1, x2) in LDS, [pair][thread].
template <class M>
__device__ __forceinline__ void polar_attempts(M &m, int need, double2 *stage,
                                               int tid = (int)threadIdx.x) {
  int np = 0;
  if constexpr (M::kPeek && M::kPeek4) {
    // four attempts per lockstep iteration from the staged doubles
    // (~3 iterations for 5 pairs), consumed only as far as they are used
    while (__builtin_amdgcn_ballot_w64(np < need)) {   // wave-uniform
      if (np < need) {
        double x1[4], x2[4];
        m.attempts4(x1, x2);
        int used = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const double r2 = x1[i] * x1[i] + x2[i] * x2[i];
          if (np < need) {
            used += 4;
            if (r2 < 1.0 && r2 != 0.0) {
              stage[np * kBlockLegacy + tid] = make_double2(x1[i], x2[i]);
              ++np;
            }
          }
        }
        m.advance(used);
      }
    }
  } else if constexpr (M::kPeek) {
    // two attempts per lockstep iteration (read ahead from the window,
    // consumed only as far as they are used): ~5.5 iterations for 5
    // pairs instead of ~9.5, and two independent chains of arithmetic
    while (__builtin_amdgcn_ballot_w64(np < need)) {   // wave-uniform
      if (np < need) {
        double x1a, x2a, x1b, x2b;
        m.attempts2(x1a, x2a, x1b, x2b);
        const double r2a = x1a * x1a + x2a * x2a;
        const double r2b = x1b * x1b + x2b * x2b;
        if (r2a < 1.0 && r2a != 0.0) {
          stage[np * kBlockLegacy + tid] = make_double2(x1a, x2a);
          ++np;
        }
        int used = 4;
        if (np < need) {
          used = 8;
          if (r2b < 1.0 && r2b != 0.0) {
            stage[np * kBlockLegacy + tid] = make_double2(x1b, x2b);
            ++np;
          }
        }
        m.advance(used);
      }
    }
  } else {
    while (__builtin_amdgcn_ballot_w64(np < need)) {   // wave-uniform
      if (np < need) {
        const double x1 = 2.0 * m.next_double() - 1.0;
        const double x2 = 2.0 * m.next_double() - 1.0;
        const double r2 = x1 * x1 + x2 * x2;
        if (r2 < 1.0 && r2 != 0.0) {
          stage[np * kBlockLegacy + tid] = make_double2(x1, x2);
          ++np;
        }
      }
    }
  }
}

// The transcendental part of accepted pair k: f = sqrt(-2 ln r2 / r2), the
// deviates (f x2, f x1) in legacy_gauss's order.
template <class M>
__device__ __forceinline__ void polar_pair(const double2 *stage, int k, const double *s_lg,
                                           double &g0, double &g1) {
  const double2 p = stage[k * kBlockLegacy + threadIdx.x];
  const double r2 = p.x * p.x + p.y * p.y;
  double lr;
  if constexpr (M::kLogTab) lr = log_leg(r2, s_lg);   // Mt4: the table log
  else lr = log(r2);
  const double f = sqrt(-2.0 * lr / r2);
  g0 = f * p.y;
  g1 = f * p.x;
}

// s_ord (the windowed kernels): order[j] n per draw j, staged in LDS at the
// kernel's start.  Read from a.order, every row index was a vector load
// whose s_waitcnt vmcnt(0) also waited for the step's earlier trace stores
// to be acknowledged (gfx9's vmcnt counts stores too) -- ten store round
// trips per cfg2 step; so was blockDim.x (an implicit-argument load).
template <class M, int MODE = kModeAny, bool SORD = false>
__device__ __forceinline__ void legacy_gen_body(const LegacyArgs &a, int64_t c, M &m,
                                                double2 *stage = nullptr,
                                                const uint32_t *s_ord = nullptr,
                                                const double *s_lg = nullptr) {
  constexpr bool kAny = MODE == kModeAny;
  auto ord = [&](int j) -> int64_t {
    if constexpr (SORD) return (int64_t)s_ord[j];
    else return (int64_t)a.order[j] * a.n;
  };
  double gauss = a.gauss[c];
  int has = a.has_gauss[c];
  // every load before the step loop completes here, once: a load result
  // carried into the loop (gauss, has) otherwise made the wait pass put an
  // s_waitcnt vmcnt(0) at its first use in EVERY step -- which also waited
  // for the previous step's trace stores and the prefetch just issued
  __builtin_amdgcn_s_waitcnt(0);
  const int64_t rowlen = (int64_t)a.R * a.n;
  for (int64_t t = 0; t < a.n_steps; ++t) {
    double *row = a.out + t * rowlen + c;
    m.maintain();   // wave-uniform: every active lane is here
    if ((kAny || MODE == kModeGibbs) && (!kAny || a.gibbs)) {
      // rf.py:446-452: block (step0 + t) mod ceil(d / tsteps) of the cycle
      const int64_t nblk = (a.d + a.R - 1) / a.R;
      const int cm = (int)(((a.step0 + t) % nblk) * a.R);
      const int cnt = (cm + a.R < a.d ? cm + a.R : a.d) - cm;
      for (int j = 0; j < a.R; ++j)
        row[(int64_t)j * a.n] = j < cnt ? m.next_double() : __builtin_nan("");
      continue;
    }
    if constexpr (kAny || MODE == kModeVardelta) {
      if (!kAny || a.vardelta) {
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
    }
    if (M::kLockstep && (kAny || MODE == kModeNormal) && (!kAny || a.normal)) {
      // the step's d polar-method normals.  Lanes run the ATTEMPTS in
      // lockstep (one per iteration until each holds its pairs: a wave loops
      // ~max over lanes of the step's attempts, about 9.5 for 5 pairs, not
      // the sum over pairs of per-pair maxima, about 18), keeping only the
      // accepted (x1, x2) in LDS; the transcendental part f = sqrt(-2 ln r2 /
      // r2) then runs over the step's pairs as independent chains.  The
      // draws, their order, the arithmetic and the cached deviate are
      // legacy_gauss's exactly.
      // every chain draws d normals per step from the same start, so the
      // cached-deviate flag is the same in every lane: made wave-uniform, the
      // row indices order[j] below are scalar loads
      has = __builtin_amdgcn_readfirstlane(has);
      int j0 = 0;
      if (has) {
        row[ord(0)] = gauss;
        has = 0;
        gauss = 0.0;
        j0 = 1;
      }
      const int need = (a.d - j0 + 1) / 2;   // pairs this lane draws
      polar_attempts(m, need, stage);
      // Wait here for this step's window prefetch (issued at the step top,
      // complete by now) and the previous step's trace stores (issued ~a step
      // ago): vmcnt(0) only, once per step, before this step's stores.  The
      // prefetched chunks are then complete in the compiler's view, so the
      // commit that consumes them in a later step needs no vmcnt(0) -- which
      // there also waited for the round trip of the stores just issued.
      __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0), expcnt / lgkmcnt untouched
      // the pairs' transcendental part, two independent pairs per
      // iteration (one basic block: the scheduler interleaves their log /
      // division / square-root chains); a last pair whose second deviate is
      // cached (odd d - j0) after them
      const int half = (a.d - j0) & 1;
      const int nfull = need - half;
      auto polar = [&](int k, double &g0, double &g1) { polar_pair<M>(stage, k, s_lg, g0, g1); };
      int k = 0;
      for (; k + 2 <= nfull; k += 2) {
        double a0, a1, b0, b1;
        polar(k, a0, a1);
        polar(k + 1, b0, b1);
        const int j = j0 + 2 * k;
        row[ord(j)] = a0;
        row[ord(j + 1)] = a1;
        row[ord(j + 2)] = b0;
        row[ord(j + 3)] = b1;
      }
      if (k < nfull) {
        double a0, a1;
        polar(k, a0, a1);
        row[ord(j0 + 2 * k)] = a0;
        row[ord(j0 + 2 * k + 1)] = a1;
        ++k;
      }
      if (half) {
        double a0, a1;
        polar(k, a0, a1);
        row[ord(j0 + 2 * k)] = a0;
        gauss = a1;   // cached for the next draw (odd d)
        has = 1;
      }
      row[(int64_t)a.d * a.n] = m.next_double();   // the MH threshold
      continue;
    }
    if constexpr (!kAny && MODE != kModeRaw) continue;   // not reached
    for (int j = 0; j < a.d; ++j) {
      const double v = (kAny && a.normal) ? legacy_gauss(m, gauss, has) : m.next_double();
      row[ord(j)] = v;    // draw j feeds dim order[j]
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
  Mt2 m{reinterpret_cast<uint4 *>(a.key), a.n, c, st & 0xFFFF, (st >> 16) & 1,
        (st >> 17) & 1, make_uint4(0u, 0u, 0u, 0u)};
  m.load_cur();
  // accepted polar pairs of one step, [pair][thread] (bank-conflict free)
  __shared__ double2 s_stage[(PBH_MAX_DIM + 1) / 2 * 256];
  legacy_gen_body(a, c, m, s_stage);
  a.pos[c] = m.packed();
}

// The windowed generator (Mt3): dynamic LDS = the lanes' rings (2H quads
// each) followed by the polar stage ((d + 1) / 2 pairs each).
template <int H, int MODE>
__global__ __launch_bounds__(kBlockLegacy) __attribute__((amdgpu_waves_per_eu(1, 1)))
void legacy_gen_win_kernel(LegacyArgs a) {
  extern __shared__ w4 s_lw[];
  __shared__ uint32_t s_ord[PBH_MAX_DIM];   // order[j] n (a multiple of 16 B)
  if (!a.gibbs && threadIdx.x < (unsigned)a.d) s_ord[threadIdx.x] = (uint32_t)(a.order[threadIdx.x] * a.n);
  __syncthreads();
  const int64_t c = (int64_t)blockIdx.x * kBlockLegacy + threadIdx.x;
  if (c >= a.n) return;
  Mt3<H> m;
  m.key = reinterpret_cast<w4 *>(a.key);
  m.n = a.n;
  m.c = c;
  m.init(a.pos[c], s_lw + threadIdx.x);
  legacy_gen_body<Mt3<H>, MODE, true>(a, c, m, reinterpret_cast<double2 *>(s_lw + 2 * H * kBlockLegacy), s_ord);
  a.pos[c] = m.packed();
}

template <int H, int MODE>
__global__ __launch_bounds__(kBlockLegacy) __attribute__((amdgpu_waves_per_eu(1, 1)))
void legacy_gen_k4_kernel(LegacyArgs a) {
  extern __shared__ w4 s_lw[];
  __shared__ uint32_t s_ord[PBH_MAX_DIM];   // order[j] n (a multiple of 16 B)
  __shared__ double s_lg[kLegLogDoubles];   // log_leg's table (a multiple of 16 B)
  if (!a.gibbs && threadIdx.x < (unsigned)a.d) s_ord[threadIdx.x] = (uint32_t)(a.order[threadIdx.x] * a.n);
  for (int i = threadIdx.x; i < kLegLogDoubles; i += kBlockLegacy) s_lg[i] = a.lgtab[i];
  __syncthreads();
  const int64_t c = (int64_t)blockIdx.x * kBlockLegacy + threadIdx.x;
  if (c >= a.n) return;
  // the staged-double ring for every stream of double draws (not randint's words)
  Mt4<H, MODE != kModeVardelta && MODE != kModeAny> m;
  m.key = reinterpret_cast<w4 *>(a.key);
  m.n = a.n;
  m.c = c;
  m.init(a.pos[c], s_lw + threadIdx.x);
  legacy_gen_body<Mt4<H, MODE != kModeVardelta && MODE != kModeAny>, MODE, true>(
      a, c, m, reinterpret_cast<double2 *>(s_lw + 2 * H * kBlockLegacy), s_ord, s_lg);
  a.pos[c] = m.packed();
}

template <int H, int MODE>
hipError_t launch_k4_mode(const LegacyArgs &a, hipStream_t s) {
  const int pairs = a.normal ? (a.d + 1) / 2 : 0;
  const size_t lds = (size_t)(2 * H + pairs) * kBlockLegacy * sizeof(uint4);
  hipError_t err = hipFuncSetAttribute(
      reinterpret_cast<const void *>(&legacy_gen_k4_kernel<H, MODE>),
      hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (err != hipSuccess) return err;
  const dim3 grid((unsigned)((a.n + kBlockLegacy - 1) / kBlockLegacy)), block(kBlockLegacy);
  hipLaunchKernelGGL((legacy_gen_k4_kernel<H, MODE>), grid, block, lds, s, a);
  return hipGetLastError();
}

template <int H>
hipError_t launch_k4(const LegacyArgs &a, hipStream_t s) {
  if (a.gibbs) return launch_k4_mode<H, kModeGibbs>(a, s);
  if (a.vardelta) return launch_k4_mode<H, kModeVardelta>(a, s);
  if (a.normal) return launch_k4_mode<H, kModeNormal>(a, s);
  return launch_k4_mode<H, kModeRaw>(a, s);
}

template <int H, int MODE>
hipError_t launch_win_mode(const LegacyArgs &a, hipStream_t s) {
  const int pairs = a.normal ? (a.d + 1) / 2 : 0;
  const size_t lds = (size_t)(2 * H + pairs) * kBlockLegacy * sizeof(uint4);
  hipError_t err = hipFuncSetAttribute(
      reinterpret_cast<const void *>(&legacy_gen_win_kernel<H, MODE>),
      hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (err != hipSuccess) return err;
  const dim3 grid((unsigned)((a.n + kBlockLegacy - 1) / kBlockLegacy)), block(kBlockLegacy);
  hipLaunchKernelGGL((legacy_gen_win_kernel<H, MODE>), grid, block, lds, s, a);
  return hipGetLastError();
}

template <int H>
hipError_t launch_win(const LegacyArgs &a, hipStream_t s) {
  if (a.gibbs) return launch_win_mode<H, kModeGibbs>(a, s);
  if (a.vardelta) return launch_win_mode<H, kModeVardelta>(a, s);
  if (a.normal) return launch_win_mode<H, kModeNormal>(a, s);
  return launch_win_mode<H, kModeRaw>(a, s);
}

// legacy_standard_exponential (legacy-distributions.c): -log(1 - random_sample)
template <class M>
__device__ __forceinline__ double legacy_exponential(M &m) {
  return -log(1.0 - m.next_double());
}

// NumPy's legacy_standard_gamma (random/src/legacy/legacy-distributions.c,
// the numpy 2.2.6 pinned in SURVEY.md §8c): Marsaglia-Tsang for shape > 1
// over the polar legacy gauss (its cached deviate included) and
// random_sample -- the squeeze 1 - 0.0331 x^4, then the log test -- and
// Johnk-style rejection for shape < 1; shape 1 is the exponential.  The
// operations and their order are NumPy's (-ffp-contract=off: no FMA).
template <class M>
__device__ double legacy_gamma(M &m, double &gauss, int &has, double shape) {
  if (shape == 1.0) return legacy_exponential(m);
  if (shape == 0.0) return 0.0;
  if (shape < 1.0) {
    for (;;) {
      const double U = m.next_double();
      const double V = legacy_exponential(m);
      if (U <= 1.0 - shape) {
        const double X = pow(U, 1. / shape);
        if (X <= V) return X;
      } else {
        const double Y = -log((1 - U) / shape);
        const double X = pow(1.0 - shape + shape * Y, 1. / shape);
        if (X <= (V + Y)) return X;
      }
    }
  }
  const double b = shape - 1. / 3.;
  const double c = 1. / sqrt(9 * b);
  for (;;) {
    double X, V;
    do {
      X = legacy_gauss(m, gauss, has);
      V = 1.0 + c * X;
    } while (V <= 0.0);
    V = V * V * V;
    const double U = m.next_double();
    if (U < 1.0 - 0.0331 * (X * X) * (X * X)) return (b * V);
    if (log(U) < 0.5 * X * X + b * (1. - V + log(V))) return (b * V);
  }
}

// pbh_legacy_draws: one chain per lane on Mt4's state through its window,
// the draws of each step in the reference's order, out [n_steps][n]
template <int H>
__global__ __launch_bounds__(kBlockLegacy) __attribute__((amdgpu_waves_per_eu(1, 1)))
void legacy_draws_kernel(LegacyArgs a, int32_t kind, double param) {
  extern __shared__ w4 s_lw[];
  const int64_t c = (int64_t)blockIdx.x * kBlockLegacy + threadIdx.x;
  if (c >= a.n) return;
  Mt4<H, true> m;
  m.key = reinterpret_cast<w4 *>(a.key);
  m.n = a.n;
  m.c = c;
  m.init(a.pos[c], s_lw + threadIdx.x);
  double gauss = a.gauss[c];
  int has = a.has_gauss[c];
  __builtin_amdgcn_s_waitcnt(0);
  for (int64_t t = 0; t < a.n_steps; ++t) {
    m.maintain();   // wave-uniform: every active lane is here
    const bool gam = kind == PBH_DRAWS_LINREG && (a.step0 + t) % 3 == 2;
    a.out[t * a.n + c] = gam ? legacy_gamma(m, gauss, has, param) : legacy_gauss(m, gauss, has);
  }
  a.pos[c] = m.packed();
  a.gauss[c] = gauss;
  a.has_gauss[c] = has;
}

// ---------------------------------------------------------------------------
// Fused REPLAY (legacy_mh_kernel): the generator and the REPLAY chain-step in
// one kernel.  The two-kernel form writes the [T][R][N] stream (1.44 GB per
// 250 cfg2-width steps) and the REPLAY kernel reads it back; here each
// step's draws go from the Mt4 window straight into the step's registers.
// mh_body (pbh_kernels_impl.h) is the REPLAY kernel's own body -- the same
// proposal, density, score and trace code -- with LegacyDraws as its draw
// source, which runs legacy_gen_body's per-step generation for the normal
// (callable Gaussian Delta) and raw (tuple / list delta) modes with the
// identity draw order (draw j feeds dim j): the values, their order and the
// cached deviate are the stream kernel's, so chains, traces and the legacy
// state equal legacy_replay + run.  Lanes past the last chain leave at once
// (the generator's ballots count active lanes only), so mh_body sees active
// lanes only and runs without the LDS observation stage (its
// __syncthreads); one chain per lane at one wavefront per SIMD (the window
// and the polar stage take ~155 KB of LDS per 256 lanes).
// ---------------------------------------------------------------------------
template <class M, bool NORMAL>
struct LegacyDraws {
  M &m;
  double2 *stage;
  const double *s_lg;
  double gauss;
  int has;
  double *thr_out;   // [n_steps][n] thresholds (pbh_set_record_threshold) or nullptr
  int64_t n;

  // every load before the step loop completes here, once (see legacy_gen_body)
  __device__ __forceinline__ void begin() { __builtin_amdgcn_s_waitcnt(0); }

  // the step's D normals with J0 = 1 when the cached deviate leads
  template <int D, int J0>
  __device__ __forceinline__ void normals(double (&r)[D]) {
    constexpr int need = (D - J0 + 1) / 2, half = (D - J0) & 1, nfull = need - half;
    if constexpr (J0 == 1) {
      r[0] = gauss;
      has = 0;
      gauss = 0.0;
    }
    polar_attempts(m, need, stage);
    __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0): as legacy_gen_body
#pragma unroll
    for (int k = 0; k < nfull; ++k) {
      double g0, g1;
      polar_pair<M>(stage, k, s_lg, g0, g1);
      r[J0 + 2 * k] = g0;
      r[J0 + 2 * k + 1] = g1;
    }
    if constexpr (half != 0) {
      double g0, g1;
      polar_pair<M>(stage, nfull, s_lg, g0, g1);
      r[J0 + 2 * nfull] = g0;
      gauss = g1;   // cached for the next draw (odd d)
      has = 1;
    }
  }

  template <int D>
  __device__ __forceinline__ void draws(const KArgs &, int s, int64_t cc, double (&r)[D],
                                        double &thr) {
    m.maintain();   // wave-uniform: every active lane is here
    if constexpr (NORMAL) {
      // the same flag in every lane (each chain draws D per step from the
      // same start): wave-uniform
      has = __builtin_amdgcn_readfirstlane(has);
      if (has) normals<D, 1>(r);
      else normals<D, 0>(r);
    } else {
#pragma unroll
      for (int k = 0; k < D; ++k) r[k] = m.next_double();
    }
    thr = m.next_double();   // the MH threshold
    if (thr_out) thr_out[(int64_t)s * n + cc] = thr;
  }
};

// ---------------------------------------------------------------------------
// Timing-only probe (PBH_LEGACY_FAKE=1; wrong streams, never a result): the
// fused kernel with the Mt4 generator replaced by a counter hash of the same
// interface -- no state in HBM, no twist, no window -- so that its time is
// what the polar method, the REPLAY step and the trace cost without MT19937.
// ---------------------------------------------------------------------------
struct FakeM {
  static constexpr bool kLockstep = true, kPeek = true, kPeek4 = true, kLogTab = true;
  uint32_t ctr, key;
  __device__ __forceinline__ static uint32_t mix(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    return x;
  }
  __device__ __forceinline__ double dbl(uint32_t i) const {
    const uint32_t a = mix(i ^ key), b = mix(i + 0x9E3779B9u * key);
    return ((double)(a >> 5) * 67108864.0 + (double)(b >> 6)) * (1.0 / 9007199254740992.0);
  }
  __device__ __forceinline__ void maintain() {}
  __device__ __forceinline__ double next_double() { return dbl(ctr++); }
  __device__ __forceinline__ void attempts4(double (&x1)[4], double (&x2)[4]) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      x1[i] = 2.0 * dbl(ctr + 2 * i) - 1.0;
      x2[i] = 2.0 * dbl(ctr + 2 * i + 1) - 1.0;
    }
  }
  __device__ __forceinline__ void advance(int nw) { ctr += (uint32_t)nw / 2; }
};

template <int D, bool NORMAL, int TGT, int PROP>
__global__ __launch_bounds__(kBlockLegacy) __attribute__((amdgpu_waves_per_eu(1, 1)))
void legacy_mh_fake_kernel(LegacyArgs la, KArgs a) {
  extern __shared__ w4 s_lw[];
  __shared__ double s_lg[kLegLogDoubles];
  for (int i = threadIdx.x; i < kLegLogDoubles; i += kBlockLegacy) s_lg[i] = la.lgtab[i];
  __syncthreads();
  const int64_t c = (int64_t)blockIdx.x * kBlockLegacy + threadIdx.x;
  if (c >= la.n) return;
  FakeM m{(uint32_t)la.step0 * 64u, (uint32_t)c * 0x85ebca6bu + 1u};
  LegacyDraws<FakeM, NORMAL> src{m, reinterpret_cast<double2 *>(s_lw), s_lg,
                                 la.gauss[c], la.has_gauss[c], la.thr, la.n};
  mh_body<D, PBH_RNG_REPLAY, TGT, PROP>(a, src, nullptr, false);
  la.gauss[c] = src.gauss;
  la.has_gauss[c] = src.has;
}

bool legacy_fake_on() {
  static const bool on = [] {
    const char *p = std::getenv("PBH_LEGACY_FAKE");
    return p && p[0] == '1';
  }();
  return on;
}

template <int D, int H, bool NORMAL, int TGT, int PROP>
__global__ __launch_bounds__(kBlockLegacy) __attribute__((amdgpu_waves_per_eu(1, 1)))
void legacy_mh_kernel(LegacyArgs la, KArgs a) {
  static_assert(kBlockLegacy == kBlock, "mh_body's chain index");
  extern __shared__ w4 s_lw[];
  __shared__ double s_lg[kLegLogDoubles];
  for (int i = threadIdx.x; i < kLegLogDoubles; i += kBlockLegacy) s_lg[i] = la.lgtab[i];
  __syncthreads();
  const int64_t c = (int64_t)blockIdx.x * kBlockLegacy + threadIdx.x;
  if (c >= la.n) return;
  using M = Mt4<H, true>;
  M m;
  m.key = reinterpret_cast<w4 *>(la.key);
  m.n = la.n;
  m.c = c;
  m.init(la.pos[c], s_lw + threadIdx.x);
  LegacyDraws<M, NORMAL> src{m, reinterpret_cast<double2 *>(s_lw + 2 * H * kBlockLegacy), s_lg,
                             la.gauss[c], la.has_gauss[c], la.thr, la.n};
  mh_body<D, PBH_RNG_REPLAY, TGT, PROP>(a, src, nullptr, false);
  la.pos[c] = m.packed();
  la.gauss[c] = src.gauss;
  la.has_gauss[c] = src.has;
}

template <int D, int H, bool NORMAL, int TGT, int PROP>
hipError_t launch_legacy_mh_t(const LegacyArgs &la, const KArgs &a, hipStream_t s) {
  const void *fn = reinterpret_cast<const void *>(&legacy_mh_kernel<D, H, NORMAL, TGT, PROP>);
  const size_t lds = (size_t)(2 * H + (NORMAL ? (D + 1) / 2 : 0)) * kBlockLegacy * sizeof(uint4);
  static const hipError_t attr =
      hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (attr != hipSuccess) return attr;
  const dim3 grid((unsigned)((la.n + kBlockLegacy - 1) / kBlockLegacy)), block(kBlockLegacy);
  // the timed region's events on the dispatch packet, as pbh_launch
  LaunchEvents &ev = launch_events();
  if (ev.start || ev.stop)
    (void)hipExtLaunchKernelGGL((legacy_mh_kernel<D, H, NORMAL, TGT, PROP>), grid, block,
                                (uint32_t)lds, s, ev.start, ev.stop, 0u, la, a);
  else
    hipLaunchKernelGGL((legacy_mh_kernel<D, H, NORMAL, TGT, PROP>), grid, block, lds, s, la, a);
  ev.start = nullptr;
  return hipGetLastError();
}

template <int D>
hipError_t launch_legacy_mh_d(const LegacyArgs &la, const KArgs &a, hipStream_t s) {
  constexpr int H = D <= 12 ? 16 : 8;   // the window while the stage leaves room
  if constexpr (D == 10) {
    if (legacy_fake_on() && la.normal && a.target == PBH_TARGET_DIAG_GAUSS &&
        a.prop == PBH_PROP_GAUSS) {   // timing-only probe (see FakeM)
      constexpr size_t lds = (size_t)((D + 1) / 2) * kBlockLegacy * sizeof(uint4);
      const dim3 grid((unsigned)((la.n + kBlockLegacy - 1) / kBlockLegacy)), block(kBlockLegacy);
      hipLaunchKernelGGL((legacy_mh_fake_kernel<D, true, PBH_TARGET_DIAG_GAUSS, PBH_PROP_GAUSS>),
                         grid, block, lds, s, la, a);
      return hipGetLastError();
    }
  }
  if (la.normal) {
    if (a.target == PBH_TARGET_DIAG_GAUSS && a.prop == PBH_PROP_GAUSS)   // cfg2's form
      return launch_legacy_mh_t<D, H, true, PBH_TARGET_DIAG_GAUSS, PBH_PROP_GAUSS>(la, a, s);
    return launch_legacy_mh_t<D, H, true, 0, 0>(la, a, s);
  }
  return launch_legacy_mh_t<D, 16, false, 0, 0>(la, a, s);
}



// ---------------------------------------------------------------------------
// Twist-ahead (legacy_ahead_kernel, round 6): before a fused REPLAY launch,
// every chain's Mt4 buffers after its current block are twisted in advance
// (`ready` raised to the launch's need), so that the fused kernel -- one
// chain per lane, one wavefront per SIMD at 65 536 chains, latency-bound --
// only consumes (window refills: load, temper, convert) and never twists in
// its own step loop.  Here ONE WAVEFRONT twists ONE chain's blocks: the block
// sits in LDS (624 words), the 64 lanes twist it in five 128-word iterations
// (the sequential twist's three ranges are whole iterations apart: words i <
// 227 read the old words i + 397, the rest the new words i - 227, and word
// 623 the new word 0), and each new block is stored to its buffer as whole
// 128-byte lines.  The buffers' contents and the packed state are exactly
// what the fused kernel's own twist rounds would have left (the twist is a
// pure function of the previous block), so streams are unchanged.
// ---------------------------------------------------------------------------
constexpr int kAheadW = 4;   // chains (wavefronts) per workgroup

__global__ __launch_bounds__(64 * kAheadW) void legacy_ahead_kernel(uint32_t *key_, int32_t *pos,
                                                                     int64_t n, int32_t want) {
  __shared__ uint32_t sh[kAheadW][kN];
  const int lane = threadIdx.x & 63;
  uint32_t *const mt = sh[threadIdx.x >> 6];
  const int64_t c = (int64_t)blockIdx.x * kAheadW + (threadIdx.x >> 6);
  if (c >= n) return;   // the whole wave
  w4 *const key = reinterpret_cast<w4 *>(key_);
  const int st = pos[c];
  const int cb = (st >> 16) & kBufMask, ready = (st >> 20) & kBufMask;
  if (ready >= want) return;   // wave-uniform
  // the last twisted block (current + ready) into LDS
  const int src = (cb + ready) & kBufMask;
  for (int i = lane; i < kQ; i += 64)
    *reinterpret_cast<w4 *>(&mt[4 * i]) = k4q(key, n, c, src, i);
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  for (int r = ready; r < want; ++r) {
#pragma unroll
    for (int it = 0; it < 5; ++it) {
      const int k = lane + 64 * it;
      if (k < kN / 2) {
        const int i0 = 2 * k;
        const uint2 o = *reinterpret_cast<const uint2 *>(&mt[i0]);
        const uint32_t o2 = mt[i0 + 2 < kN ? i0 + 2 : 0];
        const uint32_t f0 = mt[i0 < kN - kM ? i0 + kM : i0 - (kN - kM)];
        const uint32_t f1 = mt[i0 + 1 < kN - kM ? i0 + 1 + kM : i0 + 1 - (kN - kM)];
        *reinterpret_cast<uint2 *>(&mt[i0]) = make_uint2(f0 ^ mt_f(o.x, o.y), f1 ^ mt_f(o.y, o2));
      }
      // this iteration's words before the next one's reads (one wavefront:
      // its LDS operations complete in order)
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    const int dst = (cb + r + 1) & kBufMask;
    for (int i = lane; i < kQ; i += 64)
      k4q(key, n, c, dst, i) = *reinterpret_cast<const w4 *>(&mt[4 * i]);
  }
  if (lane == 0) pos[c] = (st & 0xFFFF) | (cb << 16) | (want << 20);
}

// The checkpoint form of the Mt4 state: every chain's current block moved
// into buffer 0 (quad per thread) and its packed position's buffer and
// ready fields cleared (the blocks twisted ahead are dropped: the next run
// twists them again, the same words), so that the state is the prefix of
// 20 chunks x 32 words per chain of the key array
__global__ __launch_bounds__(256) void legacy_norm_copy_kernel(w4 *key, const int32_t *pos,
                                                              int64_t n) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n * kCh * 8) return;
  const int64_t c = t / (kCh * 8);
  const int i = (int)(t - c * (kCh * 8));
  const int cb = (pos[c] >> 16) & kBufMask;
  if (cb != 0) k4q(key, n, c, 0, i) = k4q(key, n, c, cb, i);
}
__global__ __launch_bounds__(256) void legacy_norm_pos_kernel(int32_t *pos, int64_t n) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c < n) pos[c] &= 0xFFFF;
}

}  // namespace

hipError_t launch_legacy_normalize(uint32_t *key, int32_t *pos, int64_t n, hipStream_t s) {
  const int64_t q = n * kCh * 8;
  hipLaunchKernelGGL(legacy_norm_copy_kernel, dim3((unsigned)((q + 255) / 256)), dim3(256), 0, s,
                     reinterpret_cast<w4 *>(key), pos, n);
  hipLaunchKernelGGL(legacy_norm_pos_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s,
                     pos, n);
  return hipGetLastError();
}

hipError_t launch_legacy_ahead(uint32_t *key, int32_t *pos, int64_t n, int32_t want,
                               hipStream_t s) {
  if (want < 1 || want > kK4 - 1) return hipErrorInvalidValue;
  const dim3 grid((unsigned)((n + kAheadW - 1) / kAheadW)), block(64 * kAheadW);
  hipLaunchKernelGGL(legacy_ahead_kernel, grid, block, 0, s, key, pos, n, want);
  return hipGetLastError();
}

hipError_t launch_legacy_seed(uint32_t *key, int32_t *pos, double *gauss,
                              int32_t *has_gauss, const uint32_t *seeds,
                              int64_t n, int32_t db, hipStream_t s) {
  const dim3 grid((unsigned)((n + 255) / 256)), block(256);
  if (db == 2)
    hipLaunchKernelGGL(mt_seed_k4_kernel, grid, block, 0, s, key, pos, gauss,
                       has_gauss, seeds, n);
  else if (db)
    hipLaunchKernelGGL(mt_seed_db_kernel, grid, block, 0, s, key, pos, gauss,
                       has_gauss, seeds, n);
  else
    hipLaunchKernelGGL(mt_seed_kernel, grid, block, 0, s, key, pos, gauss,
                       has_gauss, seeds, n);
  return hipGetLastError();
}

// the word-parallel generator (pbh_legacy_wp.hip)
hipError_t launch_legacy_wp(const LegacyArgs &a, hipStream_t s);

hipError_t launch_legacy_draws(const LegacyArgs &a, int32_t kind, double param,
                               hipStream_t s) {
  if (a.db != 2) return hipErrorNotSupported;   // the Mt4 state
  constexpr int H = 16;
  const size_t lds = (size_t)(2 * H) * kBlockLegacy * sizeof(uint4);
  hipError_t err = hipFuncSetAttribute(reinterpret_cast<const void *>(&legacy_draws_kernel<H>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (err != hipSuccess) return err;
  const dim3 grid((unsigned)((a.n + kBlockLegacy - 1) / kBlockLegacy)), block(kBlockLegacy);
  hipLaunchKernelGGL(legacy_draws_kernel<H>, grid, block, lds, s, a, kind, param);
  return hipGetLastError();
}

hipError_t launch_legacy_gen(const LegacyArgs &a, hipStream_t s) {
  // the word-parallel generator: Mt4's state, MH streams of doubles
  if (a.db == 2 && a.wp && !a.gibbs && !a.vardelta) return launch_legacy_wp(a, s);
  if (a.db == 2) {   // Mt4: four chunked blocks through the window
    if (!a.normal || a.d <= 12) return launch_k4<16>(a, s);
    return launch_k4<8>(a, s);
  }
  if (a.db && a.win) {
    // 2H = 32 quads (128 words) per lane while the stage leaves room
    if (!a.normal || a.d <= 12) return launch_win<16>(a, s);
    return launch_win<8>(a, s);
  }
  const dim3 grid((unsigned)((a.n + 255) / 256)), block(256);
  if (a.db)
    hipLaunchKernelGGL(legacy_gen_db_kernel, grid, block, 0, s, a);
  else
    hipLaunchKernelGGL(legacy_gen_kernel, grid, block, 0, s, a);
  return hipGetLastError();
}

// The fused REPLAY kernel for the forms it covers (see legacy_mh_kernel):
// Mt4 state, MH with normal or raw draws, identity draw order, d of an
// instantiated kernel.  check: only report whether it applies.
bool legacy_mh_dim(int d) {
  switch (d) {
    case 1: case 2: case 3: case 4: case 5: case 6: case 8: case 10: return true;
    default: return false;
  }
}

hipError_t launch_legacy_mh(const LegacyArgs &la, const KArgs &a, hipStream_t s, bool check) {
  if (la.db != 2 || la.gibbs || la.vardelta || la.d != a.d || !legacy_mh_dim(la.d) ||
      !(la.normal ? a.prop == PBH_PROP_GAUSS
                  : (a.prop == PBH_PROP_UNIFORM || a.prop == PBH_PROP_SPHERE)))
    return hipErrorNotSupported;
  if (check) return hipSuccess;
  switch (la.d) {
    case 1: return launch_legacy_mh_d<1>(la, a, s);
    case 2: return launch_legacy_mh_d<2>(la, a, s);
    case 3: return launch_legacy_mh_d<3>(la, a, s);
    case 4: return launch_legacy_mh_d<4>(la, a, s);
    case 5: return launch_legacy_mh_d<5>(la, a, s);
    case 6: return launch_legacy_mh_d<6>(la, a, s);
    case 8: return launch_legacy_mh_d<8>(la, a, s);
    default: return launch_legacy_mh_d<10>(la, a, s);
  }
}

}  // namespace pbh
