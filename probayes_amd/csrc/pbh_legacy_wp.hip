// pbh_legacy_wp.hip -- the word-parallel generator of the reference's
// random streams (NumPy legacy RandomState per chain, see pbh_legacy.hip).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pbh_kernels.h"
#include "pbh_mt.h"
#include "pbhip.h"

namespace pbh {
namespace {

// ---------------------------------------------------------------------------
// The word-parallel generator (WP, round 6; the default for the Normal and
// Raw MH streams of the Mt4 state).  The chain-per-lane generators of
// pbh_legacy.hip run 65 536 chains as one wavefront per SIMD, each lane
// walking its own stream word by word (the polar method's rejections make
// every lane's position its own), and are latency-bound there (VALU active
// ~0.35).  Here ONE WAVEFRONT owns ONE chain (four chains per workgroup,
// sharing the log table) and works on its stream a whole MT block at a
// time, a "round":
//  1. the pass: the 64 lanes twist the block in LDS (the sequential twist's
//     three ranges: words i < 227 from the old words i + 397, the rest from
//     the new words i - 227 -- every range is whole iterations apart, so five
//     128-word iterations in order are the sequential twist) and temper +
//     convert it into its 312 random_sample doubles (d[1 + k]; d[0] keeps the
//     previous block's last double: a pair may straddle two blocks);
//  2. the polar method's accept test for the pair starting at EVERY buffer
//     position (r2 = x1^2 + x2^2 < 1, != 0: the same operations); ballots
//     give, per parity, the accepted positions in order (A[parity]) and every
//     position's rank among them -- a step's attempts run b, b + 2, ... so
//     its pairs are consecutive entries of A[b & 1] from rank[b];
//  3. per position b: n1[b] = the end of the first accepted pair at or after
//     b (its parity), e[b] = the end of the nd-th (a whole step of nd pairs:
//     where its threshold lies);
//  4. the parse, wave-uniform, one table read per whole step (e), draw by
//     draw (n1, descriptors) only for a step that straddles the block end;
//  5. sweeps of 64 lanes over the round's draws: whole steps expand by rank
//     and A, descriptors carry their draw; every lane runs the polar
//     method's transcendental part (polar_pair's operations: log_leg, the
//     IEEE division and square root) branch-free and stores its values into
//     the [T][R][N] rows.
// The values, their order and the cached deviate are legacy_gauss's: the
// streams equal the chain-per-lane generators' bit for bit (and NumPy's
// RandomState's, tests/test_gpu_legacy.py, test_gpu_legacy_wp.py).  The
// state is written back in Mt4's layout (the current block in its buffer,
// nothing twisted ahead), so either generator continues the other's streams.
// Positions must be even (streams of doubles only: no randint words since
// seeding -- the engine tracks that).
// ---------------------------------------------------------------------------
constexpr int kWpW = 4;         // chains (wavefronts) per workgroup
constexpr int kWpTab = 320;     // table entries (positions 0 .. 313 are used)
constexpr int kWpOob = 0x3FF;   // "no accepted pair of that parity before the block end"
constexpr uint32_t kWpSingle = 0, kWpSame = 1, kWpNext = 2, kWpGauss = 3;

struct WpWave {
  uint32_t mt[kN];                // the block (untempered)
  double d[kWpTab];               // [0] carry, [1 + k] the block's doubles
  uint32_t en1[kWpTab];           // e[b] << 16 | n1[b]
  uint16_t rank[kWpTab];          // accepted positions of b's parity below b
  uint16_t A[2][kWpTab / 2];      // accepted positions per parity, ascending
};

struct WpLds {
  WpWave w[kWpW];
  double lg[kLegLogDoubles];      // log_leg's table
  int32_t ord[PBH_MAX_DIM];       // draw j -> replay row
};

// the wave's own LDS hand-offs: its LDS operations complete in order; this
// keeps the compiler from moving memory operations across the point
__device__ __forceinline__ void wsync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// lane l (wave-uniform) of v takes the wave-uniform x
__device__ __forceinline__ uint32_t wp_put(uint32_t v, uint32_t x, int l, int lane) {
  return lane == l ? x : v;
}

// a descriptor: buffer position b (9 bits), the step relative to the
// round's first (8 bits), the draw index (6 bits), the kind (2 bits)
__device__ __forceinline__ uint32_t wp_desc(int b, int tr, int r, uint32_t kind) {
  return (uint32_t)b | ((uint32_t)tr << 9) | ((uint32_t)r << 17) | (kind << 23);
}

template <bool NORMAL>
__global__ __launch_bounds__(64 * kWpW) void legacy_gen_wp_kernel(LegacyArgs a) {
  __shared__ WpLds sh;
  for (int i = threadIdx.x; i < kLegLogDoubles; i += 64 * kWpW) sh.lg[i] = a.lgtab[i];
  if ((int)threadIdx.x < a.d) sh.ord[threadIdx.x] = a.order[threadIdx.x];
  __syncthreads();   // the only workgroup barrier: the waves run apart from here
  const int lane = threadIdx.x & 63;
  WpWave &W = sh.w[threadIdx.x >> 6];
  // consecutive chains on one XCD (their 8-byte stores share 128-byte lines
  // of the rows; dispatch deals workgroups to the XCDs in turn)
  int64_t g = blockIdx.x;
  const int64_t nwg = gridDim.x;
  if ((nwg & 7) == 0) g = (g & 7) * (nwg >> 3) + (g >> 3);
  const int64_t c = g * kWpW + (threadIdx.x >> 6);
  if (c >= a.n) return;   // the whole wave
  const int64_t n = a.n;
  const int d = a.d;
  const int64_t R = a.R;
  const int nsteps = (int)a.n_steps;
  double *const out = a.out + c;
  // the chain's state: the current block from buffer cb (Mt4's layout)
  const int st = a.pos[c];
  const int pos0 = st & 0xFFFF, cb = (st >> 16) & kBufMask;
  w4 *const key = reinterpret_cast<w4 *>(a.key);
  for (int i = lane; i < kQ; i += 64)
    *reinterpret_cast<w4 *>(&W.mt[4 * i]) = k4q(key, n, c, cb, i);
  if (lane == 0) W.d[0] = 0.0;
  int has = NORMAL ? a.has_gauss[c] : 0;
  const int has0 = has;
  // even d: every step draws nd = d / 2 polar pairs (the cached deviate, if
  // any, leads each step and the last pair's second deviate is cached for
  // the next): whole steps take the table path; odd d runs draw by draw
  const bool fast = NORMAL ? (d & 1) == 0 : true;
  const int nd = d >> 1;
  const int per = NORMAL ? nd + 1 : d + 1;   // draws of a whole step
  if (NORMAL && has && lane == 0) out[(int64_t)sh.ord[0] * n] = a.gauss[c];
  wsync();

  // ---- one draw per lane (branch-free apart from the masked stores): a
  // single double at position b, or the polar pair at b whose first deviate
  // goes to draw rr and whose second to the next normal draw
  auto draw = [&](bool valid, int b, int tt, int rr, uint32_t kind) {
    const int bb = valid ? b : 1;
    const double da = W.d[bb];
    double v1 = da, v2 = 0.0;
    if constexpr (NORMAL) {
      const double x1 = 2.0 * da - 1.0;
      const double x2 = 2.0 * W.d[bb + 1 <= 312 ? bb + 1 : 312] - 1.0;
      double r2 = x1 * x1 + x2 * x2;
      if (kind == kWpSingle) r2 = 0.5;   // (a value the pair path never sees)
      const double lr = log_leg(r2, sh.lg);
      const double f = sqrt(-2.0 * lr / r2);
      if (kind != kWpSingle) v1 = f * x2;
      v2 = f * x1;
    }
    const int row1 = rr < d ? sh.ord[rr] : d;
    const int tt2 = kind == kWpNext ? tt + 1 : tt;
    const int row2 = kind == kWpNext ? sh.ord[0] : sh.ord[rr + 1 < d ? rr + 1 : 0];
    if (valid) out[((int64_t)tt * R + row1) * n] = v1;
    if constexpr (NORMAL) {
      if (valid && (kind == kWpSame || kind == kWpNext)) out[((int64_t)tt2 * R + row2) * n] = v2;
      if (valid && kind == kWpGauss) a.gauss[c] = v2;   // cached past the launch
    }
  };

  int b = (pos0 >> 1) + 1;   // 1 .. 313
  bool twist = false;
  if (b > 312) {   // pos 624: the block is used up
    twist = true;
    b -= 312;
  }
  int t = 0, r = 0;

  for (;;) {
    // ---- 1. twist (after the first block) and convert: d[1 + k] = D[k]
    {
      const double carry = W.d[312];
      wsync();
      if (twist) {
#pragma unroll
        for (int i = 0; i < 5; ++i) {
          const int k = lane + 64 * i;
          if (k < kN / 2) {
            const int i0 = 2 * k;
            const uint2 o = *reinterpret_cast<const uint2 *>(&W.mt[i0]);
            const uint32_t o2 = W.mt[i0 + 2 < kN ? i0 + 2 : 0];
            const uint32_t f0 = W.mt[i0 < kN - kM ? i0 + kM : i0 - (kN - kM)];
            const uint32_t f1 = W.mt[i0 + 1 < kN - kM ? i0 + 1 + kM : i0 + 1 - (kN - kM)];
            const uint32_t w0 = f0 ^ mt_f(o.x, o.y), w1 = f1 ^ mt_f(o.y, o2);
            *reinterpret_cast<uint2 *>(&W.mt[i0]) = make_uint2(w0, w1);
            W.d[1 + k] = mt_dbl(w0, w1);
          }
          wsync();   // this iteration's words before the next's loads
        }
        if (lane == 0) W.d[0] = carry;
      } else {
#pragma unroll
        for (int i = 0; i < 5; ++i) {
          const int k = lane + 64 * i;
          if (k < kN / 2) {
            const uint2 o = *reinterpret_cast<const uint2 *>(&W.mt[2 * k]);
            W.d[1 + k] = mt_dbl(o.x, o.y);
          }
        }
      }
      wsync();
    }
    // ---- 2-3. the accept map by parity, the ranks, the tables
    if constexpr (NORMAL) {
      int rk[5];
      int cnt0 = 0, cnt1 = 0;
      const uint64_t below = (1ull << lane) - 1ull;
#pragma unroll
      for (int i = 0; i < 5; ++i) {
        const int p = lane + 64 * i;
        bool ok = false;
        if (p <= 311) {
          const double x1 = 2.0 * W.d[p] - 1.0;
          const double x2 = 2.0 * W.d[p + 1] - 1.0;
          const double r2 = x1 * x1 + x2 * x2;
          ok = r2 < 1.0 && r2 != 0.0;
        }
        const uint64_t F = __builtin_amdgcn_ballot_w64(ok);
        const uint64_t m0 = F & 0x5555555555555555ull, m1 = F & 0xAAAAAAAAAAAAAAAAull;
        const uint64_t mine = (lane & 1) ? m1 : m0;
        rk[i] = ((lane & 1) ? cnt1 : cnt0) + __builtin_popcountll(mine & below);
        W.rank[p] = (uint16_t)rk[i];
        if (ok) W.A[lane & 1][rk[i]] = (uint16_t)p;
        cnt0 += __builtin_popcountll(m0);
        cnt1 += __builtin_popcountll(m1);
      }
      wsync();
#pragma unroll
      for (int i = 0; i < 5; ++i) {
        const int p = lane + 64 * i;
        const int par = lane & 1, cnt = par ? cnt1 : cnt0;
        const int n1 = rk[i] < cnt ? W.A[par][rk[i]] + 2 : kWpOob;
        const int j = rk[i] + nd - 1;
        const int e = (fast && nd > 0 && j < cnt) ? W.A[par][j] + 2 : kWpOob;
        W.en1[p] = ((uint32_t)e << 16) | (uint32_t)n1;
      }
      wsync();
    }
    // ---- 4. the parse (wave-uniform): whole steps by table, a step that
    // straddles the block end draw by draw
    const int tround = t;
    uint32_t vstart = 0u, vdesc = 0u;   // lane s: the s-th whole step's start
    int S = 0, tfast = 0, ne = 0;
    // ---- 5. a sweep of up to 64 draws: whole steps first, then descriptors
    auto sweep = [&](int first) {
      const int item = first + lane;
      bool valid = false;
      int pb = 1, tt = 0, rr = 0;
      uint32_t kind = kWpSingle;
      // (the lane reads happen with every lane active: ds_bpermute does not
      // read lanes the exec mask has switched off)
      const int si = item / per, k = item - si * per;
      const int bs = __shfl((int)vstart, si < 64 ? si : 0);
      const int di = item - S * per;
      const uint32_t dd = (uint32_t)__shfl((int)vdesc, di >= 0 && di < 64 ? di : 0);
      if (item < S * per) {
        tt = tfast + si;
        valid = true;
        if constexpr (NORMAL) {
          const int par = bs & 1, rb = W.rank[bs];
          if (k < nd) {
            pb = W.A[par][rb + k];
            rr = 2 * k + has0;
            kind = rr + 1 < d ? kWpSame : (tt + 1 < nsteps ? kWpNext : kWpGauss);
          } else {
            pb = W.A[par][rb + nd - 1] + 2;   // the threshold after the last pair
            rr = d;
          }
        } else {
          pb = bs + k;
          rr = k;
        }
      } else if (di < ne) {
        valid = true;
        pb = (int)(dd & 511u);
        tt = tround + (int)((dd >> 9) & 255u);
        rr = (int)((dd >> 17) & 63u);
        kind = dd >> 23;
      }
      draw(valid, pb, tt, rr, kind);
    };
    auto flush = [&]() {
      const int total = S * per + ne;
      for (int f = 0; f < total; f += 64) sweep(f);
      S = 0;
      ne = 0;
    };
    while (t < nsteps) {
      if (fast && r == 0) {
        int x;
        if constexpr (NORMAL) x = __builtin_amdgcn_readfirstlane((int)(W.en1[b] >> 16));
        else x = b + d <= 312 ? b + d : kWpOob;
        if (x <= 312) {   // a whole step inside the block: its threshold at x
          if (S == 64) flush();
          if (S == 0) tfast = t;
          vstart = wp_put(vstart, (uint32_t)b, S, lane);
          ++S;
          ++t;
          b = x + 1;
          continue;
        }
      }
      if (NORMAL && r < d) {
        if (has) {   // the cached deviate (routed here by the pair that made it)
          ++r;
          has = 0;
          continue;
        }
        const int y = __builtin_amdgcn_readfirstlane((int)(W.en1[b] & 0xFFFFu));
        if (y > 313) {   // no accepted pair of this parity before the block end
          b = 312 + (b & 1);
          break;
        }
        const uint32_t kind = r + 1 < d ? kWpSame : (t + 1 < nsteps ? kWpNext : kWpGauss);
        if (ne == 64) flush();
        vdesc = wp_put(vdesc, wp_desc(y - 2, t - tround, r, kind), ne, lane);
        ++ne;
        b = y;
        ++r;
        has = 1;
        continue;
      }
      if (b > 312) break;   // a single draw past the block
      if (ne == 64) flush();
      vdesc = wp_put(vdesc, wp_desc(b, t - tround, r, kWpSingle), ne, lane);
      ++ne;
      ++b;
      if (r == d) {
        r = 0;
        ++t;
      } else {
        ++r;
      }
    }
    flush();   // the round's draws read this block's doubles
    if (t >= nsteps) break;
    b -= 312;
    twist = true;
  }
  // the state, in Mt4's layout: the current block back into buffer cb
  wsync();
  for (int i = lane; i < kQ; i += 64)
    k4q(key, n, c, cb, i) = *reinterpret_cast<const w4 *>(&W.mt[4 * i]);
  if (lane == 0) {
    a.pos[c] = (2 * (b - 1)) | (cb << 16);   // nothing twisted ahead
    if constexpr (NORMAL) {
      a.has_gauss[c] = has;
      if (!has) a.gauss[c] = 0.0;
    }
  }
}

}  // namespace

hipError_t launch_legacy_wp(const LegacyArgs &a, hipStream_t s) {
  const dim3 grid((unsigned)((a.n + kWpW - 1) / kWpW)), block(64 * kWpW);
  if (a.normal)
    hipLaunchKernelGGL(legacy_gen_wp_kernel<true>, grid, block, 0, s, a);
  else
    hipLaunchKernelGGL(legacy_gen_wp_kernel<false>, grid, block, 0, s, a);
  return hipGetLastError();
}

}  // namespace pbh
