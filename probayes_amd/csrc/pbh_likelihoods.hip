// pbh_likelihoods.hip -- bool_perm_freq (likelihoods.py:45-101) on gfx950.
//
// counts[i] = number of rows of bool2d [rows][cols] whose pattern, read as
// a binary number with the FIRST column most significant, equals i: the
// C-order flat index of counts[tuple(sequence)] (likelihoods.py:67-70).
//
// HBM-bound byte work: the input is read once (cols bytes per row) and the
// histogram is tiny.  Three kernels by table size:
//   cols = 1, 2, 4  `bool_perm_direct`: rows never straddle a 16-B chunk, so
//        every lane streams 16-B chunks (four loads in flight), turns each
//        byte into one bit and counts in registers -- popcounts for cols 1
//        and 2 (the 2 x 2 table follows from the counts of column A, column
//        B and A & B), a 16-way compare-add for cols 4;
//   other cols <= 13  `bool_perm_tiled`: each workgroup stages 256-row tiles
//        in LDS with dword loads (256 * cols bytes keeps tiles 4-B aligned)
//        and every lane decodes one row; cols 3 counts with wave ballots
//        (popcount(ballot(idx == bin)) in the register of lane `bin`),
//        cols 5..13 in an LDS u32 histogram per workgroup;
//   cols > 13  the same tiles with u64 global atomics per row (the table no
//        longer fits LDS; the bins are many, so contention is low).
// Small tables are NOT summed with global atomics: thousands of waves adding
// to the same few addresses serialise at the memory side.  Each workgroup
// writes its partial table to a scratch row [grid][16] instead, and one
// small workgroup sums the rows in a second launch (deterministic order).
// The grid is capped at 8 workgroups per CU and strides over the input.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pbh_kernels.h"

namespace pbh {
namespace {

constexpr int kTile = 256;          // rows per tile = threads per workgroup
constexpr int kMaxCols = 26;
constexpr int kLdsBinsLog2 = 13;    // 8192 u32 bins = 32 KB of LDS
constexpr int kPart = 16;           // partial slots per workgroup
constexpr int kWaves = kTile / 64;

// Sums v[0..NC) over the workgroup and stores them to part[blockIdx.x][..].
template <int NC>
__device__ __forceinline__ void store_partials(const uint32_t (&v)[NC],
                                               unsigned long long *part) {
  __shared__ unsigned long long s_red[kWaves][NC];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int b = 0; b < NC; ++b) {
    uint32_t x = v[b];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
    if (lane == 0) s_red[wave][b] = x;
  }
  __syncthreads();
  if (threadIdx.x < NC) {
    unsigned long long t = 0;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) t += s_red[w][threadIdx.x];
    part[(int64_t)blockIdx.x * kPart + threadIdx.x] = t;
  }
}

// bytes of w -> bit 0 of each byte = (byte != 0)
__device__ __forceinline__ uint32_t byte_bits(uint32_t w) {
  uint32_t t = w | (w >> 4);
  t |= t >> 2;
  t |= t >> 1;
  return t & 0x01010101u;
}

template <int COLS>
struct DirectCount {
  static constexpr int NC = COLS == 4 ? 16 : (COLS == 2 ? 3 : 1);
  // COLS 1: c[0] = ones;  COLS 2: c[0] = A, c[1] = B, c[2] = A & B;
  // COLS 4: c[b] = rows with index b
  uint32_t c[NC] = {};
  __device__ __forceinline__ void word(uint32_t w) {
    const uint32_t t = byte_bits(w);
    if (COLS == 1) {
      c[0] += __popc(t);
    } else if (COLS == 2) {
      const uint32_t a = t & 0x00010001u, b = (t >> 8) & 0x00010001u;
      c[0] += __popc(a);
      c[1] += __popc(b);
      c[2] += __popc(a & b);
    } else {
      // byte 0 (first column) is the most significant index bit
      const uint32_t idx = ((t & 1u) << 3) | ((t >> 6) & 4u) | ((t >> 15) & 2u) |
                           (t >> 24);
#pragma unroll
      for (int b = 0; b < 16; ++b) c[b] += (idx == (uint32_t)b) ? 1u : 0u;
    }
  }
};

template <int COLS>
__global__ __launch_bounds__(kTile) void bool_perm_direct(
    const uint8_t *__restrict__ in, int64_t rows,
    unsigned long long *__restrict__ part) {
  typedef uint32_t u4 __attribute__((ext_vector_type(4)));
  const int64_t n16 = (rows * COLS) >> 4;
  const u4 *src = reinterpret_cast<const u4 *>(in);
  const int64_t stride = (int64_t)gridDim.x * kTile;
  int64_t i = (int64_t)blockIdx.x * kTile + threadIdx.x;
  DirectCount<COLS> dc;
  // u32 lane counters: a lane sees n16 / (grid lanes) chunks of <= 16 rows
  for (; i + 3 * stride < n16; i += 4 * stride) {
    u4 v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = src[i + k * stride];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      dc.word(v[k].x); dc.word(v[k].y); dc.word(v[k].z); dc.word(v[k].w);
    }
  }
  for (; i < n16; i += stride) {
    const u4 v = src[i];
    dc.word(v.x); dc.word(v.y); dc.word(v.z); dc.word(v.w);
  }
  // tail (< 16 bytes, whole rows): the first lane of the grid.  One row in
  // the low bytes of w, the other bytes zero: cols 1, 2 count set bits only
  // (counts[0] follows from rows), cols 4 fills all four bytes.
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    for (int64_t r = (n16 << 4) / COLS; r < rows; ++r) {
      uint32_t w = 0;
      for (int j = 0; j < COLS; ++j) w |= (uint32_t)(in[r * COLS + j] != 0) << (8 * j);
      dc.word(w);
    }
  }
  store_partials<DirectCount<COLS>::NC>(dc.c, part);
}

template <int MODE>   // 0 ballot (cols <= 4), 1 LDS histogram, 2 global atomics
__global__ __launch_bounds__(kTile) void bool_perm_tiled(
    const uint8_t *__restrict__ in, int64_t rows, int cols,
    unsigned long long *__restrict__ counts,
    unsigned long long *__restrict__ part) {
  __shared__ uint32_t s_tile[kTile * kMaxCols / 4];
  __shared__ uint32_t s_hist[MODE == 1 ? (1 << kLdsBinsLog2) : 1];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int nbins = 1 << cols;
  if (MODE == 1) {
    for (int b = tid; b < nbins; b += kTile) s_hist[b] = 0;
  }
  uint32_t mine = 0;   // MODE 0: count of bin `lane` seen by this wave
  const int64_t n_tiles = (rows + kTile - 1) / kTile;
  const uint8_t *s_bytes = reinterpret_cast<const uint8_t *>(s_tile);
  for (int64_t t = blockIdx.x; t < n_tiles; t += gridDim.x) {
    const int64_t r0 = t * kTile;
    const int nrow = (int)((rows - r0) < kTile ? (rows - r0) : kTile);
    const int nbytes = nrow * cols;
    const uint8_t *src = in + r0 * cols;
    __syncthreads();                       // previous tile fully decoded
    if (nrow == kTile) {
      const uint32_t *src4 = reinterpret_cast<const uint32_t *>(src);
      for (int i = tid; i < nbytes / 4; i += kTile) s_tile[i] = src4[i];
    } else {
      uint8_t *dst = reinterpret_cast<uint8_t *>(s_tile);
      for (int i = tid; i < nbytes; i += kTile) dst[i] = src[i];
    }
    __syncthreads();
    const bool valid = tid < nrow;
    int idx = 0;
    if (valid) {
      const uint8_t *row = s_bytes + tid * cols;
      for (int j = 0; j < cols; ++j) idx = (idx << 1) | (row[j] != 0);
    }
    if (MODE == 0) {
      for (int b = 0; b < nbins; ++b) {
        const uint64_t m = __ballot(valid && idx == b);
        if (lane == b) mine += (uint32_t)__popcll(m);
      }
    } else if (MODE == 1) {
      if (valid) atomicAdd(&s_hist[idx], 1u);
    } else {
      if (valid) atomicAdd(&counts[idx], 1ull);
    }
  }
  if (MODE == 0) {
    // lane b of every wave holds bin b: gather them per workgroup
    __shared__ uint32_t s_bins[kWaves][16];
    if (lane < 16) s_bins[tid >> 6][lane] = lane < nbins ? mine : 0u;
    __syncthreads();
    if (tid < 16) {
      unsigned long long t = 0;
      for (int w = 0; w < kWaves; ++w) t += s_bins[w][tid];
      part[(int64_t)blockIdx.x * kPart + tid] = t;
    }
  } else if (MODE == 1) {
    __syncthreads();
    for (int b = tid; b < nbins; b += kTile)
      if (s_hist[b]) atomicAdd(&counts[b], (unsigned long long)s_hist[b]);
  }
}

// Sums the [grid][16] partials in a fixed order and writes the table.
// form 1: cols 1 popcount; 2: cols 2 (A, B, AB); 0: bins as they are.
// One workgroup of kRed threads: thread (g0, b) sums rows g0, g0 + 64, ...
// of bin b with eight loads in flight, then LDS folds the 64 row groups.
constexpr int kRed = 1024;
__global__ __launch_bounds__(kRed) void bool_perm_reduce(
    const unsigned long long *__restrict__ part, int grid, int form,
    int nbins, int64_t rows, unsigned long long *__restrict__ counts) {
  __shared__ unsigned long long s[kRed];
  const int b = threadIdx.x & 15, g0 = threadIdx.x >> 4;
  constexpr int G = kRed / 16;
  unsigned long long t = 0;
  int g = g0;
  for (; g + 7 * G < grid; g += 8 * G) {
    unsigned long long v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = part[(int64_t)(g + k * G) * kPart + b];
#pragma unroll
    for (int k = 0; k < 8; ++k) t += v[k];
  }
  for (; g < grid; g += G) t += part[(int64_t)g * kPart + b];
  s[threadIdx.x] = t;
  __syncthreads();
  unsigned long long v = 0;
  if (threadIdx.x < 16)
    for (int k = 0; k < G; ++k) v += s[k * 16 + threadIdx.x];
  __syncthreads();
  if (threadIdx.x < 16) s[threadIdx.x] = v;
  __syncthreads();
  if (threadIdx.x != 0) return;
  const unsigned long long r = (unsigned long long)rows;
  if (form == 1) {
    counts[1] = s[0];
    counts[0] = r - s[0];
  } else if (form == 2) {
    const unsigned long long a = s[0], bb = s[1], ab = s[2];
    counts[3] = ab;
    counts[2] = a - ab;         // first column True, second False
    counts[1] = bb - ab;
    counts[0] = r - a - bb + ab;
  } else {
    for (int k = 0; k < nbins; ++k) counts[k] = s[k];
  }
}

}  // namespace

int bool_perm_max_cols() { return kMaxCols; }

int64_t bool_perm_scratch_words(int n_cu) {
  return (int64_t)(n_cu > 0 ? n_cu : 256) * 8 * kPart;
}

hipError_t launch_bool_perm_freq(const uint8_t *in, int64_t rows, int cols,
                                 unsigned long long *counts,
                                 unsigned long long *scratch, int n_cu,
                                 hipStream_t s) {
  const int64_t cap = (int64_t)(n_cu > 0 ? n_cu : 256) * 8;
  const dim3 block(kTile);
  if (cols == 1 || cols == 2 || cols == 4) {
    const int64_t n16 = rows * cols / 16;
    const int64_t want = (n16 + 4 * kTile - 1) / (4 * kTile);
    const int grid = (int)(want < 1 ? 1 : (want < cap ? want : cap));
    if (cols == 1)
      hipLaunchKernelGGL(bool_perm_direct<1>, dim3(grid), block, 0, s, in, rows, scratch);
    else if (cols == 2)
      hipLaunchKernelGGL(bool_perm_direct<2>, dim3(grid), block, 0, s, in, rows, scratch);
    else
      hipLaunchKernelGGL(bool_perm_direct<4>, dim3(grid), block, 0, s, in, rows, scratch);
    hipLaunchKernelGGL(bool_perm_reduce, dim3(1), dim3(kRed), 0, s, scratch, grid,
                       cols == 4 ? 0 : cols, 1 << cols, rows, counts);
    return hipGetLastError();
  }
  const int64_t n_tiles = (rows + kTile - 1) / kTile;
  const int grid = (int)(n_tiles < cap ? n_tiles : cap);
  if (cols <= 4) {
    hipLaunchKernelGGL(bool_perm_tiled<0>, dim3(grid), block, 0, s, in, rows, cols,
                       counts, scratch);
    hipLaunchKernelGGL(bool_perm_reduce, dim3(1), dim3(kRed), 0, s, scratch, grid, 0,
                       1 << cols, rows, counts);
  } else if (cols <= kLdsBinsLog2) {
    hipLaunchKernelGGL(bool_perm_tiled<1>, dim3(grid), block, 0, s, in, rows, cols,
                       counts, scratch);
  } else {
    hipLaunchKernelGGL(bool_perm_tiled<2>, dim3(grid), block, 0, s, in, rows, cols,
                       counts, scratch);
  }
  return hipGetLastError();
}

}  // namespace pbh
