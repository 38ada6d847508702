// Trace-store pattern of the lane-pair MH kernel without its arithmetic:
// 2048 waves (32 chains each, lanes l / l+32 = the two halves of a chain),
// each step writes d = 10 fp64 rows [step][dim][chain] + a log-prob row +
// a 32-bit mask word, as mh_pair_kernel<10> does.  Compares plain stores,
// non-temporal stores and a VALU spacer between steps (what the real
// kernel's arithmetic does to the store stream).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <int NT, int SPACER>
__global__ __launch_bounds__(256) void k_trace(double *tx, double *tlp, uint32_t *tacc,
                                               int64_t n, int steps) {
  constexpr int D = 10, H = 5;
  const int lane = threadIdx.x & 63;
  const bool hi = lane >= 32;
  const int64_t wave = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
  const int64_t c = wave * 32 + (lane & 31);
  double x[H];
  for (int i = 0; i < H; ++i) x[i] = (double)(c + i);
  double lp = (double)c;
  for (int s = 0; s < steps; ++s) {
    for (int i = 0; i < H; ++i) {
      double v = x[i];
#pragma unroll
      for (int r = 0; r < SPACER; ++r) v = __builtin_fma(v, 1.0000001, 1e-9);
      x[i] = v;
    }
    lp += 1.0;
    double *row = tx + (int64_t)s * D * n;
    for (int i = 0; i < H; ++i) {
      double *p = row + (hi ? H + i : i) * n + c;
      if (NT) __builtin_nontemporal_store(x[i], p);
      else *p = x[i];
    }
    if (hi) {
      if (NT) __builtin_nontemporal_store(lp, tlp + (int64_t)s * n + c);
      else tlp[(int64_t)s * n + c] = lp;
    }
    if (lane == 32) tacc[(int64_t)s * (n / 32) + wave] = (uint32_t)s;
  }
}

// Same bytes, layout [step][wave][dim][32 chains] (+ lp [step][n]): each
// wave's x rows of one step form one contiguous 2 560-B block.
template <int NT>
__global__ __launch_bounds__(256) void k_trace_blk(double *tx, double *tlp, uint32_t *tacc,
                                                   int64_t n, int steps) {
  constexpr int D = 10, H = 5;
  const int lane = threadIdx.x & 63;
  const bool hi = lane >= 32;
  const int64_t wave = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
  const int64_t c = wave * 32 + (lane & 31);
  double x[H];
  for (int i = 0; i < H; ++i) x[i] = (double)(c + i);
  double lp = (double)c;
  for (int s = 0; s < steps; ++s) {
    lp += 1.0;
    double *blk = tx + (int64_t)s * D * n + wave * D * 32;
    for (int i = 0; i < H; ++i) {
      double *p = blk + (hi ? H + i : i) * 32 + (lane & 31);
      if (NT) __builtin_nontemporal_store(x[i] + s, p);
      else *p = x[i] + s;
    }
    if (hi) {
      if (NT) __builtin_nontemporal_store(lp, tlp + (int64_t)s * n + c);
      else tlp[(int64_t)s * n + c] = lp;
    }
    if (lane == 32) tacc[(int64_t)s * (n / 32) + wave] = (uint32_t)s;
  }
}

// Upper bound: every store instruction writes 512 contiguous bytes.
template <int NT>
__global__ __launch_bounds__(256) void k_trace_512(double *tx, double *tlp, uint32_t *tacc,
                                                   int64_t n, int steps) {
  constexpr int D = 10;
  const int lane = threadIdx.x & 63;
  const int64_t wave = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
  // half the waves' worth of 64-chain groups, 11 rows per step each
  const int64_t g = wave >> 1, half = wave & 1;
  const int64_t c = g * 64 + lane;
  for (int s = 0; s < steps; ++s) {
    double *row = tx + (int64_t)s * D * n;
    for (int i = 0; i < 5; ++i) {
      double *p = row + (half * 5 + i) * n + c;
      if (NT) __builtin_nontemporal_store((double)(s + i), p);
      else *p = (double)(s + i);
    }
    if (half) {
      if (NT) __builtin_nontemporal_store((double)s, tlp + (int64_t)s * n + c);
      else tlp[(int64_t)s * n + c] = (double)s;
    }
    if (lane == 0 && half) tacc[(int64_t)s * (n / 32) + g] = (uint32_t)s;
  }
}

// The lane-pair layout written with 16-B stores: adjacent lanes (chains c,
// c + 1) swap so that the even lane holds dim i of both chains and the odd
// lane dim i + 1 of both: dims (0,1), (2,3) as dwordx4, dim 4 as dwordx2.
template <int NT>
__global__ __launch_bounds__(256) void k_trace_x4(double *tx, double *tlp, uint32_t *tacc,
                                                  int64_t n, int steps) {
  constexpr int D = 10, H = 5;
  const int lane = threadIdx.x & 63;
  const bool hi = lane >= 32, odd = lane & 1;
  const int64_t wave = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
  const int64_t c = wave * 32 + (lane & 31);
  const int64_t c0 = c & ~(int64_t)1;
  double x[H];
  for (int i = 0; i < H; ++i) x[i] = (double)(c + i);
  double lp = (double)c;
  typedef double d2 __attribute__((ext_vector_type(2)));
  for (int s = 0; s < steps; ++s) {
    lp += 1.0;
    double *row = tx + (int64_t)s * D * n;
    const int k0 = hi ? H : 0;
#pragma unroll
    for (int i = 0; i + 1 < H; i += 2) {
      // even lane keeps dim i, sends dim i+1; odd lane keeps dim i+1
      const double send = odd ? x[i] : x[i + 1];
      const double got = __shfl_xor(send, 1);
      d2 v;
      v.x = odd ? got : x[i];        // chain c0's value of this lane's dim
      v.y = odd ? x[i + 1] : got;    // chain c0 + 1's
      d2 *p = (d2 *)(row + (k0 + i + (odd ? 1 : 0)) * n + c0);
      if (NT) __builtin_nontemporal_store(v, p);
      else *p = v;
    }
    double *p4 = row + (k0 + H - 1) * n + c;
    if (NT) __builtin_nontemporal_store(x[H - 1] + s, p4);
    else *p4 = x[H - 1] + s;
    if (hi) {
      if (NT) __builtin_nontemporal_store(lp, tlp + (int64_t)s * n + c);
      else tlp[(int64_t)s * n + c] = lp;
    }
    if (lane == 32) tacc[(int64_t)s * (n / 32) + wave] = (uint32_t)s;
  }
}

// 1 KB contiguous per store instruction (16 B per lane): an upper bound.
template <int NT>
__global__ __launch_bounds__(256) void k_trace_1k(double *tx, double *tlp, uint32_t *tacc,
                                                  int64_t n, int steps) {
  typedef double d2 __attribute__((ext_vector_type(2)));
  const int lane = threadIdx.x & 63;
  const int64_t wave = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
  // 2048 waves; per step 11 rows of n doubles = 11 n / 128 instructions
  const int64_t per_step = 11 * n / 128;   // 1-KB pieces per step
  for (int s = 0; s < steps; ++s) {
    for (int64_t q = wave; q < per_step; q += 2048) {
      d2 v = {(double)s, (double)q};
      d2 *p = (d2 *)(tx + (int64_t)s * 11 * n + q * 128) + lane;
      if (NT) __builtin_nontemporal_store(v, p);
      else *p = v;
    }
  }
}

template <class K>
void run(const char *name, K k, double *tx, double *tlp, uint32_t *tacc,
         int64_t n, int steps) {
  const int64_t waves = n / 32;
  const dim3 grid((unsigned)(waves * 64 / 256)), block(256);
  hipLaunchKernelGGL(k, grid, block, 0, 0, tx, tlp, tacc, n, steps);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  const int reps = 5;
  for (int r = 0; r < reps; ++r)
    hipLaunchKernelGGL(k, grid, block, 0, 0, tx, tlp, tacc, n, steps);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  ms /= reps;
  const double bytes = (double)n * steps * (8.0 * 10 + 8.0 + 1.0 / 8.0);
  printf("%-28s %8.3f ms/launch  %7.2f TB/s\n", name, ms, bytes / (ms * 1e-3) / 1e12);
}

int main() {
  const int64_t n = 65536;
  const int steps = 250;
  double *tx, *tlp;
  uint32_t *tacc;
  hipMalloc(&tx, (size_t)n * steps * 11 * 8);
  hipMalloc(&tlp, (size_t)n * steps * 8);
  hipMalloc(&tacc, (size_t)n / 32 * steps * 4);
  run("plain", k_trace<0, 0>, tx, tlp, tacc, n, steps);
  run("nontemporal", k_trace<1, 0>, tx, tlp, tacc, n, steps);
  run("plain + 20 fma/dim", k_trace<0, 20>, tx, tlp, tacc, n, steps);
  run("nontemporal + 20 fma/dim", k_trace<1, 20>, tx, tlp, tacc, n, steps);
  run("plain + 40 fma/dim", k_trace<0, 40>, tx, tlp, tacc, n, steps);
  run("block layout", k_trace_blk<0>, tx, tlp, tacc, n, steps);
  run("block layout nt", k_trace_blk<1>, tx, tlp, tacc, n, steps);
  run("16-B stores (x4 swap)", k_trace_x4<0>, tx, tlp, tacc, n, steps);
  run("16-B stores (x4 swap) nt", k_trace_x4<1>, tx, tlp, tacc, n, steps);
  run("1-KB pieces", k_trace_1k<0>, tx, tlp, tacc, n, steps);
  run("1-KB pieces nt", k_trace_1k<1>, tx, tlp, tacc, n, steps);
  run("512-B rows", k_trace_512<0>, tx, tlp, tacc, n, steps);
  run("512-B rows nt", k_trace_512<1>, tx, tlp, tacc, n, steps);
  run("nontemporal + 40 fma/dim", k_trace<1, 40>, tx, tlp, tacc, n, steps);
  return 0;
}
