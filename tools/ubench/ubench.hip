// Micro-benchmarks of the instruction mixes in the MH step loop (gfx950).
// Each kernel runs R iterations of a dependent-but-4-way-interleaved body
// per lane over a full grid; prints ns per (wave64 instruction-group).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include "../../probayes_amd/csrc/pbh_device.h"

using namespace pbh;
constexpr int R = 4096;

__global__ void k_mad64(uint32_t *out, uint32_t s) {
  uint32_t a = threadIdx.x + s, b = blockIdx.x, c = a ^ 7, d = b + 3;
  for (int i = 0; i < R; ++i) {
    uint64_t p = (uint64_t)0xD2511F53u * a; a = (uint32_t)(p >> 32) ^ (uint32_t)p;
    uint64_t q = (uint64_t)0xCD9E8D57u * b; b = (uint32_t)(q >> 32) ^ (uint32_t)q;
    uint64_t r = (uint64_t)0xD2511F53u * c; c = (uint32_t)(r >> 32) ^ (uint32_t)r;
    uint64_t t = (uint64_t)0xCD9E8D57u * d; d = (uint32_t)(t >> 32) ^ (uint32_t)t;
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a ^ b ^ c ^ d;
}
__global__ void k_xor(uint32_t *out, uint32_t s) {
  uint32_t a = threadIdx.x + s, b = blockIdx.x, c = a ^ 7, d = b + 3;
  for (int i = 0; i < R; ++i) {
    a = (a ^ s) + 1u; b = (b ^ s) + 3u; c = (c ^ s) + 5u; d = (d ^ s) + 7u;
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a ^ b ^ c ^ d;
}
__global__ void k_fma64(double *out, double s) {
  double a = threadIdx.x * s, b = blockIdx.x * s, c = a + 1, d = b + 1;
  for (int i = 0; i < R; ++i) {
    a = __builtin_fma(a, s, 0.5); b = __builtin_fma(b, s, 0.5);
    c = __builtin_fma(c, s, 0.5); d = __builtin_fma(d, s, 0.5);
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a + b + c + d;
}
__global__ void k_fma32(float *out, float s) {
  float a = threadIdx.x * s, b = blockIdx.x * s, c = a + 1, d = b + 1;
  for (int i = 0; i < R; ++i) {
    a = __builtin_fmaf(a, s, 0.5f); b = __builtin_fmaf(b, s, 0.5f);
    c = __builtin_fmaf(c, s, 0.5f); d = __builtin_fmaf(d, s, 0.5f);
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a + b + c + d;
}
__global__ void k_philox(uint32_t *out, uint32_t s) {
  uint32_t acc = 0;
  for (int i = 0; i < R / 16; ++i) {
    u32x4 w = philox4x32_10(u32x4{(uint32_t)i, threadIdx.x, blockIdx.x, s}, s, s + 1);
    acc ^= w.x ^ w.y ^ w.z ^ w.w;
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}
__global__ void k_exp64(double *out, double s) {
  double a = threadIdx.x * 1e-3 - s, acc = 0;
  for (int i = 0; i < R / 16; ++i) { acc += exp(a); a += 1e-4; }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

__global__ void k_expcheck(double *out, const double *x, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) { out[2 * i] = exp(x[i]); out[2 * i + 1] = fast_exp(x[i]); }
}

__global__ void k_mullo(uint32_t *out, uint32_t s) {
  uint32_t a = threadIdx.x + s, b = blockIdx.x, c = a ^ 7, d = b + 3;
  for (int i = 0; i < R; ++i) {
    a = a * 0xD2511F53u + s; b = b * 0xCD9E8D57u + s; c = c * 0xD2511F53u + s; d = d * 0xCD9E8D57u + s;
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a ^ b ^ c ^ d;
}
__global__ void k_mulhi(uint32_t *out, uint32_t s) {
  uint32_t a = threadIdx.x + s, b = blockIdx.x, c = a ^ 7, d = b + 3;
  for (int i = 0; i < R; ++i) {
    a = __umulhi(a, 0xD2511F53u) ^ s; b = __umulhi(b, 0xCD9E8D57u) ^ s; c = __umulhi(c, 0xD2511F53u) ^ s; d = __umulhi(d, 0xCD9E8D57u) ^ s;
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a ^ b ^ c ^ d;
}
__global__ void k_xor3(uint32_t *out, uint32_t s) {
  uint32_t a = threadIdx.x + s, b = blockIdx.x, c = a ^ 7, d = b + 3;
  for (int i = 0; i < R; ++i) {
    a = a ^ b ^ s; b = b ^ c ^ s; c = c ^ d ^ s; d = d ^ a ^ s;
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a ^ b ^ c ^ d;
}
__global__ void k_add64(double *out, double s) {
  double a = threadIdx.x * s, b = blockIdx.x * s, c = a + 1, d = b + 1;
  for (int i = 0; i < R; ++i) { a = a + s; b = b + s; c = c + s; d = d + s; }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a + b + c + d;
}
__global__ void k_trans32(float *out, float s) {
  float a = threadIdx.x * s, b = blockIdx.x * s, c = a + 1, d = b + 1;
  for (int i = 0; i < R; ++i) {
    a = __builtin_amdgcn_logf(a); b = __builtin_amdgcn_logf(b); c = __builtin_amdgcn_logf(c); d = __builtin_amdgcn_logf(d);
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a + b + c + d;
}
__global__ void k_cvt(double *out, double s) {
  float a = threadIdx.x * (float)s, b = blockIdx.x, c = a + 1, d = b + 1;
  double acc = 0;
  for (int i = 0; i < R; ++i) {
    double x = (double)a, y = (double)b, z = (double)c, w = (double)d;
    a = (float)x + 1.f; b = (float)y + 1.f; c = (float)z + 1.f; d = (float)w + 1.f;
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a + b + c + d;
}
__global__ void k_xoshiro(uint32_t *out, uint32_t s) {
  Xo x{threadIdx.x + s, blockIdx.x | 1u, s, 7u};
  uint32_t acc = 0;
  for (int i = 0; i < R / 4; ++i) acc ^= xo_next(x);
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <class K, class T>
float timeit(K k, T *buf, T s, int blocks) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, buf, s);
  hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, buf, s);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  return ms / 5;
}

int main() {
  const int blocks = 2048;   // 8 waves / SIMD
  uint32_t *u; double *d; float *f;
  hipMalloc(&u, blocks * 256 * 4); hipMalloc(&d, blocks * 256 * 8); hipMalloc(&f, blocks * 256 * 4);
  const double waves = blocks * 4.0, simds = 1024.0;
  auto rep = [&](const char *n, float ms, double ops_per_iter, double iters) {
    double wave_ops = waves * iters * ops_per_iter;
    printf("%-10s %8.3f ms  %.2f cycles/wave-instr/SIMD @2.4GHz\n", n, ms,
           ms * 1e-3 * 2.4e9 * simds / wave_ops);
  };
  rep("mad_u64", timeit(k_mad64, u, 3u, blocks), 4 * 2, R);   // mad + xor
  rep("xor+add", timeit(k_xor, u, 3u, blocks), 4 * 2, R);
  rep("fma_f64", timeit(k_fma64, d, 0.999, blocks), 4, R);
  rep("fma_f32", timeit(k_fma32, f, 0.999f, blocks), 4, R);
  rep("mul_lo", timeit(k_mullo, u, 3u, blocks), 4 * 2, R);
  rep("mul_hi+x", timeit(k_mulhi, u, 3u, blocks), 4 * 2, R);
  rep("xor3", timeit(k_xor3, u, 3u, blocks), 4, R);
  rep("add_f64", timeit(k_add64, d, 0.999, blocks), 4, R);
  rep("log_f32", timeit(k_trans32, f, 0.999f, blocks), 4, R);
  rep("cvt64+32+a", timeit(k_cvt, d, 0.999, blocks), 4 * 3, R);
  float xm = timeit(k_xoshiro, u, 3u, blocks);
  printf("xoshiro   %8.3f ms  %.1f ns per word per wave-slot\n", xm, xm * 1e6 / (waves * R / 4) * simds);
  float pm = timeit(k_philox, u, 3u, blocks);
  printf("philox    %8.3f ms  %.1f ns per call per wave-slot\n", pm, pm * 1e6 / (waves * R / 16) * simds);
  float em = timeit(k_exp64, d, 0.5, blocks);
  printf("exp_f64   %8.3f ms  %.1f ns per call per wave-slot\n", em, em * 1e6 / (waves * R / 16) * simds);
  // fast_exp accuracy against ocml exp over [-746, 710]
  const int n = 1 << 20;
  double *hx = new double[n], *ho = new double[2 * n], *dx, *dout;
  for (int i = 0; i < n; ++i) hx[i] = -746.0 + 1456.0 * (i + 0.5) / n;
  hipMalloc(&dx, n * 8); hipMalloc(&dout, 2 * n * 8);
  hipMemcpy(dx, hx, n * 8, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k_expcheck, dim3(n / 256), dim3(256), 0, 0, dout, dx, n);
  hipMemcpy(ho, dout, 2 * n * 8, hipMemcpyDeviceToHost);
  long long maxulp = 0;
  for (int i = 0; i < n; ++i) {
    long long a = *(long long *)&ho[2 * i], b = *(long long *)&ho[2 * i + 1];
    long long dd = a > b ? a - b : b - a;
    if (ho[2 * i] > 2.3e-308 && dd > maxulp) maxulp = dd;
  }
  printf("fast_exp max ulp vs ocml exp (normal range): %lld\n", maxulp);
  return 0;
}
