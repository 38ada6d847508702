// Per-instruction VALU cost on gfx950, measured with inline asm so the
// compiler cannot substitute forms: throughput (cycles per wave-instruction
// per SIMD) at W waves per SIMD, 8 independent register chains per lane.
// Used to price the MH step's instruction mix.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <cstdint>

constexpr int R = 2048;

#define K32(NAME, ASM)                                                      \
  __global__ void NAME(uint32_t *out, uint32_t s) {                         \
    uint32_t v0 = threadIdx.x + s, v1 = v0 ^ 1, v2 = v0 ^ 2, v3 = v0 ^ 3,   \
             v4 = v0 ^ 4, v5 = v0 ^ 5, v6 = v0 ^ 6, v7 = v0 ^ 7;            \
    uint32_t k = s * 3 + threadIdx.x;                                       \
    for (int i = 0; i < R; ++i) {                                           \
      asm volatile(ASM : "+v"(v0) : "v"(k), "s"(s));                        \
      asm volatile(ASM : "+v"(v1) : "v"(k), "s"(s));                        \
      asm volatile(ASM : "+v"(v2) : "v"(k), "s"(s));                        \
      asm volatile(ASM : "+v"(v3) : "v"(k), "s"(s));                        \
      asm volatile(ASM : "+v"(v4) : "v"(k), "s"(s));                        \
      asm volatile(ASM : "+v"(v5) : "v"(k), "s"(s));                        \
      asm volatile(ASM : "+v"(v6) : "v"(k), "s"(s));                        \
      asm volatile(ASM : "+v"(v7) : "v"(k), "s"(s));                        \
    }                                                                       \
    out[blockIdx.x * blockDim.x + threadIdx.x] =                            \
        v0 ^ v1 ^ v2 ^ v3 ^ v4 ^ v5 ^ v6 ^ v7;                              \
  }

#define K64(NAME, ASM)                                                      \
  __global__ void NAME(uint32_t *out, uint32_t s) {                         \
    uint64_t v0 = threadIdx.x + s, v1 = v0 ^ 1, v2 = v0 ^ 2, v3 = v0 ^ 3,   \
             v4 = v0 ^ 4, v5 = v0 ^ 5, v6 = v0 ^ 6, v7 = v0 ^ 7;            \
    uint64_t k = s * 3ull + threadIdx.x;                                    \
    for (int i = 0; i < R; ++i) {                                           \
      asm volatile(ASM : "+v"(v0) : "v"(k), "s"(s));                        \
      asm volatile(ASM : "+v"(v1) : "v"(k), "s"(s));                        \
      asm volatile(ASM : "+v"(v2) : "v"(k), "s"(s));                        \
      asm volatile(ASM : "+v"(v3) : "v"(k), "s"(s));                        \
      asm volatile(ASM : "+v"(v4) : "v"(k), "s"(s));                        \
      asm volatile(ASM : "+v"(v5) : "v"(k), "s"(s));                        \
      asm volatile(ASM : "+v"(v6) : "v"(k), "s"(s));                        \
      asm volatile(ASM : "+v"(v7) : "v"(k), "s"(s));                        \
    }                                                                       \
    out[blockIdx.x * blockDim.x + threadIdx.x] =                            \
        (uint32_t)(v0 ^ v1 ^ v2 ^ v3 ^ v4 ^ v5 ^ v6 ^ v7);                  \
  }

// 32-bit forms: %0 = acc (in/out), %1 = vector operand, %2 = scalar
K32(k_xor, "v_xor_b32 %0, %0, %1")
K32(k_add, "v_add_u32 %0, %0, %1")
K32(k_bitop3, "v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96")
K32(k_alignbit, "v_alignbit_b32 %0, %0, %0, 7")
K32(k_lshladd, "v_lshl_add_u32 %0, %0, 2, %1")
K32(k_mullo, "v_mul_lo_u32 %0, %0, %1")
K32(k_mulhi, "v_mul_hi_u32 %0, %0, %1")
K32(k_cndmask, "v_cndmask_b32 %0, %0, %1, vcc")
K32(k_fma32, "v_fma_f32 %0, %0, %1, %1")
K32(k_mul32, "v_mul_f32 %0, %0, %1")
K32(k_exp32, "v_exp_f32 %0, %0")
K32(k_log32, "v_log_f32 %0, %0")
K32(k_sin32, "v_sin_f32 %0, %0")
K32(k_sqrt32, "v_sqrt_f32 %0, %0")
K32(k_cvtf32u, "v_cvt_f32_u32 %0, %0")
K32(k_dpp, "v_mov_b32_dpp %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf")
K32(k_perm32, "s_nop 1\n\tv_permlane32_swap_b32 %0, %1")
K32(k_perm16, "s_nop 1\n\tv_permlane16_swap_b32 %0, %1")
// 64-bit forms
K64(k_fma64, "v_fma_f64 %0, %0, %1, %1")
K64(k_add64, "v_add_f64 %0, %0, %1")
K64(k_mul64, "v_mul_f64 %0, %0, %1")
K64(k_cvtf64f32, "v_cvt_f64_f32 %0, %2")
K64(k_ldexp64, "v_ldexp_f64 %0, %0, %2")
K64(k_rcp64, "v_rcp_f64 %0, %0")
K64(k_lshladd64, "v_lshl_add_u64 %0, %0, 3, %1")
K64(k_pkfma32, "v_pk_fma_f32 %0, %0, %1, %1")
K64(k_mov64, "v_mov_b64 %0, %1")

// v_mad_u64_u32: 32 x 32 + 64 -> 64 (the Philox round's multiply)
__global__ void k_mad64(uint32_t *out, uint32_t s) {
  uint64_t v[8];
  uint32_t a = threadIdx.x * 7 + s;
  for (int j = 0; j < 8; ++j) v[j] = a + j;
  for (int i = 0; i < R; ++i) {
#pragma unroll
    for (int j = 0; j < 8; ++j)
      asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(v[j]) : "v"(a), "v"(s) : "vcc");
  }
  uint64_t x = 0;
  for (int j = 0; j < 8; ++j) x ^= v[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)x;
}

// v_cndmask_b32 with a real lane mask: e64 form reading an SGPR pair, and
// the e32 form reading VCC written once by a v_cmp before the loop.
__global__ void k_cnd_sgpr(uint32_t *out, uint32_t s) {
  uint32_t v[8];
  const uint32_t a = threadIdx.x * 7 + s;
  const uint64_t m = __ballot(threadIdx.x & 1);
  for (int j = 0; j < 8; ++j) v[j] = a + j;
  for (int i = 0; i < R; ++i) {
#pragma unroll
    for (int j = 0; j < 8; ++j)
      asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(v[j]) : "v"(a), "s"(m));
  }
  uint32_t x = 0;
  for (int j = 0; j < 8; ++j) x ^= v[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}
__global__ void k_cnd_vcc(uint32_t *out, uint32_t s) {
  uint32_t v[8];
  const uint32_t a = threadIdx.x * 7 + s;
  for (int j = 0; j < 8; ++j) v[j] = a + j;
  asm volatile("v_cmp_gt_u32 vcc, %0, %1" :: "v"(a), "v"(s) : "vcc");
  for (int i = 0; i < R; ++i) {
#pragma unroll
    for (int j = 0; j < 8; ++j)
      asm volatile("v_cndmask_b32_e32 %0, %0, %1, vcc" : "+v"(v[j]) : "v"(a) : );
  }
  uint32_t x = 0;
  for (int j = 0; j < 8; ++j) x ^= v[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}
// e64 encoding reading VCC itself
__global__ void k_cnd_e64_vcc(uint32_t *out, uint32_t s) {
  uint32_t v[8];
  const uint32_t a = threadIdx.x * 7 + s;
  for (int j = 0; j < 8; ++j) v[j] = a + j;
  asm volatile("v_cmp_gt_u32 vcc, %0, %1" :: "v"(a), "v"(s) : "vcc");
  for (int i = 0; i < R; ++i) {
#pragma unroll
    for (int j = 0; j < 8; ++j)
      asm volatile("v_cndmask_b32_e64 %0, %0, %1, vcc" : "+v"(v[j]) : "v"(a) : );
  }
  uint32_t x = 0;
  for (int j = 0; j < 8; ++j) x ^= v[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}
// the kernel's pattern: a SALU op writes the mask, then 8 selects read it
// (vcc / e32 against an SGPR pair / e64)
__global__ void k_cnd_salu_vcc(uint32_t *out, uint32_t s) {
  uint32_t v[8];
  const uint32_t a = threadIdx.x * 7 + s;
  for (int j = 0; j < 8; ++j) v[j] = a + j;
  const uint64_t m = 0x5555555555555555ull ^ s;
  for (int i = 0; i < R; ++i) {
    asm volatile("s_mov_b64 vcc, %0" :: "s"(m) : "vcc");
#pragma unroll
    for (int j = 0; j < 8; ++j)
      asm volatile("v_cndmask_b32_e32 %0, %0, %1, vcc" : "+v"(v[j]) : "v"(a) : );
  }
  uint32_t x = 0;
  for (int j = 0; j < 8; ++j) x ^= v[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}
__global__ void k_cnd_salu_sgpr(uint32_t *out, uint32_t s) {
  uint32_t v[8];
  const uint32_t a = threadIdx.x * 7 + s;
  for (int j = 0; j < 8; ++j) v[j] = a + j;
  uint64_t m = 0x5555555555555555ull ^ s;
  for (int i = 0; i < R; ++i) {
    uint64_t mm;
    asm volatile("s_mov_b64 %0, %1" : "=s"(mm) : "s"(m));
#pragma unroll
    for (int j = 0; j < 8; ++j)
      asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(v[j]) : "v"(a), "s"(mm));
  }
  uint32_t x = 0;
  for (int j = 0; j < 8; ++j) x ^= v[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}
// other VOP2 forms with an implicit VCC operand: carry-in add (64-bit address
// arithmetic), against its VOP3 form with an SGPR-pair carry
__global__ void k_addc_e32(uint32_t *out, uint32_t s) {
  uint32_t v[8];
  const uint32_t a = threadIdx.x * 7 + s;
  for (int j = 0; j < 8; ++j) v[j] = a + j;
  asm volatile("v_cmp_gt_u32 vcc, %0, %1" :: "v"(a), "v"(s) : "vcc");
  for (int i = 0; i < R; ++i) {
#pragma unroll
    for (int j = 0; j < 8; ++j)
      asm volatile("v_addc_co_u32_e32 %0, vcc, %0, %1, vcc" : "+v"(v[j]) : "v"(a) : "vcc");
  }
  uint32_t x = 0;
  for (int j = 0; j < 8; ++j) x ^= v[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}
__global__ void k_addc_e64(uint32_t *out, uint32_t s) {
  uint32_t v[8];
  const uint32_t a = threadIdx.x * 7 + s;
  for (int j = 0; j < 8; ++j) v[j] = a + j;
  for (int i = 0; i < R; ++i) {
#pragma unroll
    for (int j = 0; j < 8; ++j)
      asm volatile("v_addc_co_u32_e64 %0, s[40:41], %0, %1, s[42:43]" : "+v"(v[j]) : "v"(a) : "s40", "s41");
  }
  uint32_t x = 0;
  for (int j = 0; j < 8; ++j) x ^= v[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}
__global__ void k_add_co_e32(uint32_t *out, uint32_t s) {
  uint32_t v[8];
  const uint32_t a = threadIdx.x * 7 + s;
  for (int j = 0; j < 8; ++j) v[j] = a + j;
  for (int i = 0; i < R; ++i) {
#pragma unroll
    for (int j = 0; j < 8; ++j)
      asm volatile("v_add_co_u32_e32 %0, vcc, %0, %1" : "+v"(v[j]) : "v"(a) : "vcc");
  }
  uint32_t x = 0;
  for (int j = 0; j < 8; ++j) x ^= v[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}
// cmp + cndmask pair as the compiler emits a select (v_cmp -> s[..] -> cndmask)
__global__ void k_sel(uint32_t *out, uint32_t s) {
  uint32_t v[8];
  const uint32_t a = threadIdx.x * 7 + s;
  for (int j = 0; j < 8; ++j) v[j] = a + j;
  for (int i = 0; i < R; ++i) {
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (v[j] > s) ? v[j] : a;
    asm volatile("" :: "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]), "v"(v[4]), "v"(v[5]), "v"(v[6]), "v"(v[7]));
  }
  uint32_t x = 0;
  for (int j = 0; j < 8; ++j) x ^= v[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}
// dependent fp64 fma chain (latency at 1 wave/SIMD)
__global__ void k_fma64_lat(uint32_t *out, uint32_t s) {
  double v = threadIdx.x * 1e-3, k = 0.999;
  for (int i = 0; i < R * 8; ++i) asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(v) : "v"(k));
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)v;
}
__global__ void k_xor_lat(uint32_t *out, uint32_t s) {
  uint32_t v = threadIdx.x;
  for (int i = 0; i < R * 8; ++i) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(v) : "v"(s));
  out[blockIdx.x * blockDim.x + threadIdx.x] = v;
}
__global__ void k_mad64_lat(uint32_t *out, uint32_t s) {
  uint64_t v = threadIdx.x;
  uint32_t a = s;
  for (int i = 0; i < R * 8; ++i) asm volatile("v_mad_u64_u32 %0, vcc, %1, %1, %0" : "+v"(v) : "v"(a) : "vcc");
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)v;
}

template <class K>
double cyc(K k, uint32_t *buf, int wps) {
  const int blocks = 256 * wps;   // 256 CUs x wps blocks of 4 waves
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, buf, 3u);
  hipEventRecord(e0);
  for (int r = 0; r < 4; ++r)
    hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, buf, 3u);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const double per_simd = (double)wps * R * 8;   // wave-instructions per SIMD
  return ms / 4 * 1e-3 * 2.4e9 / per_simd;
}

int main(int argc, char **argv) {
  uint32_t *u;
  hipMalloc(&u, 256 * 8 * 256 * 4);
  struct E { const char *n; void (*k)(uint32_t *, uint32_t); };
  const E es[] = {
      {"v_xor_b32", k_xor}, {"v_add_u32", k_add}, {"v_bitop3_b32", k_bitop3},
      {"v_alignbit_b32", k_alignbit}, {"v_lshl_add_u32", k_lshladd},
      {"v_mul_lo_u32", k_mullo}, {"v_mul_hi_u32", k_mulhi},
      {"v_cndmask_b32", k_cndmask}, {"v_fma_f32", k_fma32},
      {"v_mul_f32", k_mul32}, {"v_exp_f32", k_exp32}, {"v_log_f32", k_log32},
      {"v_sin_f32", k_sin32}, {"v_sqrt_f32", k_sqrt32},
      {"v_cvt_f32_u32", k_cvtf32u}, {"v_mov_b32_dpp", k_dpp},
      {"v_permlane32_swap+nop", k_perm32}, {"v_permlane16_swap+nop", k_perm16},
      {"v_fma_f64", k_fma64}, {"v_add_f64", k_add64}, {"v_mul_f64", k_mul64},
      {"v_mad_u64_u32", k_mad64}, {"v_cvt_f64_f32", k_cvtf64f32},
      {"v_ldexp_f64", k_ldexp64}, {"v_rcp_f64", k_rcp64},
      {"v_lshl_add_u64", k_lshladd64}, {"v_pk_fma_f32", k_pkfma32},
      {"v_mov_b64", k_mov64}, {"v_cndmask_e64(sgpr)", k_cnd_sgpr},
      {"v_cndmask_e32(vcc)", k_cnd_vcc}, {"select(cmp+cnd)/2", k_sel},
      {"v_cndmask_e64(vcc)", k_cnd_e64_vcc}, {"s_mov vcc+8 e32(vcc)", k_cnd_salu_vcc},
      {"s_mov sgpr+8 e64(sgpr)", k_cnd_salu_sgpr},
      {"v_addc_co_u32_e32(vcc)", k_addc_e32}, {"v_addc_co_u32_e64(sgpr)", k_addc_e64},
      {"v_add_co_u32_e32(vcc)", k_add_co_e32},
      {"LAT v_fma_f64", k_fma64_lat}, {"LAT v_xor_b32", k_xor_lat},
      {"LAT v_mad_u64_u32", k_mad64_lat}};
  printf("%-24s %8s %8s %8s %8s\n", "instruction", "1w/SIMD", "2w/SIMD",
         "4w/SIMD", "8w/SIMD");
  for (const E &e : es) {
    if (argc > 1 && !strstr(e.n, argv[1])) continue;
    printf("%-24s", e.n);
    for (int w : {1, 2, 4, 8}) printf(" %8.2f", cyc(e.k, u, w));
    printf("\n");
  }
  return 0;
}
