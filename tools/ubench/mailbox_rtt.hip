// mailbox_rtt.hip -- host round trip of one command to a resident kernel of
// 256 workgroups and its completion back, for the resident sampling server's
// protocols (the host path of the driver-shape bench).
//   mode 0 relay:   the command in pinned host memory; workgroup 0 polls it
//                   and relays it to a device mailbox, the others poll the
//                   mailbox; per-workgroup completion words, the host scans
//                   them all (the shipped protocol, pbh_kernels_impl.h SRV)
//   mode 1 direct:  the host writes the command straight into fine-grained
//                   device memory, every workgroup polls it; per-workgroup
//                   completion words
//   mode 2 relay  + one completion word (the last workgroup to finish, by a
//                   device atomic counter, writes it)
//   mode 3 direct + one completion word
// Each command runs `work_us` of busy work per workgroup.  Prints one JSON
// line: the host round trip per command (mean / p10 / p50 / p90, us).
// Build: hipcc --offload-arch=gfx950 -O3 -o bin/mailbox_rtt mailbox_rtt.hip
// Usage: mailbox_rtt MODE [iters] [work_us] [wgs]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <csignal>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <unistd.h>
#include <vector>

typedef uint32_t u4 __attribute__((ext_vector_type(4)));
struct alignas(16) Cmd {
  uint32_t seq, n, a, b;
};
struct alignas(64) Done {
  uint32_t seq, pad[15];
};

__device__ __forceinline__ u4 ld16_sys(const void *p) {
  u4 v;
  asm volatile("global_load_dwordx4 %0, %1, off sc0 sc1\n\ts_waitcnt vmcnt(0)"
               : "=v"(v) : "v"(p) : "memory");
  return v;
}
__device__ __forceinline__ void st16_sys(void *p, u4 v) {
  asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" : : "v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ void st4_sys(void *p, uint32_t v) {
  asm volatile("global_store_dword %0, %1, off sc0 sc1" : : "v"(p), "v"(v) : "memory");
}

__global__ __launch_bounds__(256) void server(const Cmd *hcmd, Cmd *mail, Done *done,
                                              uint32_t *cnt, uint32_t *fin, int mode,
                                              uint64_t work, uint64_t idle) {
  __shared__ uint32_t s_q;
  const bool relay = (mode & 1) == 0, single = mode >= 2;
  const bool poller_wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x) < 64;
  const Cmd *src = (relay && blockIdx.x == 0) ? hcmd : mail;
  uint32_t seen = 0u;
  for (;;) {
    if (poller_wave) {
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      uint32_t q;
      u4 v;
      for (;;) {
        v = ld16_sys(src);
        q = (uint32_t)__builtin_amdgcn_readfirstlane((int)v.x);
        if (q != seen) break;
        if (__builtin_amdgcn_s_memrealtime() - t0 > idle) {
          q = 0u;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      if (relay && blockIdx.x == 0 && q) st16_sys(mail, v);
      if (threadIdx.x == 0) s_q = q;
    }
    __syncthreads();
    const uint32_t q = (uint32_t)__builtin_amdgcn_readfirstlane((int)s_q);
    __syncthreads();   // every wave read s_q before the poller writes it again
    if (q == 0u || q == 0xFFFFFFFFu) break;
    const uint64_t tw = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - tw < work) __builtin_amdgcn_s_sleep(1);
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    if (threadIdx.x == 0) {
      if (!single) {
        st4_sys(&done[blockIdx.x].seq, q);
      } else {
        const uint32_t old =
            __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (old + 1u == q * gridDim.x) st4_sys(fin, q);
      }
    }
    seen = q;
  }
}

static const char *const kNames[4] = {"relay", "direct", "relay+single", "direct+single"};

static void on_segv(int) {
  static const char m[] = "{\"error\": \"SIGSEGV: the host cannot write this device memory\"}\n";
  (void)!write(1, m, sizeof m - 1);
  _exit(3);
}

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      std::printf("{\"error\": \"%s: %s\"}\n", #x, hipGetErrorString(e_));     \
      return 2;                                                                \
    }                                                                          \
  } while (0)

int main(int argc, char **argv) {
  const int mode = argc > 1 ? std::atoi(argv[1]) : 0;
  const int iters = argc > 2 ? std::atoi(argv[2]) : 2000;
  const double work_us = argc > 3 ? std::atof(argv[3]) : 20.0;
  const int wgs = argc > 4 ? std::atoi(argv[4]) : 256;
  const bool direct = (mode & 1) != 0, single = mode >= 2;
  std::signal(SIGSEGV, on_segv);
  Cmd *hcmd = nullptr, *mail = nullptr;
  Done *done = nullptr;
  uint32_t *fin = nullptr, *cnt = nullptr;
  CK(hipHostMalloc((void **)&hcmd, sizeof(Cmd), hipHostMallocCoherent));
  CK(hipHostMalloc((void **)&done, wgs * sizeof(Done), hipHostMallocCoherent));
  CK(hipHostMalloc((void **)&fin, 64, hipHostMallocCoherent));
  std::memset(hcmd, 0, sizeof(Cmd));
  std::memset(done, 0, wgs * sizeof(Done));
  *fin = 0u;
  if (direct)
    CK(hipExtMallocWithFlags((void **)&mail, 64, hipDeviceMallocFinegrained));
  else
    CK(hipMalloc((void **)&mail, 64));
  CK(hipMemset(mail, 0, 64));
  CK(hipMalloc((void **)&cnt, 64));
  CK(hipMemset(cnt, 0, 64));
  CK(hipDeviceSynchronize());
  Cmd *wr = hcmd;
  if (direct) {
    // the host writes the device mailbox through its own mapping of it
    hipPointerAttribute_t at{};
    CK(hipPointerGetAttributes(&at, mail));
    wr = reinterpret_cast<Cmd *>(at.hostPointer ? at.hostPointer : (void *)mail);
    volatile uint32_t *probe = &wr->b;
    *probe = 7u;   // SIGSEGV here: not host-accessible
    __builtin_ia32_sfence();
    uint32_t back = 0;
    CK(hipMemcpy(&back, &mail->b, 4, hipMemcpyDeviceToHost));
    if (back != 7u) {
      std::printf("{\"error\": \"host write to device memory not seen (%u)\"}\n", back);
      return 4;
    }
    *probe = 0u;
  }
  Done *ddone = nullptr;
  uint32_t *dfin = nullptr;
  Cmd *dcmd = nullptr;
  CK(hipHostGetDevicePointer((void **)&ddone, done, 0));
  CK(hipHostGetDevicePointer((void **)&dfin, fin, 0));
  CK(hipHostGetDevicePointer((void **)&dcmd, hcmd, 0));
  const uint64_t work = (uint64_t)(work_us * 100.0);   // 100 MHz ticks
  const uint64_t idle = 200000000ull;                   // 2 s
  hipLaunchKernelGGL(server, dim3(wgs), dim3(256), 0, 0, dcmd, mail, ddone, cnt, dfin, mode,
                     work, idle);
  CK(hipGetLastError());
  std::vector<double> rtt;
  rtt.reserve(iters);
  using clk = std::chrono::steady_clock;
  for (int it = 1; it <= iters + 100; ++it) {
    const auto t0 = clk::now();
    __atomic_store_n(&wr->seq, (uint32_t)it, __ATOMIC_RELEASE);
    if (direct) __builtin_ia32_sfence();   // out of any write-combining buffer
    // (a command not completed in 1 s: stop; the kernel's idle exit ends it)
    bool late = false;
    if (single) {
      while (__atomic_load_n(fin, __ATOMIC_ACQUIRE) != (uint32_t)it)
        if ((late = clk::now() - t0 > std::chrono::seconds(1))) break;
    } else {
      for (int w = 0; w < wgs;) {
        if (__atomic_load_n(&done[w].seq, __ATOMIC_ACQUIRE) == (uint32_t)it) ++w;
        else if ((late = clk::now() - t0 > std::chrono::seconds(1))) break;
      }
    }
    if (late) {
      std::printf("{\"error\": \"command %d not completed in 1 s\"}\n", it);
      (void)hipDeviceSynchronize();   // the kernel's 2 s idle exit
      return 5;
    }
    const auto t1 = clk::now();
    if (it > 100) rtt.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
  }
  __atomic_store_n(&wr->seq, 0xFFFFFFFFu, __ATOMIC_RELEASE);
  __builtin_ia32_sfence();
  CK(hipDeviceSynchronize());
  std::sort(rtt.begin(), rtt.end());
  double m = 0;
  for (double v : rtt) m += v;
  m /= rtt.size();
  auto pct = [&](double p) { return rtt[(size_t)(p * (rtt.size() - 1))]; };
  std::printf("{\"mode\": %d, \"name\": \"%s\", \"wgs\": %d, \"work_us\": %.2f, \"iters\": %d, "
              "\"rtt_us_mean\": %.3f, \"p10\": %.3f, \"p50\": %.3f, \"p90\": %.3f}\n",
              mode, kNames[mode & 3],
              wgs, work_us, iters, m, pct(0.1), pct(0.5), pct(0.9));
  return 0;
}
