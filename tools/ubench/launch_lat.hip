// Launch / completion latency of one short kernel on gfx950 under the HIP
// runtime: how long the host spends enqueuing (event markers + launch, or a
// graph), and how long after the GPU is done the host sees it, for several
// completion checks.  The kernel busy-waits a given time on the 100 MHz
// real-time counter over a full grid (2 048 waves), so "wall - busy" is the
// fixed cost of one timed launch.  Writes one JSON line per variant.
// build: hipcc --offload-arch=gfx950 -O2 -o launch_lat launch_lat.hip
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                               \
  do {                                                                      \
    hipError_t e_ = (x);                                                    \
    if (e_ != hipSuccess) {                                                 \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));          \
      std::exit(1);                                                         \
    }                                                                       \
  } while (0)

struct Args {
  double *out;
  long ticks;   // busy time in 10 ns ticks
  long pad[80]; // a kernarg block of the engine's size (KArgs: 664 bytes)
};

__global__ __launch_bounds__(256) void busy(Args a) {
  const long t0 = __builtin_amdgcn_s_memrealtime();
  while ((long)__builtin_amdgcn_s_memrealtime() - t0 < a.ticks) {
  }
  if (threadIdx.x == 0) a.out[blockIdx.x] = (double)t0;
}

using clk = std::chrono::steady_clock;
static double us(clk::time_point a, clk::time_point b) {
  return std::chrono::duration<double, std::micro>(b - a).count();
}

enum Sync { SQ, EQ, SS, FLAG };
static const char *sync_name[] = {"stream_query", "event_query", "stream_sync", "host_flag"};
enum Launch { MARKERS, GRAPH, EXT };
static const char *launch_name[] = {"markers", "graph", "ext_events"};

int main(int argc, char **argv) {
  const long busy_us = argc > 1 ? std::atol(argv[1]) : 20;
  const int reps = argc > 2 ? std::atoi(argv[2]) : 50;
  const bool spin_flag = argc > 3 && std::atoi(argv[3]);
  if (spin_flag) CK(hipSetDeviceFlags(hipDeviceScheduleSpin));
  CK(hipSetDevice(0));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  Args a{};
  CK(hipMalloc(&a.out, 8192 * sizeof(double)));
  a.ticks = busy_us * 100;
  const dim3 grid(512), block(256);
  volatile int *flag = nullptr;
  CK(hipHostMalloc((void **)&flag, 64, hipHostMallocCoherent | hipHostMallocMapped));
  int *dflag = nullptr;
  CK(hipHostGetDevicePointer((void **)&dflag, (void *)flag, 0));
  // graph of [event, kernel, event]
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
  CK(hipEventRecord(e0, st));
  hipLaunchKernelGGL(busy, grid, block, 0, st, a);
  CK(hipEventRecord(e1, st));
  CK(hipStreamEndCapture(st, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  for (int w = 0; w < 5; ++w) {
    hipLaunchKernelGGL(busy, grid, block, 0, st, a);
    CK(hipGraphLaunch(ge, st));
  }
  CK(hipStreamSynchronize(st));

  for (int L = 0; L < 3; ++L) {
    for (int S = 0; S < 4; ++S) {
      std::vector<double> enq, wall, ev;
      for (int r = 0; r < reps + 3; ++r) {
        CK(hipStreamSynchronize(st));
        *flag = 0;
        const auto t0 = clk::now();
        if (L == MARKERS) {
          CK(hipEventRecord(e0, st));
          hipLaunchKernelGGL(busy, grid, block, 0, st, a);
          CK(hipEventRecord(e1, st));
        } else if (L == GRAPH) {
          CK(hipGraphLaunch(ge, st));
        } else {
          hipExtLaunchKernelGGL(busy, grid, block, 0, st, e0, e1, 0, a);
        }
        if (S == FLAG) CK(hipStreamWriteValue32(st, dflag, 1, 0));
        const auto t1 = clk::now();
        if (S == SQ) {
          while (hipStreamQuery(st) == hipErrorNotReady) {
          }
        } else if (S == EQ) {
          while (hipEventQuery(e1) == hipErrorNotReady) {
          }
        } else if (S == SS) {
          CK(hipStreamSynchronize(st));
        } else {
          while (*flag == 0) {
          }
        }
        const auto t2 = clk::now();
        CK(hipStreamSynchronize(st));
        float ms = 0.f;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (r >= 3) {
          enq.push_back(us(t0, t1));
          wall.push_back(us(t0, t2));
          ev.push_back(ms * 1e3);
        }
      }
      auto med = [](std::vector<double> v) {
        std::sort(v.begin(), v.end());
        return v[v.size() / 2];
      };
      std::printf("{\"launch\": \"%s\", \"sync\": \"%s\", \"busy_us\": %ld, \"spin_flag\": %d, "
                  "\"enqueue_us\": %.2f, \"wall_us\": %.2f, \"events_us\": %.2f}\n",
                  launch_name[L], sync_name[S], busy_us, (int)spin_flag, med(enq),
                  med(wall), med(ev));
      std::fflush(stdout);
    }
  }
  return 0;
}
