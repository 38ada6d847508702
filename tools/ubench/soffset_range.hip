// Does the raw-buffer range check of gfx950 include the SGPR offset?
// One wave stores lane-indexed words through a resource of num_records =
// 256 bytes with voffset = 4 * lane and soffset = 0, 128, 512; the words
// that land say which lanes passed the check.
// build: hipcc --offload-arch=gfx950 -O2 -o soffset_range soffset_range.hip
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void probe(unsigned *buf, int soff) {
  const unsigned lane = threadIdx.x;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(buf, 0, 256, 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b32(lane + 1, rs, (int)(lane * 4), soff, 0);
}

int main() {
  unsigned *d;
  hipMalloc(&d, 4096);
  const int soffs[3] = {0, 128, 512};
  for (int s : soffs) {
    hipMemset(d, 0, 4096);
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d, s);
    unsigned h[1024];
    hipMemcpy(h, d, 4096, hipMemcpyDeviceToHost);
    int n = 0, first = -1, last = -1;
    for (int i = 0; i < 1024; ++i)
      if (h[i]) { ++n; if (first < 0) first = i; last = i; }
    std::printf("{\"soffset\": %d, \"words_written\": %d, \"first_word\": %d, \"last_word\": %d, "
                "\"first_lane\": %d, \"last_lane\": %d}\n",
                s, n, first, last, first >= 0 ? (int)h[first] - 1 : -1, last >= 0 ? (int)h[last] - 1 : -1);
  }
  return 0;
}
