// DTW dynamic-programme microbenchmark (launch_dtw_dp_only: the token-time DP and backtrace of one
// window, [rows][1500] f32 cost matrix), alone on the GPU; per-launch time.  WDR_DTW_DP_OLD=1 times
// the 256-thread barrier-per-diagonal form; WDR_DTW_WAVE_MAX=R the one-wave form up to R rows a lane.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/dtw_bench.cpp -Lwhisper-diarize-rs_amd -lwdr
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../whisper-diarize-rs_amd/csrc/common.h"
#include "../whisper-diarize-rs_amd/csrc/kernels/kernels.h"

using namespace wdr;

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);          \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

int main() {
  const int M = 1500;
  // a background load on another stream keeps the clocks up (a lone 1-block kernel leaves the GPU
  // in a low power state: several times slower)
  hipStream_t bg;
  CK(hipStreamCreateWithFlags(&bg, hipStreamNonBlocking));
  float* sink;
  CK(hipMalloc(&sink, 1 << 16));
  for (int k = 0; k < 200; ++k) launch_busy(128, 4000000, sink, bg);
  for (int rows : {24, 60, 100, 160, 221}) {
    std::vector<float> h((size_t)rows * M);
    unsigned v = 12345u + rows;
    for (auto& f : h) {
      v = v * 1664525u + 1013904223u;
      f = (float)((v >> 8) & 0xffff) / 65536.0f - 0.5f;
    }
    float* x;
    int *t, *nt;
    CK(hipMalloc(&x, h.size() * 4));
    CK(hipMalloc(&t, 4096));
    CK(hipMalloc(&nt, 4));
    CK(hipMemcpy(x, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    launch_dtw_dp_only(x, rows, M, 0, t, nt, nullptr);
    CK(hipDeviceSynchronize());
    const int it = 20;
    CK(hipEventRecord(a, nullptr));
    for (int k = 0; k < it; ++k) launch_dtw_dp_only(x, rows, M, 0, t, nt, nullptr);
    CK(hipEventRecord(b, nullptr));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    int n = 0;
    CK(hipMemcpy(&n, nt, 4, hipMemcpyDeviceToHost));
    std::vector<int> ht(n);
    CK(hipMemcpy(ht.data(), t, n * 4, hipMemcpyDeviceToHost));
    long long cs = 0;
    for (int k = 0; k < n; ++k) cs = cs * 31 + ht[k];
    printf("dtw_dp rows %3d M %d: %8.1f us per window  (%d times, checksum %lld)\n", rows, M, ms * 1e3 / it, n, cs);
    CK(hipFree(x));
    CK(hipFree(t));
    CK(hipFree(nt));
  }
  CK(hipDeviceSynchronize());
  return 0;
}
