// im2col microbenchmark: CAM++'s batched FCM im2col (k_im2col_2d_b, the shapes CamModel issues
// for a batch of utterances) and whisper's conv2 im2col (k_im2col_conv2, nb windows of large-v3),
// alone on the GPU; per-launch time and GB/s of the bytes written.  Linked against libwdr.so, so
// the same binary times another build of the library (LD_LIBRARY_PATH); -DNO_CONV2 drops the conv2
// part for a library whose conv2 launcher has the older (one window) signature.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/im2col_bench.cpp -Lwhisper-diarize-rs_amd -lwdr
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

template <typename F>
static double time_us(F f, int iters) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  f();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a, nullptr));
  for (int i = 0; i < iters; ++i) f();
  CK(hipEventRecord(b, nullptr));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms * 1e3 / iters;
}

int main() {
  // a CAM++ batch: B utterances of ~T/B frames each (16 000 frames, the embedding worker's cap)
  const int B = 64, Tt = 16000;
  std::vector<int> off(B), len(B);
  for (int b = 0; b < B; ++b) {
    off[b] = b * (Tt / B);
    len[b] = Tt / B;
  }
  int *d_off, *d_len;
  CK(hipMalloc(&d_off, B * 4));
  CK(hipMalloc(&d_len, B * 4));
  CK(hipMemcpy(d_off, off.data(), B * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_len, len.data(), B * 4, hipMemcpyHostToDevice));
  SegRows sr{d_off, d_len, B};
  float *X, *col;
  CK(hipMalloc(&X, (size_t)Tt * 80 * 32 * 4));
  CK(hipMalloc(&col, (size_t)Tt * 80 * 288 * 4));
  CK(hipMemset(X, 0x3c, (size_t)Tt * 80 * 32 * 4));
  struct Shape {
    int F, C, kf, kt, sf, Fo;
  } shapes[] = {{80, 1, 3, 3, 1, 80}, {80, 32, 3, 3, 2, 40}, {80, 32, 1, 1, 2, 40}, {40, 32, 3, 3, 1, 40},
                {40, 32, 3, 3, 2, 20}, {20, 32, 3, 3, 1, 20}, {20, 32, 3, 3, 2, 10}};
  for (const Shape& s : shapes) {
    const double us = time_us([&] { launch_im2col_2d_b(X, sr, Tt, s.F, s.C, s.kf, s.kt, s.sf, s.Fo, col, nullptr); }, 20);
    const double wb = (double)Tt * s.Fo * s.C * s.kf * s.kt * 4;
    printf("im2col_2d_b T %d F %2d C %2d k %dx%d sf %d Fo %2d: %8.1f us  write %7.1f MB  %6.2f TB/s\n", Tt, s.F, s.C,
           s.kf, s.kt, s.sf, s.Fo, us, wb / 1e6, wb / us * 1e-6);
  }
#ifndef NO_CONV2
  const int d = 1280;
  for (int nb : {1, 6}) {
    f16 *x, *out;
    CK(hipMalloc(&x, (size_t)nb * 3000 * d * 2));
    CK(hipMalloc(&out, (size_t)nb * 1500 * 3 * d * 2));
    CK(hipMemset(x, 0x3c, (size_t)nb * 3000 * d * 2));
    const double us = time_us([&] { launch_im2col_conv2(x, d, nb, out, nullptr); }, 50);
    const double wb = (double)nb * 1500 * 3 * d * 2, rb = (double)nb * 3000 * d * 2;
    printf("im2col_conv2 nb %d d %d: %8.1f us  write %6.1f MB read %6.1f MB  %6.2f TB/s\n", nb, d, us, wb / 1e6, rb / 1e6,
           (wb + rb) / us * 1e-6);
    CK(hipFree(x));
    CK(hipFree(out));
  }
#endif
  return 0;
}
