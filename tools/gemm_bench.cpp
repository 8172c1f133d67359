// Encoder GEMM microbenchmark (large-v3, 4 windows batched: M = 6000 rows): per-launch time and
// TFLOP/s of the production launch_proj path at the encoder / cross-K/V shapes, uniform random
// f16 operands (MI355X_MICROARCH.md: zero-filled operands read high).
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/gemm_bench.cpp -Lwhisper-diarize-rs_amd -lwdr
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>
#include <cmath>
#include <algorithm>

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

__global__ void k_rand(f16* p, long long n, unsigned seed) {
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    unsigned x = (unsigned)i * 2654435761u + seed;
    x ^= x >> 13;
    x *= 0x5bd1e995u;
    x ^= x >> 15;
    p[i] = (f16)(((x & 0xffff) / 65536.0f - 0.5f) * 0.2f);
  }
}

int main(int argc, char** argv) {
  const int M = argc > 1 ? atoi(argv[1]) : 6000;
  struct Shape {
    const char* name;
    int N, K, epi;
  } shapes[] = {{"qkv   3d x d", 3840, 1280, EPI_F16},        {"o      d x d resid", 1280, 1280, EPI_F32_RESID},
                {"fc1  4d x d gelu", 5120, 1280, EPI_F16_GELU}, {"fc2   d x 4d resid", 1280, 5120, EPI_F32_RESID},
                {"xkv  64d x d", 81920, 1280, EPI_F16}};
  hipStream_t s;
  CK(hipStreamCreate(&s));
  f16 *A, *W;
  float *out, *bias;
  CK(hipMalloc(&A, (size_t)M * 5120 * 2));
  CK(hipMalloc(&W, (size_t)81920 * 1280 * 2));
  CK(hipMalloc(&out, (size_t)M * 81920 * 4 / 2 + (size_t)M * 5120 * 4));
  CK(hipMalloc(&bias, 81920 * 4));
  CK(hipMemset(bias, 0, 81920 * 4));
  hipLaunchKernelGGL(k_rand, dim3(4096), dim3(256), 0, s, A, (long long)M * 5120, 1u);
  hipLaunchKernelGGL(k_rand, dim3(4096), dim3(256), 0, s, W, (long long)81920 * 1280, 2u);
  CK(hipMemsetAsync(out, 0, (size_t)M * 5120 * 4, s));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  std::vector<float> ref, r;
  const char* vname[6] = {"gemm ", "gemm2", "gemm3", "gemm4", "gemm5", "g4gm8"};
  for (const Shape& sh : shapes) {
    for (int variant = 0; variant < 6; ++variant) {
      // 0: k_gemm (register staging, WDR_GEMM1=1); 1: k_gemm2 / k_gemm (WDR_GEMM3=0);
      // 2: k_gemm3 / k_gemm2 (256 x 256 tiles where the shape allows); 3: k_gemm4 (ping-pong)
      unsetenv("WDR_GEMM1");
      unsetenv("WDR_GEMM3");
      // 3: k_gemm4 forced on every shape; 4: the default dispatch (k_gemm5 on the narrow shapes)
      setenv("WDR_GEMM4", variant == 3 || variant == 5 ? "1" : variant == 4 ? "-1" : "0", 1);
      setenv("WDR_GEMM5", variant == 3 ? "0" : "1", 1);
      setenv("WDR_GEMM4_GM", variant == 5 ? "8" : "4", 1);
      if (variant == 0) setenv("WDR_GEMM1", "1", 1);
      if (variant == 1) setenv("WDR_GEMM3", "0", 1);
      gemm_knobs_reload();   // launch_proj reads the knobs once per process
      // EPI_F32 into a zeroed buffer for the cross-check (the timed runs use the real epilogue)
      const size_t on = (size_t)M * sh.N;
      if (sh.N <= 5120) {
        CK(hipMemsetAsync(out, 0, on * 4, s));
        ProjArgs c{A, sh.K, W, sh.K, bias, out, sh.N, nullptr, 0, M, sh.N, sh.K, EPI_F32};
        launch_proj(c, s);
        std::vector<float>& rr = variant == 0 ? ref : r;
        rr.resize(on);
        CK(hipMemcpyAsync(rr.data(), out, on * 4, hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
        if (variant > 0) {
          size_t nd = 0;
          double md = 0, mr = 0;
          for (size_t i = 0; i < ref.size(); ++i) {
            const double dd = std::fabs((double)ref[i] - r[i]);
            if (dd > 0) ++nd;
            md = std::max(md, dd);
            mr = std::max(mr, std::fabs((double)ref[i]));
          }
          printf("   %s vs k_gemm: %zu of %zu differ, max |diff| %.3g (max |ref| %.3g)\n", vname[variant], nd, ref.size(),
                 md, mr);
        }
      }
      // GB_HOT=1: every row of A and B is the same K-vector (lda = ldb = 0), so every operand
      // load hits in cache: the launch time without the memory latency (a diagnostic only)
      const int ldz = getenv("GB_HOT") ? 0 : sh.K;
      ProjArgs p{A, ldz, W, ldz, bias, out, sh.N, nullptr, 0, M, sh.N, sh.K, sh.epi};
      for (int i = 0; i < 3; ++i) launch_proj(p, s);
      const int reps = 20;
      CK(hipEventRecord(a, s));
      for (int i = 0; i < reps; ++i) launch_proj(p, s);
      CK(hipEventRecord(b, s));
      CK(hipEventSynchronize(b));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, a, b));
      const double us = ms * 1e3 / reps, tf = 2.0 * M * sh.N * sh.K / (us * 1e-6) / 1e12;
      printf("%-20s %s M=%d N=%5d K=%4d  %9.1f us  %7.1f TFLOP/s\n", sh.name, vname[variant], M, sh.N, sh.K, us, tf);
    }
  }
  {
    // fp8 MX encoder GEMMs (BASELINE configs[4], k_gemm8): operands quantised once (launch_quant_f8),
    // the production epilogues (fc1: GELU written as the e4m3 fc2 operand); relative error of the
    // f32 product against the f16 kernel's
    const int mp = (M + 255) / 256 * 256;
    uint8_t *A8, *W8, *O8;
    uint32_t *As, *Ws, *Os;
    CK(hipMalloc(&A8, (size_t)mp * 5120));
    CK(hipMalloc(&W8, (size_t)5120 * 5120));
    CK(hipMalloc(&O8, (size_t)mp * 5120));
    CK(hipMalloc(&As, (size_t)40 * mp * 4));
    CK(hipMalloc(&Ws, (size_t)40 * 5120 * 4));
    CK(hipMalloc(&Os, (size_t)40 * mp * 4));
    for (int si = 0; si < 4; ++si) {
      const Shape& sh = shapes[si];
      launch_quant_f8(A, sh.K, M, sh.K, A8, sh.K, As, mp, s);
      launch_quant_f8(W, sh.K, sh.N, sh.K, W8, sh.K, Ws, sh.N, s);
      const size_t on = (size_t)M * sh.N;
      // cross-check in f32 against the f16 GEMM (k_gemm reference path)
      ProjArgs c8{nullptr, sh.K, nullptr, sh.K, bias, out, sh.N, nullptr, 0, M, sh.N, sh.K, EPI_F32};
      c8.A8 = A8; c8.a_sc = As; c8.ld_asc = mp; c8.B8 = W8; c8.b_sc = Ws; c8.ld_bsc = sh.N;
      CK(hipMemsetAsync(out, 0, on * 4, s));
      launch_proj_fp8(c8, s);
      r.resize(on);
      CK(hipMemcpyAsync(r.data(), out, on * 4, hipMemcpyDeviceToHost, s));
      setenv("WDR_GEMM1", "1", 1);
      gemm_knobs_reload();
      ProjArgs c{A, sh.K, W, sh.K, bias, out, sh.N, nullptr, 0, M, sh.N, sh.K, EPI_F32};
      launch_proj(c, s);
      ref.resize(on);
      CK(hipMemcpyAsync(ref.data(), out, on * 4, hipMemcpyDeviceToHost, s));
      CK(hipStreamSynchronize(s));
      unsetenv("WDR_GEMM1");
      gemm_knobs_reload();
      double num = 0, den = 0;
      for (size_t i = 0; i < on; ++i) {
        num += ((double)r[i] - ref[i]) * ((double)r[i] - ref[i]);
        den += (double)ref[i] * ref[i];
      }
      const int epi = sh.epi == EPI_F16_GELU ? EPI_F8_GELU : sh.epi;
      ProjArgs p{nullptr, sh.K, nullptr, sh.K, bias, epi == EPI_F8_GELU ? (void*)O8 : (void*)out, sh.N, nullptr, 0,
                 M, sh.N, sh.K, epi};
      p.A8 = A8; p.a_sc = As; p.ld_asc = mp; p.B8 = W8; p.b_sc = Ws; p.ld_bsc = sh.N; p.o_sc = Os; p.ld_osc = mp;
      for (int i = 0; i < 3; ++i) launch_proj_fp8(p, s);
      const int reps = 20;
      CK(hipEventRecord(a, s));
      for (int i = 0; i < reps; ++i) launch_proj_fp8(p, s);
      CK(hipEventRecord(b, s));
      CK(hipEventSynchronize(b));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, a, b));
      const double us = ms * 1e3 / reps, tf = 2.0 * M * sh.N * sh.K / (us * 1e-6) / 1e12;
      printf("%-20s fp8mx M=%d N=%5d K=%4d  %9.1f us  %7.1f TFLOP/s  (rel. err vs f16 %.4f)\n", sh.name, M, sh.N, sh.K,
             us, tf, std::sqrt(num / std::max(den, 1e-30)));
    }
  }
  {
    // encoder self-attention of the same batch: nb = M / 1500 windows x 20 heads x 1500^2
    const int nb = M / 1500, d = 1280;
    f16* att;
    CK(hipMalloc(&att, (size_t)M * d * 2));
    const long long bs = 1500ll * 3 * d, obs = 1500ll * d;
    FlashArgs fa{A, 3 * d, bs, A + d, 3 * d, bs, A + 2 * d, 3 * d, bs, att, d, obs, nullptr, 1500, 1500, 20, 0, 0.125f};
    for (int i = 0; i < 3; ++i) launch_flash_attn(fa, nb, s);
    const int reps = 20;
    CK(hipEventRecord(a, s));
    for (int i = 0; i < reps; ++i) launch_flash_attn(fa, nb, s);
    CK(hipEventRecord(b, s));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    const double us = ms * 1e3 / reps, tf = 4.0 * nb * 20 * 1500.0 * 1500.0 * 64 / (us * 1e-6) / 1e12;
    printf("%-20s       nb=%d T=1500 H=20      %9.1f us  %7.1f TFLOP/s\n", "flash attention", nb, us, tf);
  }
  return 0;
}
