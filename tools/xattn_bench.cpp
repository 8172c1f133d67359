// Decode-step cross-attention microbenchmark (large-v3: 32 layers, 20 heads, 1500 keys): R rows,
// each with its OWN cross-K/V slot (the multi-chain batched step), one launch per layer as the
// step issues them; per-launch time and GB/s of the K/V bytes, head-major slots (common.h XKV_*)
// vs the previous key-major [1500][L*2d] slots.  Slots are filled with random f16.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/xattn_bench.cpp -Lwhisper-diarize-rs_amd -lwdr
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

__global__ void k_rand(f16* p, long long n, unsigned seed) {
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    unsigned x = (unsigned)i * 2654435761u + seed;
    x ^= x >> 13;
    x *= 0x5bd1e995u;
    x ^= x >> 15;
    p[i] = (f16)(((x & 0xffff) / 65536.0f - 0.5f) * 2.0f);
  }
}

int main(int argc, char** argv) {
  const int L = 32, H = 20, d = H * 64, T = 1500;
  const int S = getenv("XB_SLOTS") ? atoi(getenv("XB_SLOTS")) : 48;
  const size_t slot = (size_t)T * L * 2 * d;
  f16* xkv;
  CK(hipMalloc(&xkv, slot * S * 2));
  hipLaunchKernelGGL(k_rand, dim3(8192), dim3(256), 0, nullptr, xkv, (long long)(slot * S), 7u);
  f16 *q, *o;
  float *po;
  float2* pml;
  CK(hipMalloc(&q, (size_t)S * d * 2));
  CK(hipMalloc(&o, (size_t)S * d * 2));
  CK(hipMalloc(&po, (size_t)64 * S * H * 64 * 4));
  CK(hipMalloc(&pml, (size_t)64 * S * H * 8));
  hipLaunchKernelGGL(k_rand, dim3(64), dim3(256), 0, nullptr, q, (long long)S * d, 3u);
  const f16** rk;
  CK(hipMalloc(&rk, S * sizeof(void*)));
  std::vector<const f16*> h(S);
  for (int r = 0; r < S; ++r) h[r] = xkv + (size_t)r * slot;
  CK(hipMemcpy(rk, h.data(), S * sizeof(void*), hipMemcpyHostToDevice));
  // the batched step's tables (launch_xattn_rows): every row its own group, leaders 0..S-1
  int *grp1, *lead1;
  CK(hipMalloc(&grp1, S * 4));
  CK(hipMalloc(&lead1, S * 4));
  {
    std::vector<int> g1(S, 1), l1(S);
    for (int r = 0; r < S; ++r) l1[r] = r;
    CK(hipMemcpy(grp1, g1.data(), S * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(lead1, l1.data(), S * 4, hipMemcpyHostToDevice));
  }
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const int rows_list[] = {1, 4, 8, 16, 32, 48};
  for (int layout = 0; layout < 1; ++layout) {
    for (int R : rows_list) {
      if (R > S) continue;
      auto run = [&](int l) {
        XAttnArgs xa{q, d, nullptr, nullptr, 64, T, R, H, 0.125f, po, pml, o, d};
        xa.row_k = rk;
        if (layout == 0) {   // head-major
          xa.hs = XKV_HS;
          xa.layer_off = xkv_k_off(l, H);
          xa.v_off = xkv_v_off(l, H) - xkv_k_off(l, H);
        } else {             // key-major [1500][L*2d]
          xa.ldkv = L * 2 * d;
          xa.hs = 64;
          xa.layer_off = (long long)l * 2 * d;
          xa.v_off = d;
        }
        if (layout == 0) {   // the batched step's path (rows_forward)
          xa.grp = grp1;
          xa.lead = lead1;
          xa.n_grp = xa.n_vgrp = R;
          xa.vgrp_max = 1;
          launch_xattn_rows(xa, nullptr);
        } else {
          launch_xattn(xa, nullptr);
        }
      };
      for (int l = 0; l < L; ++l) run(l);
      CK(hipEventRecord(a, nullptr));
      const int reps = 5;
      for (int i = 0; i < reps; ++i)
        for (int l = 0; l < L; ++l) run(l);
      CK(hipEventRecord(b, nullptr));
      CK(hipEventSynchronize(b));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, a, b));
      const double us = ms * 1e3 / (reps * L);
      const double bytes = (double)R * T * d * 2 * 2;
      printf("%s R=%2d  %8.2f us per layer (partial + combine)  %7.1f GB/s  step share %.3f ms\n",
             layout == 0 ? "head-major" : "key-major ", R, us, bytes / us / 1e3, us * L / 1e3);
    }
  }
  // beam groups: 16 segments x 5 beams (80 rows), each group's rows share its slot
  {
    const int G = 5, R = 16 * G;
    f16 *qg, *og;
    float* pog;
    float2* pmlg;
    CK(hipMalloc(&qg, (size_t)R * d * 2));
    CK(hipMalloc(&og, (size_t)R * d * 2));
    CK(hipMalloc(&pog, (size_t)24 * R * H * 64 * 4));
    CK(hipMalloc(&pmlg, (size_t)24 * R * H * 8));
    hipLaunchKernelGGL(k_rand, dim3(64), dim3(256), 0, nullptr, qg, (long long)R * d, 5u);
    const f16** rkg;
    int* grp;
    CK(hipMalloc(&rkg, R * sizeof(void*)));
    CK(hipMalloc(&grp, R * 4));
    std::vector<const f16*> hk(R);
    std::vector<int> hg(R, 0);
    for (int r = 0; r < R; ++r) hk[r] = xkv + (size_t)(r / G) * slot;
    for (int g = 0; g < 16; ++g) hg[g * G] = G;
    CK(hipMemcpy(rkg, hk.data(), R * sizeof(void*), hipMemcpyHostToDevice));
    CK(hipMemcpy(grp, hg.data(), R * 4, hipMemcpyHostToDevice));
    for (int grouped = 0; grouped < 2; ++grouped) {
      auto run = [&](int l) {
        XAttnArgs xa{qg, d, nullptr, nullptr, 64, T, R, H, 0.125f, pog, pmlg, og, d};
        xa.row_k = rkg;
        xa.hs = XKV_HS;
        xa.layer_off = xkv_k_off(l, H);
        xa.v_off = xkv_v_off(l, H) - xkv_k_off(l, H);
        if (grouped) {
          xa.grp = grp;
          xa.n_grp = 16;
        }
        launch_xattn(xa, nullptr);
      };
      for (int l = 0; l < L; ++l) run(l);
      CK(hipEventRecord(a, nullptr));
      for (int i = 0; i < 5; ++i)
        for (int l = 0; l < L; ++l) run(l);
      CK(hipEventRecord(b, nullptr));
      CK(hipEventSynchronize(b));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, a, b));
      const double us = ms * 1e3 / (5 * L);
      printf("beams %s R=%d (16 x 5)  %8.2f us per layer\n", grouped ? "grouped  " : "ungrouped", R, us);
    }
  }
  return 0;
}
