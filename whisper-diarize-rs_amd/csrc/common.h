// Shared HIP helpers for libwdr (gfx950 / CDNA4 only).
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>

#include <cstdint>
#include <cstdio>
#include <stdexcept>
#include <string>

namespace wdr {

struct HipError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

#define WDR_HIP(call)                                                                       \
  do {                                                                                      \
    hipError_t e_ = (call);                                                                 \
    if (e_ != hipSuccess)                                                                   \
      throw ::wdr::HipError(std::string("HIP error ") + hipGetErrorString(e_) + " at " +    \
                            __FILE__ + ":" + std::to_string(__LINE__) + " (" #call ")");    \
  } while (0)

#define WDR_CHECK(cond, msg)                                                                \
  do {                                                                                      \
    if (!(cond)) throw std::runtime_error(std::string(msg));                                \
  } while (0)

typedef _Float16 f16;
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// Epilogue selectors for the projection kernels (GEMM / GEMV).
enum Epi : int {
  EPI_F16 = 0,          // out16 = acc + bias
  EPI_F16_GELU = 1,     // out16 = gelu_tanh(acc + bias)
  EPI_F32_RESID = 2,    // out32 += acc + bias          (pre-LN residual stream update)
  EPI_F32 = 3,          // out32 = acc + bias
  EPI_F32_GELU_POS = 4, // out32 = gelu_tanh(acc + bias) + pos[row % pos_rows]  (conv2 + positional)
  EPI_QKV_CACHE = 5,    // cols [0,d) -> out16 (Q); [d,2d) / [2d,3d) -> K / V self-attention cache rows
  EPI_XKV = 6,          // cross K/V of all layers (N = L*2d) into head-major slots (XKV_* below):
                        // row = window*1500 + key -> slot out + window*seq_stride
  EPI_F8_GELU = 7       // fp8 GEMM only: out8 = e4m3(gelu_tanh(acc + bias)) with MX scales o_sc
                        // (the encoder fc1 -> fc2 operand, Fp8Operand layout)
};

// Cross-K/V slot layout (one per encoded 30-s window): head-major [L][2][H][1500][64] f16, so
// one head's keys (or values) of one layer are 192 KB contiguous -- a cross-attention chunk of
// 64 keys is one 8-KB run.  Layer l, head h: K at xkv_k_off(l, H) + h * XKV_HS, V at
// xkv_v_off(l, H) + h * XKV_HS, key stride 64.  GEMM column c of the N = L*2d projection is
// (layer, K|V, head, dim) = (c / 2d, c / d % 2, c / 64 % H, c % 64): its block is c / 64.
constexpr int XKV_T = 1500;
constexpr long long XKV_HS = (long long)XKV_T * 64;   // head stride (elements)
__host__ __device__ inline long long xkv_k_off(int l, int H) { return (long long)(2 * l) * H * XKV_HS; }
__host__ __device__ inline long long xkv_v_off(int l, int H) { return (long long)(2 * l + 1) * H * XKV_HS; }

__host__ __device__ inline int cdiv(int a, int b) { return (a + b - 1) / b; }

__device__ __forceinline__ float gelu_tanh(float x) {
  // ggml_gelu (tanh form): 0.5 x (1 + tanh(u)), u = sqrt(2/pi) (x + 0.044715 x^3), evaluated as
  // x * sigmoid(2u) = x / (1 + exp(-2u)) -- the same function without the cancellation of
  // 1 + tanh at large negative u, in 7 instructions (v_exp_f32 + v_rcp_f32) where tanhf takes ~30:
  // the GELU epilogue of the encoder fc1 GEMM is MFMA-shadow work (within 5e-7 absolute of the
  // tanhf form over |x| <= 12, far under the f16 rounding of the output)
  // Contraction off and the one fma explicit: every kernel's epilogue (scalar or 4-wide) then
  // evaluates the same instruction sequence, so the GEMM family stays bit-identical under GELU.
#pragma clang fp contract(off)
  const float c2 = 2.0f * 0.7978845608028654f;
  const float u2 = c2 * __builtin_fmaf(0.044715f * x, x * x, x);
  float g = x * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(u2 * -1.4426950408889634f));
  // materialised in f32: the caller's f16 conversion must not fuse with the multiply into a
  // single-rounding v_fma_mix (the compiler does so in some epilogues and not in others)
  asm("" : "+v"(g));
  return g;
}

__device__ __forceinline__ float wave_sum(float v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
// A workgroup barrier that orders LDS only: waits for this wave's LDS operations, not for its
// outstanding global loads (__syncthreads' workgroup fence waits vmcnt(0), which in a recurrence
// with prefetched inputs stalls every step on the prefetch it just issued)
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__device__ __forceinline__ double wave_sum_d(double v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Projection launchers (kernels/gemm.hip).
struct ProjArgs {
  const f16* A; int lda;            // activations [M][K] f16
  const f16* B; int ldb;            // weights     [N][K] f16 (nn.Linear / ggml layout)
  const float* bias;                // [N] or null
  void* out; int ldo;               // f16 or f32 [M][N]
  const float* pos; int pos_rows;   // EPI_F32_GELU_POS only
  int M, N, K;
  int epi;
  // fused LayerNorm prologue (decoder rows, k_skinny): A is ignored, rows come from the f32
  // residual stream ln_x [M][ldln] normalised with (ln_g, ln_b) -- ggml_norm eps 1e-5.
  const float* ln_x = nullptr; int ldln = 0; const float* ln_g = nullptr; const float* ln_b = nullptr;
  // EPI_QKV_CACHE
  f16* kc = nullptr; f16* vc = nullptr; long long seq_stride = 0; const int* row_seq = nullptr;
  const int* row_pos = nullptr; int d = 0;
  unsigned long long* ts = nullptr;   // live kernel clock of a sampled launch (ProfClock)
  // fp8 (OCP e4m3) MX operands (launch_proj_fp8): A8 [M][lda] and B8 [N][ldb] bytes, each row
  // with one E8M0 scale per 32 k, as u32 words [K/128][ld_*sc] (byte b of word (t, r): k = 128 t
  // + 32 b .. +32 of row r; ld_asc >= M rounded up to 256) applied inside the MFMA; EPI_F8_GELU
  // writes out [M][ldo] bytes and the scales o_sc [N/128][ld_osc]
  const uint8_t* A8 = nullptr; const uint8_t* B8 = nullptr;
  const uint32_t* a_sc = nullptr; const uint32_t* b_sc = nullptr; int ld_asc = 0, ld_bsc = 0;
  uint32_t* o_sc = nullptr; int ld_osc = 0;
  // k_gemm4 tile order: groups of tile_gm row tiles walked column by column (0: row-major)
  int tile_gm = 0;
  // M > 64: the register-staged reference tile k_gemm whatever the dispatch rule picks
  // (wdr_dbg_proj WDR_DBG_PROJ_GEMM1: the bit-identity tests of the tiled GEMM family)
  int gemm_ref = 0;
  // decoder rows of any count (steps, prompt prefills, DTW re-forwards) on the row kernel
  // (k_skinny's arithmetic: 8 or 16 waves split K, fixed k order, fixed wave order in the
  // reduce), so a row's result never depends on how many rows share the launch (the LN
  // prologue normalises each workgroup's own row tiles)
  int rows_mma = 0;
  // optional row map: A / ln_x row m is row_map[m] (logit rows gathered from the residual stream)
  const int* row_map = nullptr;
};

// Live kernel clock (csrc/prof.cpp): a launch the profiler samples carries ts -> {earliest wave
// start, latest wave end} in wall_clock64() ticks (the constant-rate clock), i.e. the span
// rocprofv3's dispatch timestamps measure, free of the queueing that HIP start/stop events of a
// launch absorb under multi-stream concurrency.  Thread 0 of every workgroup stamps the start
// when its wave (the first dispatched) starts, and lane 0 of the workgroup's LAST wave stamps the
// end when that wave retires -- the wave that finishes last in the multi-wave kernels (k_gemm4 /
// k_gemm5 run waves 4-7 one barrier behind waves 0-3; the k_skinny / flash / cross-attention
// waves end together after their final barrier), so the span is the workgroup's, not wave 0's
//  -- two vector atomics per workgroup,
// spread over PROF_CLK_LANES words (one stamp per wave, on 32 words, serialised at L2 on the
// 11 520-workgroup cross-attention launches and inflated their spans ~3x against the trace);
// unsampled launches (ts null) skip it.
constexpr int PROF_CLK_LANES = 128;   // stamp addresses per sampled launch (csrc/prof.cpp ring)
struct ProfClock {
  unsigned long long* ts;
  __device__ __forceinline__ explicit ProfClock(unsigned long long* t) : ts(t) {
    if (ts && threadIdx.x == 0) atomicMin(ts + lane_of_block(), (unsigned long long)wall_clock64());
  }
  __device__ __forceinline__ ~ProfClock() {
    if (ts && threadIdx.x == ((blockDim.x - 1) & ~63u)) atomicMax(ts + PROF_CLK_LANES + lane_of_block(), (unsigned long long)wall_clock64());
  }
  __device__ __forceinline__ static int lane_of_block() {
    return (int)((blockIdx.x + blockIdx.y * 7u + blockIdx.z * 13u) % PROF_CLK_LANES);
  }
};
unsigned long long* prof_slot();   // next clock slot of the sampled-launch ring (null when full)
template <typename A>
inline unsigned long long* prof_attach(A&) { return nullptr; }
inline unsigned long long* prof_attach(ProjArgs& a) { return a.ts = prof_slot(); }
// M <= 64 (or rows_mma) on the row kernel k_skinny, larger M on the MFMA GEMM tiles
void launch_proj(const ProjArgs& a, hipStream_t s);
// re-read the encoder GEMM dispatch knobs (WDR_GEMM*), which launch_proj reads once per process:
// tools/gemm_bench's per-variant A/B only
void gemm_knobs_reload();
// fp8 MX encoder GEMM (BASELINE configs[4], k_gemm8): ProjArgs::A8 / B8 / a_sc / b_sc, M > 64,
// N % 256 == 0, K % 128 == 0; epilogues as launch_proj plus EPI_F8_GELU
void launch_proj_fp8(const ProjArgs& a, hipStream_t s);
// f16 rows -> e4m3 + one E8M0 scale per 32 k (the smallest power of two that maps the block's
// max |x| to <= 448), scale words [K/128][ld_sc]
void launch_quant_f8(const f16* x, int ldx, int rows, int K, uint8_t* y, int ldy, uint32_t* sc, int ld_sc,
                     hipStream_t s);
// one scaled MFMA on raw per-lane operands (a / b [64][32] bytes, sa / sb [64], out [64][4])
void launch_probe_mfma_scale(const void* a, const void* b, const int* sa, const int* sb, float* out, hipStream_t s);
// LayerNorm (k_layernorm's arithmetic) written as e4m3 + MX scales
void launch_layernorm_f8(const float* x, int ldx, const float* g, const float* b, uint8_t* y, int ldy, uint32_t* sc,
                         int ld_sc, int rows, int d, hipStream_t s);

}  // namespace wdr
