// Projection kernels: the dense contractions of the Whisper encoder / decoder
// (SURVEY.md §8(a) a5-a7, a9, a12).
//
//  * k_gemm  — MFMA GEMM for M > 64 rows (encoder windows, cross-K/V; the general fallback
//              of the tiled family k_gemm2..5):  C[M][N] = A[M][K] . B[N][K]^T  (+ fused epilogue).
//              f16 operands (what ggml's mul_mat feeds: f16 weights, activations cast to
//              f16), f32 accumulation, v_mfma_f32_32x32x16_f16.  128x128x32 block tile,
//              4 waves of 64x64, register-staged double-buffered LDS, row padding for
//              conflict-free ds_read_b128.  Roofline: MFMA (2.5 PF/s dense f16).
//  * k_skinny — the decoder row kernel (any row count; decode steps, prompt prefills, DTW
//              re-forwards, language detection) and every other projection of <= 64 rows:
//              16-row MFMA tiles, K split over 8 or 16 waves in a fixed order (optionally a
//              fused LayerNorm prologue), so a row's result does not depend on the launch's
//              other rows.  Roofline: HBM (N*K*2 per launch).
#include "../common.h"
#include "../prof.h"

#include <algorithm>
#include <cstdlib>

namespace wdr {

typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));

constexpr int GB_M = 128, GB_N = 128, GB_K = 32;
constexpr int GLDS = GB_K + 8;   // LDS row stride in halfs (80 B): conflict-free b128 fragment reads

template <int EPI>
__device__ __forceinline__ void epi_store(const ProjArgs& a, int row, int col, float v) {
  if (row >= a.M || col >= a.N) return;
  if (a.bias) v += a.bias[col];
  if constexpr (EPI == EPI_F16) {
    ((f16*)a.out)[(size_t)row * a.ldo + col] = (f16)v;
  } else if constexpr (EPI == EPI_F16_GELU) {
    ((f16*)a.out)[(size_t)row * a.ldo + col] = (f16)gelu_tanh(v);
  } else if constexpr (EPI == EPI_F32_RESID) {
    float* o = (float*)a.out + (size_t)row * a.ldo + col;
    *o = *o + v;
  } else if constexpr (EPI == EPI_F32) {
    ((float*)a.out)[(size_t)row * a.ldo + col] = v;
  } else if constexpr (EPI == EPI_F32_GELU_POS) {
    ((float*)a.out)[(size_t)row * a.ldo + col] =
        gelu_tanh(v) + a.pos[(size_t)(row % a.pos_rows) * a.N + col];
  } else if constexpr (EPI == EPI_XKV) {
    const int w = row / XKV_T, t = row - w * XKV_T;
    ((f16*)a.out)[w * a.seq_stride + (long long)(col >> 6) * XKV_HS + t * 64 + (col & 63)] = (f16)v;
  } else {  // EPI_QKV_CACHE
    if (col < a.d) {
      ((f16*)a.out)[(size_t)row * a.ldo + col] = (f16)v;
    } else {
      const long long dst = a.row_seq[row] * a.seq_stride + (long long)a.row_pos[row] * a.d;
      if (col < 2 * a.d) a.kc[dst + col - a.d] = (f16)v;
      else a.vc[dst + col - 2 * a.d] = (f16)v;
    }
  }
}

// Four consecutive columns col..col+3 of one row (col % 4 == 0; N, ldo, d, pos and bias rows
// multiples of 4 elements): the epilogue of the transposed-accumulator tiles (k_gemm4 / k_gemm5),
// one 8-B (f16) or 16-B (f32) access per lane where epi_store makes four scalar ones; per element
// the same arithmetic as epi_store, so the same bits.
template <int EPI>
__device__ __forceinline__ void epi_store4(const ProjArgs& a, int row, int col, f32x4 v, bool has_bias, f32x4 bias) {
  if (row >= a.M) return;
  if (has_bias) v += bias;
  if constexpr (EPI == EPI_F16 || EPI == EPI_F16_GELU) {
    f16x4 h;
#pragma unroll
    for (int r = 0; r < 4; ++r) h[r] = (f16)(EPI == EPI_F16_GELU ? gelu_tanh(v[r]) : v[r]);
    *(f16x4*)((f16*)a.out + (size_t)row * a.ldo + col) = h;
  } else if constexpr (EPI == EPI_F32_RESID) {
    f32x4* o = (f32x4*)((float*)a.out + (size_t)row * a.ldo + col);
    *o = *o + v;
  } else if constexpr (EPI == EPI_F32) {
    *(f32x4*)((float*)a.out + (size_t)row * a.ldo + col) = v;
  } else if constexpr (EPI == EPI_F32_GELU_POS) {
    const f32x4 p = *(const f32x4*)(a.pos + (size_t)(row % a.pos_rows) * a.N + col);
    f32x4 g;
#pragma unroll
    for (int r = 0; r < 4; ++r) g[r] = gelu_tanh(v[r]) + p[r];
    *(f32x4*)((float*)a.out + (size_t)row * a.ldo + col) = g;
  } else {
    f16x4 h;
#pragma unroll
    for (int r = 0; r < 4; ++r) h[r] = (f16)v[r];
    if constexpr (EPI == EPI_XKV) {
      const int w = row / XKV_T, t = row - w * XKV_T;
      *(f16x4*)((f16*)a.out + w * a.seq_stride + (long long)(col >> 6) * XKV_HS + t * 64 + (col & 63)) = h;
    } else {  // EPI_QKV_CACHE: d % 4 == 0, so the four columns lie in one of Q / K / V
      if (col < a.d) {
        *(f16x4*)((f16*)a.out + (size_t)row * a.ldo + col) = h;
      } else {
        const long long dst = a.row_seq[row] * a.seq_stride + (long long)a.row_pos[row] * a.d;
        if (col < 2 * a.d) *(f16x4*)(a.kc + dst + col - a.d) = h;
        else *(f16x4*)(a.vc + dst + col - 2 * a.d) = h;
      }
    }
  }
}

template <int EPI>
__global__ __launch_bounds__(256, 2) void k_gemm(ProjArgs a) {
  ProfClock prof_clock_(a.ts);   // sampled launches only (csrc/prof.cpp)
  __shared__ __attribute__((aligned(16))) f16 sA[2][GB_M * GLDS];
  __shared__ __attribute__((aligned(16))) f16 sB[2][GB_N * GLDS];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int bn = blockIdx.x, bm = blockIdx.y;
  const int wr = wid >> 1, wc = wid & 1;

  // staging: 512 16-B chunks per operand tile, 2 per thread
  int a_off[2], b_off[2], s_off[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int c = tid + 256 * i;
    const int r = c >> 2, kc = (c & 3) * 8;
    int gm = bm * GB_M + r;
    gm = gm < a.M ? gm : a.M - 1;
    const int gn = bn * GB_N + r;   // N % 128 == 0 (host-checked)
    a_off[i] = gm * a.lda + kc;
    b_off[i] = gn * a.ldb + kc;
    s_off[i] = r * GLDS + kc;
  }
  const int nk = a.K / GB_K;
  f16x8 ra[2], rb[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    ra[i] = *(const f16x8*)(a.A + a_off[i]);
    rb[i] = *(const f16x8*)(a.B + b_off[i]);
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    *(f16x8*)(&sA[0][s_off[i]]) = ra[i];
    *(f16x8*)(&sB[0][s_off[i]]) = rb[i];
  }
  __syncthreads();

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int fr = lane & 31, fk = 8 * (lane >> 5);
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const bool more = kt + 1 < nk;
    if (more) {
      const int ko = (kt + 1) * GB_K;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        ra[i] = *(const f16x8*)(a.A + a_off[i] + ko);
        rb[i] = *(const f16x8*)(a.B + b_off[i] + ko);
      }
    }
    const f16* As = sA[cur];
    const f16* Bs = sB[cur];
#pragma unroll
    for (int ks = 0; ks < GB_K / 16; ++ks) {
      f16x8 af[2], bf[2];
#pragma unroll
      for (int i = 0; i < 2; ++i)
        af[i] = *(const f16x8*)(As + (wr * 64 + i * 32 + fr) * GLDS + ks * 16 + fk);
#pragma unroll
      for (int j = 0; j < 2; ++j)
        bf[j] = *(const f16x8*)(Bs + (wc * 64 + j * 32 + fr) * GLDS + ks * 16 + fk);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[i], bf[j], acc[i][j], 0, 0, 0);
    }
    if (more) {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        *(f16x8*)(&sA[cur ^ 1][s_off[i]]) = ra[i];
        *(f16x8*)(&sB[cur ^ 1][s_off[i]]) = rb[i];
      }
    }
    __syncthreads();
  }

  const int h = lane >> 5;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = bm * GB_M + wr * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        const int col = bn * GB_N + wc * 64 + j * 32 + fr;
        epi_store<EPI>(a, row, col, acc[i][j][r]);
      }
}


// ---------------------------------------------------------------- MFMA GEMM, LDS-DMA staged
// The encoder / cross-K/V GEMM (M > 64): 128x128 block tile, BK = 64, 4 waves of 64x64
// (2x2 v_mfma_f32_32x32x16_f16 per 16-deep k-step, the same k order as k_gemm), operand tiles
// staged global -> LDS by global_load_lds (16 B per lane, no VGPR round trip) into two buffers:
// the loads of tile k+1 fly while tile k is multiplied.  LDS images are lane-linear (what the
// DMA writes: 1 KB per wave-instruction = 8 rows x 128 B); bank conflicts of the fragment reads
// are removed by an XOR swizzle applied on the global SOURCE address: logical 16-B chunk c of
// row r sits at chunk c ^ ((r >> 1) & 7).  Workgroups are remapped so that each XCD owns a
// contiguous run of tiles (row-major over N tiles): the A rows and B columns a tile reuses stay
// in that XCD's L2.
constexpr int G2_BK = 64;
__device__ __forceinline__ int g2_swz(int r, int c) { return c ^ ((r >> 1) & 7); }

template <int EPI>
__global__ __launch_bounds__(256, 2) void k_gemm2(ProjArgs a) {
  ProfClock prof_clock_(a.ts);   // sampled launches only (csrc/prof.cpp)
  __shared__ __attribute__((aligned(16))) f16 lds[2][2][GB_M * G2_BK];   // [buf][A,B][128 x 64]
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  // XCD-aware tile order (bijective for any tile count)
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int q = nwg / 8, rr = nwg % 8, xcd = orig % 8;
  const int id = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + orig / 8;
  const int ntn = a.N / GB_N;
  const int bm = id / ntn, bn = id % ntn;
  const int wr = wid >> 1, wc = wid & 1;
  // this wave's 4 DMA blocks per operand: block j = wid*4 + jj covers rows 8*j .. 8*j + 7
  const f16* ga[4];
  const f16* gb[4];
#pragma unroll
  for (int jj = 0; jj < 4; ++jj) {
    const int row = (wid * 4 + jj) * 8 + (lane >> 3);
    const int c = g2_swz(row, lane & 7);
    int gm = bm * GB_M + row;
    gm = gm < a.M ? gm : a.M - 1;
    ga[jj] = a.A + (size_t)gm * a.lda + c * 8;
    gb[jj] = a.B + (size_t)(bn * GB_N + row) * a.ldb + c * 8;
  }
  auto stage = [&](int buf, int k0) {
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      __builtin_amdgcn_global_load_lds((const void*)(ga[jj] + k0), (void*)&lds[buf][0][(wid * 4 + jj) * 512], 16, 0, 0);
      __builtin_amdgcn_global_load_lds((const void*)(gb[jj] + k0), (void*)&lds[buf][1][(wid * 4 + jj) * 512], 16, 0, 0);
    }
  };
  const int nk = a.K / G2_BK;
  stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int fr = lane & 31, fh = lane >> 5;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) stage(cur ^ 1, (kt + 1) * G2_BK);
    const f16* As = lds[cur][0];
    const f16* Bs = lds[cur][1];
#pragma unroll
    for (int ks = 0; ks < G2_BK / 16; ++ks) {
      const int c = 2 * ks + fh;   // logical 16-B chunk of this lane's 8 k values
      f16x8 af[2], bf[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int r = wr * 64 + i * 32 + fr;
        af[i] = *(const f16x8*)(As + r * G2_BK + g2_swz(r, c) * 8);
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int r = wc * 64 + j * 32 + fr;
        bf[j] = *(const f16x8*)(Bs + r * G2_BK + g2_swz(r, c) * 8);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(bf[j], af[i], acc[i][j], 0, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // transposed accumulators (B fragment first): element 4g..4g+3 of a 32 x 32 tile is row fr,
  // columns 8g + 4h .. +3 -- four consecutive columns, one vector access (epi_store4)
  const int h = lane >> 5;
  const bool hb = a.bias != nullptr;
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int col = bn * GB_N + wc * 64 + j * 32 + 8 * g + 4 * h;
      const f32x4 bz = hb ? *(const f32x4*)(a.bias + col) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const f32x4 v = {acc[i][j][4 * g], acc[i][j][4 * g + 1], acc[i][j][4 * g + 2], acc[i][j][4 * g + 3]};
        epi_store4<EPI>(a, bm * GB_M + wr * 64 + i * 32 + fr, col, v, hb, bz);
      }
    }
}


// ---------------------------------------------------------------- MFMA GEMM, 256 x 256 tile
// The big encoder GEMMs (M = windows x 1500 > 2048, N % 256 == 0): 256 x 256 block tile, BK 64,
// 8 waves (2 along M x 4 along N) of 128 x 64 outputs, v_mfma_f32_16x16x32_f16 (8 x 4
// accumulator tiles per wave: 128 acc registers), one workgroup per CU.  Operand tiles are
// staged by global_load_lds into two LDS buffers (2 x (32 + 32) KB = 128 KB, one dynamic LDS
// array); lane-linear images (8 rows x 128 B per wave-instruction) with the g2_swz XOR applied to
// the global source address, so the 16-row fragment reads (ds_read_b128) are conflict-free.
// The loads of tile k+1 are issued before tile k's MFMAs and retired once per K-tile by a
// counted wait + a raw s_barrier (no __syncthreads fence that would drain them early).
// Twice the output per staged byte of k_gemm2 (128 x 128) and 4x the MFMAs per barrier.
constexpr int G3_M = 256, G3_N = 256, G3_BK = 64;
constexpr uint32_t G3_LDS = 2u * 2u * G3_M * G3_BK * 2u;   // bytes

template <int EPI>
__global__ __launch_bounds__(512, 1) void k_gemm3(ProjArgs a) {
  ProfClock prof_clock_(a.ts);   // sampled launches only (csrc/prof.cpp)
  extern __shared__ __attribute__((aligned(16))) f16 lds3[];   // [buf][A, B][256 x 64]
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int q = nwg / 8, rr = nwg % 8, xcd = orig % 8;
  const int id = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + orig / 8;
  const int ntn = a.N / G3_N;
  const int bm = id / ntn, bn = id % ntn;
  const int wm = wid >> 2, wn = wid & 3;
  // DMA blocks of this wave: block j = wid * 4 + jj holds rows 8 j .. 8 j + 7 of each operand
  const f16* ga[4];
  const f16* gb[4];
#pragma unroll
  for (int jj = 0; jj < 4; ++jj) {
    const int row = (wid * 4 + jj) * 8 + (lane >> 3);
    const int c = g2_swz(row, lane & 7);
    int gm = bm * G3_M + row;
    gm = gm < a.M ? gm : a.M - 1;
    ga[jj] = a.A + (size_t)gm * a.lda + c * 8;
    gb[jj] = a.B + (size_t)(bn * G3_N + row) * a.ldb + c * 8;
  }
  constexpr int OP = G3_M * G3_BK;   // halfs per operand image
  auto stage = [&](int buf, int k0) {
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      __builtin_amdgcn_global_load_lds((const void*)(ga[jj] + k0), (void*)(lds3 + (buf * 2 + 0) * OP + (wid * 4 + jj) * 512),
                                       16, 0, 0);
      __builtin_amdgcn_global_load_lds((const void*)(gb[jj] + k0), (void*)(lds3 + (buf * 2 + 1) * OP + (wid * 4 + jj) * 512),
                                       16, 0, 0);
    }
  };
  const int nk = a.K / G3_BK;
  stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fq = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) stage(cur ^ 1, (kt + 1) * G3_BK);
    const f16* As = lds3 + (cur * 2 + 0) * OP;
    const f16* Bs = lds3 + (cur * 2 + 1) * OP;
#pragma unroll
    for (int ks = 0; ks < G3_BK / 32; ++ks) {
      const int c = ks * 4 + fq;   // logical 16-B chunk: k = 8 fq .. 8 fq + 7 of this 32-deep step
      f16x8 bf[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int r = wn * 64 + j * 16 + fr;
        bf[j] = *(const f16x8*)(Bs + r * G3_BK + g2_swz(r, c) * 8);
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int r = wm * 128 + i * 16 + fr;
        const f16x8 af = *(const f16x8*)(As + r * G3_BK + g2_swz(r, c) * 8);
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af, bf[j], acc[i][j], 0, 0, 0);
      }
    }
    // own loads of tile k+1 landed and own reads of tile k retired; the barrier then publishes
    // every wave's loads and frees buffer `cur` for the next stage
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }

#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = bm * G3_M + wm * 128 + i * 16 + fq * 4 + r;
        const int col = bn * G3_N + wn * 64 + j * 16 + fr;
        epi_store<EPI>(a, row, col, acc[i][j][r]);
      }
}


// ---------------------------------------------------------------- MFMA GEMM, 256 x 256 ping-pong
// k_gemm3's tile and wave layout (8 waves: 2 along M x 4 along N, 128 x 64 outputs each,
// v_mfma_f32_16x16x32_f16, the same k order, so bit-identical to k_gemm) in a phased schedule:
//  * a K-tile (BK 64) is four phases, one output quadrant each -- Q(a, b) = the wave's rows
//    64a..64a+63 x columns 32b..32b+31, 16 MFMAs over the tile's 64 k -- in the order Q00, Q01,
//    Q11, Q10, so a phase reads 12, 4, 8 or 4 fragments (A kept from Q00 to Q01, B1 from Q01 to
//    Q11; B0 re-read for Q10);
//  * a phase is {LDS fragment reads + one half-tile of LDS-DMA staging} barrier {16 MFMAs}
//    barrier, and waves 4-7 run one barrier behind waves 0-3: the two waves of every SIMD
//    alternate, one multiplying while the other reads and stages (a ping-pong on the matrix pipe);
//  * the LDS tile of each operand is cut into the halves the quadrants read -- AH[a] = rows
//    64a..64a+63 of both wave groups, BH[b] = columns 32b..32b+31 of every wave -- so a half is
//    restaged one phase after its last read: BH0 of tile t+1 in phase 1 of tile t, AH0 / BH1 /
//    AH1 of tile t+2 in phases 2 / 3 / 4 (two LDS buffers, two tiles in flight);
//  * one counted wait per tile (vmcnt(6): the three half-tiles staged after BH0 of tile t+1 stay
//    in flight across the barriers), raw s_barrier, all LDS in one dynamic array.
// Image: 128 rows x 128 B per half, lane-linear LDS-DMA pieces of 8 rows, g2_swz on the source.
constexpr int G4_HALF = 128 * 64;                   // halfs per half-tile image
constexpr uint32_t G4_LDS = 2u * 4u * G4_HALF * 2u;   // 2 buffers x {AH0, AH1, BH0, BH1}: 128 KB

template <int EPI>
__device__ __forceinline__ void gemm4_tile(const ProjArgs& a, f16* lds4, int orig, int nwg) {
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int q = nwg / 8, rr = nwg % 8, xcd = orig % 8;
  const int id = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + orig / 8;
  const int ntn = a.N / G3_N;
  int bm = id / ntn, bn = id % ntn;
  if (a.tile_gm > 1) {
    // grouped order: consecutive ids (one XCD's concurrent workgroups) cover tile_gm row tiles
    // x a few column tiles, so the K-slices they stage are shared through that XCD's L2
    const int ntm = cdiv(a.M, G3_M), gsz = a.tile_gm * ntn, g = id / gsz, m0 = g * a.tile_gm;
    const int gm = min(a.tile_gm, ntm - m0), l = id - g * gsz;
    bm = m0 + l % gm;
    bn = l / gm;
  }
  const int grp = wid >> 2, wn = wid & 3;
  // staging: wave w writes pieces 2w, 2w+1 (8 image rows each) of every half-tile
  //   AH[h] image row q -> A row bm*256 + (q >> 6)*128 + 64h + (q & 63)
  //   BH[h] image row q -> B row bn*256 + (q >> 5)*64 + 32h + (q & 31)
  // as buffer-resource DMA (buffer_load_dwordx4 ... lds): the piece's row base and k0 a
  // wave-uniform scalar offset, one loop-invariant 32-bit lane offset per piece jj (row lane/8,
  // g2_swz chunk (lane & 7) ^ ((4 jj + lane/16) & 7) -- wid drops out of the swizzle).  No VGPR an
  // LDS DMA reads is ever rewritten: hipcc treats those operands like store data and waits
  // vmcnt(0) before redefining one, which with per-K-tile 64-bit addresses put a full drain of
  // the two tiles in flight at the head of every K-tile (round 4's k_gemm4 carried it).  Rows
  // past M read zeros (the descriptor's bounds) and are never stored.
  // A: the descriptor starts at the tile's first row and ends at row M (rows past it read zeros:
  // the buffer range check covers the VGPR offset, which carries the row), k0 in the scalar offset
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(a.A + (size_t)bm * G3_M * a.lda), (short)0, max(0, a.M - bm * G3_M) * a.lda * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc((void*)a.B, (short)0, a.N * a.ldb * 2, 0x00020000);
  uint32_t offa[2][2], offb[2];   // offa[half][jj]: the row inside the tile and the chunk
#pragma unroll
  for (int jj = 0; jj < 2; ++jj) {
    const uint32_t ca = (lane & 7) ^ ((4 * jj + (lane >> 4)) & 7);
    const int p = 2 * wid + jj;
#pragma unroll
    for (int h = 0; h < 2; ++h)
      offa[h][jj] = (uint32_t)((p >> 3) * 128 + 64 * h + (p & 7) * 8 + (lane >> 3)) * (uint32_t)a.lda * 2u + ca * 16u;
    offb[jj] = (uint32_t)(lane >> 3) * (uint32_t)a.ldb * 2u + ca * 16u;
  }
  typedef __attribute__((address_space(3))) void* lds_ptr;
  auto stage = [&](int buf, int half, int k0) {   // half: 0 AH0, 1 AH1, 2 BH0, 3 BH1
    f16* dst = lds4 + (buf * 4 + half) * G4_HALF + (2 * wid) * 512;
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
      const int p = 2 * wid + jj;
      if (half < 2) {
        __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (lds_ptr)(dst + jj * 512), 16, offa[half][jj], k0 * 2, 0, 0);
      } else {
        const int row = bn * G3_N + (p >> 2) * 64 + 32 * (half - 2) + (p & 3) * 8;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, (lds_ptr)(dst + jj * 512), 16, offb[jj], (row * a.ldb + k0) * 2, 0, 0);
      }
    }
  };
  const int nk = a.K / G3_BK;
  // prologue: tile 0 and the halves of tile 1 staged ahead of the loop (AH0, BH1, AH1)
  stage(0, 0, 0);
  stage(0, 2, 0);
  stage(0, 3, 0);
  stage(0, 1, 0);
  if (nk > 1) {
    stage(1, 0, G3_BK);
    stage(1, 3, G3_BK);
    stage(1, 1, G3_BK);
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  if (grp == 1) __builtin_amdgcn_s_barrier();   // waves 4-7 run one barrier behind
  __builtin_amdgcn_sched_barrier(0);

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fq = lane >> 4;
  f16x8 af[2][4], bf[2][2];   // [ks][row tile], [ks][column tile] of the current quadrant
  auto read_a = [&](const f16* img) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = grp * 64 + i * 16 + fr;
        af[ks][i] = *(const f16x8*)(img + r * 64 + g2_swz(r, ks * 4 + fq) * 8);
      }
  };
  auto read_b = [&](const f16* img) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int r = wn * 32 + j * 16 + fr;
        bf[ks][j] = *(const f16x8*)(img + r * 64 + g2_swz(r, ks * 4 + fq) * 8);
      }
  };
  auto mfma_q = [&](int qa, int qb) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[qa * 4 + i][qb * 2 + j] =
              __builtin_amdgcn_mfma_f32_16x16x32_f16(bf[ks][j], af[ks][i], acc[qa * 4 + i][qb * 2 + j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  // end of a load section: fragments in registers, then the barrier into the MFMA section
  auto sync_in = [&]() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  auto sync_out = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };

  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const f16* img = lds4 + cur * 4 * G4_HALF;
    const bool n1 = kt + 1 < nk, n2 = kt + 2 < nk;
    // phase 1: Q00 -- read AH0 + BH0; stage BH0 of tile kt+1
    read_b(img + 2 * G4_HALF);
    read_a(img);
    if (n1) stage(cur ^ 1, 2, (kt + 1) * G3_BK);
    sync_in();
    mfma_q(0, 0);
    sync_out();
    // phase 2: Q01 -- read BH1; stage AH0 of tile kt+2
    read_b(img + 3 * G4_HALF);
    if (n2) stage(cur, 0, (kt + 2) * G3_BK);
    sync_in();
    mfma_q(0, 1);
    sync_out();
    // phase 3: Q11 -- read AH1; stage BH1 of tile kt+2
    read_a(img + G4_HALF);
    if (n2) stage(cur, 3, (kt + 2) * G3_BK);
    sync_in();
    mfma_q(1, 1);
    sync_out();
    // phase 4: Q10 -- read BH0; stage AH1 of tile kt+2; retire everything up to BH0 of tile kt+1
    read_b(img + 2 * G4_HALF);
    if (n2) {
      stage(cur, 1, (kt + 2) * G3_BK);
      asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    sync_in();
    mfma_q(1, 0);
    sync_out();
  }
  if (grp == 0) __builtin_amdgcn_s_barrier();   // matches the stagger barrier of waves 4-7

  // transposed accumulators (B fragment first): lane (fr, fq) holds row fr, columns fq*4..+3 of
  // every 16 x 16 tile -- four consecutive columns, one vector access
  const bool hb = a.bias != nullptr;
  f32x4 bz[4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
    bz[j] = hb ? *(const f32x4*)(a.bias + bn * G3_N + wn * 64 + j * 16 + fq * 4) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
      epi_store4<EPI>(a, bm * G3_M + grp * 128 + i * 16 + fr, bn * G3_N + wn * 64 + j * 16 + fq * 4, acc[i][j], hb, bz[j]);
}

// Persistent form: gridDim.x workgroups (a multiple of 8, <= the tile count) walk the tiles
// blockIdx.x, blockIdx.x + gridDim.x, ... -- every tile of a workgroup keeps its XCD, so the
// XCD-grouped order holds.  Fewer workgroups than CUs leave CUs to the decode-step kernels that
// run beside the encoder (WDR_GEMM_CUS).
template <int EPI>
__global__ __launch_bounds__(512, 1) void k_gemm4(ProjArgs a) {
  ProfClock prof_clock_(a.ts);   // sampled launches only (csrc/prof.cpp)
  extern __shared__ __attribute__((aligned(16))) f16 lds4[];   // [buf][AH0, AH1, BH0, BH1][128 x 64]
  const int ntiles = (a.N / G3_N) * cdiv(a.M, G3_M);
  for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
    gemm4_tile<EPI>(a, lds4, t, ntiles);
    __builtin_amdgcn_s_barrier();   // every wave's last LDS reads done before the next prologue
  }
}


// ---------------------------------------------------------------- MFMA GEMM, 256 x 128 ping-pong
// k_gemm4's schedule on a 256 x 128 tile for the narrow encoder projections (o, fc2: N = d =
// 1280), which fill only 120 of 256 CUs with 256 x 256 tiles at M = 6000 (240 with these).
// 8 waves, 2 along M x 4 along N, 128 x 32 outputs each; a K-tile (BK 64) is two phases, one per
// 64-row half of the wave's rows (16 MFMAs each: 4 row x 2 column tiles x 2 k-steps); the B
// fragments are read in phase 1 and kept for phase 2.  LDS per buffer: AH0 / AH1 (the two row
// halves of both wave groups) and BT (the 128 B rows), 16 KB each, two buffers (96 KB); a half is
// restaged one phase after its last read -- AH1 of tile t+1 in phase 1 of tile t, AH0 and BT of
// tile t+2 in phase 2 -- and every phase ends its load section with a counted wait (vmcnt(6):
// three half-tiles in flight across the barriers).  Same k order as k_gemm: bit-identical.
constexpr uint32_t G5_LDS = 2u * 3u * G4_HALF * 2u;   // 96 KB

template <int EPI>
__device__ __forceinline__ void gemm5_tile(const ProjArgs& a, f16* lds5, int orig, int nwg) {
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int q = nwg / 8, rr = nwg % 8, xcd = orig % 8;
  const int id = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + orig / 8;
  const int ntn = a.N / 128;
  int bm = id / ntn, bn = id % ntn;
  if (a.tile_gm > 1) {
    const int ntm = cdiv(a.M, G3_M), gsz = a.tile_gm * ntn, g = id / gsz, m0 = g * a.tile_gm;
    const int gm = min(a.tile_gm, ntm - m0), l = id - g * gsz;
    bm = m0 + l % gm;
    bn = l / gm;
  }
  const int grp = wid >> 2, wn = wid & 3;
  // staging: wave w writes pieces 2w, 2w+1 (8 image rows each) of every half
  //   AH[h] image row q -> A row bm*256 + (q >> 6)*128 + 64h + (q & 63);  BT row q -> B row bn*128 + q
  // buffer-resource DMA with loop-invariant lane offsets, as k_gemm4
  // A: the descriptor starts at the tile's first row and ends at row M (rows past it read zeros:
  // the buffer range check covers the VGPR offset, which carries the row), k0 in the scalar offset
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(a.A + (size_t)bm * G3_M * a.lda), (short)0, max(0, a.M - bm * G3_M) * a.lda * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc((void*)a.B, (short)0, a.N * a.ldb * 2, 0x00020000);
  uint32_t offa[2][2], offb[2];   // offa[half][jj]: the row inside the tile and the chunk
#pragma unroll
  for (int jj = 0; jj < 2; ++jj) {
    const uint32_t ca = (lane & 7) ^ ((4 * jj + (lane >> 4)) & 7);
    const int p = 2 * wid + jj;
#pragma unroll
    for (int h = 0; h < 2; ++h)
      offa[h][jj] = (uint32_t)((p >> 3) * 128 + 64 * h + (p & 7) * 8 + (lane >> 3)) * (uint32_t)a.lda * 2u + ca * 16u;
    offb[jj] = (uint32_t)(lane >> 3) * (uint32_t)a.ldb * 2u + ca * 16u;
  }
  typedef __attribute__((address_space(3))) void* lds_ptr;
  auto stage = [&](int buf, int half, int k0) {   // half: 0 AH0, 1 AH1, 2 BT
    f16* dst = lds5 + (buf * 3 + half) * G4_HALF + (2 * wid) * 512;
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
      const int p = 2 * wid + jj;
      if (half < 2) {
        __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (lds_ptr)(dst + jj * 512), 16, offa[half][jj], k0 * 2, 0, 0);
      } else {
        const int row = bn * 128 + p * 8;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, (lds_ptr)(dst + jj * 512), 16, offb[jj], (row * a.ldb + k0) * 2, 0, 0);
      }
    }
  };
  const int nk = a.K / G3_BK;
  stage(0, 0, 0);
  stage(0, 2, 0);
  stage(0, 1, 0);
  if (nk > 1) {
    stage(1, 0, G3_BK);
    stage(1, 2, G3_BK);
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  if (grp == 1) __builtin_amdgcn_s_barrier();   // waves 4-7 run one barrier behind
  __builtin_amdgcn_sched_barrier(0);

  f32x4 acc[8][2];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fq = lane >> 4;
  f16x8 af[2][4], bf[2][2];
  auto read_a = [&](const f16* img) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = grp * 64 + i * 16 + fr;
        af[ks][i] = *(const f16x8*)(img + r * 64 + g2_swz(r, ks * 4 + fq) * 8);
      }
  };
  auto read_b = [&](const f16* img) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int r = wn * 32 + j * 16 + fr;
        bf[ks][j] = *(const f16x8*)(img + r * 64 + g2_swz(r, ks * 4 + fq) * 8);
      }
  };
  auto mfma_h = [&](int qa) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[qa * 4 + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bf[ks][j], af[ks][i], acc[qa * 4 + i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  auto sync_in = [&]() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  auto sync_out = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };

  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const f16* img = lds5 + cur * 3 * G4_HALF;
    const bool n1 = kt + 1 < nk, n2 = kt + 2 < nk;
    // phase 1: rows 0..63 of the wave's half -- read AH0 + BT; stage AH1 of tile kt+1; retire AH1
    // of tile kt (read in phase 2)
    read_b(img + 2 * G4_HALF);
    read_a(img);
    if (n1) {
      stage(cur ^ 1, 1, (kt + 1) * G3_BK);
      asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    sync_in();
    mfma_h(0);
    sync_out();
    // phase 2: rows 64..127 -- read AH1; stage AH0 + BT of tile kt+2; retire AH0 / BT of tile kt+1
    read_a(img + G4_HALF);
    if (n2) {
      stage(cur, 0, (kt + 2) * G3_BK);
      stage(cur, 2, (kt + 2) * G3_BK);
      asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    } else if (n1) {
      asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    sync_in();
    mfma_h(1);
    sync_out();
  }
  if (grp == 0) __builtin_amdgcn_s_barrier();   // matches the stagger barrier of waves 4-7

  // transposed accumulators, as k_gemm4
  const bool hb = a.bias != nullptr;
  f32x4 bz[2];
#pragma unroll
  for (int j = 0; j < 2; ++j)
    bz[j] = hb ? *(const f32x4*)(a.bias + bn * 128 + wn * 32 + j * 16 + fq * 4) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
      epi_store4<EPI>(a, bm * G3_M + grp * 128 + i * 16 + fr, bn * 128 + wn * 32 + j * 16 + fq * 4, acc[i][j], hb, bz[j]);
}

template <int EPI>
__global__ __launch_bounds__(512, 1) void k_gemm5(ProjArgs a) {
  ProfClock prof_clock_(a.ts);   // sampled launches only (csrc/prof.cpp)
  extern __shared__ __attribute__((aligned(16))) f16 lds5[];   // [buf][AH0, AH1, BT][128 x 64]
  const int ntiles = (a.N / 128) * cdiv(a.M, G3_M);
  for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
    gemm5_tile<EPI>(a, lds5, t, ntiles);
    __builtin_amdgcn_s_barrier();   // every wave's last LDS reads done before the next prologue
  }
}


// ---------------------------------------------------------------- fp8 (e4m3) MX MFMA GEMM
// The encoder GEMMs of BASELINE configs[4] on the block-scaled fp8 MFMA
// (v_mfma_scale_f32_16x16x128_f8f6f4: twice the f16 MFMA rate, MI355X_MICROARCH.md "Matrix
// cores") with MX scaling: every operand row carries one E8M0 (power-of-two) scale per 32
// consecutive k (an F8 block), applied by the MFMA itself -- no dequantisation in the epilogue,
// and the producers of the A operand quantise as they write it (the LayerNorm k_layernorm_f8,
// the fc1 GEMM's GELU epilogue EPI_F8_GELU, k_quant_f8 behind the attention), so no separate
// quantisation pass runs before a projection.
// Operand layout (Fp8Operand): bytes [rows][ld] e4m3 (OCP e4m3fn) and scales as u32 words
// [K / 128][ld_sc] (ld_sc = rows rounded up to 256): byte b of word (kt, r) is the E8M0 scale of
// k = 128 kt + 32 b .. +32 of row r, so one K-tile's scales of a 256-row tile are one 1-KB run --
// one LDS-DMA wave instruction.
//
// k_gemm8 is k_gemm4's ping-pong schedule byte for byte: a BK = 128 fp8 K-tile is the 128-B row
// of k_gemm4's BK = 64 f16 tile, so the half-tile images, the g2_swz source swizzle, the four
// quadrant phases, the stagger of waves 4-7 and the counted vmcnt(6) are unchanged; a quadrant is
// 8 scaled MFMAs (4 row x 2 column tiles, K = 128: 32 cycles each -- the 256 cycles of k_gemm4's
// 16 f16 MFMAs for twice the k).  A K-tile's two scale images are staged with its first half (BH0,
// phase 1 of the tile before; waves 0 / 1, one DMA each) into a 4-KB double buffer behind the
// tile images, retired by the same vmcnt(6), and read into registers in phase 1 of the tile.
// Lane (fr, fq) of a 16 x 16 x 128 operand holds k = 16 fq .. +15 and 64 + 16 fq .. +15 of row fr
// (bytes 0-15 / 16-31) and its scale register scales k-block fq (k = 32 fq .. +31), so the
// fragment is the row's 16-B chunks fq and 4 + fq (test_mfma_scale_lane_map pins both maps).
typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef int i32x4 __attribute__((ext_vector_type(4)));
constexpr int G8_BK = 128;                              // k per K-tile (bytes per row)
constexpr uint32_t G8_SC = 2u * 2u * 1024u;             // scale images: [buf][A | B][256 words]
constexpr uint32_t G8_LDS = G4_LDS + G8_SC;             // 132 KB

// E8M0 exponent of an F8 block whose largest magnitude is amax: the smallest e with
// amax / 2^e <= 448 (e4m3's largest finite value), exactly -- amax = m 2^x, m in [0.5, 1), and
// 448 = 0.875 2^9 -- clamped to [-126, 126] so that 2^-e is a normal f32.
__device__ __forceinline__ int f8_block_exp(float amax) {
  if (!(amax > 0.f)) return -126;   // an all-zero block (a NaN propagates through the values)
  int x;
  const float m = frexpf(amax, &x);
  const int e = m <= 0.875f ? x - 9 : x - 8;
  return max(-126, min(126, e));
}
__device__ __forceinline__ float f8_pow2(int e) { return __int_as_float((127 + e) << 23); }   // 2^e
// four values (already multiplied by 2^-e) to e4m3, round to nearest even, little-endian bytes
__device__ __forceinline__ uint32_t f8_pack4(float a, float b, float c, float d) {
  uint32_t w = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
  return __builtin_amdgcn_cvt_pk_fp8_f32(c, d, w, true);
}

// LDS reads the compiler does not see as LDS loads: hipcc (ROCm 7.2) cannot tell a ds_read of the
// current K-tile's image from the LDS-DMA writes still in flight into the other images, and puts
// an s_waitcnt vmcnt(0) at the head of every K-tile in front of the first compiler-visible
// ds_read (k_gemm4 carries it too) -- which drains the two tiles in flight the counted vmcnt(6)
// schedule is built for.  The phases order these reads themselves: every load section ends in
// s_waitcnt lgkmcnt(0) + sched_barrier(0) (sync_in) before the MFMAs that use them.
__device__ __forceinline__ i32x4 lds_read16(const void* p) {
  i32x4 v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"((uint32_t)(uintptr_t)p));
  return v;
}
__device__ __forceinline__ uint32_t lds_read4(const void* p) {
  uint32_t v;
  asm volatile("ds_read_b32 %0, %1" : "=v"(v) : "v"((uint32_t)(uintptr_t)p));
  return v;
}

template <int EPI>
__device__ __forceinline__ void gemm8_tile(const ProjArgs& a, uint8_t* lds, int orig, int nwg) {
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int q = nwg / 8, rr = nwg % 8, xcd = orig % 8;
  const int id = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + orig / 8;
  const int ntn = a.N / G3_N;
  int bm = id / ntn, bn = id % ntn;
  if (a.tile_gm > 1) {
    const int ntm = cdiv(a.M, G3_M), gsz = a.tile_gm * ntn, g = id / gsz, m0 = g * a.tile_gm;
    const int gm = min(a.tile_gm, ntm - m0), l = id - g * gsz;
    bm = m0 + l % gm;
    bn = l / gm;
  }
  const int grp = wid >> 2, wn = wid & 3;
  // staging as k_gemm4 (bytes): AH[h] image row q -> A row bm*256 + (q >> 6)*128 + 64h + (q & 63),
  // BH[h] image row q -> B row bn*256 + (q >> 5)*64 + 32h + (q & 31), q = (2 wid + jj)*8 + lane/8.
  // Buffer-resource DMA (buffer_load_dwordx4 ... lds): the row base and k0 are a wave-uniform
  // scalar offset, a lane adds one loop-invariant 32-bit offset per piece jj -- its row lane/8 and
  // its g2_swz chunk ((lane & 7) ^ ((4 jj + lane/16) & 7): wid drops out).  A VGPR that an LDS
  // DMA reads is then never rewritten: hipcc treats an LDS-DMA's VGPR operands like store data and
  // puts an s_waitcnt vmcnt(0) in front of any redefinition, which with per-K-tile 64-bit
  // addresses sat at the head of every K-tile and drained the two tiles in flight.  Rows past M
  // read zeros (the descriptor's bounds), and are never stored.
  // A: the descriptor starts at the tile's first row and ends at row M (rows past it read zeros:
  // the buffer range check covers the VGPR offset, which carries the row), k0 in the scalar offset
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(a.A8 + (size_t)bm * G3_M * a.lda), (short)0, max(0, a.M - bm * G3_M) * a.lda, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc((void*)a.B8, (short)0, a.N * a.ldb, 0x00020000);
  uint32_t offa[2][2], offb[2];   // offa[half][jj]: the row inside the tile and the chunk
#pragma unroll
  for (int jj = 0; jj < 2; ++jj) {
    const uint32_t ca = (lane & 7) ^ ((4 * jj + (lane >> 4)) & 7);
    const int p = 2 * wid + jj;
#pragma unroll
    for (int h = 0; h < 2; ++h)
      offa[h][jj] = (uint32_t)((p >> 3) * 128 + 64 * h + (p & 7) * 8 + (lane >> 3)) * (uint32_t)a.lda + ca * 16u;
    offb[jj] = (uint32_t)(lane >> 3) * (uint32_t)a.ldb + ca * 16u;
  }
  constexpr int HB = G4_HALF * 2;   // bytes per half-tile image
  typedef __attribute__((address_space(3))) void* lds_ptr;
  auto stage = [&](int buf, int half, int k0) {   // half: 0 AH0, 1 AH1, 2 BH0, 3 BH1; k0 in bytes
    uint8_t* dst = lds + (buf * 4 + half) * HB + (2 * wid) * 1024;
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
      const int p = 2 * wid + jj;
      if (half < 2) {
        __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (lds_ptr)(dst + jj * 1024), 16, offa[half][jj], k0, 0, 0);
      } else {
        const int row = bn * G3_N + (p >> 2) * 64 + 32 * (half - 2) + (p & 3) * 8;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, (lds_ptr)(dst + jj * 1024), 16, offb[jj], row * a.ldb + k0, 0, 0);
      }
    }
  };
  uint8_t* sc_lds = lds + G4_LDS;
  const int nk = a.K / G8_BK;
  const __amdgpu_buffer_rsrc_t rsa = __builtin_amdgcn_make_buffer_rsrc((void*)a.a_sc, (short)0, nk * a.ld_asc * 4, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsb = __builtin_amdgcn_make_buffer_rsrc((void*)a.b_sc, (short)0, nk * a.ld_bsc * 4, 0x00020000);
  const uint32_t offs = (uint32_t)lane * 16u;
  auto stage_sc = [&](int buf, int kt) {   // wave 0: A scales of the tile's 256 rows, wave 1: B's
    if (wid == 0)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsa, (lds_ptr)(sc_lds + buf * 2048), 16, offs, (kt * a.ld_asc + bm * G3_M) * 4, 0, 0);
    else if (wid == 1)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsb, (lds_ptr)(sc_lds + buf * 2048 + 1024), 16, offs, (kt * a.ld_bsc + bn * G3_N) * 4, 0, 0);
  };
  stage_sc(0, 0);
  stage(0, 0, 0);
  stage(0, 2, 0);
  stage(0, 3, 0);
  stage(0, 1, 0);
  if (nk > 1) {
    stage(1, 0, G8_BK);
    stage(1, 3, G8_BK);
    stage(1, 1, G8_BK);
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  if (grp == 1) __builtin_amdgcn_s_barrier();   // waves 4-7 run one barrier behind
  __builtin_amdgcn_sched_barrier(0);

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fq = lane >> 4;
  i32x8 af[4], bf[2];            // the current quadrant's fragments (one K = 128 step)
  int sa[4], sb[2];              // the quadrant's scale bytes (in bits 0..7) per row / column tile
  // lane (fr, fq) of a 16 x 16 x 128 operand holds k = 16 fq .. +15 in its bytes 0-15 and
  // k = 64 + 16 fq .. +15 in bytes 16-31, and its scale register scales the k-block fq (32 k):
  // measured, tests/test_gpu_kernels.py test_mfma_scale_lane_map -- so the fragment is the 16-B
  // chunks fq and 4 + fq of the row, and the hardware k is the memory k
  auto frag = [&](const uint8_t* img, int r) {
    const i32x4 lo = lds_read16(img + r * 128 + g2_swz(r, fq) * 16);
    const i32x4 hi = lds_read16(img + r * 128 + g2_swz(r, 4 + fq) * 16);
    return (i32x8)__builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  };
  auto read_a = [&](const uint8_t* img) {
#pragma unroll
    for (int i = 0; i < 4; ++i) af[i] = frag(img, grp * 64 + i * 16 + fr);
  };
  auto read_b = [&](const uint8_t* img) {
#pragma unroll
    for (int j = 0; j < 2; ++j) bf[j] = frag(img, wn * 32 + j * 16 + fr);
  };
  // the quadrant's scales: rows grp*128 + (4 qa + i)*16 + fr, columns wn*64 + (2 qb + j)*16 + fr
  // (read per phase: 6 registers where a whole tile's 12 would spill beside the accumulators)
  auto read_sc = [&](int buf, int qa, int qb) {
    const uint32_t* s = (const uint32_t*)(sc_lds + buf * 2048);
#pragma unroll
    for (int i = 0; i < 4; ++i) sa[i] = (int)(lds_read4(s + grp * 128 + (qa * 4 + i) * 16 + fr) >> (8 * fq));
#pragma unroll
    for (int j = 0; j < 2; ++j) sb[j] = (int)(lds_read4(s + 256 + wn * 64 + (qb * 2 + j) * 16 + fr) >> (8 * fq));
  };
  auto mfma_q = [&](int qa, int qb) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        acc[qa * 4 + i][qb * 2 + j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(
            bf[j], af[i], acc[qa * 4 + i][qb * 2 + j], 0, 0, 0, sb[j], 0, sa[i]);
    // pin the quadrant's MFMAs inside their phase: without a use here the (pure) scaled-MFMA
    // calls sink past the phase barriers to the end of the K-tile, which keeps all four phases'
    // fragments live at once and spills
#pragma unroll
    for (int i = 0; i < 4; ++i)
      asm volatile("" : "+v"(acc[qa * 4 + i][qb * 2]), "+v"(acc[qa * 4 + i][qb * 2 + 1]));
    __builtin_amdgcn_s_setprio(0);
  };
  auto sync_in = [&]() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  auto sync_out = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };

  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const uint8_t* img = lds + cur * 4 * HB;
    const bool n1 = kt + 1 < nk, n2 = kt + 2 < nk;
    // phase 1: Q00 -- read AH0 + BH0 (and the quadrant's scales); stage the scales and BH0 of
    // tile kt+1
    read_sc(cur, 0, 0);
    read_b(img + 2 * HB);
    read_a(img);
    if (n1) {
      stage_sc(cur ^ 1, kt + 1);
      stage(cur ^ 1, 2, (kt + 1) * G8_BK);
    }
    sync_in();
    mfma_q(0, 0);
    sync_out();
    // phase 2: Q01 -- read BH1; stage AH0 of tile kt+2
    read_sc(cur, 0, 1);
    read_b(img + 3 * HB);
    if (n2) stage(cur, 0, (kt + 2) * G8_BK);
    sync_in();
    mfma_q(0, 1);
    sync_out();
    // phase 3: Q11 -- read AH1; stage BH1 of tile kt+2
    read_sc(cur, 1, 1);
    read_a(img + HB);
    if (n2) stage(cur, 3, (kt + 2) * G8_BK);
    sync_in();
    mfma_q(1, 1);
    sync_out();
    // phase 4: Q10 -- read BH0; stage AH1 of tile kt+2; retire everything up to BH0 (and the
    // scales) of tile kt+1
    read_sc(cur, 1, 0);
    read_b(img + 2 * HB);
    if (n2) {
      stage(cur, 1, (kt + 2) * G8_BK);
      asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    sync_in();
    mfma_q(1, 0);
    sync_out();
  }
  if (grp == 0) __builtin_amdgcn_s_barrier();   // matches the stagger barrier of waves 4-7

  // transposed accumulators (B fragment first): lane (fr, fq) holds row fr, columns fq*4..+3 of
  // every 16 x 16 tile
  const bool hb = a.bias != nullptr;
  f32x4 bz[4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
    bz[j] = hb ? *(const f32x4*)(a.bias + bn * G3_N + wn * 64 + j * 16 + fq * 4) : f32x4{0.f, 0.f, 0.f, 0.f};
  if constexpr (EPI == EPI_F8_GELU) {
    // fc1 -> the fc2 operand: GELU, then e4m3 with one E8M0 scale per 32 columns (column tiles
    // 2p, 2p+1 of the wave: 8 values per lane, the block's 4 lanes fq = 0..3 of row fr)
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int row = bm * G3_M + grp * 128 + i * 16 + fr;
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        f32x4 g[2];
        float am = 0.f;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const f32x4 v = acc[i][2 * p + h] + bz[2 * p + h];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            g[h][r] = gelu_tanh(v[r]);
            am = fmaxf(am, fabsf(g[h][r]));
          }
        }
        am = fmaxf(am, __shfl_xor(am, 16, 64));
        am = fmaxf(am, __shfl_xor(am, 32, 64));
        const int e = f8_block_exp(am);
        const float inv = f8_pow2(-e);
        if (row < a.M) {
          const int col = bn * G3_N + wn * 64 + 32 * p;
#pragma unroll
          for (int h = 0; h < 2; ++h)
            *(uint32_t*)((uint8_t*)a.out + (size_t)row * a.ldo + col + 16 * h + fq * 4) =
                f8_pack4(g[h][0] * inv, g[h][1] * inv, g[h][2] * inv, g[h][3] * inv);
          if (fq == 0) {
            const int blk = col >> 5;
            ((uint8_t*)a.o_sc)[((size_t)(blk >> 2) * a.ld_osc + row) * 4 + (blk & 3)] = (uint8_t)(e + 127);
          }
        }
      }
    }
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        epi_store4<EPI>(a, bm * G3_M + grp * 128 + i * 16 + fr, bn * G3_N + wn * 64 + j * 16 + fq * 4, acc[i][j], hb, bz[j]);
  }
}

template <int EPI>
__global__ __launch_bounds__(512, 1) void k_gemm8(ProjArgs a) {
  ProfClock prof_clock_(a.ts);   // sampled launches only (csrc/prof.cpp)
  extern __shared__ __attribute__((aligned(16))) uint8_t lds8[];   // [buf][AH0, AH1, BH0, BH1] + scales
  const int ntiles = (a.N / G3_N) * cdiv(a.M, G3_M);
  for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
    gemm8_tile<EPI>(a, lds8, t, ntiles);
    __builtin_amdgcn_s_barrier();   // every wave's last LDS reads done before the next prologue
  }
}

// k_gemm8n: the narrow fp8 projections (o, fc2: N = d = 1280) on k_gemm5's 256 x 128 tile and
// two-phase schedule (8 waves of 128 x 32, B fragments kept across the two 64-row phases): 240
// tiles at M = 6000 where k_gemm8's 256 x 256 tiles leave half the CUs idle.  Scale images: A
// (256 rows) and B (128 rows, the first 512 B of the image) per K-tile, in a 3-deep ring: a
// K-tile's scales are staged with its AH0 / BT (phase 2 of the tile two before), so the tile in
// between still reads its own.
constexpr uint32_t G8N_LDS = 2u * 3u * G4_HALF * 2u + 3u * 2048u;   // 96 KB + 6 KB

template <int EPI>
__device__ __forceinline__ void gemm8n_tile(const ProjArgs& a, uint8_t* lds, int orig, int nwg) {
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int q = nwg / 8, rr = nwg % 8, xcd = orig % 8;
  const int id = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + orig / 8;
  const int ntn = a.N / 128;
  int bm = id / ntn, bn = id % ntn;
  if (a.tile_gm > 1) {
    const int ntm = cdiv(a.M, G3_M), gsz = a.tile_gm * ntn, g = id / gsz, m0 = g * a.tile_gm;
    const int gm = min(a.tile_gm, ntm - m0), l = id - g * gsz;
    bm = m0 + l % gm;
    bn = l / gm;
  }
  const int grp = wid >> 2, wn = wid & 3;
  // staging (bytes) as k_gemm5: AH[h] image row q -> A row bm*256 + (q >> 6)*128 + 64h + (q & 63);
  // BT row q -> B row bn*128 + q; buffer-resource DMA as k_gemm8 (rows past M read zeros)
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(a.A8 + (size_t)bm * G3_M * a.lda), (short)0, max(0, a.M - bm * G3_M) * a.lda, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc((void*)a.B8, (short)0, a.N * a.ldb, 0x00020000);
  uint32_t offa[2][2], offb[2];
#pragma unroll
  for (int jj = 0; jj < 2; ++jj) {
    const uint32_t ca = (lane & 7) ^ ((4 * jj + (lane >> 4)) & 7);
    const int p = 2 * wid + jj;
#pragma unroll
    for (int h = 0; h < 2; ++h)
      offa[h][jj] = (uint32_t)((p >> 3) * 128 + 64 * h + (p & 7) * 8 + (lane >> 3)) * (uint32_t)a.lda + ca * 16u;
    offb[jj] = (uint32_t)(p * 8 + (lane >> 3)) * (uint32_t)a.ldb + ca * 16u;
  }
  constexpr int HB = G4_HALF * 2;
  typedef __attribute__((address_space(3))) void* lds_ptr;
  auto stage = [&](int buf, int half, int k0) {   // half: 0 AH0, 1 AH1, 2 BT; k0 in bytes
    uint8_t* dst = lds + (buf * 3 + half) * HB + (2 * wid) * 1024;
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
      if (half < 2)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (lds_ptr)(dst + jj * 1024), 16, offa[half][jj], k0, 0, 0);
      else
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, (lds_ptr)(dst + jj * 1024), 16, offb[jj], bn * 128 * a.ldb + k0, 0, 0);
    }
  };
  uint8_t* sc_lds = lds + 2 * 3 * HB;
  const int nk = a.K / G8_BK;
  const __amdgpu_buffer_rsrc_t rsa = __builtin_amdgcn_make_buffer_rsrc((void*)a.a_sc, (short)0, nk * a.ld_asc * 4, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsb = __builtin_amdgcn_make_buffer_rsrc((void*)a.b_sc, (short)0, nk * a.ld_bsc * 4, 0x00020000);
  const uint32_t offs = (uint32_t)lane * 16u;
  auto stage_sc = [&](int kt) {   // wave 0: A scales (256 rows), wave 1 lanes 0-31: B scales (128 rows)
    uint8_t* dst = sc_lds + (kt % 3) * 2048;
    if (wid == 0)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsa, (lds_ptr)dst, 16, offs, (kt * a.ld_asc + bm * G3_M) * 4, 0, 0);
    else if (wid == 1 && lane < 32)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsb, (lds_ptr)(dst + 1024), 16, offs, (kt * a.ld_bsc + bn * 128) * 4, 0, 0);
  };
  stage_sc(0);
  stage(0, 0, 0);
  stage(0, 2, 0);
  stage(0, 1, 0);
  if (nk > 1) {
    stage_sc(1);
    stage(1, 0, G8_BK);
    stage(1, 2, G8_BK);
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  if (grp == 1) __builtin_amdgcn_s_barrier();   // waves 4-7 run one barrier behind
  __builtin_amdgcn_sched_barrier(0);

  f32x4 acc[8][2];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fq = lane >> 4;
  i32x8 af[4], bf[2];
  int sa[4], sb[2];
  auto frag = [&](const uint8_t* img, int r) {   // chunks fq and 4 + fq: k_gemm8's lane map
    const i32x4 lo = lds_read16(img + r * 128 + g2_swz(r, fq) * 16);
    const i32x4 hi = lds_read16(img + r * 128 + g2_swz(r, 4 + fq) * 16);
    return (i32x8)__builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  };
  auto read_a = [&](const uint8_t* img, const uint32_t* sc, int h) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      af[i] = frag(img, grp * 64 + i * 16 + fr);
      sa[i] = (int)(lds_read4(sc + grp * 128 + 64 * h + i * 16 + fr) >> (8 * fq));
    }
  };
  auto read_b = [&](const uint8_t* img, const uint32_t* sc) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      bf[j] = frag(img, wn * 32 + j * 16 + fr);
      sb[j] = (int)(lds_read4(sc + 256 + wn * 32 + j * 16 + fr) >> (8 * fq));
    }
  };
  auto mfma_h = [&](int h) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        acc[h * 4 + i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(bf[j], af[i], acc[h * 4 + i][j], 0, 0, 0,
                                                                             sb[j], 0, sa[i]);
#pragma unroll
    for (int i = 0; i < 4; ++i) asm volatile("" : "+v"(acc[h * 4 + i][0]), "+v"(acc[h * 4 + i][1]));
    __builtin_amdgcn_s_setprio(0);
  };
  auto sync_in = [&]() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  auto sync_out = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };

  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const uint8_t* img = lds + cur * 3 * HB;
    const uint32_t* sc = (const uint32_t*)(sc_lds + (kt % 3) * 2048);
    const bool n1 = kt + 1 < nk, n2 = kt + 2 < nk;
    // phase 1: rows 0..63 of the wave's half -- read BT + AH0 (+ scales); stage AH1 of tile kt+1;
    // retire AH1 of tile kt
    read_b(img + 2 * HB, sc);
    read_a(img, sc, 0);
    if (n1) {
      stage(cur ^ 1, 1, (kt + 1) * G8_BK);
      asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    sync_in();
    mfma_h(0);
    sync_out();
    // phase 2: rows 64..127 -- read AH1; stage the scales, AH0 and BT of tile kt+2; retire AH0 /
    // BT (and the scales) of tile kt+1
    read_a(img + HB, sc, 1);
    if (n2) {
      stage_sc(kt + 2);
      stage(cur, 0, (kt + 2) * G8_BK);
      stage(cur, 2, (kt + 2) * G8_BK);
      asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    } else if (n1) {
      asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    sync_in();
    mfma_h(1);
    sync_out();
  }
  if (grp == 0) __builtin_amdgcn_s_barrier();   // matches the stagger barrier of waves 4-7

  const bool hb = a.bias != nullptr;
  f32x4 bz[2];
#pragma unroll
  for (int j = 0; j < 2; ++j)
    bz[j] = hb ? *(const f32x4*)(a.bias + bn * 128 + wn * 32 + j * 16 + fq * 4) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
      epi_store4<EPI>(a, bm * G3_M + grp * 128 + i * 16 + fr, bn * 128 + wn * 32 + j * 16 + fq * 4, acc[i][j], hb, bz[j]);
}

template <int EPI>
__global__ __launch_bounds__(512, 1) void k_gemm8n(ProjArgs a) {
  ProfClock prof_clock_(a.ts);   // sampled launches only (csrc/prof.cpp)
  extern __shared__ __attribute__((aligned(16))) uint8_t lds8n[];   // [buf][AH0, AH1, BT] + scale ring
  const int ntiles = (a.N / 128) * cdiv(a.M, G3_M);
  for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
    gemm8n_tile<EPI>(a, lds8n, t, ntiles);
    __builtin_amdgcn_s_barrier();
  }
}

template <int EPI>
static void launch_epi8(const ProjArgs& a, hipStream_t s) {
  // algorithmic bytes: fp8 operands + their scales, the output at its epilogue's width
  const double ob = EPI == EPI_F8_GELU ? 1.0 : (EPI == EPI_F32_RESID || EPI == EPI_F32) ? 4.0 : 2.0;
  const double bytes = ((double)a.N + a.M) * a.K * (1.0 + 1.0 / 32) + (double)a.M * a.N * ob;
  const double flops = 2.0 * a.M * a.N * a.K;
  static bool attr = [] {
    WDR_HIP(hipFuncSetAttribute((const void*)k_gemm8<EPI>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)G8_LDS));
    return true;
  }();
  (void)attr;
  static const int tile_gm = getenv("WDR_GEMM4_GM") ? atoi(getenv("WDR_GEMM4_GM")) : 4;   // as k_gemm4
  ProjArgs g = a;
  g.tile_gm = tile_gm;
  if constexpr (EPI != EPI_F8_GELU) {
    // the narrow projections (o, fc2: N = 1280) on 256 x 128 tiles: 240 at M = 6000 where 256 x 256
    // tiles fill 120 CUs (WDR_GEMM8N=0: k_gemm8 for every shape)
    // N % 256 != 0 (tiny's qkv, N = 1152) has only the 256 x 128 tiling
    static const bool narrow_on = !getenv("WDR_GEMM8N") || atoi(getenv("WDR_GEMM8N")) != 0;
    if ((narrow_on && a.N < 2048) || a.N % G3_N != 0) {
      static bool attrn = [] {
        WDR_HIP(hipFuncSetAttribute((const void*)k_gemm8n<EPI>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)G8N_LDS));
        return true;
      }();
      (void)attrn;
      const int ntn = (a.N / 128) * cdiv(a.M, G3_M);
      wdr_launch(PROF_GEMM, bytes, flops, k_gemm8n<EPI>, dim3(ntn), dim3(512), G8N_LDS, s, g);
      return;
    }
  }
  const int ntiles = (a.N / G3_N) * cdiv(a.M, G3_M);
  wdr_launch(PROF_GEMM, bytes, flops, k_gemm8<EPI>, dim3(ntiles), dim3(512), G8_LDS, s, g);
}

void launch_proj_fp8(const ProjArgs& a, hipStream_t s) {
  WDR_CHECK(a.A8 && a.B8 && a.a_sc && a.b_sc, "fp8 projection: operands / scales missing");
  // N % 128: k_gemm8n's 256 x 128 tiles; the 256 x 256 k_gemm8 (every N >= 2048, and fc1's GELU ->
  // fp8 epilogue) needs N % 256
  WDR_CHECK(a.M > 64 && a.N % 128 == 0 && (a.epi != EPI_F8_GELU || a.N % G3_N == 0) && a.K % G8_BK == 0 &&
                a.lda % 16 == 0 && a.ldb % 16 == 0,
            "fp8 projection: M > 64, N % 128 == 0 (N % 256 for the GELU -> fp8 epilogue), K % 128 == 0, "
            "lda / ldb % 16 required");
  WDR_CHECK(a.ld_asc >= cdiv(a.M, G3_M) * G3_M && a.ld_bsc >= a.N && a.ld_asc % 4 == 0 && a.ld_bsc % 4 == 0,
            "fp8 projection: scale images need the rows rounded up to 256");
  WDR_CHECK(a.epi != EPI_F8_GELU || (a.o_sc && a.ld_osc >= cdiv(a.M, G3_M) * G3_M && a.ldo % 16 == 0),
            "fp8 projection: GELU -> fp8 epilogue needs an output scale image");
  switch (a.epi) {
    case EPI_F16: launch_epi8<EPI_F16>(a, s); break;
    case EPI_F16_GELU: launch_epi8<EPI_F16_GELU>(a, s); break;
    case EPI_F32_RESID: launch_epi8<EPI_F32_RESID>(a, s); break;
    case EPI_F32: launch_epi8<EPI_F32>(a, s); break;
    case EPI_F8_GELU: launch_epi8<EPI_F8_GELU>(a, s); break;
    default: throw std::runtime_error("fp8 projection: unsupported epilogue");
  }
  WDR_HIP(hipGetLastError());
}

// f16 rows -> e4m3 + MX scales (Fp8Operand layout): one wave per row, 8 values per lane per
// step; a 32-k block is 4 lanes (max by two xor shuffles), a scale word 16 lanes (gathered by
// shuffles, stored by the group's first lane).  The weights (once, Context::fp8_build) and the
// attention output ahead of the o projection.
__global__ __launch_bounds__(256) void k_quant_f8(const f16* x, int ldx, int rows, int K, uint8_t* y, int ldy,
                                                  uint32_t* sc, int ld_sc) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= rows) return;
  const f16* xr = x + (size_t)row * ldx;
  for (int c0 = 0; c0 < K; c0 += 512) {
    const int c = c0 + lane * 8;
    const bool ok = c < K;
    f16x8 v = ok ? *(const f16x8*)(xr + c) : f16x8{};
    float am = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) am = fmaxf(am, fabsf((float)v[e]));
    am = fmaxf(am, __shfl_xor(am, 1, 64));
    am = fmaxf(am, __shfl_xor(am, 2, 64));
    const int e = f8_block_exp(am);
    const float inv = f8_pow2(-e);
    const uint32_t lo = f8_pack4((float)v[0] * inv, (float)v[1] * inv, (float)v[2] * inv, (float)v[3] * inv);
    const uint32_t hi = f8_pack4((float)v[4] * inv, (float)v[5] * inv, (float)v[6] * inv, (float)v[7] * inv);
    if (ok) *(uint2*)(y + (size_t)row * ldy + c) = make_uint2(lo, hi);
    // scale word of k 128 t .. +128 (lanes 16 u .. 16 u + 15): the bytes of lanes +0, 4, 8, 12
    const int b = e + 127, base = lane & ~15;
    const uint32_t w = (uint32_t)__shfl(b, base, 64) | (uint32_t)__shfl(b, base + 4, 64) << 8 |
                       (uint32_t)__shfl(b, base + 8, 64) << 16 | (uint32_t)__shfl(b, base + 12, 64) << 24;
    if ((lane & 15) == 0 && ok) sc[(size_t)(c >> 7) * ld_sc + row] = w;
  }
}

// one v_mfma_scale_f32_16x16x128_f8f6f4 (e4m3 x e4m3) on raw per-lane operands: lane l's 32 A
// bytes a[l], B bytes b[l], scale registers sa[l] / sb[l] (op_sel 0), its 4 accumulators out[l]
// -- the probe that pins the lane -> (row, k-block) map of the data and the scales
__global__ __launch_bounds__(64) void k_probe_mfma_scale(const i32x8* a, const i32x8* b, const int* sa, const int* sb,
                                                          f32x4* out) {
  const int l = threadIdx.x;
  out[l] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a[l], b[l], f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0, sa[l], 0,
                                                             sb[l]);
}
void launch_probe_mfma_scale(const void* a, const void* b, const int* sa, const int* sb, float* out, hipStream_t s) {
  WDR_KLAUNCH(k_probe_mfma_scale, dim3(1), dim3(64), 0, s, (const i32x8*)a, (const i32x8*)b, sa, sb, (f32x4*)out);
  WDR_HIP(hipGetLastError());
}

void launch_quant_f8(const f16* x, int ldx, int rows, int K, uint8_t* y, int ldy, uint32_t* sc, int ld_sc,
                     hipStream_t s) {
  WDR_CHECK(rows >= 1 && K % 128 == 0 && ldx % 8 == 0 && ldy % 16 == 0 && ld_sc >= rows,
            "fp8 quantisation: K % 128, ldx % 8, ldy % 16, scale rows");
  WDR_KLAUNCH(k_quant_f8, dim3(cdiv(rows, 4)), dim3(256), 0, s, x, ldx, rows, K, y, ldy, sc, ld_sc);
  WDR_HIP(hipGetLastError());
}

// LayerNorm (k_layernorm's arithmetic: ggml_norm, eps 1e-5, gamma / beta) quantised as it is
// written: the encoder's LN1 / LN2 straight into the qkv / fc1 fp8 operands.  One wave per row,
// 4 consecutive columns per lane and step (lanes 0-31 cover a 128-column scale word, a 32-column
// block is 8 lanes).
__global__ __launch_bounds__(256) void k_layernorm_f8(const float* x, int ldx, const float* g, const float* b,
                                                      uint8_t* y, int ldy, uint32_t* sc, int ld_sc, int rows, int d) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const float* xr = x + (long long)row * ldx;
  float v[5][4];
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < 5; ++j) {
    const int c = lane * 4 + j * 256;
    const bool ok = c < d;
    const int cc = ok ? c : 0;
    const float4 q = *(const float4*)(xr + cc);
    v[j][0] = ok ? q.x : 0.f; v[j][1] = ok ? q.y : 0.f; v[j][2] = ok ? q.z : 0.f; v[j][3] = ok ? q.w : 0.f;
    s += (v[j][0] + v[j][1]) + (v[j][2] + v[j][3]);
  }
  s = wave_sum(s);
  const float mean = s / d;
  float s2 = 0.f;
#pragma unroll
  for (int j = 0; j < 5; ++j)
    if (lane * 4 + j * 256 < d)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float t = v[j][e] - mean;
        s2 += t * t;
      }
  s2 = wave_sum(s2);
  const float scale = 1.0f / sqrtf(s2 / d + 1e-5f);
#pragma unroll
  for (int j = 0; j < 5; ++j) {
    const int c = lane * 4 + j * 256;
    if (j * 256 >= d) break;   // wave-uniform: the shuffles below need every lane
    const bool ok = c < d;
    const int cc = ok ? c : 0;
    const float4 g4 = *(const float4*)(g + cc);
    const float4 b4 = *(const float4*)(b + cc);
    const float gg[4] = {g4.x, g4.y, g4.z, g4.w}, bb[4] = {b4.x, b4.y, b4.z, b4.w};
    float o[4], am = 0.f;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      o[e] = ok ? (v[j][e] - mean) * scale * gg[e] + bb[e] : 0.f;
      am = fmaxf(am, fabsf(o[e]));
    }
    am = fmaxf(am, __shfl_xor(am, 1, 64));
    am = fmaxf(am, __shfl_xor(am, 2, 64));
    am = fmaxf(am, __shfl_xor(am, 4, 64));
    const int e = f8_block_exp(am);
    const float inv = f8_pow2(-e);
    if (ok) *(uint32_t*)(y + (size_t)row * ldy + c) = f8_pack4(o[0] * inv, o[1] * inv, o[2] * inv, o[3] * inv);
    const int bb8 = e + 127, base = lane & 32;
    const uint32_t w = (uint32_t)__shfl(bb8, base, 64) | (uint32_t)__shfl(bb8, base + 8, 64) << 8 |
                       (uint32_t)__shfl(bb8, base + 16, 64) << 16 | (uint32_t)__shfl(bb8, base + 24, 64) << 24;
    if ((lane & 31) == 0 && ok) sc[(size_t)(c >> 7) * ld_sc + row] = w;
  }
}

void launch_layernorm_f8(const float* x, int ldx, const float* g, const float* b, uint8_t* y, int ldy, uint32_t* sc,
                         int ld_sc, int rows, int d, hipStream_t s) {
  WDR_CHECK(d % 128 == 0 && d <= 1280 && ldx % 4 == 0 && ldy % 16 == 0 && ld_sc >= rows,
            "fp8 layernorm: d % 128, d <= 1280");
  WDR_KLAUNCH(k_layernorm_f8, dim3(cdiv(rows, 4)), dim3(256), 0, s, x, ldx, g, b, y, ldy, sc, ld_sc, rows, d);
  WDR_HIP(hipGetLastError());
}

// ---------------------------------------------------------------- skinny MFMA GEMM (8 < M <= 64)
// Prompt prefill / DTW re-forward rows.  A workgroup owns 16*NT output columns for ALL rows;
// its 4 waves split K (interleaved 32-wide steps), stream the weight fragments straight from
// HBM into v_mfma_f32_16x16x32_f16 (B operand = 16 contiguous bytes of one weight row per
// lane) and reduce through LDS.  N/16 workgroups instead of N/128 keep every CU streaming.
// LN: the A rows are LayerNorm(ln_x rows) -- each workgroup normalises its 16*MT rows into LDS
// first (k_layernorm's arithmetic, so the f16 operands are bit-identical to the unfused path) --
// which removes the separate LayerNorm launch and its f16 round trip.  The rows sit unpadded,
// [16*MT][K] with the 16-B chunk index XOR (row & 15) (the 16-row fragment reads stay
// conflict-free), and the waves' partial sums reuse that LDS after the K loop: 32 rows of K = 1280
// are exactly 80 KB, so two such workgroups share a CU (with padded rows and a separate
// reduction buffer one did).
template <int EPI, int MT, int NT, int W>
constexpr uint32_t skinny_red_bytes() { return (uint32_t)W * MT * NT * 4 * 64 * 4; }
template <int EPI, int MT, int NT, int W>
static uint32_t skinny_ln_lds(int K) {
  return std::max((uint32_t)16 * MT * K * 2, skinny_red_bytes<EPI, MT, NT, W>());
}

template <int EPI, int MT, int NT, int W = 4, bool LN = false, int UU = 0>
__global__ __launch_bounds__(W * 64) void k_skinny(ProjArgs a) {
  ProfClock prof_clock_(a.ts);   // sampled launches only (csrc/prof.cpp)
  __shared__ float red_s[LN ? 1 : W * MT * NT * 4 * 64];
  extern __shared__ __attribute__((aligned(16))) f16 xln[];   // LN: [16*MT][K], chunk-swizzled
  float* red = LN ? (float*)xln : red_s;   // [W][MT][NT][4][64]
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int n0 = blockIdx.x * 16 * NT;
  const int m0 = blockIdx.y * 16 * MT;   // row tiles split over gridDim.y workgroups (narrow N)
  const int fr = lane & 15, fk = 8 * (lane >> 4);
  f32x4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  const int lds_ld = a.K;
  if constexpr (LN) {
    const int d = a.K;
    // rows past M are never stored (an MFMA output row depends on its own A row only): only
    // the live rows are normalised, the rest of the tile stays whatever LDS holds
    const int live = min(16 * MT, a.M - m0);
    for (int rr = wid; rr < live; rr += W) {
      int row = m0 + rr;
      if (a.row_map) row = a.row_map[row];
      const float* xr = a.ln_x + (long long)row * a.ldln;
      float v[5][4];
      float sm = 0.f;
#pragma unroll
      for (int j = 0; j < 5; ++j) {
        const int c = lane * 4 + j * 256;
        const bool ok = c < d;
        const int cc = ok ? c : 0;
        const float4 q = *(const float4*)(xr + cc);
        v[j][0] = ok ? q.x : 0.f; v[j][1] = ok ? q.y : 0.f; v[j][2] = ok ? q.z : 0.f; v[j][3] = ok ? q.w : 0.f;
        sm += (v[j][0] + v[j][1]) + (v[j][2] + v[j][3]);
      }
      sm = wave_sum(sm);
      const float mean = sm / d;
      float s2 = 0.f;
#pragma unroll
      for (int j = 0; j < 5; ++j)
        if (lane * 4 + j * 256 < d)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float t = v[j][e] - mean;
            s2 += t * t;
          }
      s2 = wave_sum(s2);
      const float scale = 1.0f / sqrtf(s2 / d + 1e-5f);
#pragma unroll
      for (int j = 0; j < 5; ++j) {
        const int c = lane * 4 + j * 256;
        if (c >= d) continue;
        const float4 g4 = *(const float4*)(a.ln_g + c);
        const float4 b4 = *(const float4*)(a.ln_b + c);
        const float gg[4] = {g4.x, g4.y, g4.z, g4.w}, bb[4] = {b4.x, b4.y, b4.z, b4.w};
        f16x4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = (f16)((v[j][e] - mean) * scale * gg[e] + bb[e]);
        *(f16x4*)(xln + rr * lds_ld + ((((c >> 3) ^ (rr & 15))) << 3) + (c & 7)) = o;
      }
    }
    __syncthreads();
  }
  const f16* arow[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    int m = m0 + i * 16 + fr;
    m = m < a.M ? m : a.M - 1;
    if (!LN && a.row_map) m = a.row_map[m];
    arow[i] = LN ? xln + (i * 16 + fr) * lds_ld : a.A + (size_t)m * a.lda + fk;
  }
  const f16* brow[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    int n = n0 + j * 16 + fr;
    n = n < a.N ? n : a.N - 1;
    brow[j] = a.B + (size_t)n * a.ldb + fk;
  }
  // U k-steps per batch: all of a batch's fragment loads are issued before its MFMAs, so each
  // wave keeps U*(NT+MT) 16-B loads in flight instead of one dependent round trip per step
  // (UU: a fixed batch, e.g. all of a wave's k-steps in one batch; the k order is the same)
  constexpr int U = UU > 0 ? UU : (MT + NT) <= 3 ? 8 : 4;
  for (int k0 = wid * 32; k0 < a.K; k0 += 32 * W * U) {
    f16x8 bf[U][NT], af[U][MT];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = k0 + u * 32 * W;
      const bool ok = k < a.K;
      const int kk = ok ? k : 0;
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const f16x8 t = *(const f16x8*)(brow[j] + kk);
        bf[u][j] = ok ? t : (f16x8){};
      }
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        // LN: the fragment's 16-B chunk (kk + fk) / 8 of row i*16 + fr, swizzled by the row
        const f16x8 t = LN ? *(const f16x8*)(arow[i] + ((((kk >> 3) | (lane >> 4)) ^ fr) << 3))
                           : *(const f16x8*)(arow[i] + kk);
        af[u][i] = ok ? t : (f16x8){};
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[u][i], bf[u][j], acc[i][j], 0, 0, 0);
  }
  if constexpr (LN) __syncthreads();   // every wave's reads of the rows done before red reuses them
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) red[(((wid * MT + i) * NT + j) * 4 + r) * 64 + lane] = acc[i][j][r];
  __syncthreads();
  for (int e = threadIdx.x; e < MT * NT * 4 * 64; e += W * 64) {
    const int l = e & 63, r = (e >> 6) & 3, j = (e >> 8) % NT, i = (e >> 8) / NT;
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < W; ++w) v += red[(((w * MT + i) * NT + j) * 4 + r) * 64 + l];
    const int row = m0 + i * 16 + (l >> 4) * 4 + r, col = n0 + j * 16 + (l & 15);
    epi_store<EPI>(a, row, col, v);
  }
}



// A/B knobs of the encoder GEMM dispatch, read once per process (gemm_knobs_reload: tools/gemm_bench
// A/B runs set them per variant): WDR_GEMM1=1 every M > 64 projection on k_gemm; WDR_GEMM3=0 the
// big shapes off k_gemm3; WDR_GEMM4=0|1 the ping-pong 256 x 256 GEMM off / forced on for every
// shape it takes (unset: the measured dispatch rule); WDR_GEMM4_GM row tiles per group of the
// k_gemm4 / k_gemm5 tile order (default 4); WDR_GEMM5=1 the narrow projections on k_gemm5's
// 256 x 128 tiles; WDR_GEMM_CUS persistent k_gemm4 / k_gemm5 workgroups (multiple of 8; default one per
// tile)
struct GemmKnobs {
  bool gemm1, gemm3, gemm5, gemm5w;
  int gemm4, tile_gm, cus;
};
static int env_int(const char* name, int def) {
  const char* e = getenv(name);
  return e ? atoi(e) : def;
}
static GemmKnobs read_knobs() {
  GemmKnobs k;
  k.gemm1 = env_int("WDR_GEMM1", 0) != 0;
  k.gemm3 = env_int("WDR_GEMM3", 1) != 0 && !k.gemm1;
  k.gemm4 = env_int("WDR_GEMM4", -1);
  k.tile_gm = env_int("WDR_GEMM4_GM", 4);
  // k_gemm5 off by default since round 4: on the encode-ahead streams' 224 CUs its 240 tiles of
  // o / fc2 take two rounds where k_gemm4's 120 take one and leave ~100 CUs to the decode chain
  // (1-h bench 737-739 vs 725-731 xRT, profiles/r04/ab_gemm5.txt)
  k.gemm5 = env_int("WDR_GEMM5", 0) != 0;
  k.gemm5w = env_int("WDR_GEMM5_WIDE", 1) != 0;
  k.cus = env_int("WDR_GEMM_CUS", 0) / 8 * 8;
  return k;
}
static GemmKnobs& knobs() {
  static GemmKnobs k = read_knobs();
  return k;
}
void gemm_knobs_reload() { knobs() = read_knobs(); }

template <int EPI>
static void launch_epi(const ProjArgs& a, hipStream_t s) {
  const int ob = (EPI == EPI_F32_RESID || EPI == EPI_F32 || EPI == EPI_F32_GELU_POS) ? 4 : 2;
  const double bytes = (double)a.N * a.K * 2 + (double)a.M * a.K * 2 + (double)a.M * a.N * ob;
  const double flops = 2.0 * a.M * a.N * a.K;
  WDR_CHECK(a.M > 64, "encoder GEMM: more than 64 rows (fewer go to the row kernel)");
  const GemmKnobs& kn = knobs();
  const bool ref = kn.gemm1 || a.gemm_ref;
  const bool vec4 = a.ldo % 4 == 0 && (a.epi != EPI_QKV_CACHE || a.d % 4 == 0);   // epi_store4
  // fc1 (N = 4d) on k_gemm5's 256 x 128 tiles (WDR_GEMM5_WIDE, default on): on the encode-ahead
  // streams' 224 CUs k_gemm4's 480 tiles take 3 rounds where k_gemm5's 960 half-size tiles take
  // 5 (2.5 of the big ones); alone both run at the same per-tile rate (875 TFLOP/s)
  const bool wide5 = kn.gemm5w && a.N >= 4096 && a.N < 16384 && a.M >= 4096;
  if (a.N % 128 == 0 && a.K % G3_BK == 0 && a.M >= 4096 && !ref && vec4 && kn.gemm4 != 0 &&
      (wide5 || (a.N < 2048 && kn.gemm5 && (a.N / G3_N) * cdiv(a.M, G3_M) < 192))) {
    // the narrow encoder projections (o, fc2) where 256 x 256 tiles would leave CUs idle: 256 x
    // 128 tiles fill 240 of 256 CUs at M = 6000 (tools/gemm_bench: o 53 vs 62 us on k_gemm2, fc2
    // 107 vs 126 us; at M = 12000 k_gemm4's 235 tiles are faster: fc2 194 vs 216 us)
    static bool attr5 = [] {
      WDR_HIP(hipFuncSetAttribute((const void*)k_gemm5<EPI>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)G5_LDS));
      return true;
    }();
    (void)attr5;
    ProjArgs g = a;
    g.tile_gm = kn.tile_gm;
    const int ntiles5 = (a.N / 128) * cdiv(a.M, G3_M);
    dim3 grid(kn.cus > 0 && kn.cus < ntiles5 ? kn.cus : ntiles5);
    wdr_launch(PROF_GEMM, bytes, flops, k_gemm5<EPI>, grid, dim3(512), G5_LDS, s, g);
  } else if (a.N % G3_N == 0 && a.K % G3_BK == 0 && !ref && vec4 &&
             (kn.gemm4 == 1 ||
              (kn.gemm4 != 0 && (a.M >= 4096 || a.N >= 16384 || (a.N >= 4096 && a.M > 1024) ||
                                 (a.N >= 3072 && a.M >= 2560))))) {
    // round 6, partial encode batches and on-demand windows (profiles/r06/gemm_bench_mid_m.txt,
    // bit-identical outputs): fc1 (N = 4d) at M = 1500 / 3000 39.7 / 44.4 us on k_gemm4 vs 45.0 /
    // 67.3 on k_gemm / k_gemm3; qkv (3d) at M = 3000 41.9 vs 50.2 (k_gemm2), at M = 1500 29.2 on
    // k_gemm2 stays; o / fc2 (N = d) below M = 4096 stay on k_gemm2 (25.7 / 68.5 vs 43.3 / 110.4)
    // ping-pong 256 x 256 tiles (tools/gemm_bench, large-v3, alone on the GPU): M = 6000 qkv 600
    // vs 557 (k_gemm2), fc1 616 vs 574 (k_gemm3), cross-K/V 818 vs 742 TFLOP/s; M = 12000 every
    // shape (o 394 vs 382, fc2 811 vs 743); M = 1500 cross-K/V 773 vs 616.  The N = 1280 shapes
    // at M = 6000 fill only 120 of 256 CUs (alone: 209 / 478 vs 314 / 618 TFLOP/s on k_gemm2),
    // but inside the pipeline the CUs they leave run decode steps: 1-h bench 480 vs 476 xRT.
    static bool attr4 = [] {
      WDR_HIP(hipFuncSetAttribute((const void*)k_gemm4<EPI>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)G4_LDS));
      return true;
    }();
    (void)attr4;
    const int ntiles = (a.N / G3_N) * cdiv(a.M, G3_M);
    dim3 grid(kn.cus > 0 && kn.cus < ntiles ? kn.cus : ntiles);
    ProjArgs g = a;
    g.tile_gm = kn.tile_gm;
    wdr_launch(PROF_GEMM, bytes, flops, k_gemm4<EPI>, grid, dim3(512), G4_LDS, s, g);
  } else if ((a.N >= 5120 || a.M >= 9000) && a.M > 2048 && a.N % G3_N == 0 && a.K % G3_BK == 0 && kn.gemm3 && !ref) {
    // 256 x 256 tiles where they measured faster (tools/gemm_bench, large-v3 shapes): M = 6000
    // fc1 574 vs 509 TFLOP/s, cross-K/V 743 vs 641; at M = 12000 every encoder shape (qkv 667 vs
    // 520, o 387 vs 335, fc1 550 vs 527, fc2 746 vs 620).  Below that the 120..360 tiles of the
    // N <= 3840 shapes leave CUs idle and k_gemm2's 128 x 128 tiles win.
    static bool attr = [] {
      WDR_HIP(hipFuncSetAttribute((const void*)k_gemm3<EPI>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)G3_LDS));
      return true;
    }();
    (void)attr;
    dim3 grid((a.N / G3_N) * cdiv(a.M, G3_M));
    wdr_launch(PROF_GEMM, bytes, flops, k_gemm3<EPI>, grid, dim3(512), G3_LDS, s, a);
  } else if (a.K % G2_BK == 0 && a.N <= 4096 && !ref && vec4) {
    // LDS-DMA GEMM where it measured faster (tools/gemm_bench, M = 6000: qkv -5 %, o -11 %,
    // fc2 -23 %; fc1 and the 82k-column cross-K/V GEMM stay on k_gemm, +8 % / +7 % there)
    dim3 grid((a.N / GB_N) * cdiv(a.M, GB_M));
    wdr_launch(PROF_GEMM, bytes, flops, k_gemm2<EPI>, grid, dim3(256), 0, s, a);
  } else {
    dim3 grid(a.N / GB_N, cdiv(a.M, GB_M));
    wdr_launch(PROF_GEMM, bytes, flops, k_gemm<EPI>, grid, dim3(256), 0, s, a);
  }
}

// Decoder rows of any count on the row kernel (k_skinny, 8 or 16 waves splitting K): the k
// order of a wave (k = 32 wid + 32 W t, t = 0, 1, ...) and the wave order of the reduce depend
// only on the projection's shape (N, K), never on the tile shape (MT) or the row count, so every
// row's result is the same whatever the launch holds -- a prompt prefill of n rows equals n
// one-row steps, bit for bit.  (Round 4 tried a 4-wave, <= 64-VGPR variant with split-K slabs
// for the residual projections, to share CUs with the encoder GEMM tiles: slower alone --
// tools/rows_bench, o 15.0 vs 5.1 us, fc2 21.1 vs 13.7 us at 16 rows -- and 5 % slower in the
// 1-h pipeline, profiles/r04/ab_epi4.txt.)
// WDR_ROWS_PAIR=0: narrow projections of more than 32 rows one row tile per workgroup (A/B; read
// once)
static bool rows_pair_tiles() {
  static const bool v = env_int("WDR_ROWS_PAIR", 1) != 0;
  return v;
}
// WDR_ROWS_MT (A/B, read once): the most 16-row tiles one workgroup of a narrow projection
// (N < 4096, no LayerNorm prologue) takes above 32 rows, 2..5 (default 2).  A row's k order
// depends on (N, K) only, so every value gives the same bits; fewer workgroups stream each
// column tile's weights fewer times and take fewer rounds of the CUs the encoder leaves free.
static int rows_mt_max() {
  static const int v = std::max(2, std::min(5, env_int("WDR_ROWS_MT", 2)));
  return v;
}

template <int EPI>
static void launch_rows_epi(const ProjArgs& a, hipStream_t s) {
  // algorithmic bytes of the rows class (bench.py's live roofline and its trace counterpart,
  // bench.py rows_weight_bytes): the weights, streamed once per launch -- the activation rows and
  // outputs (<= 4 % of it at the batches' 10-60 rows) are L2 traffic
  const double bytes = (double)a.N * a.K * 2;
  const double flops = 2.0 * a.M * a.N * a.K;
  const int mt = cdiv(a.M, 16);
  const bool ln = a.ln_x != nullptr;
  const bool wide = a.N >= 4096;
  const int prof = PROF_GEMV;   // the "rows" class of bench.py's live roofline (any row count)
  if (!wide) {
    // one 16-row tile per workgroup: the row tiles of a column tile re-read its weights from L2.
    // K > 2048 (fc2): 16 waves, each wave's 10 k-steps as ONE batch of loads (8 waves took three
    // dependent batches: fc2 at 1 row 9.8 us against 5.4 us)
    if (a.K > 2048) {
      WDR_CHECK(!ln, "row projection: LN prologue needs K <= 1280");
      if (mt >= 4 && rows_pair_tiles()) {
        // above 48 rows two row tiles per workgroup: N/16 x mt one-CU workgroups would take a
        // second round on 256 CUs (tools/rows_bench fc2 at 56 / 64 rows: 16.8 / 17.8 vs 20.3 /
        // 22.1 us; at 33-48 rows the mt <= 3 tiles fit one round and stay faster alone, 12.2 vs
        // 16.6 us).  Each wave's 10 k-steps as two batches of 5 (10 at MT = 2 spills)
        const int m2 = std::min(mt, rows_mt_max());
        const dim3 g2(cdiv(a.N, 16), cdiv(mt, m2));
        if (m2 >= 4) wdr_launch(prof, bytes, flops, k_skinny<EPI, 4, 1, 16, false, 2>, g2, dim3(1024), 0, s, a);
        else if (m2 == 3) wdr_launch(prof, bytes, flops, k_skinny<EPI, 3, 1, 16, false, 5>, g2, dim3(1024), 0, s, a);
        else wdr_launch(prof, bytes, flops, k_skinny<EPI, 2, 1, 16, false, 5>, g2, dim3(1024), 0, s, a);
        return;
      }
      wdr_launch(prof, bytes, flops, k_skinny<EPI, 1, 1, 16, false, 12>, dim3(cdiv(a.N, 16), mt), dim3(1024), 0, s, a);
      return;
    }
    if (!ln && mt > 2 && rows_pair_tiles()) {
      // above 32 rows (the batched steps that carry a prompt prefill, ~56 rows): two (up to
      // WDR_ROWS_MT) row tiles per workgroup, so a column tile's weights are read half as often
      const int m2 = std::min(mt, rows_mt_max());
      const dim3 g2(cdiv(a.N, 16), cdiv(mt, m2));
      if (m2 >= 5) wdr_launch(prof, bytes, flops, k_skinny<EPI, 5, 1, 8>, g2, dim3(512), 0, s, a);
      else if (m2 == 4) wdr_launch(prof, bytes, flops, k_skinny<EPI, 4, 1, 8>, g2, dim3(512), 0, s, a);
      else if (m2 == 3) wdr_launch(prof, bytes, flops, k_skinny<EPI, 3, 1, 8>, g2, dim3(512), 0, s, a);
      else wdr_launch(prof, bytes, flops, k_skinny<EPI, 2, 1, 8>, g2, dim3(512), 0, s, a);
      return;
    }
    dim3 grid(cdiv(a.N, 16), mt), blk(512);
    if (ln) wdr_launch(prof, bytes, flops, k_skinny<EPI, 1, 1, 8, true>, grid, blk, skinny_ln_lds<EPI, 1, 1, 8>(a.K), s, a);
    else wdr_launch(prof, bytes, flops, k_skinny<EPI, 1, 1, 8>, grid, blk, 0, s, a);
    return;
  }
  // wide N (fc1, logits): 32 columns per workgroup, up to 4 row tiles per workgroup
  const int mtw = std::min(mt, ln ? 2 : 4);
  dim3 grid(cdiv(a.N, 32), cdiv(mt, mtw)), blk(512);
#define WDR_RW(MTV)                                                                                        \
  if (ln) wdr_launch(prof, bytes, flops, k_skinny<EPI, MTV, 2, 8, true>, grid, blk, skinny_ln_lds<EPI, MTV, 2, 8>(a.K), s, a); \
  else wdr_launch(prof, bytes, flops, k_skinny<EPI, MTV, 2, 8>, grid, blk, 0, s, a);
  if (mtw == 1) { WDR_RW(1) }
  else if (mtw == 2) { WDR_RW(2) }
  else if (mtw == 3) { WDR_RW(3) }
  else { WDR_RW(4) }
#undef WDR_RW
}

static void launch_rows(const ProjArgs& a, hipStream_t s) {
  WDR_CHECK(a.K % 32 == 0 && a.lda % 8 == 0 && a.ldb % 8 == 0, "row projection: K % 32, lda / ldb % 8");
  // LN prologue: every workgroup normalises only its own <= 32 rows (any M)
  WDR_CHECK(!a.ln_x || (a.K <= 1280 && a.K % 128 == 0), "row projection LN prologue: K <= 1280, K % 128 == 0");
  WDR_CHECK(a.epi != EPI_QKV_CACHE || (a.kc && a.vc && a.row_seq && a.row_pos && a.d > 0), "qkv-cache epilogue args");
  switch (a.epi) {
    case EPI_F16: launch_rows_epi<EPI_F16>(a, s); break;
    case EPI_F16_GELU: launch_rows_epi<EPI_F16_GELU>(a, s); break;
    case EPI_F32_RESID: launch_rows_epi<EPI_F32_RESID>(a, s); break;
    case EPI_F32: launch_rows_epi<EPI_F32>(a, s); break;
    case EPI_QKV_CACHE: launch_rows_epi<EPI_QKV_CACHE>(a, s); break;
    default: throw std::runtime_error("row projection: bad epilogue");
  }
  WDR_HIP(hipGetLastError());
}

void launch_proj(const ProjArgs& a, hipStream_t s) {
  WDR_CHECK(a.M > 0 && a.K > 0 && a.N > 0, "projection: empty shape");
  // decoder rows (any count, rows_mma) and every other projection of <= 64 rows run on the row
  // kernel; the encoder's M > 64 GEMMs on the MFMA tile family
  if (a.rows_mma || a.M <= 64) {
    launch_rows(a, s);
    return;
  }
  WDR_CHECK(a.K % 8 == 0 && a.lda % 8 == 0 && a.ldb % 8 == 0, "projection: K/lda/ldb must be multiples of 8");
  WDR_CHECK(a.N % GB_N == 0, "gemm: N must be a multiple of 128");
  WDR_CHECK(a.K % GB_K == 0, "gemm: K must be a multiple of 32");
  WDR_CHECK(a.epi != EPI_QKV_CACHE || (a.kc && a.vc && a.row_seq && a.row_pos && a.d > 0), "qkv-cache epilogue args");
  switch (a.epi) {
    case EPI_F16: launch_epi<EPI_F16>(a, s); break;
    case EPI_F16_GELU: launch_epi<EPI_F16_GELU>(a, s); break;
    case EPI_F32_RESID: launch_epi<EPI_F32_RESID>(a, s); break;
    case EPI_F32: launch_epi<EPI_F32>(a, s); break;
    case EPI_F32_GELU_POS: launch_epi<EPI_F32_GELU_POS>(a, s); break;
    case EPI_QKV_CACHE: launch_epi<EPI_QKV_CACHE>(a, s); break;
    case EPI_XKV:
      WDR_CHECK(a.M > 64 && a.seq_stride > 0, "cross-K/V epilogue: encoder GEMM rows and a slot stride");
      launch_epi<EPI_XKV>(a, s);
      break;
    default: throw std::runtime_error("projection: bad epilogue");
  }
  WDR_HIP(hipGetLastError());
}

}  // namespace wdr
