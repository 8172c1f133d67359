// Projection kernels: the dense contractions of the Whisper encoder / decoder
// (SURVEY.md §8(a) a5-a7, a9, a12).
//
//  * k_gemm  — MFMA GEMM for M > 8 rows (encoder windows, cross-K/V, prompt prefill,
//              DTW re-forward):  C[M][N] = A[M][K] . B[N][K]^T  (+ fused epilogue).
//              f16 operands (what ggml's mul_mat feeds: f16 weights, activations cast to
//              f16), f32 accumulation, v_mfma_f32_32x32x16_f16.  128x128x32 block tile,
//              4 waves of 64x64, register-staged double-buffered LDS, row padding for
//              conflict-free ds_read_b128.  Roofline: MFMA (2.5 PF/s dense f16).
//  * k_gemv  — M <= 8 rows (decoder step, one row per decoder): each wave streams one
//              weight row with 16-B loads, v_dot2_f32_f16, wave-shuffle reduction.
//              Roofline: HBM (bytes = N*K*2 per launch).
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
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[i], bf[j], acc[i][j], 0, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
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
  const f16* ga[2][2];   // [half][piece]; rows past M read row M - 1
  const f16* gb[2];      // [piece]; BH1 = BH0 + 32 rows
#pragma unroll
  for (int jj = 0; jj < 2; ++jj) {
    const int qa = (2 * wid + jj) * 8 + (lane >> 3);
    const int ca = g2_swz(qa, lane & 7);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      int gm = bm * G3_M + (qa >> 6) * 128 + 64 * h + (qa & 63);
      gm = gm < a.M ? gm : a.M - 1;
      ga[h][jj] = a.A + (size_t)gm * a.lda + ca * 8;
    }
    const int gn = bn * G3_N + (qa >> 5) * 64 + (qa & 31);
    gb[jj] = a.B + (size_t)gn * a.ldb + ca * 8;
  }
  const size_t b_half = (size_t)32 * a.ldb;
  auto stage = [&](int buf, int half, int k0) {   // half: 0 AH0, 1 AH1, 2 BH0, 3 BH1
    f16* dst = lds4 + (buf * 4 + half) * G4_HALF + (2 * wid) * 512;
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
      const f16* src = half < 2 ? ga[half][jj] + k0 : gb[jj] + (half - 2) * b_half + k0;
      __builtin_amdgcn_global_load_lds((const void*)src, (void*)(dst + jj * 512), 16, 0, 0);
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
              __builtin_amdgcn_mfma_f32_16x16x32_f16(af[ks][i], bf[ks][j], acc[qa * 4 + i][qb * 2 + j], 0, 0, 0);
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

#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = bm * G3_M + grp * 128 + i * 16 + fq * 4 + r;
        const int col = bn * G3_N + wn * 64 + j * 16 + fr;
        epi_store<EPI>(a, row, col, acc[i][j][r]);
      }
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
  const f16* ga[2][2];
  const f16* gb[2];
#pragma unroll
  for (int jj = 0; jj < 2; ++jj) {
    const int qa = (2 * wid + jj) * 8 + (lane >> 3);
    const int ca = g2_swz(qa, lane & 7);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      int gm = bm * G3_M + (qa >> 6) * 128 + 64 * h + (qa & 63);
      gm = gm < a.M ? gm : a.M - 1;
      ga[h][jj] = a.A + (size_t)gm * a.lda + ca * 8;
    }
    gb[jj] = a.B + (size_t)(bn * 128 + qa) * a.ldb + ca * 8;
  }
  auto stage = [&](int buf, int half, int k0) {   // half: 0 AH0, 1 AH1, 2 BT
    f16* dst = lds5 + (buf * 3 + half) * G4_HALF + (2 * wid) * 512;
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
      const f16* src = half < 2 ? ga[half][jj] + k0 : gb[jj] + k0;
      __builtin_amdgcn_global_load_lds((const void*)src, (void*)(dst + jj * 512), 16, 0, 0);
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
          acc[qa * 4 + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[ks][i], bf[ks][j], acc[qa * 4 + i][j], 0, 0, 0);
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

#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = bm * G3_M + grp * 128 + i * 16 + fq * 4 + r;
        const int col = bn * 128 + wn * 32 + j * 16 + fr;
        epi_store<EPI>(a, row, col, acc[i][j][r]);
      }
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


// ---------------------------------------------------------------- fp8 (e4m3) MFMA GEMM
// The encoder GEMMs of BASELINE configs[4]: k_gemm3's structure (8 waves of 128 x BN/4, operand
// tiles staged by global_load_lds into two LDS buffers, g2_swz source swizzle, XCD-aware tile
// order) on fp8 operands: a K-tile is 128 k = 128 B per row (the bytes of k_gemm3's f16 BK = 64
// tile), one v_mfma_scale_f32_16x16x128_f8f6f4 per 16 x 16 output tile and K-tile -- the
// block-scaled form runs twice the f16 MFMA rate (MI355X_MICROARCH.md, matrix cores); its
// block scales are all 1 (E8M0 127) and the per-row / per-channel scales of the quantisation
// are applied in the epilogue.  Lane l holds bytes 32 (l >> 4) .. +32 of row (l & 15) of both
// operands: the same k for A and B, so the dot product is that of the rows whatever k order the
// hardware sums them in.  BN = 128 for the N = d projections (o, fc2), so M = 6000 fills 240
// tiles, BN = 256 otherwise.
typedef int i32x8 __attribute__((ext_vector_type(8)));
constexpr int G8_M = 256, G8_BK = 128;

template <int EPI, int BN>
__global__ __launch_bounds__(512, 1) void k_gemm8(ProjArgs a) {
  ProfClock prof_clock_(a.ts);   // sampled launches only (csrc/prof.cpp)
  extern __shared__ __attribute__((aligned(16))) uint8_t lds8[];   // [buf][A 256 x 128 B, B BN x 128 B]
  constexpr int NJ = BN / 64;          // 16-column tiles per wave
  constexpr int BI = BN / 64;          // B DMA instructions (8 rows each) per wave
  constexpr int BUF = (G8_M + BN) * G8_BK;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int q = nwg / 8, rr = nwg % 8, xcd = orig % 8;
  const int id = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + orig / 8;
  const int ntn = a.N / BN;
  const int bm = id / ntn, bn = id % ntn;
  const int wm = wid >> 2, wn = wid & 3;
  const uint8_t* ga[4];
  const uint8_t* gb[BI];
#pragma unroll
  for (int jj = 0; jj < 4; ++jj) {
    const int row = (wid * 4 + jj) * 8 + (lane >> 3);
    const int c = g2_swz(row, lane & 7);
    int gm = bm * G8_M + row;
    gm = gm < a.M ? gm : a.M - 1;
    ga[jj] = a.A8 + (size_t)gm * a.lda + c * 16;
  }
#pragma unroll
  for (int jj = 0; jj < BI; ++jj) {
    const int row = (wid * BI + jj) * 8 + (lane >> 3);
    const int c = g2_swz(row, lane & 7);
    gb[jj] = a.B8 + (size_t)(bn * BN + row) * a.ldb + c * 16;
  }
  auto stage = [&](int buf, int k0) {
#pragma unroll
    for (int jj = 0; jj < 4; ++jj)
      __builtin_amdgcn_global_load_lds((const void*)(ga[jj] + k0), (void*)(lds8 + buf * BUF + (wid * 4 + jj) * 1024),
                                       16, 0, 0);
#pragma unroll
    for (int jj = 0; jj < BI; ++jj)
      __builtin_amdgcn_global_load_lds((const void*)(gb[jj] + k0),
                                       (void*)(lds8 + buf * BUF + G8_M * G8_BK + (wid * BI + jj) * 1024), 16, 0, 0);
  };
  const int nk = a.K / G8_BK;
  stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();

  f32x4 acc[8][NJ];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fq = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) stage(cur ^ 1, (kt + 1) * G8_BK);
    const uint8_t* As = lds8 + cur * BUF;
    const uint8_t* Bs = As + G8_M * G8_BK;
    i32x8 bf[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int r = wn * (BN / 4) + j * 16 + fr;
      const int4 lo = *(const int4*)(Bs + r * G8_BK + g2_swz(r, 2 * fq) * 16);
      const int4 hi = *(const int4*)(Bs + r * G8_BK + g2_swz(r, 2 * fq + 1) * 16);
      bf[j] = i32x8{lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int r = wm * 128 + i * 16 + fr;
      const int4 lo = *(const int4*)(As + r * G8_BK + g2_swz(r, 2 * fq) * 16);
      const int4 hi = *(const int4*)(As + r * G8_BK + g2_swz(r, 2 * fq + 1) * 16);
      const i32x8 af = i32x8{lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
#pragma unroll
      for (int j = 0; j < NJ; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(af, bf[j], acc[i][j], 0, 0, 0, 0x7f7f7f7f, 0,
                                                                      0x7f7f7f7f);
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }

#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = bm * G8_M + wm * 128 + i * 16 + fq * 4 + r;
      const float xs = row < a.M ? a.a_scale[row] : 0.f;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int col = bn * BN + wn * (BN / 4) + j * 16 + fr;
        epi_store<EPI>(a, row, col, acc[i][j][r] * xs * a.b_scale[col]);
      }
    }
}

template <int EPI>
static void launch_epi8(const ProjArgs& a, hipStream_t s) {
  const double bytes = (double)a.N * a.K + (double)a.M * a.K + (double)a.M * a.N * 2;
  const double flops = 2.0 * a.M * a.N * a.K;
  const bool narrow = a.N % 256 != 0 || a.N <= 2048;
  const uint32_t lds = 2u * (G8_M + (narrow ? 128u : 256u)) * G8_BK;
  static bool attr = [] {
    WDR_HIP(hipFuncSetAttribute((const void*)k_gemm8<EPI, 128>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                2 * (G8_M + 128) * G8_BK));
    WDR_HIP(hipFuncSetAttribute((const void*)k_gemm8<EPI, 256>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                2 * (G8_M + 256) * G8_BK));
    return true;
  }();
  (void)attr;
  if (narrow) {
    dim3 grid((a.N / 128) * cdiv(a.M, G8_M));
    wdr_launch(PROF_GEMM, bytes, flops, k_gemm8<EPI, 128>, grid, dim3(512), lds, s, a);
  } else {
    dim3 grid((a.N / 256) * cdiv(a.M, G8_M));
    wdr_launch(PROF_GEMM, bytes, flops, k_gemm8<EPI, 256>, grid, dim3(512), lds, s, a);
  }
}

void launch_proj_fp8(const ProjArgs& a, hipStream_t s) {
  WDR_CHECK(a.A8 && a.B8 && a.a_scale && a.b_scale, "fp8 projection: operands / scales missing");
  WDR_CHECK(a.M > 64 && a.N % 128 == 0 && a.K % G8_BK == 0 && a.lda % 16 == 0 && a.ldb % 16 == 0,
            "fp8 projection: M > 64, N % 128 == 0, K % 128 == 0 required");
  switch (a.epi) {
    case EPI_F16: launch_epi8<EPI_F16>(a, s); break;
    case EPI_F16_GELU: launch_epi8<EPI_F16_GELU>(a, s); break;
    case EPI_F32_RESID: launch_epi8<EPI_F32_RESID>(a, s); break;
    case EPI_F32: launch_epi8<EPI_F32>(a, s); break;
    case EPI_XKV: launch_epi8<EPI_XKV>(a, s); break;
    default: throw std::runtime_error("fp8 projection: unsupported epilogue");
  }
  WDR_HIP(hipGetLastError());
}

// one workgroup per row: max |x| -> scale = amax / 448 (e4m3's largest finite value), then
// the row scaled by 448 / amax, rounded to nearest-even e4m3 (v_cvt_pk_fp8_f32, OCP e4m3fn)
__global__ __launch_bounds__(256) void k_quant_rows(const f16* x, int ldx, int K, uint8_t* y, int ldy, float* scale) {
  __shared__ float red[4];
  const int r = blockIdx.x, tid = threadIdx.x;
  const f16* xr = x + (size_t)r * ldx;
  float am = 0.f;
  for (int c = tid * 8; c < K; c += 2048) {
    const f16x8 v = *(const f16x8*)(xr + c);
#pragma unroll
    for (int e = 0; e < 8; ++e) am = fmaxf(am, fabsf((float)v[e]));
  }
  am = wave_max(am);
  if ((tid & 63) == 0) red[tid >> 6] = am;
  __syncthreads();
  am = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  const float inv = am > 0.f ? 448.f / am : 1.f;
  if (tid == 0) scale[r] = am > 0.f ? am / 448.f : 1.f;
  uint8_t* yr = y + (size_t)r * ldy;
  for (int c = tid * 8; c < K; c += 2048) {
    const f16x8 v = *(const f16x8*)(xr + c);
    unsigned lo = 0, hi = 0;
    lo = __builtin_amdgcn_cvt_pk_fp8_f32((float)v[0] * inv, (float)v[1] * inv, lo, false);
    lo = __builtin_amdgcn_cvt_pk_fp8_f32((float)v[2] * inv, (float)v[3] * inv, lo, true);
    hi = __builtin_amdgcn_cvt_pk_fp8_f32((float)v[4] * inv, (float)v[5] * inv, hi, false);
    hi = __builtin_amdgcn_cvt_pk_fp8_f32((float)v[6] * inv, (float)v[7] * inv, hi, true);
    *(uint2*)(yr + c) = make_uint2(lo, hi);
  }
}

void launch_quant_rows(const f16* x, int ldx, int M, int K, uint8_t* y, int ldy, float* scale, hipStream_t s) {
  WDR_CHECK(M >= 1 && K % 8 == 0 && ldx % 8 == 0 && ldy % 8 == 0, "fp8 quantisation: K, ld must be multiples of 8");
  WDR_KLAUNCH(k_quant_rows, dim3(M), dim3(256), 0, s, x, ldx, K, y, ldy, scale);
  WDR_HIP(hipGetLastError());
}

// ---------------------------------------------------------------- GEMV (M <= 8)
// Grid-stride over output rows (one weight row per wave per iteration), 16-B weight loads,
// v_dot2_f32_f16.  With the fused LayerNorm prologue (LN, K <= 1536) every wave normalises
// its input rows itself, straight into the registers that hold exactly the K-slices its lane
// multiplies (lane l owns k in [512 i + 8 l, +8)): one round of loads, no LDS, no barrier.
template <int NCH>
__device__ __forceinline__ void ln_row_regs(const ProjArgs& a, int r, int lane, f16x8 (&xo)[NCH]) {
  const float* xr = a.ln_x + (size_t)r * a.ldln;
  float v[NCH][8];
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int k = c * 512 + lane * 8;
    if (k < a.K) {
      const float4 p0 = *(const float4*)(xr + k), p1 = *(const float4*)(xr + k + 4);
      v[c][0] = p0.x; v[c][1] = p0.y; v[c][2] = p0.z; v[c][3] = p0.w;
      v[c][4] = p1.x; v[c][5] = p1.y; v[c][6] = p1.z; v[c][7] = p1.w;
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[c][e] = 0.f;
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) s += v[c][e];
  }
  s = wave_sum(s);
  const float mean = s / a.K;
  float s2 = 0.f;
#pragma unroll
  for (int c = 0; c < NCH; ++c)
    if (c * 512 + lane * 8 < a.K)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float t = v[c][e] - mean;
        s2 += t * t;
      }
  s2 = wave_sum(s2);
  const float scale = 1.0f / sqrtf(s2 / a.K + 1e-5f);
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int k = c * 512 + lane * 8;
    if (k < a.K) {
      const float4 g0 = *(const float4*)(a.ln_g + k), g1 = *(const float4*)(a.ln_g + k + 4);
      const float4 b0 = *(const float4*)(a.ln_b + k), b1 = *(const float4*)(a.ln_b + k + 4);
      const float gg[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
      const float bb[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
      for (int e = 0; e < 8; ++e) xo[c][e] = (f16)((v[c][e] - mean) * scale * gg[e] + bb[e]);
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) xo[c][e] = (f16)0.f;
    }
  }
}

__device__ __forceinline__ float dot8(f16x8 w, f16x8 x, float s) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    f16x2 wp = {w[2 * q], w[2 * q + 1]};
    f16x2 xp = {x[2 * q], x[2 * q + 1]};
    s = __builtin_amdgcn_fdot2(wp, xp, s, false);
  }
  return s;
}

template <int EPI, int MR>
__device__ __forceinline__ void gemv_store(const ProjArgs& a, float (&acc)[MR], int lane, int n) {
#pragma unroll
  for (int r = 0; r < MR; ++r) acc[r] = wave_sum(acc[r]);
  if (lane < MR && lane < a.M) {
    float v = 0.f;
#pragma unroll
    for (int r = 0; r < MR; ++r)
      if (r == lane) v = acc[r];
    epi_store<EPI>(a, lane, n, v);
  }
}

// Decode GEMV for M <= 2 (the hot path of every greedy step): each wave owns R consecutive
// weight rows and issues ALL of their loads before anything else, then (optionally) the
// LayerNorm of the activation rows -- computed once per wave and amortised over its R rows,
// its latency hidden under the weight stream -- then the dot products and the fused epilogue.
// grid = ceil(N / 4R), one pass, no grid-stride loop.
template <int EPI, int MR, int R, int NCH, bool LN>
__global__ __launch_bounds__(256) void k_dgemv(ProjArgs a) {
  ProfClock prof_clock_(a.ts);   // sampled launches only (csrc/prof.cpp)
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int n0 = (blockIdx.x * 4 + wid) * R;
  const int K = a.K, M = a.M;
  // Every load below is unconditional (clamped address, masked value): no exec-mask branch
  // per load, so the whole batch issues back to back.
  int kc[NCH];
  bool kin[NCH];
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int k = c * 512 + lane * 8;
    kin[c] = k < K;
    kc[c] = kin[c] ? k : K - 8;
  }
  // 1. activations (+ LayerNorm parameters) first: they are L2 hits, and the in-order return of
  //    vector loads means the LayerNorm can then run while the weight stream is in flight
  float xf[LN ? MR : 1][LN ? NCH : 1][8];
  float gv[LN ? NCH : 1][8], bv[LN ? NCH : 1][8];
  f16x8 xr[MR][NCH];
#pragma unroll
  for (int m = 0; m < MR; ++m) {
    const int mm = m < M ? m : M - 1;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      if constexpr (LN) {
        const float* xs = a.ln_x + (size_t)mm * a.ldln + kc[c];
        const float4 p0 = *(const float4*)xs, p1 = *(const float4*)(xs + 4);
        xf[m][c][0] = p0.x; xf[m][c][1] = p0.y; xf[m][c][2] = p0.z; xf[m][c][3] = p0.w;
        xf[m][c][4] = p1.x; xf[m][c][5] = p1.y; xf[m][c][6] = p1.z; xf[m][c][7] = p1.w;
        if (!kin[c])
#pragma unroll
          for (int e = 0; e < 8; ++e) xf[m][c][e] = 0.f;
      } else {
        const f16x8 t = *(const f16x8*)(a.A + (size_t)mm * a.lda + kc[c]);
        xr[m][c] = kin[c] ? t : (f16x8){};
      }
    }
  }
  if constexpr (LN) {
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const float4 g0 = *(const float4*)(a.ln_g + kc[c]), g1 = *(const float4*)(a.ln_g + kc[c] + 4);
      const float4 b0 = *(const float4*)(a.ln_b + kc[c]), b1 = *(const float4*)(a.ln_b + kc[c] + 4);
      gv[c][0] = g0.x; gv[c][1] = g0.y; gv[c][2] = g0.z; gv[c][3] = g0.w;
      gv[c][4] = g1.x; gv[c][5] = g1.y; gv[c][6] = g1.z; gv[c][7] = g1.w;
      bv[c][0] = b0.x; bv[c][1] = b0.y; bv[c][2] = b0.z; bv[c][3] = b0.w;
      bv[c][4] = b1.x; bv[c][5] = b1.y; bv[c][6] = b1.z; bv[c][7] = b1.w;
    }
  }
  // 2. the weight stream: every load of the wave's R rows in flight at once
  f16x8 wv[R][NCH];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int n = n0 + r < a.N ? n0 + r : a.N - 1;
    const f16* w = a.B + (size_t)n * a.ldb;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const f16x8 t = *(const f16x8*)(w + kc[c]);
      wv[r][c] = kin[c] ? t : (f16x8){};
    }
  }
  const int mrow = lane < M ? lane : 0;   // lane m stores output row m
  float pbias[R], pold[R];
  long long cdst = 0;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int n = n0 + r < a.N ? n0 + r : a.N - 1;
    pbias[r] = a.bias ? a.bias[n] : 0.f;
    pold[r] = 0.f;
    if constexpr (EPI == EPI_F32_RESID) pold[r] = ((const float*)a.out)[(size_t)mrow * a.ldo + n];
  }
  if constexpr (EPI == EPI_QKV_CACHE) cdst = a.row_seq[mrow] * a.seq_stride + (long long)a.row_pos[mrow] * a.d;
  // 3. LayerNorm (ggml_norm, eps 1e-5) once per wave, amortised over its R rows
  if constexpr (LN) {
#pragma unroll
    for (int m = 0; m < MR; ++m) {
      float sm = 0.f;
#pragma unroll
      for (int c = 0; c < NCH; ++c)
#pragma unroll
        for (int e = 0; e < 8; ++e) sm += xf[m][c][e];
      sm = wave_sum(sm);
      const float mean = sm / a.K;
      float s2 = 0.f;
#pragma unroll
      for (int c = 0; c < NCH; ++c)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float t = xf[m][c][e] - mean;
          s2 += kin[c] ? t * t : 0.f;
        }
      s2 = wave_sum(s2);
      const float scale = 1.0f / sqrtf(s2 / a.K + 1e-5f);
#pragma unroll
      for (int c = 0; c < NCH; ++c)
#pragma unroll
        for (int e = 0; e < 8; ++e) xr[m][c][e] = (f16)((xf[m][c][e] - mean) * scale * gv[c][e] + bv[c][e]);
    }
  }
  // 4. dot products, wave reductions, fused epilogue
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int n = n0 + r;
    float acc[MR];
#pragma unroll
    for (int m = 0; m < MR; ++m) {
      acc[m] = 0.f;
#pragma unroll
      for (int c = 0; c < NCH; ++c) acc[m] = dot8(wv[r][c], xr[m][c], acc[m]);
      acc[m] = wave_sum(acc[m]);
    }
    if (n >= a.N || lane >= MR || lane >= a.M) continue;
    float v = acc[0];
#pragma unroll
    for (int m = 1; m < MR; ++m)
      if (lane == m) v = acc[m];
    v += pbias[r];
    const size_t o = (size_t)lane * a.ldo + n;
    if constexpr (EPI == EPI_F16) {
      ((f16*)a.out)[o] = (f16)v;
    } else if constexpr (EPI == EPI_F16_GELU) {
      ((f16*)a.out)[o] = (f16)gelu_tanh(v);
    } else if constexpr (EPI == EPI_F32_RESID) {
      ((float*)a.out)[o] = pold[r] + v;
    } else if constexpr (EPI == EPI_F32) {
      ((float*)a.out)[o] = v;
    } else if constexpr (EPI == EPI_QKV_CACHE) {
      if (n < a.d) ((f16*)a.out)[o] = (f16)v;
      else if (n < 2 * a.d) a.kc[cdst + n - a.d] = (f16)v;
      else a.vc[cdst + n - 2 * a.d] = (f16)v;
    } else {
      epi_store<EPI>(a, lane, n, v - pbias[r]);
    }
  }
}

// Decode GEMV for 2 < M <= 8 rows (the multi-chain batched step, whisper_ctx.cpp StepBatcher):
// k_dgemv's weight stream (each wave owns R weight rows, every load issued up front) with the
// activation rows shared through LDS instead of registers.  With the LayerNorm prologue, wave w
// normalises rows w, w+4 (the same arithmetic as k_dgemv, so every row's result is bit-identical
// to the 1-row step's: multi-chain decoding equals one chain exactly) into LDS; without it the
// rows are read per 512-wide chunk from L2.  Per (weight row, activation row) the dot product
// runs over the chunks in the same order as k_dgemv, then the same wave reduction.
template <int EPI, int MR, int R, int NCH, bool LN>
__global__ __launch_bounds__(256) void k_mgemv(ProjArgs a) {
  ProfClock prof_clock_(a.ts);   // sampled launches only (csrc/prof.cpp)
  constexpr int KP = NCH * 512;
  constexpr int LR = LN ? (MR + 3) / 4 : 1;   // LayerNorm rows per wave
  extern __shared__ __attribute__((aligned(16))) f16 xsh[];   // LN: [MR][KP] normalised rows
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int n0 = (blockIdx.x * 4 + wid) * R;
  const int K = a.K, M = a.M;
  int kc[NCH];
  bool kin[NCH];
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int k = c * 512 + lane * 8;
    kin[c] = k < K;
    kc[c] = kin[c] ? k : K - 8;
  }
  // 1. this wave's LayerNorm rows (+ gamma / beta) first, then the weight stream
  float xf[LR][LN ? NCH : 1][8];
  float gv[LN ? NCH : 1][8], bv[LN ? NCH : 1][8];
  if constexpr (LN) {
#pragma unroll
    for (int j = 0; j < LR; ++j) {
      const int m = wid + 4 * j;
      const int mm = m < M ? m : M - 1;
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
        const float* xs = a.ln_x + (size_t)mm * a.ldln + kc[c];
        const float4 p0 = *(const float4*)xs, p1 = *(const float4*)(xs + 4);
        xf[j][c][0] = p0.x; xf[j][c][1] = p0.y; xf[j][c][2] = p0.z; xf[j][c][3] = p0.w;
        xf[j][c][4] = p1.x; xf[j][c][5] = p1.y; xf[j][c][6] = p1.z; xf[j][c][7] = p1.w;
        if (!kin[c])
#pragma unroll
          for (int e = 0; e < 8; ++e) xf[j][c][e] = 0.f;
      }
    }
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const float4 g0 = *(const float4*)(a.ln_g + kc[c]), g1 = *(const float4*)(a.ln_g + kc[c] + 4);
      const float4 b0 = *(const float4*)(a.ln_b + kc[c]), b1 = *(const float4*)(a.ln_b + kc[c] + 4);
      gv[c][0] = g0.x; gv[c][1] = g0.y; gv[c][2] = g0.z; gv[c][3] = g0.w;
      gv[c][4] = g1.x; gv[c][5] = g1.y; gv[c][6] = g1.z; gv[c][7] = g1.w;
      bv[c][0] = b0.x; bv[c][1] = b0.y; bv[c][2] = b0.z; bv[c][3] = b0.w;
      bv[c][4] = b1.x; bv[c][5] = b1.y; bv[c][6] = b1.z; bv[c][7] = b1.w;
    }
  }
  f16x8 wv[R][NCH];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int n = n0 + r < a.N ? n0 + r : a.N - 1;
    const f16* w = a.B + (size_t)n * a.ldb;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const f16x8 t = *(const f16x8*)(w + kc[c]);
      wv[r][c] = kin[c] ? t : (f16x8){};
    }
  }
  const int mrow = lane < M ? lane : 0;   // lane m stores output row m
  float pbias[R], pold[R];
  long long cdst = 0;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int n = n0 + r < a.N ? n0 + r : a.N - 1;
    pbias[r] = a.bias ? a.bias[n] : 0.f;
    pold[r] = 0.f;
    if constexpr (EPI == EPI_F32_RESID) pold[r] = ((const float*)a.out)[(size_t)mrow * a.ldo + n];
  }
  if constexpr (EPI == EPI_QKV_CACHE) cdst = a.row_seq[mrow] * a.seq_stride + (long long)a.row_pos[mrow] * a.d;
  // 2. LayerNorm (ggml_norm, eps 1e-5; k_dgemv's arithmetic) into LDS
  if constexpr (LN) {
#pragma unroll
    for (int j = 0; j < LR; ++j) {
      const int m = wid + 4 * j;
      float sm = 0.f;
#pragma unroll
      for (int c = 0; c < NCH; ++c)
#pragma unroll
        for (int e = 0; e < 8; ++e) sm += xf[j][c][e];
      sm = wave_sum(sm);
      const float mean = sm / a.K;
      float s2 = 0.f;
#pragma unroll
      for (int c = 0; c < NCH; ++c)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float t = xf[j][c][e] - mean;
          s2 += kin[c] ? t * t : 0.f;
        }
      s2 = wave_sum(s2);
      const float scale = 1.0f / sqrtf(s2 / a.K + 1e-5f);
      if (m < MR) {
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
          f16x8 o;
#pragma unroll
          for (int e = 0; e < 8; ++e) o[e] = (f16)((xf[j][c][e] - mean) * scale * gv[c][e] + bv[c][e]);
          *(f16x8*)(xsh + m * KP + c * 512 + lane * 8) = o;
        }
      }
    }
    __syncthreads();
  }
  // 3. dot products chunk by chunk (activation rows from LDS / L2), reductions, epilogue
  float acc[R][MR];
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int m = 0; m < MR; ++m) acc[r][m] = 0.f;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    f16x8 xv[MR];
#pragma unroll
    for (int m = 0; m < MR; ++m) {
      if constexpr (LN) {
        xv[m] = *(const f16x8*)(xsh + m * KP + c * 512 + lane * 8);
      } else {
        const int mm = m < M ? m : M - 1;
        const f16x8 t = *(const f16x8*)(a.A + (size_t)mm * a.lda + kc[c]);
        xv[m] = kin[c] ? t : (f16x8){};
      }
    }
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int m = 0; m < MR; ++m) acc[r][m] = dot8(wv[r][c], xv[m], acc[r][m]);
  }
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int n = n0 + r;
#pragma unroll
    for (int m = 0; m < MR; ++m) acc[r][m] = wave_sum(acc[r][m]);
    if (n >= a.N || lane >= MR || lane >= a.M) continue;
    float v = acc[r][0];
#pragma unroll
    for (int m = 1; m < MR; ++m)
      if (lane == m) v = acc[r][m];
    v += pbias[r];
    const size_t o = (size_t)lane * a.ldo + n;
    if constexpr (EPI == EPI_F16) {
      ((f16*)a.out)[o] = (f16)v;
    } else if constexpr (EPI == EPI_F16_GELU) {
      ((f16*)a.out)[o] = (f16)gelu_tanh(v);
    } else if constexpr (EPI == EPI_F32_RESID) {
      ((float*)a.out)[o] = pold[r] + v;
    } else if constexpr (EPI == EPI_F32) {
      ((float*)a.out)[o] = v;
    } else if constexpr (EPI == EPI_QKV_CACHE) {
      if (n < a.d) ((f16*)a.out)[o] = (f16)v;
      else if (n < 2 * a.d) a.kc[cdst + n - a.d] = (f16)v;
      else a.vc[cdst + n - 2 * a.d] = (f16)v;
    } else {
      epi_store<EPI>(a, lane, n, v - pbias[r]);
    }
  }
}


// LayerNorm of decode-step rows into f16 with k_dgemv's in-register arithmetic (same per-lane
// chunk order, sums and masks), so a GEMV over these rows gives exactly what the fused-LN GEMV
// gives.  One wave per row.  Used for 9..16-row steps, where recomputing the LayerNorm of every
// row in every GEMV workgroup (k_mgemv's LN prologue) costs more L2 traffic than the weights.
template <int NCH>
__global__ __launch_bounds__(64) void k_ln_rows(ProjArgs a, f16* y, int ldy) {
  const int lane = threadIdx.x, row = blockIdx.x;
  const int K = a.K;
  int kc[NCH];
  bool kin[NCH];
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int k = c * 512 + lane * 8;
    kin[c] = k < K;
    kc[c] = kin[c] ? k : K - 8;
  }
  float xf[NCH][8], gv[NCH][8], bv[NCH][8];
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const float* xs = a.ln_x + (size_t)row * a.ldln + kc[c];
    const float4 p0 = *(const float4*)xs, p1 = *(const float4*)(xs + 4);
    xf[c][0] = p0.x; xf[c][1] = p0.y; xf[c][2] = p0.z; xf[c][3] = p0.w;
    xf[c][4] = p1.x; xf[c][5] = p1.y; xf[c][6] = p1.z; xf[c][7] = p1.w;
    if (!kin[c])
#pragma unroll
      for (int e = 0; e < 8; ++e) xf[c][e] = 0.f;
    const float4 g0 = *(const float4*)(a.ln_g + kc[c]), g1 = *(const float4*)(a.ln_g + kc[c] + 4);
    const float4 b0 = *(const float4*)(a.ln_b + kc[c]), b1 = *(const float4*)(a.ln_b + kc[c] + 4);
    gv[c][0] = g0.x; gv[c][1] = g0.y; gv[c][2] = g0.z; gv[c][3] = g0.w;
    gv[c][4] = g1.x; gv[c][5] = g1.y; gv[c][6] = g1.z; gv[c][7] = g1.w;
    bv[c][0] = b0.x; bv[c][1] = b0.y; bv[c][2] = b0.z; bv[c][3] = b0.w;
    bv[c][4] = b1.x; bv[c][5] = b1.y; bv[c][6] = b1.z; bv[c][7] = b1.w;
  }
  float sm = 0.f;
#pragma unroll
  for (int c = 0; c < NCH; ++c)
#pragma unroll
    for (int e = 0; e < 8; ++e) sm += xf[c][e];
  sm = wave_sum(sm);
  const float mean = sm / a.K;
  float s2 = 0.f;
#pragma unroll
  for (int c = 0; c < NCH; ++c)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float t = xf[c][e] - mean;
      s2 += kin[c] ? t * t : 0.f;
    }
  s2 = wave_sum(s2);
  const float scale = 1.0f / sqrtf(s2 / a.K + 1e-5f);
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    if (!kin[c]) continue;
    f16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = (f16)((xf[c][e] - mean) * scale * gv[c][e] + bv[c][e]);
    *(f16x8*)(y + (size_t)row * ldy + kc[c]) = o;
  }
}

void launch_ln_rows(const ProjArgs& a, f16* y, int ldy, hipStream_t s) {
  WDR_CHECK(a.ln_x && a.K % 8 == 0 && a.K <= 1536, "step LayerNorm rows: K must be <= 1536");
  const int nch = cdiv(a.K, 512);
  if (nch == 1) WDR_KLAUNCH(k_ln_rows<1>, dim3(a.M), dim3(64), 0, s, a, y, ldy);
  else if (nch == 2) WDR_KLAUNCH(k_ln_rows<2>, dim3(a.M), dim3(64), 0, s, a, y, ldy);
  else WDR_KLAUNCH(k_ln_rows<3>, dim3(a.M), dim3(64), 0, s, a, y, ldy);
  WDR_HIP(hipGetLastError());
}

// Decode GEMV for 3..16 step rows without a LayerNorm prologue (o / xo / fc2, and every
// projection of a 9..16-row step after k_ln_rows): the workgroup stages its M activation rows
// into LDS once (issued before the weight stream, so the L2 reads overlap the HBM latency)
// instead of every wave re-reading all rows from L2, and the R x MR dot products of a wave
// are reduced with one reduce-scatter butterfly (V - 1 + log2(64 / V) shuffles instead of
// 6 V).  Per (weight row, activation row) the chunk order, dot8 order and the butterfly tree
// are those of k_dgemv / k_mgemv (each butterfly step adds the partner lane's partial of the
// same value), so every row's result is bit-identical to the 1-row step's.
template <int V, int O, int CNT>
__device__ __forceinline__ void reduce_scatter_step(float (&v)[V], int lane) {
  if constexpr (CNT > 1) {
    constexpr int H = CNT / 2;
    const bool up = (lane & O) != 0;
#pragma unroll
    for (int i = 0; i < H; ++i) {
      const float keep = up ? v[i + H] : v[i];
      const float send = up ? v[i] : v[i + H];
      v[i] = keep + __shfl_xor(send, O, 64);
    }
  } else {
    v[0] += __shfl_xor(v[0], O, 64);
  }
  if constexpr (O > 1) reduce_scatter_step<V, O / 2, (CNT > 1 ? CNT / 2 : 1)>(v, lane);
}
template <int V>
__device__ __forceinline__ float reduce_scatter(float (&v)[V], int lane) {
  static_assert(V >= 1 && V <= 64 && (V & (V - 1)) == 0, "V: power of two <= 64");
  reduce_scatter_step<V, 32, V>(v, lane);
  return v[0];   // the value index lane >> (6 - log2 V)
}

// NP > 1: the M <= MR * NP rows go through the LDS image MR at a time (pass p covers rows
// p*MR .. p*MR + MR - 1) with the wave's weight rows held in registers across the passes, so a
// K = 5120 projection (fc2) of a 9..16-row step streams its weights once from one launch
// within an 8-row LDS image; the next pass's rows are loaded while the current one is
// multiplied.  Per row, the arithmetic is that of the NP = 1 kernel.
template <int EPI, int MR, int R, int NCH, int NP = 1>
__global__ __launch_bounds__(256) void k_mgemv_s(ProjArgs a) {
  ProfClock prof_clock_(a.ts);   // sampled launches only (csrc/prof.cpp)
  constexpr int KP = NCH * 512, V = R * MR;
  constexpr int SH = V >= 64 ? 0 : V >= 32 ? 1 : V >= 16 ? 2 : V >= 8 ? 3 : V >= 4 ? 4 : V >= 2 ? 5 : 6;
  constexpr int NV = MR * KP / 8, PER = (NV + 255) / 256;
  extern __shared__ __attribute__((aligned(16))) f16 xsh[];   // [MR][KP] activation rows
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int n0 = (blockIdx.x * 4 + wid) * R;
  const int K = a.K, M = a.M;
  // 1. activation rows -> registers (zero past K, rows >= M not staged: their results are dropped)
  f16x8 t[PER];
  auto fetch = [&](int p) {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int v = i * 256 + threadIdx.x;
      const int m = v / (KP / 8) + p * MR, k = (v % (KP / 8)) * 8;
      t[i] = (v < NV && m < M && k < K) ? *(const f16x8*)(a.A + (size_t)m * a.lda + k) : (f16x8){};
    }
  };
  auto put = [&]() {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int v = i * 256 + threadIdx.x;
      if (v < NV) *(f16x8*)(xsh + (size_t)v * 8) = t[i];
    }
  };
  fetch(0);
  // 2. the weight stream, every load of the wave's R rows in flight at once
  int kc[NCH];
  bool kin[NCH];
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int k = c * 512 + lane * 8;
    kin[c] = k < K;
    kc[c] = kin[c] ? k : K - 8;
  }
  f16x8 wv[R][NCH];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int n = n0 + r < a.N ? n0 + r : a.N - 1;
    const f16* w = a.B + (size_t)n * a.ldb;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const f16x8 tw = *(const f16x8*)(w + kc[c]);
      wv[r][c] = kin[c] ? tw : (f16x8){};
    }
  }
  put();
  // epilogue operands of the (weight row, activation row) this lane stores, per pass
  const int j = lane >> SH, jr = j / MR, jm = j % MR;
  const bool lead = (lane & ((1 << SH) - 1)) == 0 && n0 + jr < a.N;
  const int nst = n0 + jr < a.N ? n0 + jr : a.N - 1;
  const float pbias = a.bias ? a.bias[nst] : 0.f;
  float pold[NP];
  long long cdst[NP];
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    const int mr = jm + p * MR, mst = mr < M ? mr : 0;
    pold[p] = 0.f;
    cdst[p] = 0;
    if constexpr (EPI == EPI_F32_RESID) pold[p] = ((const float*)a.out)[(size_t)mst * a.ldo + nst];
    if constexpr (EPI == EPI_QKV_CACHE) cdst[p] = a.row_seq[mst] * a.seq_stride + (long long)a.row_pos[mst] * a.d;
  }
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    if (p > 0) {
      __syncthreads();   // every wave is done with the previous pass's rows
      put();
    }
    if (p + 1 < NP) fetch(p + 1);   // in flight while this pass is multiplied
    __syncthreads();
    // 3. dot products chunk by chunk (k_mgemv's order), one reduce-scatter, fused epilogue
    float acc[V];
#pragma unroll
    for (int i = 0; i < V; ++i) acc[i] = 0.f;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
#pragma unroll
      for (int m = 0; m < MR; ++m) {
        const f16x8 xv = *(const f16x8*)(xsh + m * KP + c * 512 + lane * 8);
#pragma unroll
        for (int r = 0; r < R; ++r) acc[r * MR + m] = dot8(wv[r][c], xv, acc[r * MR + m]);
      }
    }
    float v = reduce_scatter<V>(acc, lane);
    const int mr = jm + p * MR;
    if (!lead || mr >= M) continue;
    v += pbias;
    const size_t o = (size_t)mr * a.ldo + nst;
    if constexpr (EPI == EPI_F16) {
      ((f16*)a.out)[o] = (f16)v;
    } else if constexpr (EPI == EPI_F16_GELU) {
      ((f16*)a.out)[o] = (f16)gelu_tanh(v);
    } else if constexpr (EPI == EPI_F32_RESID) {
      ((float*)a.out)[o] = pold[p] + v;
    } else if constexpr (EPI == EPI_F32) {
      ((float*)a.out)[o] = v;
    } else if constexpr (EPI == EPI_QKV_CACHE) {
      if (nst < a.d) ((f16*)a.out)[o] = (f16)v;
      else if (nst < 2 * a.d) a.kc[cdst[p] + nst - a.d] = (f16)v;
      else a.vc[cdst[p] + nst - 2 * a.d] = (f16)v;
    } else {
      epi_store<EPI>(a, mr, nst, v - pbias);
    }
  }
}

// General GEMV (optional LN prologue through LDS for 2 < M <= 8).
// A decode step of more than 16 rows (the beams of several segments, StepBatcher): k_mgemv_s's
// arithmetic with the pass count a runtime value -- ceil(M / MR) passes of MR rows through the
// LDS image, the wave's weight rows held in registers across them -- so the weights stream once
// for every row of the step (16-row launches streamed them once per 16 rows).  MR is the row
// count of the <= 16-row kernel for the same K (16, or 8 for K > 3072), so each row's result is
// bit-identical to the one it gets in a smaller step.
template <int EPI, int MR, int R, int NCH>
__global__ __launch_bounds__(256) void k_mgemv_sp(ProjArgs a) {
  ProfClock prof_clock_(a.ts);   // sampled launches only (csrc/prof.cpp)
  constexpr int KP = NCH * 512, V = R * MR;
  constexpr int SH = V >= 64 ? 0 : V >= 32 ? 1 : V >= 16 ? 2 : V >= 8 ? 3 : V >= 4 ? 4 : V >= 2 ? 5 : 6;
  constexpr int NV = MR * KP / 8, PER = (NV + 255) / 256;
  extern __shared__ __attribute__((aligned(16))) f16 xsh[];   // [MR][KP] activation rows
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int n0 = (blockIdx.x * 4 + wid) * R;
  const int K = a.K, M = a.M, np = (M + MR - 1) / MR;
  f16x8 t[PER];
  auto fetch = [&](int p) {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int v = i * 256 + threadIdx.x;
      const int m = v / (KP / 8) + p * MR, k = (v % (KP / 8)) * 8;
      t[i] = (v < NV && m < M && k < K) ? *(const f16x8*)(a.A + (size_t)m * a.lda + k) : (f16x8){};
    }
  };
  auto put = [&]() {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int v = i * 256 + threadIdx.x;
      if (v < NV) *(f16x8*)(xsh + (size_t)v * 8) = t[i];
    }
  };
  fetch(0);
  int kc[NCH];
  bool kin[NCH];
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int k = c * 512 + lane * 8;
    kin[c] = k < K;
    kc[c] = kin[c] ? k : K - 8;
  }
  f16x8 wv[R][NCH];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int n = n0 + r < a.N ? n0 + r : a.N - 1;
    const f16* w = a.B + (size_t)n * a.ldb;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const f16x8 tw = *(const f16x8*)(w + kc[c]);
      wv[r][c] = kin[c] ? tw : (f16x8){};
    }
  }
  put();
  const int j = lane >> SH, jr = j / MR, jm = j % MR;
  const bool lead = (lane & ((1 << SH) - 1)) == 0 && n0 + jr < a.N;
  const int nst = n0 + jr < a.N ? n0 + jr : a.N - 1;
  const float pbias = a.bias ? a.bias[nst] : 0.f;
  for (int p = 0; p < np; ++p) {
    if (p > 0) {
      __syncthreads();   // every wave is done with the previous pass's rows
      put();
    }
    if (p + 1 < np) fetch(p + 1);   // in flight while this pass is multiplied
    __syncthreads();
    float acc[V];
#pragma unroll
    for (int i = 0; i < V; ++i) acc[i] = 0.f;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
#pragma unroll
      for (int m = 0; m < MR; ++m) {
        const f16x8 xv = *(const f16x8*)(xsh + m * KP + c * 512 + lane * 8);
#pragma unroll
        for (int r = 0; r < R; ++r) acc[r * MR + m] = dot8(wv[r][c], xv, acc[r * MR + m]);
      }
    }
    float v = reduce_scatter<V>(acc, lane);
    const int mr = jm + p * MR;
    if (!lead || mr >= M) continue;
    v += pbias;
    const size_t o = (size_t)mr * a.ldo + nst;
    if constexpr (EPI == EPI_F16) {
      ((f16*)a.out)[o] = (f16)v;
    } else if constexpr (EPI == EPI_F16_GELU) {
      ((f16*)a.out)[o] = (f16)gelu_tanh(v);
    } else if constexpr (EPI == EPI_F32_RESID) {
      ((float*)a.out)[o] += v;
    } else if constexpr (EPI == EPI_F32) {
      ((float*)a.out)[o] = v;
    } else if constexpr (EPI == EPI_QKV_CACHE) {
      const long long cdst = a.row_seq[mr] * a.seq_stride + (long long)a.row_pos[mr] * a.d;
      if (nst < a.d) ((f16*)a.out)[o] = (f16)v;
      else if (nst < 2 * a.d) a.kc[cdst + nst - a.d] = (f16)v;
      else a.vc[cdst + nst - 2 * a.d] = (f16)v;
    } else {
      epi_store<EPI>(a, mr, nst, v - pbias);
    }
  }
}

template <int EPI, int MR, bool LN>
__global__ __launch_bounds__(256) void k_gemv(ProjArgs a) {
  ProfClock prof_clock_(a.ts);   // sampled launches only (csrc/prof.cpp)
  extern __shared__ __attribute__((aligned(16))) f16 xs[];   // [MR][K] when LN
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if constexpr (LN) {
    for (int r = wid; r < a.M; r += 4) {
      f16x8 t[3];
      ln_row_regs<3>(a, r, lane, t);
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const int k = c * 512 + lane * 8;
        if (k < a.K) *(f16x8*)(xs + r * a.K + k) = t[c];
      }
    }
    __syncthreads();
  }
  for (int n = blockIdx.x * 4 + wid; n < a.N; n += gridDim.x * 4) {
    const f16* w = a.B + (size_t)n * a.ldb;
    float acc[MR];
#pragma unroll
    for (int r = 0; r < MR; ++r) acc[r] = 0.f;
#pragma unroll 4
    for (int k = lane * 8; k < a.K; k += 512) {
      const f16x8 wv = *(const f16x8*)(w + k);
#pragma unroll
      for (int r = 0; r < MR; ++r) {
        if (r < a.M) {
          const f16x8 xv = LN ? *(const f16x8*)(xs + r * a.K + k) : *(const f16x8*)(a.A + (size_t)r * a.lda + k);
          acc[r] = dot8(wv, xv, acc[r]);
        }
      }
    }
    gemv_store<EPI, MR>(a, acc, lane, n);
  }
}

// ---------------------------------------------------------------- skinny MFMA GEMM (8 < M <= 64)
// Prompt prefill / DTW re-forward rows.  A workgroup owns 16*NT output columns for ALL rows;
// its 4 waves split K (interleaved 32-wide steps), stream the weight fragments straight from
// HBM into v_mfma_f32_16x16x32_f16 (B operand = 16 contiguous bytes of one weight row per
// lane) and reduce through LDS.  N/16 workgroups instead of N/128 keep every CU streaming.
// LN: the A rows are LayerNorm(ln_x rows) -- each workgroup normalises its 16*MT rows into LDS
// first (k_layernorm's arithmetic, so the f16 operands are bit-identical to the unfused path;
// row stride K + 8 halfs keeps the 16-row fragment reads conflict-free) -- which removes the
// separate LayerNorm launch and its f16 round trip from the prefill / DTW passes.
template <int EPI, int MT, int NT, int W = 4, bool LN = false, int UU = 0>
__global__ __launch_bounds__(W * 64) void k_skinny(ProjArgs a) {
  ProfClock prof_clock_(a.ts);   // sampled launches only (csrc/prof.cpp)
  __shared__ float red[W][MT][NT][4][64];
  extern __shared__ __attribute__((aligned(16))) f16 xln[];   // LN: [16*MT][K + 8]
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int n0 = blockIdx.x * 16 * NT;
  const int m0 = blockIdx.y * 16 * MT;   // row tiles split over gridDim.y workgroups (narrow N)
  const int fr = lane & 15, fk = 8 * (lane >> 4);
  f32x4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  const int lds_ld = a.K + 8;
  if constexpr (LN) {
    const int d = a.K;
    // rows past M are never stored (an MFMA output row depends on its own A row only): only
    // the live rows are normalised, the rest of the tile stays whatever LDS holds
    const int live = min(16 * MT, a.M - m0);
    for (int rr = wid; rr < live; rr += W) {
      int row = m0 + rr;
      if (a.row_map) row = a.row_map[row];
      const float* xr = a.ln_x + (long long)row * a.ldln;
      float v[5][4], gg[5][4], bb[5][4];
      float sm = 0.f;
#pragma unroll
      for (int j = 0; j < 5; ++j) {
        const int c = lane * 4 + j * 256;
        const bool ok = c < d;
        const int cc = ok ? c : 0;
        const float4 q = *(const float4*)(xr + cc);
        const float4 g4 = *(const float4*)(a.ln_g + cc);
        const float4 b4 = *(const float4*)(a.ln_b + cc);
        v[j][0] = ok ? q.x : 0.f; v[j][1] = ok ? q.y : 0.f; v[j][2] = ok ? q.z : 0.f; v[j][3] = ok ? q.w : 0.f;
        gg[j][0] = g4.x; gg[j][1] = g4.y; gg[j][2] = g4.z; gg[j][3] = g4.w;
        bb[j][0] = b4.x; bb[j][1] = b4.y; bb[j][2] = b4.z; bb[j][3] = b4.w;
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
        f16x4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = (f16)((v[j][e] - mean) * scale * gg[j][e] + bb[j][e]);
        *(f16x4*)(xln + rr * lds_ld + c) = o;
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
    arow[i] = LN ? xln + (i * 16 + fr) * lds_ld + fk : a.A + (size_t)m * a.lda + fk;
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
        const f16x8 t = *(const f16x8*)(arow[i] + kk);
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
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) red[wid][i][j][r][lane] = acc[i][j][r];
  __syncthreads();
  for (int e = threadIdx.x; e < MT * NT * 4 * 64; e += W * 64) {
    const int l = e & 63, r = (e >> 6) & 3, j = (e >> 8) % NT, i = (e >> 8) / NT;
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < W; ++w) v += red[w][i][j][r][l];
    const int row = m0 + i * 16 + (l >> 4) * 4 + r, col = n0 + j * 16 + (l & 15);
    epi_store<EPI>(a, row, col, v);
  }
}


// WDR_SKINNY_MSPLIT=0: narrow skinny GEMMs keep all row tiles in one workgroup (A/B runs)
// WDR_MGEMV_STAGED=0: 3..16-row GEMVs without LN on k_mgemv (rows re-read from L2 per wave)
static bool mgemv_staged() {
  static const bool on = [] {
    const char* e = getenv("WDR_MGEMV_STAGED");
    return !(e && e[0] == '0');
  }();
  return on;
}
// WDR_MGEMV_R=1|2|4: weight rows per wave of k_mgemv_s (default 2 for N >= 1024, else 1)
static int mgemv_rows() {
  static const int r = [] {
    const char* e = getenv("WDR_MGEMV_R");
    const int v = e ? atoi(e) : 0;
    return (v == 1 || v == 2 || v == 4) ? v : 0;
  }();
  return r;
}
// WDR_MGEMV_NP2=0: K > 3072 projections of 9..16-row steps as two 8-row launches (the
// previous schedule) instead of one two-pass launch
static bool mgemv_np2() {
  static const bool on = [] {
    const char* e = getenv("WDR_MGEMV_NP2");
    return !(e && e[0] == '0');
  }();
  return on;
}
static bool skinny_msplit_off() {
  const char* e = getenv("WDR_SKINNY_MSPLIT");
  return e && atoi(e) == 0;
}

// WDR_GEMM1=1: every M > 64 projection on k_gemm (A/B runs of tools/gemm_bench); read per call
static bool gemm1_forced() {
  const char* e = getenv("WDR_GEMM1");
  return e && atoi(e) != 0;
}
// WDR_GEMM3=0: keep the big encoder GEMMs on k_gemm2 / k_gemm (A/B runs); read per call
static bool gemm3_enabled() {
  const char* e = getenv("WDR_GEMM3");
  return !(e && atoi(e) == 0) && !gemm1_forced();
}

// WDR_GEMM4=0|1: the ping-pong 256 x 256 GEMM (k_gemm4) off / forced on for every M > 64 shape
// it takes (A/B runs of tools/gemm_bench); unset: the measured dispatch rule; read per call
static int gemm4_mode() {
  const char* e = getenv("WDR_GEMM4");
  return e ? atoi(e) : -1;
}

// WDR_GEMM4_GM: row tiles per group of the k_gemm4 / k_gemm5 tile order (default 4: qkv and
// cross-K/V 1 % faster than row-major in tools/gemm_bench); read per call (A/B runs)
static int gemm_tile_gm() {
  const char* e = getenv("WDR_GEMM4_GM");
  return e ? atoi(e) : 4;
}
// WDR_GEMM5=0: the narrow encoder projections on k_gemm4's 256 x 256 tiles (A/B); read per call
static bool gemm5_on() {
  const char* e = getenv("WDR_GEMM5");
  return !(e && atoi(e) == 0);
}

template <int EPI>
static void launch_epi(const ProjArgs& a, hipStream_t s) {
  const int ob = (EPI == EPI_F32_RESID || EPI == EPI_F32 || EPI == EPI_F32_GELU_POS) ? 4 : 2;
  const double bytes = (double)a.N * a.K * 2 + (double)a.M * a.K * 2 + (double)a.M * a.N * ob;
  const double flops = 2.0 * a.M * a.N * a.K;
  if (a.step_rows && a.M > 8 && !a.ln_x && a.K > 3072 && mgemv_staged() && mgemv_np2() && a.K <= 5120 &&
      a.K % 512 == 0) {
    // 9..16 step rows through a K > 3072 projection (fc2): one launch, two 8-row passes through
    // the LDS image, the weights streamed once
    const int nch = a.K / 512;
    const uint32_t lds = (uint32_t)8 * nch * 512 * 2;
    dim3 g2(cdiv(a.N, 4)), blk(256);
    switch (nch) {
      case 8: wdr_launch(PROF_GEMV, bytes, flops, k_mgemv_s<EPI, 8, 1, 8, 2>, g2, blk, lds, s, a); break;
      case 10: wdr_launch(PROF_GEMV, bytes, flops, k_mgemv_s<EPI, 8, 1, 10, 2>, g2, blk, lds, s, a); break;
      default: WDR_CHECK(false, "step GEMV: two-pass staging needs K = 4096 or 5120");
    }
    return;
  }
  if (a.step_rows && a.M > 8 && !a.ln_x && a.K > 3072) {
    // 9..16 step rows through a K > 3072 projection (fc2): two 8-row launches -- the 16-row
    // shape would spill its activation registers; per-row results are unchanged
    ProjArgs lo = a, hi = a;
    lo.M = 8;
    hi.M = a.M - 8;
    hi.A = a.A + (size_t)8 * a.lda;
    const int ob = (EPI == EPI_F32_RESID || EPI == EPI_F32 || EPI == EPI_F32_GELU_POS) ? 4 : 2;
    hi.out = (char*)a.out + (size_t)8 * a.ldo * ob;
    if (a.row_seq) hi.row_seq = a.row_seq + 8;
    if (a.row_pos) hi.row_pos = a.row_pos + 8;
    launch_epi<EPI>(lo, s);
    launch_epi<EPI>(hi, s);
    return;
  }
  if (a.M <= 8 || (a.step_rows && a.M <= 16)) {
    const int nwg = std::min(cdiv(a.N, 4), 1024);
    dim3 grid(nwg), blk(256);
    const bool ln = a.ln_x != nullptr;
    const int nch = cdiv(a.K, 512);
    if (a.M <= 2 && ((ln && a.K <= 1536) || (!ln && a.K <= 5120 && (a.K % 512 == 0 || a.K <= 1536)))) {
      // two rows per wave once there are enough rows to keep every CU busy
      const int R = a.N >= 1024 ? 2 : 1;
      dim3 g2(cdiv(a.N, 4 * R));
#define WDR_DG(MR, RR, NCH)                                                                               \
  if (ln) wdr_launch(PROF_GEMV, bytes, flops, k_dgemv<EPI, MR, RR, NCH, true>, g2, blk, 0, s, a);        \
  else wdr_launch(PROF_GEMV, bytes, flops, k_dgemv<EPI, MR, RR, NCH, false>, g2, blk, 0, s, a);
#define WDR_DG_N(MR, RR)                                                                                  \
  switch (nch) {                                                                                          \
    case 1: WDR_DG(MR, RR, 1) break;                                                                      \
    case 2: WDR_DG(MR, RR, 2) break;                                                                      \
    case 3: WDR_DG(MR, RR, 3) break;                                                                      \
    case 4: if (!ln) { wdr_launch(PROF_GEMV, bytes, flops, k_dgemv<EPI, MR, RR, 4, false>, g2, blk, 0, s, a); } break; \
    case 6: if (!ln) { wdr_launch(PROF_GEMV, bytes, flops, k_dgemv<EPI, MR, RR, 6, false>, g2, blk, 0, s, a); } break; \
    case 8: if (!ln) { wdr_launch(PROF_GEMV, bytes, flops, k_dgemv<EPI, MR, RR, 8, false>, g2, blk, 0, s, a); } break; \
    default: if (!ln) { wdr_launch(PROF_GEMV, bytes, flops, k_dgemv<EPI, MR, RR, 10, false>, g2, blk, 0, s, a); } break; \
  }
      if (a.M == 1) {
        if (R == 2) { WDR_DG_N(1, 2) } else { WDR_DG_N(1, 1) }
      } else {
        if (R == 2) { WDR_DG_N(2, 2) } else { WDR_DG_N(2, 1) }
      }
#undef WDR_DG_N
#undef WDR_DG
    } else if (!ln && mgemv_staged() && a.K <= 5120 && (a.K % 512 == 0 || a.K <= 1536) &&
               (a.M <= 8 || a.K <= 1536)) {
      // 3..16 rows without LN: activation rows staged in LDS once per workgroup, one
      // reduce-scatter per wave (k_mgemv_s)
      const int rq = mgemv_rows();
      // tools/gemv_bench GB_ROWS: one weight row per wave except the wide projections
      // (qkv / fc1) of 9..16-row steps, where two halve the activation staging per weight byte
      const int R = rq ? rq : (a.M > 8 && a.N >= 2048 ? 2 : 1);
      dim3 g2(cdiv(a.N, 4 * R));
      const int MRr = a.M <= 4 ? 4 : a.M <= 8 ? 8 : 16;
      const uint32_t lds = (uint32_t)MRr * nch * 512 * 2;
#define WDR_MS(MR, RR, NCH) wdr_launch(PROF_GEMV, bytes, flops, k_mgemv_s<EPI, MR, RR, NCH>, g2, blk, lds, s, a);
#define WDR_MS_N(MR, RR)                         \
  switch (nch) {                                 \
    case 1: WDR_MS(MR, RR, 1) break;             \
    case 2: WDR_MS(MR, RR, 2) break;             \
    case 3: WDR_MS(MR, RR, 3) break;             \
    case 4: WDR_MS(MR, RR, 4) break;             \
    case 6: WDR_MS(MR, RR, 6) break;             \
    case 8: WDR_MS(MR, RR, 8) break;             \
    default: WDR_MS(MR, RR, 10) break;           \
  }
#define WDR_MS_R(MR)                                                        \
  if (R == 1) { WDR_MS_N(MR, 1) } else if (R == 2) { WDR_MS_N(MR, 2) } else { WDR_MS_N(MR, 4) }
      if (MRr == 4) { WDR_MS_R(4) }
      else if (MRr == 8) { WDR_MS_R(8) }
      else {
        switch (nch) {
          case 1: if (R == 1) { WDR_MS(16, 1, 1) } else if (R == 2) { WDR_MS(16, 2, 1) } else { WDR_MS(16, 4, 1) } break;
          case 2: if (R == 1) { WDR_MS(16, 1, 2) } else if (R == 2) { WDR_MS(16, 2, 2) } else { WDR_MS(16, 4, 2) } break;
          default: if (R == 1) { WDR_MS(16, 1, 3) } else if (R == 2) { WDR_MS(16, 2, 3) } else { WDR_MS(16, 4, 3) } break;
        }
      }
#undef WDR_MS_R
#undef WDR_MS_N
#undef WDR_MS
    } else if ((ln && a.K <= 1536) || (!ln && a.K <= 5120 && (a.K % 512 == 0 || a.K <= 1536))) {
      // 3..8 rows (multi-chain batched steps): weight stream as k_dgemv, rows through LDS / L2
      const int R = a.N >= 1024 ? 2 : 1;
      dim3 g2(cdiv(a.N, 4 * R));
      const bool m4 = a.M <= 4;
      const uint32_t lds = ln ? (uint32_t)(m4 ? 4 : a.M <= 8 ? 8 : 16) * nch * 512 * 2 : 0;
#define WDR_MG(MR, RR, NCH)                                                                                  \
  if (ln) wdr_launch(PROF_GEMV, bytes, flops, k_mgemv<EPI, MR, RR, NCH, true>, g2, blk, lds, s, a);         \
  else wdr_launch(PROF_GEMV, bytes, flops, k_mgemv<EPI, MR, RR, NCH, false>, g2, blk, 0, s, a);
#define WDR_MG_N(MR, RR)                                                                                     \
  switch (nch) {                                                                                             \
    case 1: WDR_MG(MR, RR, 1) break;                                                                         \
    case 2: WDR_MG(MR, RR, 2) break;                                                                         \
    case 3: WDR_MG(MR, RR, 3) break;                                                                         \
    case 4: if (!ln) { wdr_launch(PROF_GEMV, bytes, flops, k_mgemv<EPI, MR, RR, 4, false>, g2, blk, 0, s, a); } break; \
    case 6: if (!ln) { wdr_launch(PROF_GEMV, bytes, flops, k_mgemv<EPI, MR, RR, 6, false>, g2, blk, 0, s, a); } break; \
    case 8: if (!ln) { wdr_launch(PROF_GEMV, bytes, flops, k_mgemv<EPI, MR, RR, 8, false>, g2, blk, 0, s, a); } break; \
    default: if (!ln) { wdr_launch(PROF_GEMV, bytes, flops, k_mgemv<EPI, MR, RR, 10, false>, g2, blk, 0, s, a); } break; \
  }
      if (m4) {
        if (R == 2) { WDR_MG_N(4, 2) } else { WDR_MG_N(4, 1) }
      } else if (a.M <= 8) {
        if (R == 2) { WDR_MG_N(8, 2) } else { WDR_MG_N(8, 1) }
      } else {
        if (R == 2) { WDR_MG_N(16, 2) } else { WDR_MG_N(16, 1) }
      }
#undef WDR_MG_N
#undef WDR_MG
    } else {
      WDR_CHECK(a.M <= 8, "gemv: more than 8 rows need the k_mgemv shapes");
      const uint32_t lds = ln ? (uint32_t)a.M * a.K * 2 : 0;
#define WDR_GEMV(MR)                                                                          \
  if (ln) wdr_launch(PROF_GEMV, bytes, flops, k_gemv<EPI, MR, true>, grid, blk, lds, s, a);  \
  else wdr_launch(PROF_GEMV, bytes, flops, k_gemv<EPI, MR, false>, grid, blk, 0, s, a);
      if (a.M <= 1) { WDR_GEMV(1) }
      else if (a.M <= 2) { WDR_GEMV(2) }
      else if (a.M <= 4) { WDR_GEMV(4) }
      else { WDR_GEMV(8) }
#undef WDR_GEMV
    }
  } else if (a.M <= 64 && a.N <= 2048 && !skinny_msplit_off()) {
    // narrow N (o / xq / xo / fc2: 80 column tiles): one 16-row tile per workgroup, the row
    // tiles of a column tile on one XCD (gridDim.x % 8 == 0 there) so its weights hit that L2
    const int mt = cdiv(a.M, 16);
    dim3 grid(cdiv(a.N, 16), mt), blk(512);
    if (a.ln_x) wdr_launch(PROF_SKINNY, bytes, flops, k_skinny<EPI, 1, 1, 8, true>, grid, blk,
                           (uint32_t)16 * (a.K + 8) * 2, s, a);
    else wdr_launch(PROF_SKINNY, bytes, flops, k_skinny<EPI, 1, 1, 8>, grid, blk, 0, s, a);
  } else if (a.M <= 64) {
    // 8 waves per workgroup split K (tools/skinny_bench: 5-12 % faster than 4 at M 24-64)
    const bool wide = a.N >= 4096;
    const int mt = cdiv(a.M, 16);
    dim3 grid(cdiv(a.N, wide ? 32 : 16)), blk(512);
    const uint32_t lds = a.ln_x ? (uint32_t)16 * mt * (a.K + 8) * 2 : 0;
#define WDR_SK(MTV)                                                                                             \
  if (a.ln_x) {                                                                                                 \
    if (wide) wdr_launch(PROF_SKINNY, bytes, flops, k_skinny<EPI, MTV, 2, 8, true>, grid, blk, lds, s, a);      \
    else wdr_launch(PROF_SKINNY, bytes, flops, k_skinny<EPI, MTV, 1, 8, true>, grid, blk, lds, s, a);           \
  } else if (wide) wdr_launch(PROF_SKINNY, bytes, flops, k_skinny<EPI, MTV, 2, 8>, grid, blk, 0, s, a);         \
  else wdr_launch(PROF_SKINNY, bytes, flops, k_skinny<EPI, MTV, 1, 8>, grid, blk, 0, s, a);
    if (mt == 1) { WDR_SK(1) }
    else if (mt == 2) { WDR_SK(2) }
    else if (mt == 3) { WDR_SK(3) }
    else { WDR_SK(4) }
#undef WDR_SK
  } else if (a.N % 128 == 0 && a.N < 2048 && a.K % G3_BK == 0 && a.M >= 4096 && !gemm1_forced() && gemm5_on() &&
             gemm4_mode() != 0 && (a.N / G3_N) * cdiv(a.M, G3_M) < 192) {
    // the narrow encoder projections (o, fc2) where 256 x 256 tiles would leave CUs idle: 256 x
    // 128 tiles fill 240 of 256 CUs at M = 6000 (tools/gemm_bench: o 53 vs 62 us on k_gemm2, fc2
    // 107 vs 126 us; at M = 12000 k_gemm4's 235 tiles are faster: fc2 194 vs 216 us)
    static bool attr5 = [] {
      WDR_HIP(hipFuncSetAttribute((const void*)k_gemm5<EPI>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)G5_LDS));
      return true;
    }();
    (void)attr5;
    ProjArgs g = a;
    g.tile_gm = gemm_tile_gm();
    dim3 grid((a.N / 128) * cdiv(a.M, G3_M));
    wdr_launch(PROF_GEMM, bytes, flops, k_gemm5<EPI>, grid, dim3(512), G5_LDS, s, g);
  } else if (a.N % G3_N == 0 && a.K % G3_BK == 0 && !gemm1_forced() &&
             (gemm4_mode() == 1 ||
              (gemm4_mode() != 0 && (a.M >= 4096 || a.N >= 16384)))) {
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
    // WDR_GEMM_CUS: persistent workgroups (multiple of 8; default one per tile)
    const int ntiles = (a.N / G3_N) * cdiv(a.M, G3_M);
    static const int cus = [] {
      const char* e = getenv("WDR_GEMM_CUS");
      return e ? atoi(e) / 8 * 8 : 0;
    }();
    dim3 grid(cus > 0 && cus < ntiles ? cus : ntiles);
    ProjArgs g = a;
    g.tile_gm = gemm_tile_gm();
    wdr_launch(PROF_GEMM, bytes, flops, k_gemm4<EPI>, grid, dim3(512), G4_LDS, s, g);
  } else if ((a.N >= 5120 || a.M >= 9000) && a.M > 2048 && a.N % G3_N == 0 && a.K % G3_BK == 0 && gemm3_enabled()) {
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
  } else if (a.K % G2_BK == 0 && a.N <= 4096 && !gemm1_forced()) {
    // LDS-DMA GEMM where it measured faster (tools/gemm_bench, M = 6000: qkv -5 %, o -11 %,
    // fc2 -23 %; fc1 and the 82k-column cross-K/V GEMM stay on k_gemm, +8 % / +7 % there)
    dim3 grid((a.N / GB_N) * cdiv(a.M, GB_M));
    wdr_launch(PROF_GEMM, bytes, flops, k_gemm2<EPI>, grid, dim3(256), 0, s, a);
  } else {
    dim3 grid(a.N / GB_N, cdiv(a.M, GB_M));
    wdr_launch(PROF_GEMM, bytes, flops, k_gemm<EPI>, grid, dim3(256), 0, s, a);
  }
}

// > 16 step rows through k_mgemv_sp: one launch, ceil(M / MR) passes, the weights streamed once.
// MR / R / NCH as the <= 16-row dispatch of launch_epi picks them for the same N, K (16 rows per
// pass up to K = 1536 -- 8 above K = 3072 with the two-pass fc2's shapes), so the per-row
// arithmetic is unchanged.  False: the shape has no multi-pass form (the caller chunks it).
template <int EPI>
static bool launch_mgemv_passes_epi(const ProjArgs& a, hipStream_t s) {
  const int ob = (EPI == EPI_F32_RESID || EPI == EPI_F32 || EPI == EPI_F32_GELU_POS) ? 4 : 2;
  const double bytes = (double)a.N * a.K * 2 + (double)a.M * a.K * 2 + (double)a.M * a.N * ob;
  const double flops = 2.0 * a.M * a.N * a.K;
  dim3 blk(256);
  if (a.K <= 1536) {
    // the 9..16-row k_mgemv_s shape: MR 16, R = 2 for N >= 2048 (unless WDR_MGEMV_R)
    const int rq = mgemv_rows();
    const int R = rq ? rq : (a.N >= 2048 ? 2 : 1);
    const int nch = cdiv(a.K, 512);
    const uint32_t lds = (uint32_t)16 * nch * 512 * 2;
    dim3 g(cdiv(a.N, 4 * R));
#define WDR_SP(RR, NCHV) wdr_launch(PROF_GEMV, bytes, flops, k_mgemv_sp<EPI, 16, RR, NCHV>, g, blk, lds, s, a)
    if (R == 1) {
      if (nch == 1) WDR_SP(1, 1); else if (nch == 2) WDR_SP(1, 2); else WDR_SP(1, 3);
    } else if (R == 2) {
      if (nch == 1) WDR_SP(2, 1); else if (nch == 2) WDR_SP(2, 2); else WDR_SP(2, 3);
    } else {
      return false;
    }
#undef WDR_SP
    return true;
  }
  if (a.K > 3072 && a.K <= 5120 && a.K % 512 == 0 && mgemv_np2()) {
    // the two-pass fc2 shape (MR 8, R 1): 8 rows per pass
    const int nch = a.K / 512;
    const uint32_t lds = (uint32_t)8 * nch * 512 * 2;
    dim3 g(cdiv(a.N, 4));
    if (nch == 8) wdr_launch(PROF_GEMV, bytes, flops, k_mgemv_sp<EPI, 8, 1, 8>, g, blk, lds, s, a);
    else if (nch == 10) wdr_launch(PROF_GEMV, bytes, flops, k_mgemv_sp<EPI, 8, 1, 10>, g, blk, lds, s, a);
    else return false;
    return true;
  }
  return false;
}

static bool launch_mgemv_passes(const ProjArgs& a, hipStream_t s) {
  static const bool on = [] {
    const char* e = getenv("WDR_MGEMV_PASSES");
    return !(e && atoi(e) == 0);
  }();
  if (!on) return false;
  switch (a.epi) {
    case EPI_F16: return launch_mgemv_passes_epi<EPI_F16>(a, s);
    case EPI_F16_GELU: return launch_mgemv_passes_epi<EPI_F16_GELU>(a, s);
    case EPI_F32_RESID: return launch_mgemv_passes_epi<EPI_F32_RESID>(a, s);
    case EPI_F32: return launch_mgemv_passes_epi<EPI_F32>(a, s);
    case EPI_QKV_CACHE: return launch_mgemv_passes_epi<EPI_QKV_CACHE>(a, s);
    default: return false;
  }
}

// Decoder rows of any count on the row kernel (k_skinny, 8 waves splitting K): the k order of a
// wave (k = 32 wid + 256 t, t = 0, 1, ...) and the wave order of the reduce do not depend on the
// tile shape (MT, NT, U) or the row split, so every row's result is the same whatever the launch
// holds -- a prompt prefill of n rows equals n one-row steps, bit for bit.
// A/B knobs of the row kernel's wave count (microbenchmark only: the arithmetic of a shape must
// not change within a run): WDR_ROWS_W16K=0 -> fc2 on 8 waves; WDR_ROWS_W16N=1 -> K <= 1280
// narrow projections on 16 waves
static bool rows_w16k() {
  const char* e = getenv("WDR_ROWS_W16K");
  return !(e && atoi(e) == 0);
}
static bool rows_w16n() {
  const char* e = getenv("WDR_ROWS_W16N");
  return e && atoi(e) != 0;
}

template <int EPI>
static void launch_rows_epi(const ProjArgs& a, hipStream_t s) {
  const int ob = (EPI == EPI_F32_RESID || EPI == EPI_F32 || EPI == EPI_F32_GELU_POS) ? 4 : 2;
  const double bytes = (double)a.N * a.K * 2 + (double)a.M * a.K * 2 + (double)a.M * a.N * ob;
  const double flops = 2.0 * a.M * a.N * a.K;
  const int mt = cdiv(a.M, 16);
  const bool ln = a.ln_x != nullptr;
  const bool wide = a.N >= 4096;
  const int prof = PROF_GEMV;   // the "rows" class of bench.py's live roofline (any row count)
  if (!wide) {
    // one 16-row tile per workgroup: the row tiles of a column tile re-read its weights from L2.
    // K > 2048 (fc2): 16 waves, each wave's 10 k-steps as ONE batch of loads (8 waves took three
    // dependent batches: fc2 at 1 row 9.8 us against 5.4 us on the GEMV)
    if (a.K > 2048) {
      WDR_CHECK(!ln, "row projection: LN prologue needs K <= 1280");
      dim3 grid(cdiv(a.N, 16), mt), blk(1024);
      if (rows_w16k()) wdr_launch(prof, bytes, flops, k_skinny<EPI, 1, 1, 16, false, 12>, grid, blk, 0, s, a);
      else wdr_launch(prof, bytes, flops, k_skinny<EPI, 1, 1, 8>, grid, dim3(512), 0, s, a);
      return;
    }
    if (rows_w16n()) {
      dim3 grid(cdiv(a.N, 16), mt), blk(1024);
      if (ln) wdr_launch(prof, bytes, flops, k_skinny<EPI, 1, 1, 16, true, 3>, grid, blk, (uint32_t)16 * (a.K + 8) * 2, s, a);
      else wdr_launch(prof, bytes, flops, k_skinny<EPI, 1, 1, 16, false, 3>, grid, blk, 0, s, a);
      return;
    }
    dim3 grid(cdiv(a.N, 16), mt), blk(512);
    if (ln) wdr_launch(prof, bytes, flops, k_skinny<EPI, 1, 1, 8, true>, grid, blk, (uint32_t)16 * (a.K + 8) * 2, s, a);
    else wdr_launch(prof, bytes, flops, k_skinny<EPI, 1, 1, 8>, grid, blk, 0, s, a);
    return;
  }
  // wide N (fc1, logits): 32 columns per workgroup, up to 4 row tiles per workgroup
  const int mtw = std::min(mt, ln ? 2 : 4);
  dim3 grid(cdiv(a.N, 32), cdiv(mt, mtw)), blk(512);
  const uint32_t lds = ln ? (uint32_t)16 * mtw * (a.K + 8) * 2 : 0;
#define WDR_RW(MTV)                                                                                        \
  if (ln) wdr_launch(prof, bytes, flops, k_skinny<EPI, MTV, 2, 8, true>, grid, blk, lds, s, a);            \
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
  WDR_CHECK(!a.ln_x || (a.K <= 1280 && a.K % 4 == 0), "row projection LN prologue: K <= 1280");
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
  if (a.rows_mma) {
    launch_rows(a, s);
    return;
  }
  if (a.step_rows && a.M > 16 && !a.ln_x && mgemv_staged() && launch_mgemv_passes(a, s)) return;
  if (a.step_rows && a.M > 16) {
    // a batched step of more than 16 rows (beams of several segments): 16-row GEMV launches,
    // so every row's arithmetic stays that of a <= 16-row step whatever the batch holds
    // (batch composition depends on timing; results must not)
    const int ob = (a.epi == EPI_F32_RESID || a.epi == EPI_F32 || a.epi == EPI_F32_GELU_POS) ? 4 : 2;
    for (int r0 = 0; r0 < a.M; r0 += 16) {
      ProjArgs c = a;
      c.M = std::min(16, a.M - r0);
      if (a.A) c.A = a.A + (size_t)r0 * a.lda;
      if (a.ln_x) c.ln_x = a.ln_x + (size_t)r0 * a.ldln;
      c.out = (char*)a.out + (size_t)r0 * a.ldo * ob;
      if (a.row_seq) c.row_seq = a.row_seq + r0;
      if (a.row_pos) c.row_pos = a.row_pos + r0;
      launch_proj(c, s);
    }
    return;
  }
  WDR_CHECK(a.K % 8 == 0 && a.lda % 8 == 0 && a.ldb % 8 == 0, "projection: K/lda/ldb must be multiples of 8");
  if (a.M > 64) {
    WDR_CHECK(a.N % GB_N == 0, "gemm: N must be a multiple of 128");
    WDR_CHECK(a.K % GB_K == 0, "gemm: K must be a multiple of 32");
  } else if (a.step_rows && a.M <= 16) {
    WDR_CHECK(!a.ln_x || a.K <= 1536, "gemv LN prologue: K must be <= 1536");
  } else if (a.M > 8) {
    WDR_CHECK(a.K % 32 == 0, "skinny gemm: K must be a multiple of 32");
    WDR_CHECK(!a.ln_x || (a.K <= 1280 && a.K % 4 == 0 && a.M <= 32), "skinny LN prologue: K <= 1280, M <= 32");
  } else if (a.ln_x) {
    WDR_CHECK(a.K <= 1536 && a.K % 8 == 0, "gemv LN prologue: K must be <= 1536");
  }
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
