// fp32 GEMM on CDNA4 matrix cores: v_mfma_f32_32x32x2_f32 (exact fp32 products,
// fp32 accumulation — the same arithmetic class as the reference's cuBLAS SGEMM;
// gfx950 has no xf32/TF32 shortcut).
//
// Tile 128x128x16 per 256-thread workgroup, 4 waves in a 2x2 grid, each wave a
// 64x64 sub-tile = 2x2 MFMA tiles (64 accumulator VGPRs).  Both operands are
// staged k-major in LDS ([k][m] / [k][n]) so a half-wave's MFMA fragment read is
// 32 consecutive floats (conflict-free ds_read_b32).  Global->register loads of
// tile k+1 are issued before the MFMAs of tile k (register double buffering).
// Operands that are k-contiguous are transposed on the LDS write; the row pad
// (+2 floats) makes those 8 ds_write_b32 per thread conflict-free.
#include "common.h"
#include "amax_rc.h"

#include <type_traits>

#include <algorithm>
#include <cstdlib>

namespace ds2 {

constexpr int BM = 128, BN = 128, BK = 16;
constexpr int LDS_PAD_T = 2;   // k-contiguous source -> transposed ds_write_b32
constexpr int LDS_PAD_N = 4;   // m/n-contiguous source -> ds_write_b128 (16 B aligned rows)

template <bool KCONTIG>
struct OperandTile {
  static constexpr int LD = (KCONTIG ? (BM + LDS_PAD_T) : (BM + LDS_PAD_N));
};

// Loads the BK x 128 slice of an operand into 8 registers per thread.
//   KCONTIG: element (r, kk) at p[(r0 + r) * ld + k0 + kk]   (r = m or n)
//  !KCONTIG: element (r, kk) at p[(k0 + kk) * ld + r0 + r]
template <bool KCONTIG, bool VEC>
__device__ __forceinline__ void load_tile(const float* __restrict__ p, int64_t ld, int rows,
                                          int K, int r0, int k0, float (&v)[8]) {
  const int t = threadIdx.x;
  if (KCONTIG) {
    const int r = t >> 1;
    const int kb = (t & 1) * 8;
    const int gr = r0 + r;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int gk = k0 + kb + 4 * q;
      if (VEC) {
        float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
        if (gr < rows && gk < K) x = *reinterpret_cast<const float4*>(p + (int64_t)gr * ld + gk);
        v[4 * q + 0] = x.x; v[4 * q + 1] = x.y; v[4 * q + 2] = x.z; v[4 * q + 3] = x.w;
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          v[4 * q + e] = (gr < rows && gk + e < K) ? p[(int64_t)gr * ld + gk + e] : 0.f;
      }
    }
  } else {
    const int c4 = (t & 31) * 4;
    const int gr = r0 + c4;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int kk = (t >> 5) + 8 * q;
      const int gk = k0 + kk;
      if (VEC) {
        float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
        if (gk < K && gr < rows) x = *reinterpret_cast<const float4*>(p + (int64_t)gk * ld + gr);
        v[4 * q + 0] = x.x; v[4 * q + 1] = x.y; v[4 * q + 2] = x.z; v[4 * q + 3] = x.w;
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          v[4 * q + e] = (gk < K && gr + e < rows) ? p[(int64_t)gk * ld + gr + e] : 0.f;
      }
    }
  }
}

template <bool KCONTIG>
__device__ __forceinline__ void store_tile(float* __restrict__ s, const float (&v)[8]) {
  constexpr int LD = OperandTile<KCONTIG>::LD;
  const int t = threadIdx.x;
  if (KCONTIG) {
    const int r = t >> 1;
    const int kb = (t & 1) * 8;
#pragma unroll
    for (int e = 0; e < 8; ++e) s[(kb + e) * LD + r] = v[e];
  } else {
    const int c4 = (t & 31) * 4;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int kk = (t >> 5) + 8 * q;
      *reinterpret_cast<float4*>(s + kk * LD + c4) =
          make_float4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
    }
  }
}

// Work items (blockIdx.x in dispatch order):
//   [0, main_wgs)       one whole output tile each (batch == 1), XCD-aware order;
//   [main_wgs, grid)    "tail" pieces: (batch, split, tile) of the tiles from tail_tile0
//                       on, K range split nsplit ways; dispatched last, they fill the
//                       slots the whole tiles leave in the final round.
// XCD-aware (bijective) remap of both ranges: the blocks the dispatcher deals to one XCD
// (ids congruent mod 8) get a contiguous run of tiles (pieces) in the grouped order below,
// so workgroups sharing an operand panel share that XCD's L2.
// Grouped tile order: tile ids run over groups of g_tile_group m-rows, inside a group column
// by column (m fastest), so the ~32 tiles one XCD runs at once span 4 m-rows x 8 n-columns
// (A: 4 panels, B: 8) instead of ~2 m-rows x every n-column (the input projection's 15 B
// panels, 7.7 MB, overflow the XCD's 4-MB L2 and were fetched again for every m-row).
constexpr int kTileGroup = 4;

__device__ __forceinline__ void tile_coords(int tile, int tn, int tm, int& tile_m, int& tile_n) {
  constexpr int G = kTileGroup;
  const int g = tile / (G * tn);
  const int rem = tile - g * G * tn;
  const int rows = min(G, tm - g * G);
  tile_n = rem / rows;
  tile_m = g * G + (rem - tile_n * rows);
}

__device__ __forceinline__ void decode_work(int M, int N, int K, int main_wgs, int tail_tile0,
                                            int tail_tiles, int nsplit, int kchunk,
                                            float* partial, int& m0, int& n0, int& kbeg,
                                            int& kend, int& bz, float*& part, int bn = BN,
                                            int bm = BM) {
  const int tn = (N + bn - 1) / bn;
  const int orig = blockIdx.x;
  int tile, z = 0;
  part = nullptr;
  if (orig < main_wgs) {
    const int q = main_wgs >> 3, r = main_wgs & 7;
    const int xcd = orig & 7;
    tile = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
  } else {
    const int np = gridDim.x - main_wgs;
    const int o = orig - main_wgs;
    const int q = np >> 3, r = np & 7;
    const int xcd = o & 7;
    const int pidx = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (o >> 3);
    z = pidx / tail_tiles;
    const int lt = pidx - z * tail_tiles;
    tile = tail_tile0 + lt;
    if (nsplit > 1) part = partial + ((int64_t)z * tail_tiles + lt) * (bm * bn);
  }
  int tile_m, tile_n;
  tile_coords(tile, tn, (M + bm - 1) / bm, tile_m, tile_n);
  // z = batch * nsplit + split
  bz = z / nsplit;
  const int sp = z - bz * nsplit;
  kbeg = orig < main_wgs ? 0 : sp * kchunk;
  kend = orig < main_wgs ? K : min(K, kbeg + kchunk);
  m0 = tile_m * bm;
  n0 = tile_n * bn;
}

// Epilogue: C/D map of the 32x32 MFMA: col = lane & 31, row = (r & 3) + 8 * (r >> 2) +
// 4 * (lane >> 5).  Split pieces write a tile-local [BM][BN] partial slab.
__device__ __forceinline__ void store_acc(const f32x16 (&acc)[2][2], int M, int N, float alpha,
                                          float beta, float* __restrict__ C, int64_t ldc,
                                          const float* __restrict__ bias, float* __restrict__ part,
                                          int m0, int n0, int wm, int wn, int lane) {
  const int lr = lane & 31;
  const int lk = lane >> 5;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int col = n0 + wn + 32 * j + lr;
      if (part != nullptr) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int rl = wm + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * lk;
          part[rl * BN + wn + 32 * j + lr] = acc[i][j][r];
        }
        continue;
      }
      if (col >= N) continue;
      const float bv = bias != nullptr ? bias[col] : 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * lk;
        if (row < M) {
          float* cp = C + (int64_t)row * ldc + col;
          float v = alpha * acc[i][j][r] + bv;
          if (beta != 0.f) v += beta * *cp;
          *cp = v;
        }
      }
    }
  }
}

template <int TA, int TB, bool VA, bool VB>
__global__ __launch_bounds__(256) void sgemm_kernel(
    int M, int N, int K, float alpha, const float* __restrict__ A, int64_t lda, int64_t sA,
    const float* __restrict__ B, int64_t ldb, int64_t sB, float beta, float* __restrict__ C,
    int64_t ldc, int64_t sC, const float* __restrict__ bias, int main_wgs, int tail_tile0,
    int tail_tiles, int nsplit, int kchunk, float* __restrict__ partial) {
  // op(A) is k-contiguous when TA == 0 ([m][k] storage); op(B) is k-contiguous
  // when TB == 1 ([n][k] storage).
  constexpr bool AK = (TA == 0);
  constexpr bool BKc = (TB == 1);
  constexpr int LDA_S = OperandTile<AK>::LD;
  constexpr int LDB_S = OperandTile<BKc>::LD;
  __shared__ __attribute__((aligned(16))) float As[2][BK * LDA_S];
  __shared__ __attribute__((aligned(16))) float Bs[2][BK * LDB_S];

  int m0, n0, kbeg, kend, bz;
  float* part;
  decode_work(M, N, K, main_wgs, tail_tile0, tail_tiles, nsplit, kchunk, partial, m0, n0, kbeg,
              kend, bz, part);
  A += bz * sA;
  B += bz * sB;
  C += bz * sC;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int wm = (wave >> 1) * 64;
  const int wn = (wave & 1) * 64;

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  float ra[8], rb[8];
  const int ktiles = (kend - kbeg + BK - 1) / BK;
  load_tile<AK, VA>(A, lda, M, kend, m0, kbeg, ra);
  load_tile<BKc, VB>(B, ldb, N, kend, n0, kbeg, rb);
  store_tile<AK>(As[0], ra);
  store_tile<BKc>(Bs[0], rb);
  __syncthreads();

  const int lr = lane & 31;
  const int lk = lane >> 5;
  for (int kt = 0; kt < ktiles; ++kt) {
    const int cur = kt & 1;
    const bool more = (kt + 1) < ktiles;
    if (more) {
      load_tile<AK, VA>(A, lda, M, kend, m0, kbeg + (kt + 1) * BK, ra);
      load_tile<BKc, VB>(B, ldb, N, kend, n0, kbeg + (kt + 1) * BK, rb);
    }
    const float* as = As[cur];
    const float* bs = Bs[cur];
#pragma unroll
    for (int kk = 0; kk < BK; kk += 2) {
      float a0 = as[(kk + lk) * LDA_S + wm + lr];
      float a1 = as[(kk + lk) * LDA_S + wm + 32 + lr];
      float b0 = bs[(kk + lk) * LDB_S + wn + lr];
      float b1 = bs[(kk + lk) * LDB_S + wn + 32 + lr];
      acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc[1][1], 0, 0, 0);
    }
    if (more) {
      store_tile<AK>(As[cur ^ 1], ra);
      store_tile<BKc>(Bs[cur ^ 1], rb);
    }
    __syncthreads();
  }

  store_acc(acc, M, N, alpha, beta, C, ldc, bias, part, m0, n0, wm, wn, lane);
}


// ---------------------------------------------------------------------------------------
// Deep-K variant (float4-aligned operands): same work plan and epilogue semantics as
// sgemm_kernel, but BK = 64 per LDS stage and v_mfma_f32_16x16x4_f32 with a 4 x WN grid
// of 16x16 tiles per wave (tile 128 x 32 WN: WN = 4 -> 128, WN = 5 -> 160, which divides
// the model's N = 800 / 1600 / 2400 exactly).  Within a k-group of 16, lane (r, q) feeds
// its four MFMAs c = 0..3 with the k values 16 g + 4 q + c of row r: one ds_read_b128
// from a k-contiguous image ([row][64 k], float4 slot XOR (row & 15): conflict-free for
// the b128 lane groups and for the b128 stores) or four ds_read_b32 from a
// row-contiguous image ([k][row], pitch rows + 4: the two 16-lane row groups of a
// half-wave land on disjoint bank halves).  Each operand keeps the orientation of its
// global layout, so every global load and LDS store is a contiguous float4.  One LDS
// stage (<= 76 KB) per workgroup, two workgroups per CU: one computes while the other
// refills; 16 WN MFMAs per wave per k-group, 64 WN between barriers.
constexpr int K64 = 64;

// LDS image of ROWS rows x KS k of one operand.  k-contiguous ([row][KS]): float4 slot
// s of row r stored at slot s ^ swz(r), swz = r & 15 (KS = 64) or (r >> 1) & 7 (KS = 32),
// which keeps both the ds_read_b128 fragment reads (16-lane groups, 64 banks) and the
// ds_write_b128 stores (8-lane groups, 32 banks) conflict-free without padding.
// Row-contiguous ([KS][ROWS + 4]).
template <bool KC, int ROWS, int KS>
struct Img {
  static constexpr int PITCH = KC ? KS : ROWS + 4;
  static constexpr int FLOATS = KC ? ROWS * KS : KS * (ROWS + 4);
  static constexpr int LOADS = ROWS * KS / 4 / 256;   // float4 per thread
  static constexpr int SLOTS = KS / 4;                // float4 per k-contiguous row
  __device__ static __forceinline__ int swz(int r) { return KS == 64 ? (r & 15) : ((r >> 1) & 7); }
};

// one stage of an operand through a buffer resource; an element outside [rows) x
// [k, kend) gets an out-of-range offset and reads as zero (no branches)
template <bool KC, int ROWS, int KS>
__device__ __forceinline__ void load_stage(__amdgpu_buffer_rsrc_t rs, int ld, int rows, int kend,
                                           int r0, int k0,
                                           f32x4 (&v)[Img<KC, ROWS, KS>::LOADS]) {
  using I = Img<KC, ROWS, KS>;
  constexpr int kOob = 0x7ffffff0;
  const int t = threadIdx.x;
#pragma unroll
  for (int q = 0; q < I::LOADS; ++q) {
    const int i = t + 256 * q;
    int r, k;
    if (KC) {
      r = r0 + i / I::SLOTS;
      k = k0 + (i % I::SLOTS) * 4;
    } else {
      k = k0 + i / (ROWS / 4);
      r = r0 + (i % (ROWS / 4)) * 4;
    }
    const int off = (r < rows && k < kend) ? (KC ? r * ld + k : k * ld + r) * 4 : kOob;
    v[q] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
  }
}

template <bool KC, int ROWS, int KS>
__device__ __forceinline__ void store_stage(float* __restrict__ s,
                                            const f32x4 (&v)[Img<KC, ROWS, KS>::LOADS]) {
  using I = Img<KC, ROWS, KS>;
  const int t = threadIdx.x;
#pragma unroll
  for (int q = 0; q < I::LOADS; ++q) {
    const int i = t + 256 * q;
    if (KC) {
      const int r = i / I::SLOTS;
      *reinterpret_cast<f32x4*>(s + r * I::PITCH + 4 * ((i % I::SLOTS) ^ I::swz(r))) = v[q];
    } else {
      *reinterpret_cast<f32x4*>(s + (i / (ROWS / 4)) * I::PITCH + (i % (ROWS / 4)) * 4) = v[q];
    }
  }
}

// fragment of rows [rb, rb + 16) (rb % 16 == 0) for k-group g of the stage
template <bool KC, int ROWS, int KS>
__device__ __forceinline__ f32x4 frag(const float* __restrict__ s, int rb, int g, int lane) {
  using I = Img<KC, ROWS, KS>;
  const int r = lane & 15, q = lane >> 4;
  if (KC)
    return *reinterpret_cast<const f32x4*>(s + (rb + r) * I::PITCH +
                                           4 * ((4 * g + q) ^ I::swz(rb + r)));
  const float* p = s + (16 * g + 4 * q) * I::PITCH + rb + r;
  return f32x4{p[0], p[I::PITCH], p[2 * I::PITCH], p[3 * I::PITCH]};
}

// Deep-K variant (float4-aligned operands): same work plan and epilogue semantics as
// sgemm_kernel; v_mfma_f32_16x16x4_f32 with a 4 x WN grid of 16x16 tiles per wave (tile
// 128 x 32 WN: WN = 4 -> 128, WN = 5 -> 160, which divides the model's N = 800 / 1600 /
// 2400 exactly).  Within a k-group of 16, lane (r, q) feeds its four MFMAs c = 0..3 with
// the k values 16 g + 4 q + c of row r: one ds_read_b128 from a k-contiguous image or
// four ds_read_b32 from a row-contiguous one.  Each operand keeps the orientation of its
// global layout, so every global load and LDS store is a contiguous float4.
//   NBUF = 1: one LDS stage of KS = 64 per workgroup (<= 76 KB, two workgroups per CU);
//             store, barrier, MFMAs, barrier.
//   NBUF = 2: two stages of KS = 32; the next stage is stored into the other buffer at
//             the top of each stage, one barrier per stage.
template <int TA, int TB, int WN, int KS, int NBUF>
__global__ __launch_bounds__(256, 2) void sgemm64_kernel(
    int M, int N, int K, float alpha, const float* __restrict__ A, int64_t lda, int64_t sA,
    const float* __restrict__ B, int64_t ldb, int64_t sB, float beta, float* __restrict__ C,
    int64_t ldc, int64_t sC, const float* __restrict__ bias, int main_wgs, int tail_tile0,
    int tail_tiles, int nsplit, int kchunk, float* __restrict__ partial) {
  constexpr bool AK = (TA == 0);
  constexpr bool BKc = (TB == 1);
  constexpr int TBN = 32 * WN;              // tile width
  using IA = Img<AK, BM, KS>;
  using IB = Img<BKc, TBN, KS>;
  __shared__ __attribute__((aligned(16))) float As[NBUF][IA::FLOATS];
  __shared__ __attribute__((aligned(16))) float Bs[NBUF][IB::FLOATS];

  int m0, n0, kbeg, kend, bz;
  float* part;
  decode_work(M, N, K, main_wgs, tail_tile0, tail_tiles, nsplit, kchunk, partial, m0, n0, kbeg,
              kend, bz, part, TBN);
  A += bz * sA;
  B += bz * sB;
  C += bz * sC;
  // host: every operand spans < 2^31 bytes (32-bit buffer offsets)
  const int a_rows = AK ? M : K, b_rows = BKc ? N : K;
  const __amdgpu_buffer_rsrc_t a_rs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(A), (short)0, static_cast<int>(a_rows * lda * 4), 0x00020000);
  const __amdgpu_buffer_rsrc_t b_rs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(B), (short)0, static_cast<int>(b_rows * ldb * 4), 0x00020000);
  const int ilda = static_cast<int>(lda), ildb = static_cast<int>(ldb);
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int wm = (wave >> 1) * 64;
  const int wn = (wave & 1) * 16 * WN;

  f32x4 acc[4][WN];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < WN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](const float* as, const float* bs, int k0) {
    // k-groups past kend hold zeros: skip them (K = 800, 1312, 2400 end on half stages)
    const int ng = min(KS / 16, (kend - k0 + 15) / 16);
#pragma unroll
    for (int g = 0; g < KS / 16; ++g) {
      if (g >= ng) break;
      f32x4 a[4], b[WN];
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = frag<AK, BM, KS>(as, wm + 16 * i, g, lane);
#pragma unroll
      for (int j = 0; j < WN; ++j) b[j] = frag<BKc, TBN, KS>(bs, wn + 16 * j, g, lane);
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < WN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i][c], b[j][c], acc[i][j], 0, 0, 0);
    }
  };

  f32x4 ra[IA::LOADS], rb[IB::LOADS];
  const int ktiles = (kend - kbeg + KS - 1) / KS;
  load_stage<AK, BM, KS>(a_rs, ilda, M, kend, m0, kbeg, ra);
  load_stage<BKc, TBN, KS>(b_rs, ildb, N, kend, n0, kbeg, rb);
  if (NBUF == 1) {
    for (int kt = 0; kt < ktiles; ++kt) {
      store_stage<AK, BM, KS>(As[0], ra);
      store_stage<BKc, TBN, KS>(Bs[0], rb);
      __syncthreads();
      if (kt + 1 < ktiles) {   // next stage's global loads fly during this stage's MFMAs
        load_stage<AK, BM, KS>(a_rs, ilda, M, kend, m0, kbeg + (kt + 1) * KS, ra);
        load_stage<BKc, TBN, KS>(b_rs, ildb, N, kend, n0, kbeg + (kt + 1) * KS, rb);
      }
      compute(As[0], Bs[0], kbeg + kt * KS);
      __syncthreads();
    }
  } else {
    store_stage<AK, BM, KS>(As[0], ra);
    store_stage<BKc, TBN, KS>(Bs[0], rb);
    if (ktiles > 1) {
      load_stage<AK, BM, KS>(a_rs, ilda, M, kend, m0, kbeg + KS, ra);
      load_stage<BKc, TBN, KS>(b_rs, ildb, N, kend, n0, kbeg + KS, rb);
    }
    for (int kt = 0; kt < ktiles; ++kt) {
      // stage kt visible; every wave is done with the other buffer (stage kt - 1)
      __syncthreads();
      const int cur = kt & 1;
      if (kt + 1 < ktiles) {
        store_stage<AK, BM, KS>(As[cur ^ 1], ra);
        store_stage<BKc, TBN, KS>(Bs[cur ^ 1], rb);
        if (kt + 2 < ktiles) {
          load_stage<AK, BM, KS>(a_rs, ilda, M, kend, m0, kbeg + (kt + 2) * KS, ra);
          load_stage<BKc, TBN, KS>(b_rs, ildb, N, kend, n0, kbeg + (kt + 2) * KS, rb);
        }
      }
      compute(As[cur], Bs[cur], kbeg + kt * KS);
    }
  }

  // epilogue (16x16 C/D map: col = lane & 15, row = 4 * (lane >> 4) + r)
  const int lc = lane & 15;
  const int lr = 4 * (lane >> 4);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
#pragma unroll
    for (int j = 0; j < WN; ++j) {
      const int cl = wn + 16 * j + lc;
      if (part != nullptr) {
#pragma unroll
        for (int r = 0; r < 4; ++r) part[(wm + 16 * i + lr + r) * TBN + cl] = acc[i][j][r];
        continue;
      }
      const int col = n0 + cl;
      if (col >= N) continue;
      const float bv = bias != nullptr ? bias[col] : 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wm + 16 * i + lr + r;
        if (row < M) {
          float* cp = C + (int64_t)row * ldc + col;
          float v = alpha * acc[i][j][r] + bv;
          if (beta != 0.f) v += beta * *cp;
          *cp = v;
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------
// bf16-operand variant (BASELINE cfg4 "bf16 MFMA RNN GEMMs", opt-in): fp32 operands in
// memory are rounded to bf16 (round-to-nearest-even, v_cvt_pk_bf16_f32) while they are
// staged, multiplied with v_mfma_f32_16x16x32_bf16 and accumulated in fp32; C, bias, the
// split-K plan and the epilogue are those of sgemm64_kernel (tile 128 x 128, 4 waves of
// 4 x 4 16x16 tiles).  Each operand is staged k-contiguous in LDS whatever its global
// layout: rows of 64 bf16 (128 B) in 16-B slots (8 k each) swizzled by (row >> 1) & 7, so a
// lane's A or B fragment (8 consecutive k of one row) is one conflict-free ds_read_b128.
//   k-contiguous source: a thread unit = (row, slot): 2 float4 loads -> 1 ds_write_b128;
//   row-contiguous source: a unit = (4 rows, slot): 8 float4 loads (one per k) -> 4 writes.
constexpr int KB16 = 64;   // k per stage
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ int bslot(int row, int s) { return row * KB16 + 8 * (s ^ ((row >> 1) & 7)); }

template <bool KC>
__device__ __forceinline__ void bload_stage(__amdgpu_buffer_rsrc_t rs, int ld, int rows, int kend,
                                            int r0, int k0, f32x4 (&v)[8]) {
  constexpr int kOob = 0x7ffffff0;
  const int t = threadIdx.x;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    int r, k;
    if (KC) {                        // units t + 256 i (i = q / 2): row u / 8, slot u % 8
      const int u = t + 256 * (q >> 1);
      r = r0 + (u >> 3);
      k = k0 + 8 * (u & 7) + 4 * (q & 1);
    } else {                         // 4-row group t % 32, slot t / 32, k row q of the slot
      r = r0 + 4 * (t & 31);
      k = k0 + 8 * (t >> 5) + q;
    }
    const int off = (r < rows && k < kend) ? (KC ? r * ld + k : k * ld + r) * 4 : kOob;
    v[q] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
  }
}

template <bool KC>
__device__ __forceinline__ void bstore_stage(unsigned short* __restrict__ s, const f32x4 (&v)[8]) {
  const int t = threadIdx.x;
  if (KC) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int u = t + 256 * i;
      const f32x4 a = v[2 * i], b = v[2 * i + 1];
      const bf16x8 p{(__bf16)a.x, (__bf16)a.y, (__bf16)a.z, (__bf16)a.w,
                     (__bf16)b.x, (__bf16)b.y, (__bf16)b.z, (__bf16)b.w};
      *reinterpret_cast<bf16x8*>(s + bslot(u >> 3, u & 7)) = p;
    }
  } else {
    const int g = t & 31, sl = t >> 5;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const bf16x8 p{(__bf16)v[0][c], (__bf16)v[1][c], (__bf16)v[2][c], (__bf16)v[3][c],
                     (__bf16)v[4][c], (__bf16)v[5][c], (__bf16)v[6][c], (__bf16)v[7][c]};
      *reinterpret_cast<bf16x8*>(s + bslot(4 * g + c, sl)) = p;
    }
  }
}

template <int TA, int TB>
__global__ __launch_bounds__(256, 2) void sbgemm_kernel(
    int M, int N, int K, float alpha, const float* __restrict__ A, int64_t lda, int64_t sA,
    const float* __restrict__ B, int64_t ldb, int64_t sB, float beta, float* __restrict__ C,
    int64_t ldc, int64_t sC, const float* __restrict__ bias, int main_wgs, int tail_tile0,
    int tail_tiles, int nsplit, int kchunk, float* __restrict__ partial) {
  constexpr bool AK = (TA == 0);
  constexpr bool BKc = (TB == 1);
  constexpr int TBN = 128;
  __shared__ __attribute__((aligned(16))) unsigned short As[BM * KB16];
  __shared__ __attribute__((aligned(16))) unsigned short Bs[TBN * KB16];

  int m0, n0, kbeg, kend, bz;
  float* part;
  decode_work(M, N, K, main_wgs, tail_tile0, tail_tiles, nsplit, kchunk, partial, m0, n0, kbeg,
              kend, bz, part, TBN);
  A += bz * sA;
  B += bz * sB;
  C += bz * sC;
  const int a_rows = AK ? M : K, b_rows = BKc ? N : K;
  const __amdgpu_buffer_rsrc_t a_rs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(A), (short)0, static_cast<int>(a_rows * lda * 4), 0x00020000);
  const __amdgpu_buffer_rsrc_t b_rs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(B), (short)0, static_cast<int>(b_rows * ldb * 4), 0x00020000);
  const int ilda = static_cast<int>(lda), ildb = static_cast<int>(ldb);
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int wm = (wave >> 1) * 64;
  const int wn = (wave & 1) * 64;
  const int fr = lane & 15, fq = lane >> 4;

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  f32x4 ra[8], rb[8];
  const int ktiles = (kend - kbeg + KB16 - 1) / KB16;
  bload_stage<AK>(a_rs, ilda, M, kend, m0, kbeg, ra);
  bload_stage<BKc>(b_rs, ildb, N, kend, n0, kbeg, rb);
  for (int kt = 0; kt < ktiles; ++kt) {
    bstore_stage<AK>(As, ra);
    bstore_stage<BKc>(Bs, rb);
    __syncthreads();
    if (kt + 1 < ktiles) {   // next stage's global loads fly during this stage's MFMAs
      bload_stage<AK>(a_rs, ilda, M, kend, m0, kbeg + (kt + 1) * KB16, ra);
      bload_stage<BKc>(b_rs, ildb, N, kend, n0, kbeg + (kt + 1) * KB16, rb);
    }
    // k-steps past kend hold zeros: skip them
    const int ns = min(KB16 / 32, (kend - kbeg - kt * KB16 + 31) / 32);
#pragma unroll
    for (int s = 0; s < KB16 / 32; ++s) {
      if (s >= ns) break;
      bf16x8 a[4], b[4];
#pragma unroll
      for (int i = 0; i < 4; ++i)
        a[i] = *reinterpret_cast<const bf16x8*>(As + bslot(wm + 16 * i + fr, 4 * s + fq));
#pragma unroll
      for (int j = 0; j < 4; ++j)
        b[j] = *reinterpret_cast<const bf16x8*>(Bs + bslot(wn + 16 * j + fr, 4 * s + fq));
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
  }

  // epilogue (16x16 C/D map: col = lane & 15, row = 4 * (lane >> 4) + r), as sgemm64_kernel
  const int lc = lane & 15;
  const int lr = 4 * (lane >> 4);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int cl = wn + 16 * j + lc;
      if (part != nullptr) {
#pragma unroll
        for (int r = 0; r < 4; ++r) part[(wm + 16 * i + lr + r) * TBN + cl] = acc[i][j][r];
        continue;
      }
      const int col = n0 + cl;
      if (col >= N) continue;
      const float bv = bias != nullptr ? bias[col] : 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wm + 16 * i + lr + r;
        if (row < M) {
          float* cp = C + (int64_t)row * ldc + col;
          float v = alpha * acc[i][j][r] + bv;
          if (beta != 0.f) v += beta * *cp;
          *cp = v;
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------
// fp32 GEMM on the bf16 matrix cores at fp32 accuracy (default for float4-staged operands;
// DS2_GEMM_X6=0 selects sgemm64_kernel).  Every fp32 operand value x is split while it is
// staged into three bf16 terms, hi = bf16(x), mid = bf16(x - hi), lo = bf16(x - hi - mid)
// (round to nearest even; x = hi + mid + lo to 2^-26 |x|), and a product a.b is formed from
// the six terms that carry fp32 weight,
//   mid.mid + lo.hi + hi.lo + mid.hi + hi.mid + hi.hi       (small terms first)
// (dropped: mid.lo, lo.mid, lo.lo, each below 2^-25 |a b|).  Each bf16 product is exact
// in the fp32 accumulator, so the result carries fp32 rounding only (the fp32-equivalent
// peak is the dense bf16 peak / 6 = 419 TF).  The same split and products run the GRU
// recurrences (gru_split.hip).  LDS: per operand three bf16 planes [rows][32 k] (64-B rows,
// 16-B slot s of row r at s ^ xswz(r), below: conflict-free ds_read_b128 fragments and
// stores).
constexpr int XS = 32;                  // k per stage

// 16-B slot s of a 64-B row, XOR-swizzled by q(row) = bit 2 | (bit 1 ^ bit 3) << 1: with it
// the fragment reads (ds_read_b128 serves lanes in four 16-lane groups, rows {0-3, 12-15,
// 20-27} and the rest of 32) and both staging stores (ds_write_b128 in 8-lane groups: 8
// consecutive rows of one slot, or 2 rows x 4 slots) hit distinct banks.  The earlier
// (row >> 2) & 3 left the row-contiguous stores 4-way conflicted (12 % of LDS cycles).
__device__ __forceinline__ int xswz(int row) { return ((row >> 2) & 1) | ((((row >> 1) ^ (row >> 3)) & 1) << 1); }
__device__ __forceinline__ int xslot(int row, int s) { return row * XS + 8 * (s ^ xswz(row)); }
// the v_mfma_f32_16x16x32_bf16 form (M16): a fragment is 16 rows x one 8-k slot per 16-lane
// quarter (lane (row l & 15, slot l >> 4)); slot s of row r at s ^ ((r >> 1) & 3) keeps its
// ds_read_b128 lane groups, the 8-lane groups of the (row, slot)-unit stores and those of the
// 8-consecutive-row stores of row-contiguous operands on distinct banks
template <bool M16>
__device__ __forceinline__ int xslot_t(int row, int s) {
  if constexpr (M16) return row * XS + 8 * (s ^ ((row >> 1) & 3));
  else return xslot(row, s);
}

// The default bf16x6 kernel: tile 256 x 128, eight waves (two per SIMD) of 2 x 2 32x32
// tiles on v_mfma_f32_32x32x16_bf16 (which holds the SIMD's vector issue for 8 of its 32
// cycles, half the share of the 16x16x32 form), ONE workgroup per CU with two LDS stages
// (2 x 72 KB).  Stage kt + 1 is split and stored into the other buffer in the same basic
// block as stage kt's MFMAs, and sched_group_barrier interleaves the split's VALU work with
// the MFMAs (three VALU per MFMA), so it issues in the MFMAs' shadow instead of in a phase
// of its own; one barrier per stage; stage kt + 2's global loads are issued behind it.
// Per-thread staging as sxgemm_kernel: k-contiguous units of (row, 8-k slot), or one row x
// (8 or 16) k of a row-contiguous operand (consecutive threads on consecutive rows).
constexpr int X2M = 256;                 // tile rows
constexpr int X2T = 512;                 // threads
constexpr int X2_AP = X2M * XS;          // bf16 per A plane
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4v __attribute__((ext_vector_type(4)));

template <bool KC, int ROWS>
struct X2Op {
  static constexpr int F = ROWS * XS / X2T;   // floats per thread per stage (16 or 8)
  static constexpr int SL = F / 8;            // 8-k slots per thread
  static constexpr int P = ROWS * XS;         // bf16 per plane
};

// One stage of an operand into registers.  The lane-dependent part of every offset is
// loop-invariant (voff: the lane's row, kOob for a row past the operand) and the
// k-dependent part is wave-uniform (the scalar offset), so a load costs no VALU work.  The
// buffer range check covers the vector offset only, never the scalar one, so a k past the
// operand (the prefetch of a stage beyond the end) must not reach the address: such a scalar
// offset is clamped to 0 (a real, unused element), and in KCHK mode a lane whose own k lies
// past K gets kOob.  KCHK: some stage may end inside [k0, k0 + 32) (K or the split chunk not
// a multiple of 32): values at k >= kend are zeroed.
template <bool KC, int ROWS, bool KCHK>
__device__ __forceinline__ void x2_load(__amdgpu_buffer_rsrc_t rs, int ld, const int (&voff)[2],
                                        int K, int kend, int k0, float (&v)[X2Op<KC, ROWS>::F]) {
  using O = X2Op<KC, ROWS>;
  constexpr int kOob = 0x7ffffff0;
  const int t = threadIdx.x;
  if (KC) {
    // voff[u] = (row_u * ld + 8 (t & 3)) * 4 of unit t + 512 u (rows 128 apart)
#pragma unroll
    for (int u = 0; u < O::SL; ++u) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int kw = k0 + 4 * h;                       // wave-uniform part of k
        const int so = kw < K ? kw * 4 : 0;
        const int kl = kw + 8 * (t & 3);                 // this lane's first k
        const int vo = (KCHK && kl >= K) ? kOob : voff[u];
        const f32x4 x = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, vo, so, 0));
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const bool ok = !KCHK || kl + c < kend;
          v[8 * u + 4 * h + c] = ok ? x[c] : 0.f;
        }
      }
    }
  } else {
    // voff[0] = row * 4; this wave's k run starts at k0 + F (t / ROWS) (wave-uniform)
    const int kb = k0 + O::F * __builtin_amdgcn_readfirstlane(t / ROWS);
#pragma unroll
    for (int j = 0; j < O::F; ++j) {
      const int k = kb + j;
      const float x = __builtin_bit_cast(
          float, __builtin_amdgcn_raw_buffer_load_b32(rs, voff[0], k < K ? k * ld * 4 : 0, 0));
      v[j] = (!KCHK || k < kend) ? x : 0.f;
    }
  }
}

// two fp32 -> (hi, mid, lo) bf16 pairs: v_cvt_pk_bf16_f32 (RNE), exact residuals
__device__ __forceinline__ void x2_split2(float x0, float x1, unsigned& h, unsigned& m,
                                          unsigned& l) {
  h = __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2{x0, x1}, bf16x2));
  const float r0 = x0 - __builtin_bit_cast(float, h << 16);
  const float r1 = x1 - __builtin_bit_cast(float, h & 0xffff0000u);
  m = __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2{r0, r1}, bf16x2));
  const float l0 = r0 - __builtin_bit_cast(float, m << 16);
  const float l1 = r1 - __builtin_bit_cast(float, m & 0xffff0000u);
  l = __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2{l0, l1}, bf16x2));
}

// NPL 3: the hi / mid / lo planes; NPL 1: the bf16 (RNE) rounding alone (the bf16-operand GEMM);
// NPL 2: the fp16 two-term split of the scaled value x sc (sc = 2^e, the operand row's scale:
// hi = f16(x sc), lo = f16(x sc - hi), RNE, the residual exact in fp32), two planes
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
template <int NPL = 3>
__device__ __forceinline__ void x2_split_store(unsigned short* __restrict__ s, int plane, int at,
                                               const float* v, float sc = 1.f) {
  if constexpr (NPL == 2) {
    u32x4v h, l;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const f32x2 x = f32x2{v[2 * j], v[2 * j + 1]} * sc;
      const f16x2 hh = __builtin_convertvector(x, f16x2);
      const f32x2 r = x - __builtin_convertvector(hh, f32x2);
      h[j] = __builtin_bit_cast(unsigned, hh);
      l[j] = __builtin_bit_cast(unsigned, __builtin_convertvector(r, f16x2));
    }
    *reinterpret_cast<u32x4v*>(s + at) = h;
    *reinterpret_cast<u32x4v*>(s + plane + at) = l;
  } else if constexpr (NPL == 1) {
    u32x4v h;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      h[j] = __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2{v[2 * j], v[2 * j + 1]}, bf16x2));
    *reinterpret_cast<u32x4v*>(s + at) = h;
  } else {
    u32x4v h, m, l;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      unsigned a, b, c;
#if defined(DS2_X6_ABL) && DS2_X6_ABL == 3
      // ablation build: the hi term only (no residual splits)
      a = __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2{v[2 * j], v[2 * j + 1]}, bf16x2));
      b = a;
      c = a;
#else
      x2_split2(v[2 * j], v[2 * j + 1], a, b, c);
#endif
      h[j] = a;
      m[j] = b;
      l[j] = c;
    }
    *reinterpret_cast<u32x4v*>(s + at) = h;
    *reinterpret_cast<u32x4v*>(s + plane + at) = m;
    *reinterpret_cast<u32x4v*>(s + 2 * plane + at) = l;
  }
}

// sc: the scales of the thread's staging rows (NPL 2): k-contiguous unit u -> sc[u]; a
// row-contiguous operand's thread row -> sc[0]
template <bool KC, int ROWS, int NPL = 3, bool M16 = false>
__device__ __forceinline__ void x2_store(unsigned short* __restrict__ s,
                                         const float (&v)[X2Op<KC, ROWS>::F],
                                         const float (&sc)[2] = {1.f, 1.f}) {
  using O = X2Op<KC, ROWS>;
  const int t = threadIdx.x;
  if (KC) {
#pragma unroll
    for (int u = 0; u < O::SL; ++u) {
      const int unit = t + X2T * u;
      x2_split_store<NPL>(s, O::P, xslot_t<M16>(unit >> 2, unit & 3), v + 8 * u, sc[u]);
    }
  } else {
    const int r = t % ROWS;
#pragma unroll
    for (int u = 0; u < O::SL; ++u)
      x2_split_store<NPL>(s, O::P, xslot_t<M16>(r, O::SL * (t / ROWS) + u), v + 8 * u, sc[0]);
  }
}

// c += a.b to fp32 accuracy on the 32x32x16 form (small terms first)
__device__ __forceinline__ void x2_mma6(const bf16x8 (&a)[3], const bf16x8 (&b)[3], f32x16& c) {
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[1], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2], b[0], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[2], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[0], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[1], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[0], c, 0, 0, 0);
}

// the same on the 16x16x32 form
__device__ __forceinline__ void x2_mma6_16(const bf16x8 (&a)[3], const bf16x8 (&b)[3], f32x4& c) {
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[1], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[2], b[0], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[2], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[0], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[1], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[0], c, 0, 0, 0);
}

// B stages of 160 rows (N = 800 / 2400 without a partial tile column): 640 (row, 8-k slot)
// units, units t and t + 512 (t < 128) per thread.  k-contiguous: as x2_load (wave-uniform
// scalar k offset); row-contiguous: rows 0..127 with the 128-row mapping (wave-uniform k),
// rows 128..159 (threads < 128, four slots per wave) with the whole offset in the vector
// register (range-checked).
template <bool KC, bool KCHK>
__device__ __forceinline__ void x2_load160(__amdgpu_buffer_rsrc_t rs, int ld, const int (&voff)[2],
                                           int rows_ok1, int K, int kend, int k0, float (&v)[16]) {
  constexpr int kOob = 0x7ffffff0;
  const int t = threadIdx.x;
  if (KC) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int kw = k0 + 4 * h;
        const int so = kw < K ? kw * 4 : 0;
        const int kl = kw + 8 * (t & 3);
        const int vo = (KCHK && kl >= K) ? kOob : voff[u];
        const f32x4 x = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, vo, so, 0));
#pragma unroll
        for (int c = 0; c < 4; ++c) v[8 * u + 4 * h + c] = (!KCHK || kl + c < kend) ? x[c] : 0.f;
      }
    }
  } else {
    const int kb = k0 + 8 * __builtin_amdgcn_readfirstlane(t >> 7);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = kb + j;
      const float x = __builtin_bit_cast(
          float, __builtin_amdgcn_raw_buffer_load_b32(rs, voff[0], k < K ? k * ld * 4 : 0, 0));
      v[j] = (!KCHK || k < kend) ? x : 0.f;
    }
    // rows 128..159: voff[1] = that row * 4 (kOob past N or for threads >= 128)
    const int k1 = k0 + 8 * ((t >> 5) & 3);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = k1 + j;
      const int vo = (rows_ok1 && k < K) ? voff[1] + k * ld * 4 : kOob;
      const float x = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, vo, 0, 0));
      v[8 + j] = (!KCHK || k < kend) ? x : 0.f;
    }
  }
}

template <bool KC, int NPL = 3, bool M16 = false>
__device__ __forceinline__ void x2_store160(unsigned short* __restrict__ s, const float (&v)[16],
                                            const float (&sc)[2] = {1.f, 1.f}) {
  constexpr int P = 160 * XS;
  const int t = threadIdx.x;
  if (KC) {
    x2_split_store<NPL>(s, P, xslot_t<M16>(t >> 2, t & 3), v, sc[0]);
    if (t < 128) x2_split_store<NPL>(s, P, xslot_t<M16>((t + X2T) >> 2, (t + X2T) & 3), v + 8, sc[1]);
  } else {
    x2_split_store<NPL>(s, P, xslot_t<M16>(t & 127, t >> 7), v, sc[0]);
    if (t < 128) x2_split_store<NPL>(s, P, xslot_t<M16>(128 + (t & 31), (t >> 5) & 3), v + 8, sc[1]);
  }
}

// NPL 3: the bf16x6 fp32-accurate GEMM; NPL 1: the bf16-operand GEMM (operands rounded to
// bf16 while staged, one product per fragment pair, fp32 accumulation -- cfg4's opt-in
// precision), one LDS plane per operand
template <int TA, int TB, bool KCHK, int TBN, int NPL = 3, bool M16 = false>
__global__ __launch_bounds__(X2T, 1) void sxgemm2_kernel(
    int M, int N, int K, float alpha, const float* __restrict__ A, int64_t lda, int64_t sA,
    const float* __restrict__ B, int64_t ldb, int64_t sB, float beta, float* __restrict__ C,
    int64_t ldc, int64_t sC, const float* __restrict__ bias, int main_wgs, int tail_tile0,
    int tail_tiles, int nsplit, int kchunk, float* __restrict__ partial,
    const unsigned* __restrict__ a_amax, const unsigned* __restrict__ b_amax) {
  constexpr bool AK = (TA == 0);
  constexpr bool BKc = (TB == 1);
  static_assert(TBN == 128 || TBN == 160, "tile width");
  static_assert(NPL != 2 || M16, "fp16x3: the 16x16x32 form");
  // waves: 4 (M) x 2 (N) of 2 x 2 32x32 tiles (TBN 128) or 8 (M) x 1 (N) of 1 x 5 (TBN 160);
  // M16: the same wave tiles as 4 x 4 / 2 x 10 16x16 tiles
  constexpr int TS = M16 ? 16 : 32;   // MFMA tile edge
  constexpr int WMT = (TBN == 128 ? 64 : 32) / TS, WNT = (TBN == 128 ? 64 : 160) / TS;
  using AccT = typename std::conditional<M16, f32x4, f32x16>::type;
  constexpr int AR = M16 ? 4 : 16;    // accumulator registers per tile
  constexpr int BP = TBN * XS;             // bf16 per B plane
  constexpr int BF = TBN == 128 ? 8 : 16;  // B floats per thread per stage
  using OA = X2Op<AK, X2M>;
  static_assert(NPL == 1 || NPL == 2 || NPL == 3, "planes");
  // the A and B stages back to back (the epilogue staging may span both)
  constexpr int SA = 2 * NPL * X2_AP, SB = 2 * NPL * BP;
  __shared__ __attribute__((aligned(16))) unsigned short smem[SA + SB];
  unsigned short (*const As)[NPL * X2_AP] = reinterpret_cast<unsigned short (*)[NPL * X2_AP]>(smem);
  unsigned short (*const Bs)[NPL * BP] = reinterpret_cast<unsigned short (*)[NPL * BP]>(smem + SA);

  // one job: C tile (m0, n0) over k in [kbeg, kend), into C or (part != null) a partial slab
  auto job = [&](const int m0, const int n0, const int kbeg, const int kend, float* const part) {
  const int a_rows = AK ? M : K, b_rows = BKc ? N : K;
  const __amdgpu_buffer_rsrc_t a_rs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(A), (short)0, static_cast<int>(a_rows * lda * 4), 0x00020000);
  const __amdgpu_buffer_rsrc_t b_rs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(B), (short)0, static_cast<int>(b_rows * ldb * 4), 0x00020000);
  const int ilda = static_cast<int>(lda), ildb = static_cast<int>(ldb);
  const int t = threadIdx.x;
  const int lane = t & 63;
  const int wave = t >> 6;
  const int wm = TBN == 128 ? (wave >> 1) * 64 : wave * 32;
  const int wn = TBN == 128 ? (wave & 1) * 64 : 0;
  const int fr = lane & 31, fk = lane >> 5;
  // loop-invariant lane offsets of the staging loads (kOob: a row past the operand); a
  // k-contiguous A unit 1 lies 128 rows below unit 0
  constexpr int kOob = 0x7ffffff0;
  int a_voff[2] = {kOob, kOob}, b_voff[2] = {kOob, kOob};
  if (AK) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int r = m0 + (t >> 2) + u * (X2T / 4);
      if (r < M) a_voff[u] = (r * ilda + 8 * (t & 3)) * 4;
    }
  } else {
    const int r = m0 + (t % X2M);
    if (r < M) a_voff[0] = r * 4;
  }
  int b_ok1 = 0;
  if (TBN == 128) {
    if (BKc) {
      const int r = n0 + (t >> 2);
      if (r < N) b_voff[0] = (r * ildb + 8 * (t & 3)) * 4;
    } else {
      const int r = n0 + (t % TBN);
      if (r < N) b_voff[0] = r * 4;
    }
  } else {
    if (BKc) {
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int unit = t + X2T * u;
        const int r = n0 + (unit >> 2);
        if (unit < 640 && r < N) b_voff[u] = (r * ildb + 8 * (t & 3)) * 4;
      }
    } else {
      const int r0 = n0 + (t & 127), r1 = n0 + 128 + (t & 31);
      if (r0 < N) b_voff[0] = r0 * 4;
      b_voff[1] = r1 * 4;
      b_ok1 = t < 128 && r1 < N;
    }
  }

  // fp16x3: the scale of each staging row (loop-invariant; NPL 3 / 1 ignore them)
  float a_sc[2] = {1.f, 1.f}, b_sc[2] = {1.f, 1.f};
  if constexpr (NPL == 2) {
    auto sc_of = [](const unsigned* am, int r, int lim) {
      return h3_scale(r < lim ? h3_exp(am[r]) : 0);
    };
    if (AK) {
#pragma unroll
      for (int u = 0; u < 2; ++u) a_sc[u] = sc_of(a_amax, m0 + (t >> 2) + u * (X2T / 4), M);
    } else {
      a_sc[0] = sc_of(a_amax, m0 + (t % X2M), M);
    }
    if (TBN == 128) {
      b_sc[0] = sc_of(b_amax, BKc ? n0 + (t >> 2) : n0 + (t % TBN), N);
    } else if (BKc) {
      b_sc[0] = sc_of(b_amax, n0 + (t >> 2), N);
      b_sc[1] = sc_of(b_amax, n0 + ((t + X2T) >> 2), N);
    } else {
      b_sc[0] = sc_of(b_amax, n0 + (t & 127), N);
      b_sc[1] = sc_of(b_amax, n0 + 128 + (t & 31), N);
    }
  }

  AccT acc[WMT][WNT];
#pragma unroll
  for (int i = 0; i < WMT; ++i)
#pragma unroll
    for (int j = 0; j < WNT; ++j)
#pragma unroll
      for (int r = 0; r < AR; ++r) acc[i][j][r] = 0.f;

  // two register sets: stage kt + 2's loads are issued at the top of stage kt (a whole
  // stage of latency) while the split of stage kt + 1 reads the other set
  float ra0[OA::F], rb0[BF], ra1[OA::F], rb1[BF];
  auto load = [&](int k0, float (&va)[OA::F], float (&vb)[BF]) {
#if defined(DS2_X6_ABL) && DS2_X6_ABL == 2
    // ablation build (scripts/gemm_ablation.sh): no global loads, run-time values instead
#pragma unroll
    for (int i = 0; i < OA::F; ++i) va[i] = __builtin_bit_cast(float, (unsigned)(t * 977 + k0 + i) | 0x3f000000u);
#pragma unroll
    for (int i = 0; i < BF; ++i) vb[i] = __builtin_bit_cast(float, (unsigned)(t * 613 + k0 + i) | 0x3f000000u);
#else
    x2_load<AK, X2M, KCHK>(a_rs, ilda, a_voff, K, kend, k0, va);
    if constexpr (TBN == 128)
      x2_load<BKc, TBN, KCHK>(b_rs, ildb, b_voff, K, kend, k0, vb);
    else
      x2_load160<BKc, KCHK>(b_rs, ildb, b_voff, b_ok1, K, kend, k0, vb);
#endif
  };
  auto bstore = [&](unsigned short* dst, const float (&vb)[BF]) {
    if constexpr (TBN == 128)
      x2_store<BKc, TBN, NPL, M16>(dst, vb, b_sc);
    else
      x2_store160<BKc, NPL, M16>(dst, vb, b_sc);
  };
  auto body = [&](int kt, int cur, float (&la)[OA::F], float (&lb)[BF],
                  const float (&sa)[OA::F], const float (&sb)[BF]) {
    // stage kt visible; every wave is done reading the other buffer (stage kt - 1)
#if defined(DS2_X6_ABL) && DS2_X6_ABL == 4
    __builtin_amdgcn_wave_barrier();   // ablation build: no workgroup barrier (results invalid)
#else
    __syncthreads();
#endif
    load(kbeg + (kt + 2) * XS, la, lb);          // stages past kend load as zeros
    const unsigned short* as = As[cur];
    const unsigned short* bs = Bs[cur];
    if constexpr (M16 && NPL == 2) {
      // fp16x3: two planes per operand, three v_mfma_f32_16x16x32_f16 per fragment pair
      // (lo.hi + hi.lo + hi.hi; lo.lo, below 2^-22 |a b|, dropped), same wave tiles and the
      // same interleave of the next stage's split and stores as the bf16x6 form below
      const int r16 = lane & 15, s16 = lane >> 4;
      f16x8 af[WMT][2];
#pragma unroll
      for (int i = 0; i < WMT; ++i) {
        const int at = xslot_t<true>(wm + 16 * i + r16, s16);
#pragma unroll
        for (int p = 0; p < 2; ++p) af[i][p] = *reinterpret_cast<const f16x8*>(as + p * X2_AP + at);
      }
#pragma unroll
      for (int j = 0; j < WNT; ++j) {
        f16x8 bq[2];
        const int bt = xslot_t<true>(wn + 16 * j + r16, s16);
#pragma unroll
        for (int p = 0; p < 2; ++p) bq[p] = *reinterpret_cast<const f16x8*>(bs + p * BP + bt);
#pragma unroll
        for (int i = 0; i < WMT; ++i) {
          AccT c = acc[i][j];
          c = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[i][1], bq[0], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[i][0], bq[1], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[i][0], bq[0], c, 0, 0, 0);
          acc[i][j] = c;
        }
      }
      x2_store<AK, X2M, NPL, true>(As[cur ^ 1], sa, a_sc);
      bstore(Bs[cur ^ 1], sb);
      constexpr int MPB = WMT * 3;   // MFMAs per B fragment
      __builtin_amdgcn_sched_group_barrier(0x020, 32, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 2 * WMT + 4, 0);
#pragma unroll
      for (int j = 0; j < WNT; ++j) {
#pragma unroll
        for (int q = 0; q < MPB; ++q) {   // 2 VALU per MFMA
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
        }
        if (j + 2 < WNT) __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
        __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);
      }
      return;
    } else if constexpr (M16) {
      static_assert(NPL == 3, "M16: bf16x6 or fp16x3 only");
      // one k-step of 32 per stage: the A fragments, then per B fragment (its three planes
      // read two fragments ahead) the WMT x 6 MFMAs it feeds, with the split VALU of stage
      // kt + 1 and its LDS stores interleaved
      const int r16 = lane & 15, s16 = lane >> 4;
      bf16x8 af[WMT][3];
#pragma unroll
      for (int i = 0; i < WMT; ++i) {
        const int at = xslot_t<true>(wm + 16 * i + r16, s16);
#pragma unroll
        for (int p = 0; p < 3; ++p) af[i][p] = *reinterpret_cast<const bf16x8*>(as + p * X2_AP + at);
      }
#pragma unroll
      for (int j = 0; j < WNT; ++j) {
        bf16x8 bq[3];
        const int bt = xslot_t<true>(wn + 16 * j + r16, s16);
#pragma unroll
        for (int p = 0; p < 3; ++p) bq[p] = *reinterpret_cast<const bf16x8*>(bs + p * BP + bt);
#pragma unroll
        for (int i = 0; i < WMT; ++i) {
#if defined(DS2_X6_ABL) && DS2_X6_ABL == 1
          // ablation build: no MFMA, the fragments kept live
          asm volatile("" ::"v"(af[i][0]), "v"(af[i][1]), "v"(af[i][2]), "v"(bq[0]), "v"(bq[1]), "v"(bq[2]));
#else
          x2_mma6_16(af[i], bq, acc[i][j]);
#endif
        }
      }
      x2_store<AK, X2M, NPL, true>(As[cur ^ 1], sa);
      bstore(Bs[cur ^ 1], sb);
      constexpr int MPB = WMT * 6;   // MFMAs per B fragment
      __builtin_amdgcn_sched_group_barrier(0x020, 32, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 3 * WMT + 6, 0);
#pragma unroll
      for (int j = 0; j < WNT; ++j) {
#pragma unroll
        for (int q = 0; q < MPB; q += 2) {   // 1.5 VALU per MFMA
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x002, 1, 0);
        }
        if (j + 2 < WNT) __builtin_amdgcn_sched_group_barrier(0x100, 3, 0);
        __builtin_amdgcn_sched_group_barrier(0x200, 2, 0);
      }
      return;
    }
    constexpr int NMF = WMT * WNT * (NPL == 3 ? 6 : 1);   // MFMAs per k-step
    constexpr int NRD = (WMT + WNT) * NPL;                 // fragment reads per k-step
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 af[WMT][3], bfr[WNT][3];
#pragma unroll
      for (int i = 0; i < WMT; ++i) {
        const int at = xslot(wm + 32 * i + fr, 2 * ks + fk);
#pragma unroll
        for (int p = 0; p < NPL; ++p) af[i][p] = *reinterpret_cast<const bf16x8*>(as + p * X2_AP + at);
      }
#pragma unroll
      for (int j = 0; j < WNT; ++j) {
        const int bt = xslot(wn + 32 * j + fr, 2 * ks + fk);
#pragma unroll
        for (int p = 0; p < NPL; ++p) bfr[j][p] = *reinterpret_cast<const bf16x8*>(bs + p * BP + bt);
      }
#pragma unroll
      for (int i = 0; i < WMT; ++i)
#pragma unroll
        for (int j = 0; j < WNT; ++j) {
          if constexpr (M16) {
          } else if constexpr (NPL == 3)
            x2_mma6(af[i], bfr[j], acc[i][j]);
          else
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i][0], bfr[j][0], acc[i][j], 0, 0, 0);
        }
    }
    // stage kt + 1 -> the other buffer (a stage past the end writes zeros nobody reads)
    x2_store<AK, X2M, NPL, M16>(As[cur ^ 1], sa);
    bstore(Bs[cur ^ 1], sb);
    // schedule: the loads, the first k-step's fragments, then each MFMA followed by up to
    // three VALU (the split of the next stage), the second k-step's fragments early, the
    // LDS stores of the split spread over the second half
    __builtin_amdgcn_sched_group_barrier(0x020, 32, 0);
    __builtin_amdgcn_sched_group_barrier(0x100, NRD, 0);
#pragma unroll
    for (int q = 0; q < NMF; ++q) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);
      if (q == NMF / 3) __builtin_amdgcn_sched_group_barrier(0x100, NRD, 0);
    }
#pragma unroll
    for (int q = 0; q < NMF; ++q) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);
      if (q % 3 == 2) __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);
    }
  };
  const int ktiles = (kend - kbeg + XS - 1) / XS;
  load(kbeg, ra0, rb0);
  x2_store<AK, X2M, NPL, M16>(As[0], ra0, a_sc);
  bstore(Bs[0], rb0);
  load(kbeg + XS, ra1, rb1);
  for (int kt = 0; kt < ktiles; kt += 2) {
    body(kt, 0, ra0, rb0, ra1, rb1);
    if (kt + 1 < ktiles) body(kt + 1, 1, ra1, rb1, ra0, rb0);
  }

  if constexpr (M16) {
    // epilogue through the now idle stage buffers, 16 rows of the wave tile per pass (16x16
    // C/D map: col = lane & 15, row = 4 (lane >> 4) + r, written row-major with a 4-float pad:
    // conflict-free), leaving as 16-B row runs -- each store instruction writes 1 KB of whole
    // row segments instead of sixteen 64-B pieces
    constexpr int EW = WNT * 16, EP = EW + 4;
    static_assert(8 * 16 * EP * 4 <= (SA + SB) * 2, "epilogue staging fits the stages");
    if constexpr (NPL == 2) {
      // undo the row scales: C = acc 2^-(e_a(row) - e_b(col)), exact unless the result
      // itself under- or overflows
#pragma unroll
      for (int i = 0; i < WMT; ++i) {
        int ea[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = m0 + wm + 16 * i + 4 * (lane >> 4) + r;
          ea[r] = row < M ? h3_exp(a_amax[row]) : 0;
        }
#pragma unroll
        for (int j = 0; j < WNT; ++j) {
          const int col = n0 + wn + 16 * j + (lane & 15);
          const int eb = col < N ? h3_exp(b_amax[col]) : 0;
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[i][j][r] = __builtin_ldexpf(acc[i][j][r], -(ea[r] + eb));
        }
      }
    }
    __syncthreads();   // every wave is done reading the last stage
    float* const stg = reinterpret_cast<float*>(smem) + wave * 16 * EP;
    const bool cv4 = ((reinterpret_cast<uintptr_t>(C) | static_cast<uintptr_t>(ldc * 4)) & 15) == 0 &&
                     (bias == nullptr || (reinterpret_cast<uintptr_t>(bias) & 15) == 0);
#pragma unroll
    for (int i = 0; i < WMT; ++i) {
#pragma unroll
      for (int j = 0; j < WNT; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) stg[(4 * (lane >> 4) + r) * EP + 16 * j + (lane & 15)] = acc[i][j][r];
#pragma unroll
      for (int q = 0; q < WNT; ++q) {
        const int idx = lane + 64 * q;
        const int rr = idx / (EW / 4), c4 = idx - (idx / (EW / 4)) * (EW / 4);
        const f32x4 v = *reinterpret_cast<const f32x4*>(stg + rr * EP + 4 * c4);
        const int rl = wm + 16 * i + rr, cl = wn + 4 * c4;
        if (part != nullptr) {
          *reinterpret_cast<f32x4*>(part + rl * TBN + cl) = v;
          continue;
        }
        const int row = m0 + rl, col = n0 + cl;
        if (row >= M || col >= N) continue;
        float* cp = C + (int64_t)row * ldc + col;
        if (cv4 && col + 3 < N) {
          f32x4 o = v * alpha;
          if (bias != nullptr) o += *reinterpret_cast<const f32x4*>(bias + col);
          if (beta != 0.f) o += beta * *reinterpret_cast<const f32x4*>(cp);
          *reinterpret_cast<f32x4*>(cp) = o;
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            if (col + e >= N) break;
            float o = alpha * v[e] + (bias != nullptr ? bias[col + e] : 0.f);
            if (beta != 0.f) o += beta * cp[e];
            cp[e] = o;
          }
        }
      }
    }
    return;
  }
  // epilogue (32x32 C/D map: col = lane & 31, row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5))
#pragma unroll
  for (int i = 0; i < WMT; ++i) {
#pragma unroll
    for (int j = 0; j < WNT; ++j) {
      const int cl = wn + 32 * j + (lane & 31);
      if (part != nullptr) {
#pragma unroll
        for (int r = 0; r < 16; ++r)
          part[(wm + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * fk) * TBN + cl] = acc[i][j][r];
        continue;
      }
      const int col = n0 + cl;
      if (col >= N) continue;
      const float bv = bias != nullptr ? bias[col] : 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * fk;
        if (row < M) {
          float* cp = C + (int64_t)row * ldc + col;
          float v = alpha * acc[i][j][r] + bv;
          if (beta != 0.f) v += beta * *cp;
          *cp = v;
        }
      }
    }
  }
  };   // job

  int m0, n0, kbeg, kend, bz;
  float* part;
  decode_work(M, N, K, main_wgs, tail_tile0, tail_tiles, nsplit, kchunk, partial, m0, n0, kbeg,
              kend, bz, part, TBN, X2M);
  A += bz * sA;
  B += bz * sB;
  C += bz * sC;
  job(m0, n0, kbeg, kend, part);
}

// Tail tiles: C[b] = alpha * sum_s partial[b][s][tile] + beta * C[b] + bias (fixed order).
// VEC (16-B aligned C rows and bias, bn % 4 == 0): each thread four consecutive columns, 16-B
// slab loads and C accesses -- the same per-element sums in the same order
template <bool VEC>
__global__ void splitk_reduce_kernel(const float* __restrict__ partial, int M, int N, int nsplit,
                                     int batch, int tail_tile0, int tail_tiles, float alpha,
                                     float beta, float* __restrict__ C, int64_t ldc, int64_t sC,
                                     const float* __restrict__ bias, int bn, int bm) {
  const int TE = bm * bn;
  const int tn = (N + bn - 1) / bn;
  if constexpr (VEC) {
    const int TE4 = TE / 4;
    const int64_t total4 = (int64_t)batch * tail_tiles * TE4;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total4;
         i += (int64_t)gridDim.x * blockDim.x) {
      const int e = static_cast<int>(i % TE4) * 4;
      const int64_t bt = i / TE4;
      const int lt = static_cast<int>(bt % tail_tiles);
      const int b = static_cast<int>(bt / tail_tiles);
      int tile_m, tile_n;
      tile_coords(tail_tile0 + lt, tn, (M + bm - 1) / bm, tile_m, tile_n);
      const int row = tile_m * bm + e / bn;
      const int col = tile_n * bn + e % bn;
      if (row >= M || col >= N) continue;
      f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 8
      for (int sp = 0; sp < nsplit; ++sp)
        acc += *reinterpret_cast<const f32x4*>(partial + (((int64_t)b * nsplit + sp) * tail_tiles + lt) * TE + e);
      float* cp = C + b * sC + (int64_t)row * ldc + col;
      if (col + 3 < N) {
        f32x4 v = alpha * acc;
        if (bias != nullptr) v += *reinterpret_cast<const f32x4*>(bias + col);
        if (beta != 0.f) v += beta * *reinterpret_cast<const f32x4*>(cp);
        *reinterpret_cast<f32x4*>(cp) = v;
      } else {
        for (int c = 0; c < 4 && col + c < N; ++c) {
          float v = alpha * acc[c] + (bias != nullptr ? bias[col + c] : 0.f);
          if (beta != 0.f) v += beta * cp[c];
          cp[c] = v;
        }
      }
    }
    return;
  }
  const int64_t total = (int64_t)batch * tail_tiles * TE;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int e = static_cast<int>(i % TE);
    const int64_t bt = i / TE;
    const int lt = static_cast<int>(bt % tail_tiles);
    const int b = static_cast<int>(bt / tail_tiles);
    const int tile = tail_tile0 + lt;
    int tile_m, tile_n;
    tile_coords(tile, tn, (M + bm - 1) / bm, tile_m, tile_n);
    const int row = tile_m * bm + e / bn;
    const int col = tile_n * bn + e % bn;
    if (row >= M || col >= N) continue;
    float acc = 0.f;
#pragma unroll 8
    for (int sp = 0; sp < nsplit; ++sp)   // loads in flight, summation order kept
      acc += partial[(((int64_t)b * nsplit + sp) * tail_tiles + lt) * TE + e];
    float* cp = C + b * sC + (int64_t)row * ldc + col;
    float v = alpha * acc + (bias != nullptr ? bias[col] : 0.f);
    if (beta != 0.f) v += beta * *cp;
    *cp = v;
  }
}

template <int TA, int TB>
static void launch_sgemm_t(bool va, bool vb, dim3 grid, hipStream_t st, int M, int N, int K,
                           float alpha, const float* A, int64_t lda, int64_t sA, const float* B,
                           int64_t ldb, int64_t sB, float beta, float* C, int64_t ldc,
                           int64_t sC, const float* bias, int main_wgs, int tail_tile0,
                           int tail_tiles, int nsplit, int kchunk, float* partial) {
#define DS2_L(VA, VB)                                                                      \
  hipLaunchKernelGGL((sgemm_kernel<TA, TB, VA, VB>), grid, dim3(256), 0, st, M, N, K, alpha, A, \
                     lda, sA, B, ldb, sB, beta, C, ldc, sC, bias, main_wgs, tail_tile0,        \
                     tail_tiles, nsplit, kchunk, partial)
  if (va && vb) DS2_L(true, true);
  else if (va) DS2_L(true, false);
  else if (vb) DS2_L(false, true);
  else DS2_L(false, false);
#undef DS2_L
}

template <int TA, int TB>
static void launch_k64(int bn, dim3 grid, hipStream_t st, int M, int N, int K,
                       float alpha, const float* A, int64_t lda, int64_t sA, const float* B,
                       int64_t ldb, int64_t sB, float beta, float* C, int64_t ldc, int64_t sC,
                       const float* bias, int main_wgs, int tail_tile0, int tail_tiles,
                       int nsplit, int kchunk, float* partial) {
#define DS2_K(WN)                                                                           \
  hipLaunchKernelGGL((sgemm64_kernel<TA, TB, WN, 64, 1>), grid, dim3(256), 0, st, M, N, K,     \
                     alpha, A, lda, sA, B, ldb, sB, beta, C, ldc, sC, bias, main_wgs,          \
                     tail_tile0, tail_tiles, nsplit, kchunk, partial)
  if (bn == 160) DS2_K(5);
  else DS2_K(4);
#undef DS2_K
}

static inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

// fp16x3 row scales (sxgemm2_kernel NPL 2): max |x| of every logical operand row, as float
// bits.  A logical row that is a stored row: one wave per row, float4 loads, a wave max.
__global__ __launch_bounds__(256) void amax_rows_kernel(const float* __restrict__ p, int rows,
                                                        int cols, int64_t ld,
                                                        unsigned* __restrict__ out) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (r >= rows) return;
  const f32x4* q = reinterpret_cast<const f32x4*>(p + (int64_t)r * ld);
  float m = 0.f;
  const int c4 = cols / 4;
  int c = lane;
  // up to 10 loads in flight per lane at once for rows up to 2560 columns (one batch instead of
  // two of 4 and two single loads; 22.6 -> 22.1 us on 16032 x 2400, 6.98 TB/s)
  if (c4 <= 640) {
    f32x4 v[10];
#pragma unroll
    for (int k = 0; k < 10; ++k)
      v[k] = c + 64 * k < c4 ? q[c + 64 * k] : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < 10; ++k)
      m = fmaxf(m, fmaxf(fmaxf(fabsf(v[k][0]), fabsf(v[k][1])), fmaxf(fabsf(v[k][2]), fabsf(v[k][3]))));
    c = c4;
  }
  // 4 loads in flight per lane (a 4800-column row is 19 per lane)
  for (; c + 192 < c4; c += 256) {
    const f32x4 v0 = q[c], v1 = q[c + 64], v2 = q[c + 128], v3 = q[c + 192];
#pragma unroll
    for (int e = 0; e < 4; ++e)
      m = fmaxf(m, fmaxf(fmaxf(fabsf(v0[e]), fabsf(v1[e])), fmaxf(fabsf(v2[e]), fabsf(v3[e]))));
  }
  for (; c < c4; c += 64) {
    const f32x4 v = q[c];
    m = fmaxf(m, fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3]))));
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  if (lane == 0) out[r] = __builtin_bit_cast(unsigned, m);
}

// Column maxima only (ds2_amax with row_amax NULL): one wave per block, a float4 column group
// per lane, `rpb` rows per block with 8 loads in flight per lane, then one unsigned atomic max
// per column (`out` zeroed first).
__global__ __launch_bounds__(64) void amax_cols8_kernel(const float* __restrict__ p, int rows,
                                                        int cols, int64_t ld, int rpb,
                                                        unsigned* __restrict__ out) {
  const int c = (blockIdx.x * 64 + threadIdx.x) * 4;
  if (c >= cols) return;
  const int r0 = blockIdx.y * rpb, r1 = min(rows, r0 + rpb);
  const float* base = p + c;
  f32x4 m = f32x4{0.f, 0.f, 0.f, 0.f};
  int r = r0;
  for (; r + 8 <= r1; r += 8) {
    f32x4 v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = *reinterpret_cast<const f32x4*>(base + (int64_t)(r + i) * ld);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) m[e] = fmaxf(m[e], fabsf(v[i][e]));
  }
  for (; r < r1; ++r) {
    const f32x4 v = *reinterpret_cast<const f32x4*>(base + (int64_t)r * ld);
#pragma unroll
    for (int e = 0; e < 4; ++e) m[e] = fmaxf(m[e], fabsf(v[e]));
  }
  // (each element copied to a scalar first: hipcc 7.2 bit_cast an ext_vector element
  // straight into the atomic's data as element 0 for every e)
  const float me[4] = {m[0], m[1], m[2], m[3]};
#pragma unroll
  for (int e = 0; e < 4; ++e)
    if (me[e] > 0.f) atomicMax(out + c + e, __float_as_uint(me[e]));
}

// Row AND column maxima in one pass (ds2_amax): a block covers 1024 columns (a float4 per
// thread) of `rpb` (<= 64) rows; each thread folds its 4 columns' maxima over the rows in
// registers and each row's maximum over the block's columns into an LDS word (ds_max_u32), and
// the block then folds both into the outputs with unsigned atomic max (both zeroed first).
__global__ __launch_bounds__(256) void amax_both_kernel(const float* __restrict__ p, int rows,
                                                        int cols, int64_t ld, int rpb,
                                                        unsigned* __restrict__ rmax,
                                                        unsigned* __restrict__ cmax) {
  __shared__ unsigned rm[64];
  const int c = (blockIdx.x * 256 + threadIdx.x) * 4;
  const bool in = c < cols;
  const int r0 = blockIdx.y * rpb, r1 = min(rows, r0 + rpb);
  if (threadIdx.x < 64) rm[threadIdx.x] = 0u;
  __syncthreads();
  f32x4 m = f32x4{0.f, 0.f, 0.f, 0.f};
  if (in) {
    for (int r = r0; r < r1; ++r) {
      const f32x4 v = *reinterpret_cast<const f32x4*>(p + (int64_t)r * ld + c);
      const float a0 = fabsf(v[0]), a1 = fabsf(v[1]), a2 = fabsf(v[2]), a3 = fabsf(v[3]);
      m[0] = fmaxf(m[0], a0);
      m[1] = fmaxf(m[1], a1);
      m[2] = fmaxf(m[2], a2);
      m[3] = fmaxf(m[3], a3);
      if (rmax != nullptr) {
        const float w = fmaxf(fmaxf(a0, a1), fmaxf(a2, a3));
        if (w > 0.f) atomicMax(&rm[r - r0], __float_as_uint(w));
      }
    }
  }
  if (cmax != nullptr && in) {
    // (each element copied to a scalar first: hipcc 7.2 bit_cast an ext_vector element
    // straight into the atomic's data as element 0 for every e)
    const float me[4] = {m[0], m[1], m[2], m[3]};
#pragma unroll
    for (int e = 0; e < 4; ++e)
      if (me[e] > 0.f) atomicMax(cmax + c + e, __float_as_uint(me[e]));
  }
  if (rmax != nullptr) {
    __syncthreads();
    if (threadIdx.x < r1 - r0 && rm[threadIdx.x] != 0u) atomicMax(rmax + r0 + threadIdx.x, rm[threadIdx.x]);
  }
}

// amax of the `lrows` logical rows of an operand stored [lrows][k] (rowwise) or [k][lrows]
static void launch_amax(const float* p, bool rowwise, int lrows, int k, int64_t ld, unsigned* out,
                        hipStream_t st) {
  if (rowwise) {
    hipLaunchKernelGGL(amax_rows_kernel, dim3(cdiv(lrows, 4)), dim3(256), 0, st, p, lrows, k, ld,
                       out);
    return;
  }
  (void)hipMemsetAsync(out, 0, (size_t)lrows * 4, st);
  hipLaunchKernelGGL(amax_cols8_kernel, dim3(cdiv(lrows, 256), cdiv(k, 64)), dim3(64), 0, st, p, k,
                     lrows, ld, 64, out);
}

}  // namespace ds2

using namespace ds2;

static int g_cus = -1;
static int device_cus() {
  if (g_cus < 0) {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess) dev = 0;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        v <= 0)
      v = 256;
    g_cus = v;
  }
  return g_cus;
}

// Work plan.  Whole tiles run in full rounds of `slots` resident workgroups (3 per CU);
// the tiles of a last, partial round ("tail") have their K range split so that the
// round is filled: e.g. the input projection 16032 x 2400 = 2394 tiles = 3 rounds of
// 768 + 90 tail tiles x 8 splits; the weight gradient 2400 x 800 (133 tiles, K = 16032)
// becomes 133 tiles x 5 splits.  Split partials are reduced in a fixed order.
struct GemmPlan {
  int main_wgs, tail_tile0, tail_tiles, nsplit, kchunk, bn, bm;
};

// DS2_GEMM_X6=0 selects the fp32-MFMA kernels (the accuracy cross-check of the tests); the
// bf16x6 kernel needs float4-staged operands (the fp32 kernels take any alignment; the
// deep-K sgemm64_kernel runs 2 workgroups per CU and BK = 64, the original one 3 per CU and
// BK = 16, for operands that are not float4-aligned)
static bool x6_enabled(bool va, bool vb) {
  if (!va || !vb) return false;
  const char* e = getenv("DS2_GEMM_X6");
  return !(e != nullptr && e[0] == '0');
}

// 32-bit buffer offsets: each operand (one batch entry) must span < 2^31 bytes
static bool fits_rsrc(int64_t rows, int64_t ld) { return rows * ld * 4 < (1ll << 31); }

// Plan for tile width bn.  The split count s of the tail is chosen by a time model in
// units of one workgroup slot's MFMA time per (128-row x k) tile step: whole rounds
// cost k each, the tail ceil(pieces / slots) * kchunk; a split adds its partial-slab
// write + read (8 B per element at ~4 TB/s) and the reduce launch.  `eff` is the tile's
// relative MFMA efficiency (160-wide tiles: 5 B fragments per 4 A, measured ~7 % faster
// per unit of work than 128-wide in isolation; 1.15 in the plan, where it also stands in
// for the 160-wide tile's smaller tail: a whole training step measured 1.0 < 1.07 < 1.15
// ~ 1.25 ~ 1.4, the last three within noise).
struct PlanChoice {
  GemmPlan p;
  double t;   // seconds (model)
};

static PlanChoice plan_bn(int m, int n, int k, int batch, int bn, int slots, int bk,
                          double eff, int bm = BM) {
  const int tiles = cdiv(m, bm) * cdiv(n, bn);
  GemmPlan p{0, 0, tiles, 1, std::max(k, 1), bn, bm};
  if (batch == 1) {
    p.main_wgs = (tiles / slots) * slots;
    p.tail_tile0 = p.main_wgs;
    p.tail_tiles = tiles - p.main_wgs;
    if (p.tail_tiles == 0) {   // full rounds only
      p.main_wgs = 0;
      p.tail_tile0 = 0;
      p.tail_tiles = tiles;
    }
  }
  // seconds per unit (one k step of one BM x bn tile on one slot)
  const double unit = 2.0 * bm * bn / (157.3e12 * eff / slots);
  const double main_t = (double)(p.main_wgs / slots) * k * unit;
  const int64_t tail = (int64_t)p.tail_tiles * batch;
  const int smax = std::max(1, std::min(32, k / 256));
  double best = 1e30;
  int bs = 1;
  for (int s = 1; s <= smax; ++s) {
    const int kc = cdiv(cdiv(k, s), bk) * bk;
    const int ns = cdiv(k, kc);
    if (s > 1 && ns != s) continue;
    const int64_t pieces = tail * ns;
    double t = (double)((pieces + slots - 1) / slots) * kc * unit;
    if (ns > 1) t += (double)pieces * bm * bn * 8.0 / 4e12 + 6e-6;
    if (t < best - 1e-12) {
      best = t;
      bs = ns;
    }
  }
  if (bs > 1) {
    p.kchunk = cdiv(cdiv(k, bs), bk) * bk;
    p.nsplit = cdiv(k, p.kchunk);
  }
  return {p, main_t + best};
}

// 160-wide tiles are ~7 % faster per unit of work than 128-wide in isolation (5 B fragments
// per 4 A); 1.15 in the time model, where it also stands in for the 160-wide tile's smaller
// tail (a whole training step measured 1.0 < 1.07 < 1.15 ~ 1.25 ~ 1.4, the last three
// within noise)
constexpr double kEff160 = 1.15;

static GemmPlan gemm_plan(int m, int n, int k, int batch, bool k64) {
  const int cus = device_cus();
  if (!k64) return plan_bn(m, n, k, batch, BN, 3 * cus, BK, 1.0).p;
  const PlanChoice a = plan_bn(m, n, k, batch, 128, 2 * cus, K64, 1.0);
  const PlanChoice b = plan_bn(m, n, k, batch, 160, 2 * cus, K64, kEff160);
  return b.t < a.t ? b.p : a.p;
}

static size_t plan_ws(const GemmPlan& p, int batch) {
  return p.nsplit > 1 ? (size_t)p.nsplit * batch * p.tail_tiles * p.bm * p.bn * sizeof(float) + 256
                      : 0;
}

// the bf16x6 kernel: 256-row tiles, one workgroup per CU, split-K in 32-k chunks; 160-wide
// tiles measured faster on every step shape with N >= 800 (scripts/bench_gemm_x6.py: 180-201
// vs 159-194 TF), 128-wide on narrow N (the FC's 29 columns)
static GemmPlan x6_plan(int m, int n, int k, int batch) {
  return plan_bn(m, n, k, batch, n >= 256 ? 160 : 128, device_cus(), XS, 1.0, X2M).p;
}

// fp16x3 (default since round 5; DS2_GEMM_H3=0 selects the bf16x6 kernel): the x6 kernel's
// plan and tiles with the operands split into two fp16 terms of row-scaled values and three
// products per pair (see x2_split_store); the row maxima come from the caller
// (ds2_sgemm_amax_ws) or from a pre-pass over each operand into the workspace after the
// split-K slabs.  On the step's shapes 1.4-1.7x the bf16x6 kernel's rate at equal or lower
// error against fp64 (scripts/bench_gemm_h3.py, profiles/r5b_gemm_h3_vs_x6.txt).
static bool h3_enabled() {
  const char* e = getenv("DS2_GEMM_H3");
  return !(e != nullptr && e[0] == '0');
}
static size_t h3_ws(int m, int n) { return (size_t)(m + n) * 4 + 512; }

extern "C" ds2_status_t ds2_amax(const float* x, int rows, int cols, int64_t ld,
                                 unsigned* row_amax, unsigned* col_amax, ds2_stream_t stream) {
  if (rows < 0 || cols < 0 || ld < cols) return DS2_INVALID_VALUE;
  if (rows == 0 || cols == 0 || (row_amax == nullptr && col_amax == nullptr)) return DS2_OK;
  if (x == nullptr || !aligned16(x) || (cols % 4) != 0 || (ld % 4) != 0)
    return DS2_UNSUPPORTED_SHAPE;
  hipStream_t st = as_stream(stream);
  if (col_amax == nullptr) {            // rows only: one wave per row, no atomics
    hipLaunchKernelGGL(amax_rows_kernel, dim3(cdiv(rows, 4)), dim3(256), 0, st, x, rows, cols,
                       ld, row_amax);
    return launch_status("ds2_amax");
  }
  (void)hipMemsetAsync(col_amax, 0, (size_t)cols * 4, st);
  if (row_amax == nullptr) {            // columns only: one wave per 256 columns x 64 rows
    hipLaunchKernelGGL(amax_cols8_kernel, dim3(cdiv(cols, 256), cdiv(rows, 64)), dim3(64), 0, st,
                       x, rows, cols, ld, 64, col_amax);
    return launch_status("ds2_amax");
  }
  if (cols <= 2048) {                   // narrow (a weight matrix): one wave per row
    launch_rows_amax<false>(x, rows, cols, ld, nullptr, nullptr, nullptr, nullptr, nullptr,
                            row_amax, col_amax, st);
    return launch_status("ds2_amax");
  }
  (void)hipMemsetAsync(row_amax, 0, (size_t)rows * 4, st);
  const int cb = cdiv(cols, 1024);
  const int rpb = std::min(64, std::max(16, cdiv((int64_t)rows * cb, 2048)));
  hipLaunchKernelGGL(amax_both_kernel, dim3(cb, cdiv(rows, rpb)), dim3(256), 0, st, x, rows, cols,
                     ld, rpb, row_amax, col_amax);
  return launch_status("ds2_amax");
}

// large enough for any kernel's plan (the choice depends on operand alignment)
extern "C" size_t ds2_sgemm_workspace_size(int m, int n, int k, int batch) {
  if (m <= 0 || n <= 0 || k <= 0 || batch <= 0) return 0;
  return std::max(std::max(plan_ws(gemm_plan(m, n, k, batch, false), batch),
                           plan_ws(gemm_plan(m, n, k, batch, true), batch)),
                  plan_ws(x6_plan(m, n, k, batch), batch) + h3_ws(m, n));
}

static ds2_status_t sgemm_run(int trans_a, int trans_b, int m, int n, int k, float alpha,
                              const float* a, int64_t lda, int64_t stride_a, const float* b,
                              int64_t ldb, int64_t stride_b, float beta, float* c, int64_t ldc,
                              int64_t stride_c, int batch, const float* bias, void* ws,
                              size_t ws_bytes, const unsigned* a_amax_in,
                              const unsigned* b_amax_in, ds2_stream_t stream);

extern "C" ds2_status_t ds2_sgemm_ws(int trans_a, int trans_b, int m, int n, int k, float alpha,
                                     const float* a, int64_t lda, int64_t stride_a,
                                     const float* b, int64_t ldb, int64_t stride_b, float beta,
                                     float* c, int64_t ldc, int64_t stride_c, int batch,
                                     const float* bias, void* ws, size_t ws_bytes,
                                     ds2_stream_t stream) {
  return sgemm_run(trans_a, trans_b, m, n, k, alpha, a, lda, stride_a, b, ldb, stride_b, beta, c,
                   ldc, stride_c, batch, bias, ws, ws_bytes, nullptr, nullptr, stream);
}

extern "C" ds2_status_t ds2_sgemm_amax_ws(int trans_a, int trans_b, int m, int n, int k,
                                          float alpha, const float* a, int64_t lda,
                                          const float* b, int64_t ldb, float beta, float* c,
                                          int64_t ldc, const float* bias, const unsigned* a_amax,
                                          const unsigned* b_amax, void* ws, size_t ws_bytes,
                                          ds2_stream_t stream) {
  return sgemm_run(trans_a, trans_b, m, n, k, alpha, a, lda, 0, b, ldb, 0, beta, c, ldc, 0, 1,
                   bias, ws, ws_bytes, a_amax, b_amax, stream);
}

static ds2_status_t sgemm_run(int trans_a, int trans_b, int m, int n, int k, float alpha,
                              const float* a, int64_t lda, int64_t stride_a, const float* b,
                              int64_t ldb, int64_t stride_b, float beta, float* c, int64_t ldc,
                              int64_t stride_c, int batch, const float* bias, void* ws,
                              size_t ws_bytes, const unsigned* a_amax_in,
                              const unsigned* b_amax_in, ds2_stream_t stream) {
  if (m < 0 || n < 0 || k < 0 || batch < 0) return DS2_INVALID_VALUE;
  if (m == 0 || n == 0 || batch == 0) return DS2_OK;
  if (ldc < n) return DS2_INVALID_VALUE;
  if (trans_a ? lda < m : lda < k) return DS2_INVALID_VALUE;
  if (trans_b ? ldb < k : ldb < n) return DS2_INVALID_VALUE;
  // vector (float4) staging is legal when every float4 is fully in or out of bounds
  const bool va = aligned16(a) && (lda % 4 == 0) && (stride_a % 4 == 0) &&
                  (trans_a ? (m % 4 == 0) : (k % 4 == 0));
  const bool vb = aligned16(b) && (ldb % 4 == 0) && (stride_b % 4 == 0) &&
                  (trans_b ? (k % 4 == 0) : (n % 4 == 0));
  const bool fits = fits_rsrc(trans_a ? k : m, lda) && fits_rsrc(trans_b ? n : k, ldb);
  const bool x6 = fits && x6_enabled(va, vb);
  const bool k64 = !x6 && va && vb && fits;
  GemmPlan p = x6 ? x6_plan(m, n, k, batch) : gemm_plan(m, n, k, batch, k64);
  if (p.nsplit > 1 && (ws == nullptr || ws_bytes < plan_ws(p, batch))) {
    p.nsplit = 1;                       // no workspace: whole-K pieces
    p.kchunk = std::max(k, 1);
  }
  float* partial = p.nsplit > 1 ? static_cast<float*>(ws) : nullptr;
  const int64_t nwg = p.main_wgs + (int64_t)p.tail_tiles * batch * p.nsplit;
  if (nwg > 0x7fffffff) return DS2_UNSUPPORTED_SHAPE;
  dim3 grid(static_cast<unsigned>(nwg));
  hipStream_t st = as_stream(stream);
  // every stage of every piece lies wholly inside [0, K): no per-element k check
  const bool kalign = k % XS == 0 && (p.nsplit == 1 || p.kchunk % XS == 0);
#define DS2_X6(TA_, TB_, KCHK_, BN_, M16_)                                                    \
  hipLaunchKernelGGL((sxgemm2_kernel<TA_, TB_, KCHK_, BN_, 3, M16_>), grid, dim3(X2T), 0, st,   \
                     m, n, k, alpha, a, lda, stride_a, b, ldb, stride_b, beta, c, ldc,          \
                     stride_c, bias, p.main_wgs, p.tail_tile0, p.tail_tiles, p.nsplit,          \
                     p.kchunk, partial, nullptr, nullptr)
#define DS2_H3(TA_, TB_, BN_)                                                                   \
  hipLaunchKernelGGL((sxgemm2_kernel<TA_, TB_, false, BN_, 2, true>), grid, dim3(X2T), 0, st,   \
                     m, n, k, alpha, a, lda, stride_a, b, ldb, stride_b, beta, c, ldc,          \
                     stride_c, bias, p.main_wgs, p.tail_tile0, p.tail_tiles, p.nsplit,          \
                     p.kchunk, partial, a_amax, b_amax)
  // the 16x16x32 form wherever every stage lies inside K (r4d: 0-15 % faster on the step's
  // shapes, profiles/r4d_gemm_x6_m16_sk_ab.txt), the 32x32x16 form for a K tail
  const bool m16 = x6 && kalign;
  const size_t slabs = p.nsplit > 1 ? plan_ws(p, batch) : 0;
  const bool h3 = m16 && batch == 1 && h3_enabled() && ws != nullptr &&
                  ws_bytes >= slabs + h3_ws(m, n);
  const unsigned* a_amax = a_amax_in;
  const unsigned* b_amax = b_amax_in;
  if (h3) {
    const uintptr_t base = (reinterpret_cast<uintptr_t>(ws) + slabs + 255) & ~uintptr_t(255);
    unsigned* wa = reinterpret_cast<unsigned*>(base);
    unsigned* wb = wa + m;
    if (a_amax == nullptr) {
      launch_amax(a, !trans_a, m, k, lda, wa, st);
      a_amax = wa;
    }
    if (b_amax == nullptr) {
      launch_amax(b, trans_b != 0, n, k, ldb, wb, st);
      b_amax = wb;
    }
  }
#define DS2_G(TA_, TB_)                                                                       \
  if (h3 && p.bn == 160) DS2_H3(TA_, TB_, 160);                                               \
  else if (h3) DS2_H3(TA_, TB_, 128);                                                         \
  else if (m16 && p.bn == 160) DS2_X6(TA_, TB_, false, 160, true);                          \
  else if (m16) DS2_X6(TA_, TB_, false, 128, true);                                          \
  else if (x6 && kalign && p.bn == 160) DS2_X6(TA_, TB_, false, 160, false);                 \
  else if (x6 && p.bn == 160) DS2_X6(TA_, TB_, true, 160, false);                            \
  else if (x6 && kalign) DS2_X6(TA_, TB_, false, 128, false);                                \
  else if (x6) DS2_X6(TA_, TB_, true, 128, false);                                           \
  else if (k64)                                                                               \
    launch_k64<TA_, TB_>(p.bn, grid, st, m, n, k, alpha, a, lda, stride_a, b, ldb, stride_b,   \
                         beta, c, ldc, stride_c, bias, p.main_wgs, p.tail_tile0, p.tail_tiles,  \
                         p.nsplit, p.kchunk, partial);                                         \
  else                                                                                        \
    launch_sgemm_t<TA_, TB_>(va, vb, grid, st, m, n, k, alpha, a, lda, stride_a, b, ldb,       \
                             stride_b, beta, c, ldc, stride_c, bias, p.main_wgs, p.tail_tile0, \
                             p.tail_tiles, p.nsplit, p.kchunk, partial)
  if (!trans_a && !trans_b) {
    DS2_G(0, 0);
  } else if (!trans_a && trans_b) {
    DS2_G(0, 1);
  } else if (trans_a && !trans_b) {
    DS2_G(1, 0);
  } else {
    DS2_G(1, 1);
  }
#undef DS2_G
#undef DS2_X6
#undef DS2_H3
  if (p.nsplit > 1) {
    const bool vec = p.bn % 4 == 0 && aligned16(c) && ldc % 4 == 0 && stride_c % 4 == 0 &&
                     (bias == nullptr || aligned16(bias));
    const int64_t total = (int64_t)batch * p.tail_tiles * p.bm * p.bn / (vec ? 4 : 1);
    int g = cdiv(total, 256);
    if (g > 4096) g = 4096;
    if (vec)
      hipLaunchKernelGGL(splitk_reduce_kernel<true>, dim3(g), dim3(256), 0, st, partial, m, n,
                         p.nsplit, batch, p.tail_tile0, p.tail_tiles, alpha, beta, c, ldc,
                         stride_c, bias, p.bn, p.bm);
    else
      hipLaunchKernelGGL(splitk_reduce_kernel<false>, dim3(g), dim3(256), 0, st, partial, m, n,
                         p.nsplit, batch, p.tail_tile0, p.tail_tiles, alpha, beta, c, ldc,
                         stride_c, bias, p.bn, p.bm);
  }
  return launch_status("ds2_sgemm");
}

// bf16-operand GEMM (sbgemm_kernel): same contract as ds2_sgemm_ws; every operand must be
// float4-staged (16-B aligned, ld and the contiguous extent multiples of 4) and span
// < 2^31 bytes, else DS2_UNSUPPORTED_SHAPE (no silent fp32 fallback).
extern "C" size_t ds2_sgemm_bf16_workspace_size(int m, int n, int k, int batch) {
  if (m <= 0 || n <= 0 || k <= 0 || batch <= 0) return 0;
  return plan_ws(plan_bn(m, n, k, batch, 128, 2 * device_cus(), KB16, 1.0).p, batch);
}

extern "C" ds2_status_t ds2_sgemm_bf16_ws(int trans_a, int trans_b, int m, int n, int k,
                                          float alpha, const float* a, int64_t lda,
                                          int64_t stride_a, const float* b, int64_t ldb,
                                          int64_t stride_b, float beta, float* c, int64_t ldc,
                                          int64_t stride_c, int batch, const float* bias,
                                          void* ws, size_t ws_bytes, ds2_stream_t stream) {
  if (m < 0 || n < 0 || k < 0 || batch < 0) return DS2_INVALID_VALUE;
  if (m == 0 || n == 0 || batch == 0) return DS2_OK;
  if (ldc < n) return DS2_INVALID_VALUE;
  if (trans_a ? lda < m : lda < k) return DS2_INVALID_VALUE;
  if (trans_b ? ldb < k : ldb < n) return DS2_INVALID_VALUE;
  const bool va = aligned16(a) && (lda % 4 == 0) && (stride_a % 4 == 0) &&
                  (trans_a ? (m % 4 == 0) : (k % 4 == 0));
  const bool vb = aligned16(b) && (ldb % 4 == 0) && (stride_b % 4 == 0) &&
                  (trans_b ? (k % 4 == 0) : (n % 4 == 0));
  if (!va || !vb || !fits_rsrc(trans_a ? k : m, lda) || !fits_rsrc(trans_b ? n : k, ldb))
    return DS2_UNSUPPORTED_SHAPE;
  GemmPlan p = plan_bn(m, n, k, batch, 128, 2 * device_cus(), KB16, 1.0).p;
  if (p.nsplit > 1 && (ws == nullptr || ws_bytes < plan_ws(p, batch))) {
    p.nsplit = 1;
    p.kchunk = std::max(k, 1);
  }
  float* partial = p.nsplit > 1 ? static_cast<float*>(ws) : nullptr;
  const int64_t nwg = p.main_wgs + (int64_t)p.tail_tiles * batch * p.nsplit;
  if (nwg > 0x7fffffff) return DS2_UNSUPPORTED_SHAPE;
  dim3 grid(static_cast<unsigned>(nwg));
  hipStream_t st = as_stream(stream);
#define DS2_B(TA_, TB_)                                                                        \
  hipLaunchKernelGGL((sbgemm_kernel<TA_, TB_>), grid, dim3(256), 0, st, m, n, k, alpha, a, lda, \
                     stride_a, b, ldb, stride_b, beta, c, ldc, stride_c, bias, p.main_wgs,      \
                     p.tail_tile0, p.tail_tiles, p.nsplit, p.kchunk, partial)
  if (!trans_a && !trans_b) DS2_B(0, 0);
  else if (!trans_a && trans_b) DS2_B(0, 1);
  else if (trans_a && !trans_b) DS2_B(1, 0);
  else DS2_B(1, 1);
#undef DS2_B
  if (p.nsplit > 1) {
    const int64_t total = (int64_t)batch * p.tail_tiles * p.bm * p.bn;
    int g = cdiv(total, 256);
    if (g > 4096) g = 4096;
    hipLaunchKernelGGL(splitk_reduce_kernel<false>, dim3(g), dim3(256), 0, st, partial, m, n, p.nsplit,
                       batch, p.tail_tile0, p.tail_tiles, alpha, beta, c, ldc, stride_c, bias,
                       p.bn, p.bm);
  }
  return launch_status("ds2_sgemm_bf16");
}

extern "C" ds2_status_t ds2_sgemm(int trans_a, int trans_b, int m, int n, int k, float alpha,
                                  const float* a, int64_t lda, int64_t stride_a, const float* b,
                                  int64_t ldb, int64_t stride_b, float beta, float* c,
                                  int64_t ldc, int64_t stride_c, int batch, const float* bias,
                                  ds2_stream_t stream) {
  return ds2_sgemm_ws(trans_a, trans_b, m, n, k, alpha, a, lda, stride_a, b, ldb, stride_b, beta,
                      c, ldc, stride_c, batch, bias, nullptr, 0, stream);
}
