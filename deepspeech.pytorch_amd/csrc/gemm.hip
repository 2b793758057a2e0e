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
// (ids congruent mod 8) get a contiguous run of tiles (pieces), n-tile fastest, so
// workgroups sharing an operand panel share that XCD's L2.
__device__ __forceinline__ void decode_work(int M, int N, int K, int main_wgs, int tail_tile0,
                                            int tail_tiles, int nsplit, int kchunk,
                                            float* partial, int& m0, int& n0, int& kbeg,
                                            int& kend, int& bz, float*& part) {
  const int tn = (N + BN - 1) / BN;
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
    if (nsplit > 1) part = partial + ((int64_t)z * tail_tiles + lt) * (BM * BN);
  }
  const int tile_m = tile / tn;
  const int tile_n = tile - tile_m * tn;
  // z = batch * nsplit + split
  bz = z / nsplit;
  const int sp = z - bz * nsplit;
  kbeg = orig < main_wgs ? 0 : sp * kchunk;
  kend = orig < main_wgs ? K : min(K, kbeg + kchunk);
  m0 = tile_m * BM;
  n0 = tile_n * BN;
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


// Tail tiles: C[b] = alpha * sum_s partial[b][s][tile] + beta * C[b] + bias (fixed order)
__global__ void splitk_reduce_kernel(const float* __restrict__ partial, int M, int N, int nsplit,
                                     int batch, int tail_tile0, int tail_tiles, float alpha,
                                     float beta, float* __restrict__ C, int64_t ldc, int64_t sC,
                                     const float* __restrict__ bias) {
  constexpr int TE = BM * BN;
  const int tn = (N + BN - 1) / BN;
  const int64_t total = (int64_t)batch * tail_tiles * TE;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int e = static_cast<int>(i % TE);
    const int64_t bt = i / TE;
    const int lt = static_cast<int>(bt % tail_tiles);
    const int b = static_cast<int>(bt / tail_tiles);
    const int tile = tail_tile0 + lt;
    const int row = (tile / tn) * BM + e / BN;
    const int col = (tile % tn) * BN + e % BN;
    if (row >= M || col >= N) continue;
    float acc = 0.f;
    for (int sp = 0; sp < nsplit; ++sp)
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

static inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

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
  int main_wgs, tail_tile0, tail_tiles, nsplit, kchunk;
};

static GemmPlan gemm_plan(int m, int n, int k, int batch) {
  const int tiles = cdiv(m, BM) * cdiv(n, BN);
  GemmPlan p{0, 0, tiles, 1, std::max(k, 1)};
  const int slots = 3 * device_cus();
  if (batch == 1) {
    p.main_wgs = (tiles / slots) * slots;
    p.tail_tile0 = p.main_wgs;
    p.tail_tiles = tiles - p.main_wgs;
    if (p.tail_tiles == 0) {   // full rounds only
      p.main_wgs = 0;
      p.tail_tile0 = 0;
      p.tail_tiles = tiles;
      return p;
    }
  }
  const int64_t tail = (int64_t)p.tail_tiles * batch;
  const int smax = std::max(1, std::min(32, k / 256));
  double best = 1e30;
  int bs = 1;
  for (int s = 1; s <= smax; ++s) {
    const double rounds = (double)((tail * s + slots - 1) / slots);
    const double cost = rounds / s + (s > 1 ? 0.005 * s : 0.0);
    if (cost < best - 1e-9) {
      best = cost;
      bs = s;
    }
  }
  if (bs > 1) {
    p.kchunk = cdiv(cdiv(k, bs), BK) * BK;
    p.nsplit = cdiv(k, p.kchunk);
  }
  return p;
}

extern "C" size_t ds2_sgemm_workspace_size(int m, int n, int k, int batch) {
  if (m <= 0 || n <= 0 || k <= 0 || batch <= 0) return 0;
  const GemmPlan p = gemm_plan(m, n, k, batch);
  return p.nsplit > 1
             ? (size_t)p.nsplit * batch * p.tail_tiles * BM * BN * sizeof(float) + 256
             : 0;
}

extern "C" ds2_status_t ds2_sgemm_ws(int trans_a, int trans_b, int m, int n, int k, float alpha,
                                     const float* a, int64_t lda, int64_t stride_a,
                                     const float* b, int64_t ldb, int64_t stride_b, float beta,
                                     float* c, int64_t ldc, int64_t stride_c, int batch,
                                     const float* bias, void* ws, size_t ws_bytes,
                                     ds2_stream_t stream) {
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
  GemmPlan p = gemm_plan(m, n, k, batch);
  if (p.nsplit > 1 && (ws == nullptr || ws_bytes < ds2_sgemm_workspace_size(m, n, k, batch))) {
    p.nsplit = 1;                       // no workspace: whole-K pieces
    p.kchunk = std::max(k, 1);
  }
  float* partial = p.nsplit > 1 ? static_cast<float*>(ws) : nullptr;
  const int64_t nwg = p.main_wgs + (int64_t)p.tail_tiles * batch * p.nsplit;
  if (nwg > 0x7fffffff) return DS2_UNSUPPORTED_SHAPE;
  dim3 grid(static_cast<unsigned>(nwg));
  hipStream_t st = as_stream(stream);
#define DS2_G(TA_, TB_)                                                                       \
  launch_sgemm_t<TA_, TB_>(va, vb, grid, st, m, n, k, alpha, a, lda, stride_a, b, ldb, stride_b, \
                           beta, c, ldc, stride_c, bias, p.main_wgs, p.tail_tile0, p.tail_tiles,  \
                           p.nsplit, p.kchunk, partial)
  if (!trans_a && !trans_b) DS2_G(0, 0);
  else if (!trans_a && trans_b) DS2_G(0, 1);
  else if (trans_a && !trans_b) DS2_G(1, 0);
  else DS2_G(1, 1);
#undef DS2_G
  if (p.nsplit > 1) {
    const int64_t total = (int64_t)batch * p.tail_tiles * BM * BN;
    int g = cdiv(total, 256);
    if (g > 4096) g = 4096;
    hipLaunchKernelGGL(splitk_reduce_kernel, dim3(g), dim3(256), 0, st, partial, m, n, p.nsplit,
                       batch, p.tail_tile0, p.tail_tiles, alpha, beta, c, ldc, stride_c, bias);
  }
  return launch_status("ds2_sgemm");
}

extern "C" ds2_status_t ds2_sgemm(int trans_a, int trans_b, int m, int n, int k, float alpha,
                                  const float* a, int64_t lda, int64_t stride_a, const float* b,
                                  int64_t ldb, int64_t stride_b, float beta, float* c,
                                  int64_t ldc, int64_t stride_c, int batch, const float* bias,
                                  ds2_stream_t stream) {
  return ds2_sgemm_ws(trans_a, trans_b, m, n, k, alpha, a, lda, stride_a, b, ldb, stride_b, beta,
                      c, ldc, stride_c, batch, bias, nullptr, 0, stream);
}
