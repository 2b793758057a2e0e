// bf16 GEMM on bf16 operands in HBM, fp32 accumulation and output: BASELINE cfg4's "bf16 MFMA
// RNN GEMMs" (7 x BiLSTM-1024, batch 64: input projection, dX, dW_ih, dW_hh).
//
//   C[M x N] = alpha * A[M x K] . B[N x K]^T + beta * C + bias     (A, B k-contiguous bf16)
//
// Structure (cdna_hip_programming.md "The 256^2 8-phase template"): a 256 x 256 tile per
// workgroup of 8 waves (2 M-halves x 4 N-quarters, each wave 128 x 64 = 8 x 4 tiles of
// v_mfma_f32_16x16x32_bf16), K-tiles of 64 in two LDS buffers (2 x 64 KB, ONE __shared__
// array), filled by LDS-DMA (buffer_load ... lds, 16 B per lane, out-of-range lanes read 0)
// with the XOR swizzle applied on the SOURCE address so the lane-linear LDS image is read
// conflict-free by ds_read_b128.  Every K-tile is four phases, one per C quadrant (4 x 2
// tiles, 16 MFMAs); a phase is [load segment: the quadrant's fragments + one 8-KB part of the
// next K-tile] barrier [MFMA segment] barrier.  The two M-half wave groups run one barrier
// apart (group 1 passes one extra barrier first), so in every barrier interval one wave per
// SIMD issues MFMAs while its partner loads: the matrix pipe never has two MFMA streams
// competing, and the loads hide behind the partner's MFMAs.
//
// Hazards (barrier b_i; group 0 phase p = load (b_2p, b_2p+1), MFMA (b_2p+1, b_2p+2); group 1
// one interval later): each group DMAs its own parts of K-tile t+1 during K-tile t -- its A rows
// 0-63 and B rows 0-63 of its 128-row B half in phase 0, B rows 64-127 in phase 1, its A rows
// 64-127 in phase 2 -- so every part has 2-3 phases to land before the wait that retires it:
// phase 3's vmcnt (first readers: phase 0 of t+1, both groups for B) and phase 1 of t+1's (A
// rows 64-127, first read in phase 2), each followed by a barrier before any reader (RAW).  The
// buffer a part overwrites held K-tile t-1, whose last reads (group 1, phase 3 of t-1) were
// retired by lgkmcnt(0) BEFORE the barrier that ends that load segment (WAR).  All LDS traffic
// of the loop is LDS-DMA + ds_read; no ordinary global load is pending in the loop (hipcc would
// drain the DMA queue at it).
#include "common.h"

#include <algorithm>

namespace ds2 {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x2v __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

constexpr int BG_M = 256, BG_N = 256, BG_K = 64, BG_T = 512;
constexpr int BG_IMG = (BG_M + BG_N) * BG_K;   // bf16 per LDS buffer (A rows, then B rows)
constexpr int kBgOob = 0x7ffffff0;

// 16-B chunk c (0..7) of image row r sits at chunk c ^ ((r >> 1) & 7): the 16 lanes of every
// ds_read_b128 lane group (16 rows x one chunk column) hit 16 distinct 16-B bank slots
__device__ __forceinline__ int bg_swz(int r) { return (r >> 1) & 7; }

// a raw s_barrier (no vmcnt(0): the LDS-DMA of later K-tiles stays in flight) that neither the
// IR passes (asm memory clobber) nor the machine scheduler (sched_barrier) move loads across
__device__ __forceinline__ void bg_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("" ::: "memory");
}

// Tile decode shared with gemm.hip's planner: whole tiles first, then the split-K tail pieces
// (the same XCD-aware bijective remap as decode_work, grouped tile order of 4 tile rows).
__device__ __forceinline__ void bg_decode(int M, int N, int K, int main_wgs, int tail_tile0,
                                          int tail_tiles, int nsplit, int kchunk, float* partial,
                                          int& m0, int& n0, int& kbeg, int& kend, float*& part) {
  const int tn = (N + BG_N - 1) / BG_N, tm = (M + BG_M - 1) / BG_M;
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
    if (nsplit > 1) part = partial + ((int64_t)z * tail_tiles + lt) * (BG_M * BG_N);
  }
  constexpr int G = 4;
  const int g = tile / (G * tn);
  const int rem = tile - g * G * tn;
  const int rows = min(G, tm - g * G);
  const int tile_n = rem / rows;
  const int tile_m = g * G + (rem - tile_n * rows);
  kbeg = orig < main_wgs ? 0 : z * kchunk;
  kend = orig < main_wgs ? K : min(K, kbeg + kchunk);
  m0 = tile_m * BG_M;
  n0 = tile_n * BG_N;
}

template <bool KCHK>
__global__ __launch_bounds__(BG_T, 1) void bgemm_nt_kernel(
    int M, int N, int K, float alpha, const unsigned short* __restrict__ A, int lda,
    const unsigned short* __restrict__ B, int ldb, float beta, float* __restrict__ C, int64_t ldc,
    const float* __restrict__ bias, int main_wgs, int tail_tile0, int tail_tiles, int nsplit,
    int kchunk, float* __restrict__ partial, int cvec) {
  __shared__ __attribute__((aligned(16))) unsigned short lds[2 * BG_IMG];   // 128 KB
  int m0, n0, kbeg, kend;
  float* part;
  bg_decode(M, N, K, main_wgs, tail_tile0, tail_tiles, nsplit, kchunk, partial, m0, n0, kbeg,
            kend, part);
  const int t = threadIdx.x;
  const int lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wr = wave >> 2, wc = wave & 3;    // M half (= wave group), N quarter
  const int w4 = wave & 3;                    // the wave's share of its group's DMA parts
  const __amdgpu_buffer_rsrc_t a_rs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<unsigned short*>(A), (short)0, static_cast<int>((int64_t)M * lda * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t b_rs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<unsigned short*>(B), (short)0, static_cast<int>((int64_t)N * ldb * 2), 0x00020000);

  // DMA source offsets (bytes, without the K-tile's k0): part q of this group, instruction j:
  // image row ir = base(q) + 16 w4 + 8 j + (lane >> 3), LDS chunk position lane & 7 holding
  // global chunk (lane & 7) ^ bg_swz(ir)
  int soff[4][2];
  int ldsoff[4][2];   // bf16 element offset of the 1-KB destination within a buffer
  int kc[2];          // the lane's k within a K-tile, per j (the same for every part)
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int ir16 = 16 * w4 + 8 * j + (lane >> 3);     // row within the 64-row part
    kc[j] = 8 * ((lane & 7) ^ bg_swz(ir16));
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const bool isb = q == 1 || q == 2;
      const int prow = 128 * wr + ((q == 2 || q == 3) ? 64 : 0);   // first image row of the part
      const int grow = (isb ? n0 : m0) + prow + ir16;
      const int lim = isb ? N : M;
      const int ld = isb ? ldb : lda;
      soff[q][j] = grow < lim ? (grow * ld + kc[j]) * 2 : kBgOob;
      ldsoff[q][j] = ((isb ? BG_M : 0) + prow + 16 * w4 + 8 * j) * BG_K;
    }
  }
  auto issue = [&](int q, int k0, int buf) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      int vo = soff[q][j];
      if (KCHK && k0 + kc[j] >= kend) vo = kBgOob;
      unsigned short* dst = lds + buf * BG_IMG + ldsoff[q][j];
      // the scalar offset (k0) is not range-checked, the vector one is: an out-of-range lane's
      // vector offset alone lies past the operand and reads 0
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          (q == 1 || q == 2) ? b_rs : a_rs,
          (__attribute__((address_space(3))) void*)dst, 16, vo, k0 * 2, 0, 0);
    }
  };

  // fragment read offsets (bf16 elements within a buffer): A m-tile mt, k-step ks; B n-tile nt
  const int fr = lane & 15, fk = lane >> 4;
  auto a_off = [&](int mt, int ks) {
    const int r = 128 * wr + 16 * mt + fr;
    return r * BG_K + 8 * ((4 * ks + fk) ^ bg_swz(r));
  };
  auto b_off = [&](int nt, int ks) {
    const int r = 64 * wc + 16 * nt + fr;
    return (BG_M + r) * BG_K + 8 * ((4 * ks + fk) ^ bg_swz(r));
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int jn = 0; jn < 4; ++jn) acc[i][jn] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int KT = (kend - kbeg + BG_K - 1) / BG_K;
  // prologue: K-tile 0 -> buffer 0 (this group's four parts), all complete before any read
#pragma unroll
  for (int q = 0; q < 4; ++q) issue(q, kbeg, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  bg_barrier();
  if (wr == 1) bg_barrier();   // group 1 runs one barrier interval behind group 0

  bf16x8 af[4][2], bfr[2][2];
  for (int kt = 0; kt < KT; ++kt) {
    const int cur = kt & 1;
    const unsigned short* img = lds + cur * BG_IMG;
    const bool more = kt + 1 < KT;
    const int knext = kbeg + (kt + 1) * BG_K;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      // ---- load segment: quadrant q = (qm, qn) of this K-tile; A fragments change at q 0, 2,
      // B fragments at q 0, 1, 3 (order (0,0), (0,1), (1,1), (1,0))
      const int qm = q >> 1, qn = (q == 1 || q == 2) ? 1 : 0;
      if (q != 2) {
#pragma unroll
        for (int ni = 0; ni < 2; ++ni)
#pragma unroll
          for (int ks = 0; ks < 2; ++ks)
            bfr[ni][ks] = *reinterpret_cast<const bf16x8*>(img + b_off(2 * qn + ni, ks));
      }
      if (q == 0 || q == 2) {
#pragma unroll
        for (int mi = 0; mi < 4; ++mi)
#pragma unroll
          for (int ks = 0; ks < 2; ++ks)
            af[mi][ks] = *reinterpret_cast<const bf16x8*>(img + a_off(4 * qm + mi, ks));
      }
      // DMA of K-tile kt + 1 (buffer cur ^ 1): phase 0 its A rows 0-63 and B rows 0-63, phase
      // 1 B rows 64-127, phase 2 A rows 64-127.  Waits: phase 1 retires A rows 64-127 of THIS
      // K-tile (issued in phase 2 of the previous one; 6 DMA after it when more), phase 3
      // retires everything of kt + 1 but its A rows 64-127 (2 DMA after them).
      if (more) {
        if (q == 0) {
          issue(0, knext, cur ^ 1);
          issue(1, knext, cur ^ 1);
        } else if (q == 1) {
          issue(2, knext, cur ^ 1);
        } else if (q == 2) {
          issue(3, knext, cur ^ 1);
        }
      }
      if (q == 1) {
        if (more) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      } else if (q == 3) {
        if (more) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      // this segment's fragment reads retire before the barrier, so a DMA the other group issues
      // right after it may overwrite what they read (WAR)
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      bg_barrier();
      // ---- MFMA segment
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int ni = 0; ni < 2; ++ni)
#pragma unroll
          for (int ks = 0; ks < 2; ++ks)
            acc[4 * qm + mi][2 * qn + ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                af[mi][ks], bfr[ni][ks], acc[4 * qm + mi][2 * qn + ni], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
      bg_barrier();
    }
  }
  if (wr == 0) bg_barrier();   // equal barrier counts for both groups

  // epilogue: the accumulators (16x16 C map: row 4 (lane >> 4) + r, col lane & 15) go through
  // the now idle LDS, 64 rows x 64 columns per wave and pass (16 KB per wave, columns XOR 16 by
  // row bit 2: conflict-free b32 writes and b128 reads), and leave as 16-B row runs -- each
  // store instruction writes four 256-B row segments instead of sixteen 64-B ones
  float* const stage = reinterpret_cast<float*>(lds) + wave * 4096;
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int lr = 16 * mt + 4 * fk + r;
          stage[lr * 64 + ((16 * nt + fr) ^ (((lr >> 2) & 1) << 4))] = acc[4 * pass + mt][nt][r];
        }
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int lr = 4 * i + (lane >> 4), cc = lane & 15;
      const f32x4 v4 = *reinterpret_cast<const f32x4*>(stage + lr * 64 + 4 * (cc ^ (((lr >> 2) & 1) << 2)));
      const int rl = 128 * wr + 64 * pass + lr, cl = 64 * wc + 4 * cc;   // within the tile
      if (part != nullptr) {
        *reinterpret_cast<f32x4*>(part + rl * BG_N + cl) = v4;
        continue;
      }
      const int row = m0 + rl, col = n0 + cl;
      if (row >= M || col >= N) continue;
      float* cp = C + (int64_t)row * ldc + col;
      if (cvec && col + 3 < N) {
        f32x4 o = v4 * alpha;
        if (bias != nullptr) o += *reinterpret_cast<const f32x4*>(bias + col);
        if (beta != 0.f) o += beta * *reinterpret_cast<const f32x4*>(cp);
        *reinterpret_cast<f32x4*>(cp) = o;
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          if (col + e >= N) break;
          float o = alpha * v4[e] + (bias != nullptr ? bias[col + e] : 0.f);
          if (beta != 0.f) o += beta * cp[e];
          cp[e] = o;
        }
      }
    }
  }
}

// fp32 [rows][cols] (row stride ld_src) -> bf16 (RNE), either as is (dst [rows][ld_dst]) or
// transposed (dst [cols][ld_dst]); 64 x 64 tiles.  vec (16-B aligned src / dst, ld_src % 4 ==
// 0, ld_dst % 8 == 0): 16-B loads and 16-B stores of 8 bf16 -- the transposed form goes
// through an fp32 LDS tile (float4 row loads in, 8-row column runs out); otherwise element
// loads and 2-B stores
__global__ __launch_bounds__(256) void cvt_bf16_kernel(const float* __restrict__ src, int rows,
                                                       int cols, int64_t ld_src,
                                                       unsigned short* __restrict__ dst,
                                                       int64_t ld_dst, int transpose, int vec) {
  __shared__ float tf[64][65];
  const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
  const int t = threadIdx.x;
  auto pack8 = [](const float* v) {
    u32x4 o;
#pragma unroll
    for (int e = 0; e < 4; ++e)
      o[e] = __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2v{v[2 * e], v[2 * e + 1]}, bf16x2v));
    return o;
  };
  if (!transpose) {
    // 64 rows x 64 cols: thread = (row t >> 2, 16 columns), two 8-column runs
    const int r = r0 + (t >> 2), cb = c0 + 16 * (t & 3);
    if (r >= rows) return;
    const float* sr = src + (int64_t)r * ld_src;
    unsigned short* d = dst + (int64_t)r * ld_dst;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int c = cb + 8 * h;
      if (c >= cols) break;
      float v[8];
      if (vec && c + 8 <= cols) {
        const f32x4 x0 = *reinterpret_cast<const f32x4*>(sr + c);
        const f32x4 x1 = *reinterpret_cast<const f32x4*>(sr + c + 4);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[e] = x0[e];
          v[4 + e] = x1[e];
        }
        *reinterpret_cast<u32x4*>(d + c) = pack8(v);
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (c + e < cols) d[c + e] = __builtin_bit_cast(unsigned short, (__bf16)sr[c + e]);
      }
    }
    return;
  }
  // transposed: in = rows r0.. (64) x cols c0.. (64) as float4 runs (16 threads per row, 16
  // rows per pass); out = for column c, rows r0 + 8 q .. + 7 as one 16-B store
  if (vec) {
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int rr = 16 * p + (t >> 4), cc = 4 * (t & 15);
      const int r = r0 + rr, c = c0 + cc;
      f32x4 x = f32x4{0.f, 0.f, 0.f, 0.f};
      if (r < rows) {
        if (c + 4 <= cols) {
          x = *reinterpret_cast<const f32x4*>(src + (int64_t)r * ld_src + c);
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) x[e] = c + e < cols ? src[(int64_t)r * ld_src + c + e] : 0.f;
        }
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) tf[rr][cc + e] = x[e];
    }
    __syncthreads();
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const int o = t + 256 * p;              // 512 outputs: (column, 8-row run)
      const int cc = o >> 3, q = o & 7;
      const int c = c0 + cc, rb = r0 + 8 * q;
      if (c >= cols || rb >= rows) continue;
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = tf[8 * q + e][cc];
      unsigned short* d = dst + (int64_t)c * ld_dst + rb;
      if (rb + 8 <= rows) {
        *reinterpret_cast<u32x4*>(d) = pack8(v);
      } else {
        for (int e = 0; e < 8 && rb + e < rows; ++e) d[e] = __builtin_bit_cast(unsigned short, (__bf16)v[e]);
      }
    }
    return;
  }
  for (int i = t; i < 64 * 64; i += 256) {
    const int rr = i >> 6, cc = i & 63;
    const int r = r0 + rr, c = c0 + cc;
    tf[cc][rr] = (r < rows && c < cols) ? src[(int64_t)r * ld_src + c] : 0.f;
  }
  __syncthreads();
  for (int i = t; i < 64 * 64; i += 256) {
    const int cc = i >> 6, rr = i & 63;
    const int r = r0 + rr, c = c0 + cc;
    if (r < rows && c < cols) dst[(int64_t)c * ld_dst + r] = __builtin_bit_cast(unsigned short, (__bf16)tf[cc][rr]);
  }
}

// split-K tail: C = alpha * sum_s partial[s][tile] + beta * C + bias, fixed summation order
__global__ void bg_reduce_kernel(const float* __restrict__ partial, int M, int N, int nsplit,
                                 int tail_tile0, int tail_tiles, float alpha, float beta,
                                 float* __restrict__ C, int64_t ldc, const float* __restrict__ bias) {
  constexpr int TE = BG_M * BG_N;
  const int tn = (N + BG_N - 1) / BG_N, tm = (M + BG_M - 1) / BG_M;
  const int64_t total = (int64_t)tail_tiles * TE;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int e = static_cast<int>(i % TE);
    const int lt = static_cast<int>(i / TE);
    const int tile = tail_tile0 + lt;
    constexpr int G = 4;
    const int g = tile / (G * tn);
    const int rem = tile - g * G * tn;
    const int rows = min(G, tm - g * G);
    const int tile_n = rem / rows;
    const int tile_m = g * G + (rem - tile_n * rows);
    const int row = tile_m * BG_M + e / BG_N;
    const int col = tile_n * BG_N + e % BG_N;
    if (row >= M || col >= N) continue;
    float acc = 0.f;
#pragma unroll 4
    for (int sp = 0; sp < nsplit; ++sp) acc += partial[((int64_t)sp * tail_tiles + lt) * TE + e];
    float* cp = C + (int64_t)row * ldc + col;
    float v = alpha * acc + (bias != nullptr ? bias[col] : 0.f);
    if (beta != 0.f) v += beta * *cp;
    *cp = v;
  }
}

struct BgPlan {
  int main_wgs, tail_tile0, tail_tiles, nsplit, kchunk;
};

static int bg_cus() {
  static int cus = -1;
  if (cus < 0) {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess) dev = 0;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0)
      v = 256;
    cus = v;
  }
  return cus;
}

// Whole tiles in full rounds of one workgroup per CU; the last partial round's tiles get their
// K range split so the pieces fill a round (time model in units of one 64-deep tile step;
// a split piece adds its 256 KB partial slab written and read back, ~1/8 of a step).
static BgPlan bg_plan(int m, int n, int k) {
  const int cus = bg_cus();
  const int tiles = cdiv(m, BG_M) * cdiv(n, BG_N);
  BgPlan p{(tiles / cus) * cus, 0, 0, 1, k};
  p.tail_tile0 = p.main_wgs;
  p.tail_tiles = tiles - p.main_wgs;
  if (p.tail_tiles == 0) {
    p.main_wgs = 0;
    p.tail_tile0 = 0;
    p.tail_tiles = tiles;
  }
  const int ksteps = cdiv(k, BG_K);
  double best = 1e30;
  for (int s = 1; s <= 32 && s <= ksteps; ++s) {
    const int kc = cdiv(ksteps, s);
    const int ns = cdiv(ksteps, kc);
    if (s > 1 && ns != s) continue;
    const int64_t pieces = (int64_t)p.tail_tiles * ns;
    const double t = (double)((pieces + cus - 1) / cus) * kc + (ns > 1 ? 0.125 * (double)pieces / cus + 1.0 : 0.0);
    if (t < best - 1e-9) {
      best = t;
      p.nsplit = ns;
      p.kchunk = kc * BG_K;
    }
  }
  if (p.nsplit == 1) p.kchunk = k;
  return p;
}

static size_t bg_ws(const BgPlan& p) {
  return p.nsplit > 1 ? (size_t)p.nsplit * p.tail_tiles * BG_M * BG_N * sizeof(float) + 256 : 0;
}

}  // namespace ds2

using namespace ds2;

extern "C" {

size_t ds2_bgemm_workspace_size(int m, int n, int k) {
  if (m <= 0 || n <= 0 || k <= 0) return 0;
  return bg_ws(bg_plan(m, n, k));
}

ds2_status_t ds2_bgemm_nt(int m, int n, int k, float alpha, const void* a, int64_t lda,
                          const void* b, int64_t ldb, float beta, float* c, int64_t ldc,
                          const float* bias, void* ws, size_t ws_bytes, ds2_stream_t stream) {
  if (m < 0 || n < 0 || k < 0) return DS2_INVALID_VALUE;
  if (m == 0 || n == 0) return DS2_OK;
  if (a == nullptr || b == nullptr || c == nullptr || lda < k || ldb < k || ldc < n)
    return DS2_INVALID_VALUE;
  // 16-B DMA granules: 16-B aligned operands, k and the row strides multiples of 8 bf16
  if ((reinterpret_cast<uintptr_t>(a) & 15) || (reinterpret_cast<uintptr_t>(b) & 15) ||
      (lda & 7) || (ldb & 7) || (k & 7) || (int64_t)m * lda * 2 >= (1ll << 31) ||
      (int64_t)n * ldb * 2 >= (1ll << 31) || lda >= (1 << 30) || ldb >= (1 << 30))
    return DS2_UNSUPPORTED_SHAPE;
  if (k == 0) return DS2_UNSUPPORTED_SHAPE;
  BgPlan p = bg_plan(m, n, k);
  if (p.nsplit > 1 && (ws == nullptr || ws_bytes < bg_ws(p))) {
    p.nsplit = 1;
    p.kchunk = k;
  }
  float* partial = p.nsplit > 1 ? static_cast<float*>(ws) : nullptr;
  const int64_t nwg = p.main_wgs + (int64_t)p.tail_tiles * p.nsplit;
  if (nwg > 0x7fffffff) return DS2_UNSUPPORTED_SHAPE;
  hipStream_t st = as_stream(stream);
  const bool kalign = k % BG_K == 0 && p.kchunk % BG_K == 0;
  // 16-B row runs of C (and of bias) when every row starts 16-B aligned
  const int cvec = !((reinterpret_cast<uintptr_t>(c) & 15) || (ldc & 3) ||
                     (bias != nullptr && (reinterpret_cast<uintptr_t>(bias) & 15)));
  const unsigned short* A = static_cast<const unsigned short*>(a);
  const unsigned short* B = static_cast<const unsigned short*>(b);
  if (kalign)
    hipLaunchKernelGGL(bgemm_nt_kernel<false>, dim3(static_cast<unsigned>(nwg)), dim3(BG_T), 0, st,
                       m, n, k, alpha, A, static_cast<int>(lda), B, static_cast<int>(ldb), beta, c,
                       ldc, bias, p.main_wgs, p.tail_tile0, p.tail_tiles, p.nsplit, p.kchunk,
                       partial, cvec);
  else
    hipLaunchKernelGGL(bgemm_nt_kernel<true>, dim3(static_cast<unsigned>(nwg)), dim3(BG_T), 0, st,
                       m, n, k, alpha, A, static_cast<int>(lda), B, static_cast<int>(ldb), beta, c,
                       ldc, bias, p.main_wgs, p.tail_tile0, p.tail_tiles, p.nsplit, p.kchunk,
                       partial, cvec);
  if (p.nsplit > 1) {
    const int64_t total = (int64_t)p.tail_tiles * BG_M * BG_N;
    const int g = static_cast<int>(std::min<int64_t>(cdiv(total, 256), 4096));
    hipLaunchKernelGGL(bg_reduce_kernel, dim3(g), dim3(256), 0, st, partial, m, n, p.nsplit,
                       p.tail_tile0, p.tail_tiles, alpha, beta, c, ldc, bias);
  }
  return launch_status("ds2_bgemm_nt");
}

ds2_status_t ds2_cvt_bf16(const float* src, int rows, int cols, int64_t ld_src, void* dst,
                          int64_t ld_dst, int transpose, ds2_stream_t stream) {
  if (rows < 0 || cols < 0 || src == nullptr || dst == nullptr) return DS2_INVALID_VALUE;
  if (rows == 0 || cols == 0) return DS2_OK;
  if (ld_src < cols || ld_dst < (transpose ? rows : cols)) return DS2_INVALID_VALUE;
  const int vec = !((reinterpret_cast<uintptr_t>(src) & 15) || (reinterpret_cast<uintptr_t>(dst) & 15) ||
                    (ld_src & 3) || (ld_dst & 7));
  const dim3 grid(cdiv(cols, 64), cdiv(rows, 64));
  if (grid.y > 65535) return DS2_UNSUPPORTED_SHAPE;
  hipLaunchKernelGGL(cvt_bf16_kernel, grid, dim3(256), 0, as_stream(stream), src, rows, cols,
                     ld_src, static_cast<unsigned short*>(dst), ld_dst, transpose, vec);
  return launch_status("ds2_cvt_bf16");
}

}  // extern "C"
