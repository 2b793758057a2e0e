// Lookahead convolution (Wang et al. 2016) + optional fused Hardtanh — SURVEY §8
// row a9, reference model.py:140-177 (+ Hardtanh(0, 20) model.py:329-333).
//
//   z[t][n][h] = sum_{j=0..C} W[h][j] * x[t+j][n][h]      (x = 0 for t+j >= T)
//   y = clamp(z, lo, hi) when fused
//
// The reference materialises a [T, C+1, N, H] stack and multiplies; here each
// thread owns one (n, h) column of the [T][N][H] activation and a tile of TT
// consecutive t, keeps the TT + C input window and the C + 1 weights in
// registers, and reads each input about (1 + C/TT) times — a streaming,
// HBM-bound kernel.  Threads run along (n, h), so every load is coalesced.
//
// Backward (dz = dy masked by lo < y < hi, Hardtanh's strict test):
//   dx[t][n][h] = sum_j W[h][j] * dz[t-j][n][h]           (t-j >= 0)
//   dW[h][j]    = sum_{t,n} dz[t][n][h] * x[t+j][n][h]
// dW goes through per-(t tile, n group) partials and a fixed-order reduce, so
// the result is deterministic.
#include "common.h"

namespace ds2 {

constexpr int LA_MAXC = 32;   // max context + 1
constexpr int LA_TT = 32;     // time steps per thread tile (fwd, dx)
constexpr int LA_TTW = 16;    // time steps per thread tile (dw partials)

// [T][N][H] tensors are addressed through buffer resources with 32-bit byte
// offsets (host checks T*N*H*4 < 2^31); an offset past the end reads 0, which
// is exactly the zero padding past T.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t la_rsrc(const float* p, int64_t elems) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p), (short)0,
                                           static_cast<int>(elems * 4), 0x00020000);
}

__device__ __forceinline__ float la_ld(__amdgpu_buffer_rsrc_t rs, int off) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, off, 0, 0));
}

constexpr int kLaOob = 0x7ffffff0;

__global__ __launch_bounds__(256) void lookahead_fwd_kernel(
    const float* __restrict__ x, int T, int64_t cols, int H, const float* __restrict__ w, int C,
    int clamp, float lo, float hi, float* __restrict__ y) {
  const int64_t col = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (col >= cols) return;
  const int h = static_cast<int>(col % H);
  const int t0 = blockIdx.y * LA_TT;
  float wr[LA_MAXC];
#pragma unroll
  for (int j = 0; j < LA_MAXC; ++j) wr[j] = j <= C ? w[(int64_t)h * (C + 1) + j] : 0.f;
  const __amdgpu_buffer_rsrc_t xr = la_rsrc(x, (int64_t)T * cols);
  const int stride = static_cast<int>(cols * 4);
  const int base = static_cast<int>(((int64_t)t0 * cols + col) * 4);
  float xw[LA_TT + LA_MAXC - 1];
#pragma unroll
  for (int i = 0; i < LA_TT + LA_MAXC - 1; ++i)
    xw[i] = la_ld(xr, (i < LA_TT + C && t0 + i < T) ? base + i * stride : kLaOob);
#pragma unroll
  for (int i = 0; i < LA_TT; ++i) {
    const int t = t0 + i;
    if (t >= T) break;
    float z = 0.f;
#pragma unroll
    for (int j = 0; j < LA_MAXC; ++j) z = fmaf(wr[j], xw[i + j], z);
    if (clamp) z = fminf(fmaxf(z, lo), hi);
    y[(int64_t)t * cols + col] = z;
  }
}

__global__ __launch_bounds__(256) void lookahead_dx_kernel(
    const float* __restrict__ dy, const float* __restrict__ y, float lo, float hi, int T,
    int64_t cols, int H, const float* __restrict__ w, int C, float* __restrict__ dx) {
  const int64_t col = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (col >= cols) return;
  const int h = static_cast<int>(col % H);
  const int t0 = blockIdx.y * LA_TT;
  float wr[LA_MAXC];
#pragma unroll
  for (int j = 0; j < LA_MAXC; ++j) wr[j] = j <= C ? w[(int64_t)h * (C + 1) + j] : 0.f;
  // window dz[t0 - (MAXC-1) .. t0 + TT - 1]; entry i holds t = t0 - (MAXC-1) + i
  const __amdgpu_buffer_rsrc_t gr = la_rsrc(dy, (int64_t)T * cols);
  const __amdgpu_buffer_rsrc_t yr = la_rsrc(y != nullptr ? y : dy, (int64_t)T * cols);
  const int stride = static_cast<int>(cols * 4);
  const int base = static_cast<int>(col * 4);
  float zw[LA_TT + LA_MAXC - 1];
#pragma unroll
  for (int i = 0; i < LA_TT + LA_MAXC - 1; ++i) {
    const int t = t0 - (LA_MAXC - 1) + i;
    const int off = (t >= 0 && t < T && i >= LA_MAXC - 1 - C) ? base + t * stride : kLaOob;
    const float g = la_ld(gr, off);
    if (y != nullptr) {
      const float v = la_ld(yr, off);
      zw[i] = (v > lo && v < hi) ? g : 0.f;
    } else {
      zw[i] = g;
    }
  }
#pragma unroll
  for (int i = 0; i < LA_TT; ++i) {
    const int t = t0 + i;
    if (t >= T) break;
    float g = 0.f;
#pragma unroll
    for (int j = 0; j < LA_MAXC; ++j) g = fmaf(wr[j], zw[i + LA_MAXC - 1 - j], g);
    dx[(int64_t)t * cols + col] = g;
  }
}

// partial[tile][h][j] over one t tile and all n of the block's h range.
// Block = 64 h x 4 n-groups; each thread loops over its n's.
__global__ __launch_bounds__(256) void lookahead_dw_partial_kernel(
    const float* __restrict__ dy, const float* __restrict__ y, float lo, float hi,
    const float* __restrict__ x, int T, int N, int H, int C, float* __restrict__ partial) {
  const int h = blockIdx.x * 64 + (threadIdx.x & 63);
  const int ng = threadIdx.x >> 6;
  const int t0 = blockIdx.y * LA_TTW;
  const int64_t cols = (int64_t)N * H;
  float acc[LA_MAXC];
#pragma unroll
  for (int j = 0; j < LA_MAXC; ++j) acc[j] = 0.f;
  const __amdgpu_buffer_rsrc_t xr = la_rsrc(x, (int64_t)T * cols);
  const __amdgpu_buffer_rsrc_t gr = la_rsrc(dy, (int64_t)T * cols);
  const __amdgpu_buffer_rsrc_t yr = la_rsrc(y != nullptr ? y : dy, (int64_t)T * cols);
  const int stride = static_cast<int>(cols * 4);
  if (h < H) {
    for (int n = ng; n < N; n += 4) {
      const int base = static_cast<int>(((int64_t)t0 * cols + (int64_t)n * H + h) * 4);
      float xw[LA_TTW + LA_MAXC - 1];
#pragma unroll
      for (int i = 0; i < LA_TTW + LA_MAXC - 1; ++i)
        xw[i] = la_ld(xr, (i < LA_TTW + C && t0 + i < T) ? base + i * stride : kLaOob);
#pragma unroll
      for (int i = 0; i < LA_TTW; ++i) {
        const int off = t0 + i < T ? base + i * stride : kLaOob;
        float z = la_ld(gr, off);
        if (y != nullptr) {
          const float v = la_ld(yr, off);
          z = (v > lo && v < hi) ? z : 0.f;
        }
#pragma unroll
        for (int j = 0; j < LA_MAXC; ++j) acc[j] = fmaf(z, xw[i + j], acc[j]);
      }
    }
  }
  __shared__ float red[4][64][LA_MAXC + 1];
#pragma unroll
  for (int j = 0; j < LA_MAXC; ++j) red[ng][threadIdx.x & 63][j] = acc[j];
  __syncthreads();
  // 256 threads write the 64 x (C+1) outputs of this block
  for (int e = threadIdx.x; e < 64 * (C + 1); e += 256) {
    const int hl = e / (C + 1);
    const int j = e - hl * (C + 1);
    const int hh = blockIdx.x * 64 + hl;
    if (hh < H) {
      const float v = red[0][hl][j] + red[1][hl][j] + red[2][hl][j] + red[3][hl][j];
      partial[((int64_t)blockIdx.y * H + hh) * (C + 1) + j] = v;
    }
  }
}

__global__ void lookahead_dw_reduce_kernel(const float* __restrict__ partial, int tiles,
                                           int64_t count, float* __restrict__ dw) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= count) return;
  double s = 0.0;
  for (int k = 0; k < tiles; ++k) s += partial[(int64_t)k * count + i];
  dw[i] = static_cast<float>(s);
}

}  // namespace ds2

using namespace ds2;

extern "C" {

ds2_status_t ds2_lookahead_fwd(const float* x, int t, int n, int h, const float* w, int context,
                               int clamp, float lo, float hi, float* y, ds2_stream_t stream) {
  if (t < 0 || n < 0 || h < 0 || context < 1) return DS2_INVALID_VALUE;
  if (context + 1 > LA_MAXC) return DS2_UNSUPPORTED_SHAPE;
  if (t == 0 || n == 0 || h == 0) return DS2_OK;
  if (x == nullptr || w == nullptr || y == nullptr) return DS2_INVALID_VALUE;
  const int64_t cols = (int64_t)n * h;
  if ((int64_t)t * cols * 4 >= (1ll << 31) - 64) return DS2_UNSUPPORTED_SHAPE;
  hipLaunchKernelGGL(lookahead_fwd_kernel, dim3(cdiv(cols, 256), cdiv(t, LA_TT)), dim3(256), 0,
                     as_stream(stream), x, t, cols, h, w, context, clamp, lo, hi, y);
  return launch_status("ds2_lookahead_fwd");
}

size_t ds2_lookahead_bwd_workspace_size(int t, int n, int h, int context) {
  (void)n;
  return (size_t)cdiv(t, LA_TTW) * h * (context + 1) * sizeof(float) + 256;
}

ds2_status_t ds2_lookahead_bwd(const float* dy, const float* y, float lo, float hi,
                               const float* x, int t, int n, int h, const float* w, int context,
                               float* dx, float* dw, void* ws, size_t ws_bytes,
                               ds2_stream_t stream) {
  if (t < 0 || n < 0 || h < 0 || context < 1) return DS2_INVALID_VALUE;
  if (context + 1 > LA_MAXC) return DS2_UNSUPPORTED_SHAPE;
  if (h == 0) return DS2_OK;
  hipStream_t st = as_stream(stream);
  if (t == 0 || n == 0) {
    if (dw != nullptr && hipMemsetAsync(dw, 0, (size_t)h * (context + 1) * sizeof(float), st) != hipSuccess)
      return launch_status("ds2_lookahead_bwd");
    return DS2_OK;
  }
  const int64_t cols = (int64_t)n * h;
  if ((int64_t)t * cols * 4 >= (1ll << 31) - 64) return DS2_UNSUPPORTED_SHAPE;
  const int tiles = cdiv(t, LA_TT);
  if (dx != nullptr)
    hipLaunchKernelGGL(lookahead_dx_kernel, dim3(cdiv(cols, 256), tiles), dim3(256), 0, st, dy, y,
                       lo, hi, t, cols, h, w, context, dx);
  if (dw != nullptr) {
    if (ws == nullptr || ws_bytes < ds2_lookahead_bwd_workspace_size(t, n, h, context))
      return DS2_WORKSPACE_TOO_SMALL;
    float* partial = static_cast<float*>(ws);
    const int wtiles = cdiv(t, LA_TTW);
    hipLaunchKernelGGL(lookahead_dw_partial_kernel, dim3(cdiv(h, 64), wtiles), dim3(256), 0, st,
                       dy, y, lo, hi, x, t, n, h, context, partial);
    const int64_t count = (int64_t)h * (context + 1);
    hipLaunchKernelGGL(lookahead_dw_reduce_kernel, dim3(cdiv(count, 256)), dim3(256), 0, st,
                       partial, wtiles, count, dw);
  }
  return launch_status("ds2_lookahead_bwd");
}

}  // extern "C"
