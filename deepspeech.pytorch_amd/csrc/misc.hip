// Status strings, small elementwise/reduction kernels, softmax and the
// clip + SGD-Nesterov optimizer tail.  All HBM-bound: float4 where the layout
// allows, grid-stride loops capped at ~2048 blocks (256 CUs x 8).
#include "common.h"

#include <stdio.h>

namespace ds2 {

static thread_local char g_last_error[256] = "";

void set_last_error(const char* where, hipError_t e) {
  snprintf(g_last_error, sizeof(g_last_error), "%s: %s", where, hipGetErrorString(e));
}

void set_last_error_text(const char* where, const char* what) {
  snprintf(g_last_error, sizeof(g_last_error), "%s: %s", where, what);
}

static inline int grid_for(int64_t work, int block) {
  int64_t g = (work + block - 1) / block;
  if (g > 2048) g = 2048;
  if (g < 1) g = 1;
  return static_cast<int>(g);
}

// ---------------------------------------------------------------------------
// y[r][j] = sum_d h_all[r][d][j]
__global__ void dirsum_kernel(const float* __restrict__ h_all, int64_t rows, int dirs, int h,
                              float* __restrict__ y) {
  const int64_t total = rows * h;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / h;
    const int j = static_cast<int>(i - r * h);
    const float* src = h_all + r * dirs * h + j;
    float acc = src[0];
    for (int d = 1; d < dirs; ++d) acc += src[(int64_t)d * h];
    y[i] = acc;
  }
}

// Column sums (bias gradients): stage 1 reduces a chunk of rows for 64 columns per
// block in fp64 (grid = column blocks x row chunks, enough blocks to fill the chip),
// stage 2 adds the chunk partials in a fixed order (deterministic, no atomics).
constexpr int kColChunks = 64;

__global__ __launch_bounds__(256) void colsum_partial_kernel(const float* __restrict__ x,
                                                             int rows, int cols, int64_t ld,
                                                             double* __restrict__ partial) {
  __shared__ double part[4][64];
  const int lane = threadIdx.x & 63;
  const int grp = threadIdx.x >> 6;
  const int col = blockIdx.x * 64 + lane;
  const int per = (rows + gridDim.y - 1) / gridDim.y;
  const int r0 = blockIdx.y * per;
  const int r1 = min(rows, r0 + per);
  double acc = 0.0;
  if (col < cols) {
    for (int r = r0 + grp; r < r1; r += 4) acc += (double)x[(int64_t)r * ld + col];
  }
  part[grp][lane] = acc;
  __syncthreads();
  if (grp == 0 && col < cols)
    partial[(int64_t)blockIdx.y * cols + col] = part[0][lane] + part[1][lane] + part[2][lane] +
                                                part[3][lane];
}

// Vector variant (ld, cols multiples of 4, 16-B aligned): each lane sums 4 adjacent
// columns with float4 loads, two rows in flight per row group.  Same per-column
// order of summation structure (fp64 partials per row chunk, fixed-order final).
__global__ __launch_bounds__(256) void colsum_partial4_kernel(const float* __restrict__ x,
                                                              int rows, int cols, int64_t ld,
                                                              double* __restrict__ partial) {
  __shared__ double part[4][256];
  const int lane = threadIdx.x & 63;
  const int grp = threadIdx.x >> 6;
  const int col = blockIdx.x * 256 + lane * 4;
  const int per = (rows + gridDim.y - 1) / gridDim.y;
  const int r0 = blockIdx.y * per;
  const int r1 = min(rows, r0 + per);
  double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
  if (col < cols) {
    int r = r0 + grp;
    for (; r + 4 < r1; r += 8) {
      const float4 u = *reinterpret_cast<const float4*>(x + (int64_t)r * ld + col);
      const float4 v = *reinterpret_cast<const float4*>(x + (int64_t)(r + 4) * ld + col);
      a0 += (double)u.x; a1 += (double)u.y; a2 += (double)u.z; a3 += (double)u.w;
      a0 += (double)v.x; a1 += (double)v.y; a2 += (double)v.z; a3 += (double)v.w;
    }
    if (r < r1) {
      const float4 u = *reinterpret_cast<const float4*>(x + (int64_t)r * ld + col);
      a0 += (double)u.x; a1 += (double)u.y; a2 += (double)u.z; a3 += (double)u.w;
    }
  }
  part[grp][lane * 4 + 0] = a0;
  part[grp][lane * 4 + 1] = a1;
  part[grp][lane * 4 + 2] = a2;
  part[grp][lane * 4 + 3] = a3;
  __syncthreads();
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c < cols)
    partial[(int64_t)blockIdx.y * cols + c] =
        part[0][threadIdx.x] + part[1][threadIdx.x] + part[2][threadIdx.x] + part[3][threadIdx.x];
}

// 64 columns per block; the 4 waves sum interleaved chunk subsets, combined in a
// fixed order (deterministic)
__global__ __launch_bounds__(256) void colsum_final_kernel(const double* __restrict__ partial,
                                                           int chunks, int cols,
                                                           float* __restrict__ out,
                                                           int accumulate) {
  __shared__ double part[4][64];
  const int lane = threadIdx.x & 63;
  const int grp = threadIdx.x >> 6;
  const int col = blockIdx.x * 64 + lane;
  double s = 0.0;
  if (col < cols) {
#pragma unroll 8
    for (int c = grp; c < chunks; c += 4) s += partial[(int64_t)c * cols + col];   // order kept
  }
  part[grp][lane] = s;
  __syncthreads();
  if (grp == 0 && col < cols) {
    const float v = static_cast<float>((part[0][lane] + part[1][lane]) +
                                       (part[2][lane] + part[3][lane]));
    out[col] = accumulate ? out[col] + v : v;
  }
}

// ---------------------------------------------------------------------------
// Softmax over C (C <= 64 fast path: one wave handles 64/C rows... we keep it
// simple: one wave per (t, n) row with lanes over C, C <= 64).
__global__ void softmax_tnc_kernel(const float* __restrict__ logits, int t_max, int n, int c,
                                   float* __restrict__ probs) {
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  const int rows = t_max * n;
  if (wave >= rows) return;
  const int t = wave / n;
  const int b = wave - t * n;
  const float* src = logits + (int64_t)wave * c;
  float v = lane < c ? src[lane] : -INFINITY;
  float m = wave_max(v);
  float e = lane < c ? expf(v - m) : 0.0f;
  float s = wave_sum(e);
  if (lane < c) probs[((int64_t)b * t_max + t) * c + lane] = e / s;
}

__global__ void softmax_tnc_bwd_kernel(const float* __restrict__ probs,
                                       const float* __restrict__ dprobs, int t_max, int n, int c,
                                       float* __restrict__ dlogits, int accumulate) {
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  const int rows = t_max * n;
  if (wave >= rows) return;
  const int t = wave / n;
  const int b = wave - t * n;
  const int64_t src = ((int64_t)b * t_max + t) * c + lane;
  float y = lane < c ? probs[src] : 0.0f;
  float dy = lane < c ? dprobs[src] : 0.0f;
  float dot = wave_sum(y * dy);
  if (lane < c) {
    float g = y * (dy - dot);
    float* dst = dlogits + (int64_t)wave * c + lane;
    *dst = accumulate ? *dst + g : g;
  }
}

// ---------------------------------------------------------------------------
// Optimizer tail.
__global__ void sqnorm_partial_kernel(const float* __restrict__ g, int64_t numel,
                                      double* __restrict__ partial) {
  double acc = 0.0;
  const int64_t n4 = numel >> 2;
  const float4* g4 = reinterpret_cast<const float4*>(g);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4;
       i += (int64_t)gridDim.x * blockDim.x) {
    float4 v = g4[i];
    acc += (double)v.x * v.x + (double)v.y * v.y + (double)v.z * v.z + (double)v.w * v.w;
  }
  for (int64_t i = (n4 << 2) + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < numel;
       i += (int64_t)gridDim.x * blockDim.x) {
    double v = g[i];
    acc += v * v;
  }
  __shared__ double red[4];
  acc = wave_sum_d(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    double s = 0.0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) s += red[w];
    partial[blockIdx.x] = s;
  }
}

__global__ void sqnorm_final_kernel(const double* __restrict__ partial, int nparts,
                                    float* __restrict__ out_norm) {
  double acc = 0.0;
#pragma unroll 8
  for (int i = threadIdx.x; i < nparts; i += blockDim.x) acc += partial[i];
  __shared__ double red[4];
  acc = wave_sum_d(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    double s = 0.0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) s += red[w];
    *out_norm = static_cast<float>(sqrt(s));
  }
}

// torch.nn.utils.clip_grad_norm_: coef = max_norm / (norm + 1e-6), clamped to 1;
// torch.optim.SGD(nesterov): buf = m*buf + g; d = g + m*buf; p -= lr*d.
__global__ void clip_sgd_nesterov_kernel(float* __restrict__ p, const float* __restrict__ g,
                                         float* __restrict__ buf, int64_t numel, float lr,
                                         float mom, float max_norm,
                                         const float* __restrict__ norm,
                                         const int* __restrict__ skip) {
  if (skip != nullptr && *skip != 0) return;
  float coef = 1.0f;
  if (norm != nullptr && max_norm > 0.0f) {
    coef = max_norm / (*norm + 1e-6f);
    coef = fminf(coef, 1.0f);
  }
  const int64_t n4 = numel >> 2;
  float4* p4 = reinterpret_cast<float4*>(p);
  const float4* g4 = reinterpret_cast<const float4*>(g);
  float4* b4 = reinterpret_cast<float4*>(buf);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4;
       i += (int64_t)gridDim.x * blockDim.x) {
    float4 gv = g4[i], bv = b4[i], pv = p4[i];
    gv.x *= coef; gv.y *= coef; gv.z *= coef; gv.w *= coef;
    bv.x = mom * bv.x + gv.x; bv.y = mom * bv.y + gv.y;
    bv.z = mom * bv.z + gv.z; bv.w = mom * bv.w + gv.w;
    pv.x -= lr * (gv.x + mom * bv.x); pv.y -= lr * (gv.y + mom * bv.y);
    pv.z -= lr * (gv.z + mom * bv.z); pv.w -= lr * (gv.w + mom * bv.w);
    b4[i] = bv;
    p4[i] = pv;
  }
  for (int64_t i = (n4 << 2) + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < numel;
       i += (int64_t)gridDim.x * blockDim.x) {
    float gv = g[i] * coef;
    float bv = mom * buf[i] + gv;
    buf[i] = bv;
    p[i] -= lr * (gv + mom * bv);
  }
}

__global__ void nan_guard_kernel(float* __restrict__ x, int64_t numel, int zero_nans,
                                 int* __restrict__ flag, unsigned char* __restrict__ mask) {
  int found = 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < numel;
       i += (int64_t)gridDim.x * blockDim.x) {
    float v = x[i];
    const bool nan = v != v;
    if (nan) {
      found = 1;
      if (zero_nans) x[i] = 0.0f;
    }
    if (mask != nullptr) mask[i] = nan ? 1 : 0;
  }
  if (__any(found) && (threadIdx.x & 63) == 0) atomicOr(flag, 1);
}

// Backward of the in-place NaN zeroing (train.py:598 `logits[isnan(logits)] = 0`): autograd's
// index_put gives the zeroed positions a zero gradient.  Nothing to do unless *flag says a NaN
// was seen (the common case reads one word and leaves).
__global__ void zero_masked_kernel(float* __restrict__ x, const unsigned char* __restrict__ mask,
                                   int64_t numel, const int* __restrict__ flag) {
  if (flag != nullptr && *flag == 0) return;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < numel;
       i += (int64_t)gridDim.x * blockDim.x)
    if (mask[i]) x[i] = 0.0f;
}

__global__ void scale_kernel(float* __restrict__ x, int64_t numel, const float* __restrict__ s) {
  const float k = *s;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < numel;
       i += (int64_t)gridDim.x * blockDim.x)
    x[i] *= k;
}

}  // namespace ds2

using namespace ds2;

extern "C" {

const char* ds2_status_string(ds2_status_t s) {
  switch (s) {
    case DS2_OK: return "DS2_OK";
    case DS2_INVALID_VALUE: return "DS2_INVALID_VALUE";
    case DS2_UNSUPPORTED_SHAPE: return "DS2_UNSUPPORTED_SHAPE";
    case DS2_HIP_ERROR: return "DS2_HIP_ERROR";
    case DS2_RCCL_ERROR: return "DS2_RCCL_ERROR";
    case DS2_WORKSPACE_TOO_SMALL: return "DS2_WORKSPACE_TOO_SMALL";
  }
  return "DS2_UNKNOWN_STATUS";
}

const char* ds2_last_error(void) { return g_last_error; }

const char* ds2_version(void) { return "libds2hip 0.1.0 gfx950"; }

ds2_status_t ds2_dirsum(const float* h_all, int rows, int num_dirs, int h, float* y,
                        ds2_stream_t stream) {
  if (rows < 0 || num_dirs < 1 || h < 0) return DS2_INVALID_VALUE;
  int64_t total = (int64_t)rows * h;
  if (total == 0) return DS2_OK;
  hipLaunchKernelGGL(dirsum_kernel, dim3(grid_for(total, 256)), dim3(256), 0, as_stream(stream),
                     h_all, (int64_t)rows, num_dirs, h, y);
  return launch_status("ds2_dirsum");
}

size_t ds2_colsum_workspace_size(int rows, int cols) {
  (void)rows;
  return (size_t)kColChunks * (cols > 0 ? cols : 0) * sizeof(double) + 256;
}

ds2_status_t ds2_colsum(const float* x, int rows, int cols, int64_t ld, float* out,
                        int accumulate, void* ws, size_t ws_bytes, ds2_stream_t stream) {
  if (rows < 0 || cols < 0 || ld < cols) return DS2_INVALID_VALUE;
  if (cols == 0) return DS2_OK;
  if (ws == nullptr || ws_bytes < ds2_colsum_workspace_size(rows, cols))
    return DS2_WORKSPACE_TOO_SMALL;
  int chunks = rows / 64;
  chunks = chunks < 1 ? 1 : (chunks > kColChunks ? kColChunks : chunks);
  double* partial = static_cast<double*>(ws);
  if ((ld % 4) == 0 && (cols % 4) == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0)
    hipLaunchKernelGGL(colsum_partial4_kernel, dim3(cdiv(cols, 256), chunks), dim3(256), 0,
                       as_stream(stream), x, rows, cols, ld, partial);
  else
    hipLaunchKernelGGL(colsum_partial_kernel, dim3(cdiv(cols, 64), chunks), dim3(256), 0,
                       as_stream(stream), x, rows, cols, ld, partial);
  hipLaunchKernelGGL(colsum_final_kernel, dim3(cdiv(cols, 64)), dim3(256), 0, as_stream(stream),
                     partial, chunks, cols, out, accumulate);
  return launch_status("ds2_colsum");
}

ds2_status_t ds2_softmax_tnc(const float* logits, int t_max, int n, int c, float* probs,
                             ds2_stream_t stream) {
  if (t_max < 0 || n < 0 || c < 1 || c > 64) return DS2_UNSUPPORTED_SHAPE;
  int rows = t_max * n;
  if (rows == 0) return DS2_OK;
  hipLaunchKernelGGL(softmax_tnc_kernel, dim3(cdiv(rows, 4)), dim3(256), 0, as_stream(stream),
                     logits, t_max, n, c, probs);
  return launch_status("ds2_softmax_tnc");
}

ds2_status_t ds2_softmax_tnc_bwd(const float* probs, const float* dprobs, int t_max, int n,
                                 int c, float* dlogits, int accumulate, ds2_stream_t stream) {
  if (t_max < 0 || n < 0 || c < 1 || c > 64) return DS2_UNSUPPORTED_SHAPE;
  int rows = t_max * n;
  if (rows == 0) return DS2_OK;
  hipLaunchKernelGGL(softmax_tnc_bwd_kernel, dim3(cdiv(rows, 4)), dim3(256), 0,
                     as_stream(stream), probs, dprobs, t_max, n, c, dlogits, accumulate);
  return launch_status("ds2_softmax_tnc_bwd");
}

size_t ds2_optim_workspace_size(int64_t numel) {
  (void)numel;
  return 2048 * sizeof(double);
}

ds2_status_t ds2_grad_norm(const float* grads, int64_t numel, float* out_norm, void* ws,
                           size_t ws_bytes, ds2_stream_t stream) {
  if (numel < 0 || out_norm == nullptr) return DS2_INVALID_VALUE;
  if (ws_bytes < ds2_optim_workspace_size(numel) || ws == nullptr) return DS2_WORKSPACE_TOO_SMALL;
  if ((reinterpret_cast<uintptr_t>(grads) & 15) != 0) return DS2_INVALID_VALUE;
  int grid = grid_for((numel >> 2) + 1, 256);
  double* partial = static_cast<double*>(ws);
  hipLaunchKernelGGL(sqnorm_partial_kernel, dim3(grid), dim3(256), 0, as_stream(stream), grads,
                     numel, partial);
  hipLaunchKernelGGL(sqnorm_final_kernel, dim3(1), dim3(256), 0, as_stream(stream), partial, grid,
                     out_norm);
  return launch_status("ds2_grad_norm");
}

ds2_status_t ds2_clip_sgd_nesterov(float* params, const float* grads, float* momentum_buf,
                                   int64_t numel, float lr, float momentum, float max_norm,
                                   const float* norm, const int* skip_flag,
                                   ds2_stream_t stream) {
  if (numel < 0) return DS2_INVALID_VALUE;
  if (((reinterpret_cast<uintptr_t>(params) | reinterpret_cast<uintptr_t>(grads) |
        reinterpret_cast<uintptr_t>(momentum_buf)) & 15) != 0)
    return DS2_INVALID_VALUE;
  if (numel == 0) return DS2_OK;
  hipLaunchKernelGGL(clip_sgd_nesterov_kernel, dim3(grid_for((numel >> 2) + 1, 256)), dim3(256),
                     0, as_stream(stream), params, grads, momentum_buf, numel, lr, momentum,
                     max_norm, norm, skip_flag);
  return launch_status("ds2_clip_sgd_nesterov");
}

ds2_status_t ds2_nan_guard(float* x, int64_t numel, int zero_nans, int* flag,
                           unsigned char* mask, ds2_stream_t stream) {
  if (numel < 0 || flag == nullptr) return DS2_INVALID_VALUE;
  if (numel == 0) return DS2_OK;
  hipLaunchKernelGGL(nan_guard_kernel, dim3(grid_for(numel, 256)), dim3(256), 0,
                     as_stream(stream), x, numel, zero_nans, flag, mask);
  return launch_status("ds2_nan_guard");
}

ds2_status_t ds2_zero_masked(float* x, const unsigned char* mask, int64_t numel, const int* flag,
                             ds2_stream_t stream) {
  if (numel < 0 || (numel > 0 && mask == nullptr)) return DS2_INVALID_VALUE;
  if (numel == 0) return DS2_OK;
  hipLaunchKernelGGL(zero_masked_kernel, dim3(grid_for(numel, 256)), dim3(256), 0,
                     as_stream(stream), x, mask, numel, flag);
  return launch_status("ds2_zero_masked");
}

ds2_status_t ds2_scale_by_device_scalar(float* x, int64_t numel, const float* scalar,
                                        ds2_stream_t stream) {
  if (numel < 0 || scalar == nullptr) return DS2_INVALID_VALUE;
  if (numel == 0) return DS2_OK;
  hipLaunchKernelGGL(scale_kernel, dim3(grid_for(numel, 256)), dim3(256), 0, as_stream(stream),
                     x, numel, scalar);
  return launch_status("ds2_scale_by_device_scalar");
}

}  // extern "C"
