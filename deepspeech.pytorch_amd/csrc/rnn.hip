// Vanilla (Elman) tanh RNN recurrence: supported_rnns['rnn'] = nn.RNN (ref model.py:15,97-109;
// nonlinearity tanh, both biases, packed sequences).  Per step
//   h_t = tanh(xproj_t + b_hh + W_hh h_{t-1})              (xproj_t = W_ih x_t + b_ih, a GEMM)
// and backward da_t = (dy_t + W_hh^T da_{t+1}) (1 - h_t^2), so dW_ih, dW_hh, dX and both bias
// gradients are the same plain GEMMs / column sums as the GRU's (ops._rnn_param_grads with
// dgx = dgh = da).  Not on the headline path (the DS2 benchmark is 5 x BiGRU-800), so the
// recurrence runs one launch per step: a workgroup computes a 16-sample x 32-unit tile of
// h_t (or of the carried gradient) as a dot over K staged through LDS in 64-wide chunks, both
// directions in one launch.  Packed semantics: outputs and gradients at t >= len are 0 and the
// reverse direction starts from h = 0 at t = len - 1 (exactly what zeroing h past the length
// gives, as in gru.hip).
#include "common.h"

namespace ds2 {

constexpr int RN_M = 16;      // samples per tile
constexpr int RN_U = 32;      // units per tile
constexpr int RN_KC = 64;     // K chunk staged in LDS
constexpr int RN_T = 256;     // threads: (sample m = tid / 16, units u and u + 16 of tid % 16)

// forward step s: h_all[t][n][d][:] for every direction d (t = s forward, T - 1 - s reverse)
__global__ __launch_bounds__(RN_T) void rnn_fwd_step_kernel(
    int s, int T, int N, int H, int D, const float* __restrict__ xproj,
    const float* __restrict__ w_f, const float* __restrict__ w_r, const float* __restrict__ b_f,
    const float* __restrict__ b_r, const int* __restrict__ lens, float* __restrict__ h_all) {
  __shared__ float hs[RN_M][RN_KC + 1];
  __shared__ float wsm[RN_U][RN_KC + 1];
  const int d = blockIdx.z;
  const int n0 = blockIdx.y * RN_M, j0 = blockIdx.x * RN_U;
  const int t = d == 0 ? s : T - 1 - s;
  const int tp = d == 0 ? t - 1 : t + 1;       // the previous step of this direction
  const float* W = d == 0 ? w_f : w_r;
  const float* bh = d == 0 ? b_f : b_r;
  const int m = threadIdx.x >> 4, u = threadIdx.x & 15;
  float acc0 = 0.f, acc1 = 0.f;
  if (s > 0) {
    for (int k0 = 0; k0 < H; k0 += RN_KC) {
      for (int i = threadIdx.x; i < RN_M * RN_KC; i += RN_T) {
        const int r = i / RN_KC, c = i - r * RN_KC;
        const int n = n0 + r, k = k0 + c;
        hs[r][c] = (n < N && k < H) ? h_all[(((int64_t)tp * N + n) * D + d) * H + k] : 0.f;
      }
      for (int i = threadIdx.x; i < RN_U * RN_KC; i += RN_T) {
        const int r = i / RN_KC, c = i - r * RN_KC;
        const int j = j0 + r, k = k0 + c;
        wsm[r][c] = (j < H && k < H) ? W[(int64_t)j * H + k] : 0.f;
      }
      __syncthreads();
#pragma unroll 16
      for (int c = 0; c < RN_KC; ++c) {
        const float hv = hs[m][c];
        acc0 = fmaf(hv, wsm[u][c], acc0);
        acc1 = fmaf(hv, wsm[u + 16][c], acc1);
      }
      __syncthreads();
    }
  }
  const int n = n0 + m;
  if (n >= N) return;
  const int len = lens[n];
  const float* xp = xproj + (((int64_t)t * N + n) * D + d) * H;
  float* ho = h_all + (((int64_t)t * N + n) * D + d) * H;
  const float acc[2] = {acc0, acc1};
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int j = j0 + u + 16 * q;
    if (j < H) ho[j] = t < len ? tanhf(xp[j] + bh[j] + acc[q]) : 0.f;
  }
}

// backward step s (the forward's steps in reverse): da[t][n][d][:] = (dy_t + W_hh^T
// da_{t+1 of this direction}) (1 - h_t^2), 0 past the length
__global__ __launch_bounds__(RN_T) void rnn_bwd_step_kernel(
    int s, int T, int N, int H, int D, const float* __restrict__ dy, int dyd,
    const float* __restrict__ w_f, const float* __restrict__ w_r,
    const float* __restrict__ h_all, const int* __restrict__ lens, float* __restrict__ da) {
  __shared__ float gs[RN_M][RN_KC + 1];
  __shared__ float wsm[RN_U][RN_KC + 1];       // wsm[k][j] = W_hh[j][k]
  const int d = blockIdx.z;
  const int n0 = blockIdx.y * RN_M, k0u = blockIdx.x * RN_U;
  const int t = d == 0 ? T - 1 - s : s;
  const int tq = d == 0 ? t + 1 : t - 1;       // the step processed before this one
  const float* W = d == 0 ? w_f : w_r;
  const int m = threadIdx.x >> 4, u = threadIdx.x & 15;
  float acc0 = 0.f, acc1 = 0.f;
  if (s > 0) {
    for (int j0 = 0; j0 < H; j0 += RN_KC) {
      for (int i = threadIdx.x; i < RN_M * RN_KC; i += RN_T) {
        const int r = i / RN_KC, c = i - r * RN_KC;
        const int n = n0 + r, j = j0 + c;
        gs[r][c] = (n < N && j < H) ? da[(((int64_t)tq * N + n) * D + d) * H + j] : 0.f;
      }
      for (int i = threadIdx.x; i < RN_U * RN_KC; i += RN_T) {
        const int c = i / RN_U, r = i - c * RN_U;   // consecutive threads: consecutive k
        const int k = k0u + r, j = j0 + c;
        wsm[r][c] = (k < H && j < H) ? W[(int64_t)j * H + k] : 0.f;
      }
      __syncthreads();
#pragma unroll 16
      for (int c = 0; c < RN_KC; ++c) {
        const float g = gs[m][c];
        acc0 = fmaf(g, wsm[u][c], acc0);
        acc1 = fmaf(g, wsm[u + 16][c], acc1);
      }
      __syncthreads();
    }
  }
  const int n = n0 + m;
  if (n >= N) return;
  const int len = lens[n];
  const float* hrow = h_all + (((int64_t)t * N + n) * D + d) * H;
  const float* dyr = dy + (((int64_t)t * N + n) * dyd + (dyd > 1 ? d : 0)) * H;
  float* o = da + (((int64_t)t * N + n) * D + d) * H;
  const float acc[2] = {acc0, acc1};
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int k = k0u + u + 16 * q;
    if (k >= H) continue;
    float v = 0.f;
    if (t < len) {
      const float hv = hrow[k];
      v = (dyr[k] + acc[q]) * (1.f - hv * hv);
    }
    o[k] = v;
  }
}

}  // namespace ds2

using namespace ds2;

extern "C" {

ds2_status_t ds2_rnn_fwd(int t_max, int n, int h, int num_dirs, const float* xproj,
                         const float* w_hh_f, const float* w_hh_r, const float* b_hh_f,
                         const float* b_hh_r, const int* lens, float* h_all,
                         ds2_stream_t stream) {
  if (t_max < 0 || n < 0 || h < 1 || (num_dirs != 1 && num_dirs != 2)) return DS2_INVALID_VALUE;
  if (t_max == 0 || n == 0) return DS2_OK;
  if (xproj == nullptr || w_hh_f == nullptr || b_hh_f == nullptr || lens == nullptr ||
      h_all == nullptr || (num_dirs == 2 && (w_hh_r == nullptr || b_hh_r == nullptr)))
    return DS2_INVALID_VALUE;
  if (num_dirs == 1) {
    w_hh_r = w_hh_f;
    b_hh_r = b_hh_f;
  }
  const dim3 grid(cdiv(h, RN_U), cdiv(n, RN_M), num_dirs);
  hipStream_t st = as_stream(stream);
  for (int s = 0; s < t_max; ++s)
    hipLaunchKernelGGL(rnn_fwd_step_kernel, grid, dim3(RN_T), 0, st, s, t_max, n, h, num_dirs,
                       xproj, w_hh_f, w_hh_r, b_hh_f, b_hh_r, lens, h_all);
  return launch_status("ds2_rnn_fwd");
}

ds2_status_t ds2_rnn_bwd(int t_max, int n, int h, int num_dirs, const float* dy, int dy_dirs,
                         const float* w_hh_f, const float* w_hh_r, const float* h_all,
                         const int* lens, float* dgates, ds2_stream_t stream) {
  if (t_max < 0 || n < 0 || h < 1 || (num_dirs != 1 && num_dirs != 2)) return DS2_INVALID_VALUE;
  if (dy_dirs != 1 && dy_dirs != num_dirs) return DS2_INVALID_VALUE;
  if (t_max == 0 || n == 0) return DS2_OK;
  if (dy == nullptr || w_hh_f == nullptr || h_all == nullptr || lens == nullptr ||
      dgates == nullptr || (num_dirs == 2 && w_hh_r == nullptr))
    return DS2_INVALID_VALUE;
  if (num_dirs == 1) w_hh_r = w_hh_f;
  const dim3 grid(cdiv(h, RN_U), cdiv(n, RN_M), num_dirs);
  hipStream_t st = as_stream(stream);
  for (int s = 0; s < t_max; ++s)
    hipLaunchKernelGGL(rnn_bwd_step_kernel, grid, dim3(RN_T), 0, st, s, t_max, n, h, num_dirs, dy,
                       dy_dirs, w_hh_f, w_hh_r, h_all, lens, dgates);
  return launch_status("ds2_rnn_bwd");
}

}  // extern "C"
