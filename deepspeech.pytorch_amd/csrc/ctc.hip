// CTC loss (warp-ctc semantics) and greedy CTC decoding.
//
// CTC: one workgroup per utterance.  log-softmax rows are materialised once in
// the workspace; alpha is scanned forward (one LDS row per step, stored to the
// workspace), beta is scanned backward keeping only the current LDS row, and the
// gradient row for frame t is produced right after beta_t is known:
//   grad[t][c] = softmax[t][c] - sum_{s: l'_s = c} exp(alpha_t(s) + beta_t(s) + nll - lp[t][c])
// which is d(-log p)/d(acts) through the internal softmax (ref: warpctc_pytorch,
// called at train.py:600-602; torch's ctc_loss backward formula is identical).
// Per-class sums walk a per-utterance class->state list in LDS, so results are
// deterministic (no float atomics).
//
// Greedy: one wave per utterance; argmax (first maximum) per frame, then a
// ballot/mbcnt compaction of the frames that survive blank/repeat removal
// (ref decoder.py:165-197).
#include "common.h"

namespace ds2 {

constexpr int kCtcThreads = 256;
constexpr int kCtcMaxS = 2 * 1024 + 1;  // max label length 1024

struct CtcWs {
  float* lp;      // [n][t_max][c]
  float* alpha;   // [n][t_max][s_max]
  int s_max;
};

__device__ __forceinline__ int label_at(const int* lab, int s, int blank) {
  return (s & 1) ? lab[s >> 1] : blank;
}

__global__ __launch_bounds__(kCtcThreads) void ctc_kernel(
    const float* __restrict__ acts, int t_max, int n, int c, const int* __restrict__ labels,
    const int* __restrict__ label_lens, const int* __restrict__ act_lens, int blank,
    int zero_infinity, float* __restrict__ costs, float* __restrict__ grads,
    float* __restrict__ lp_ws, float* __restrict__ alpha_ws, int s_max) {
  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  __shared__ float row_a[kCtcMaxS];
  __shared__ float row_b[kCtcMaxS];
  __shared__ int lab_s[1024];
  __shared__ int cls_count[64];
  __shared__ int cls_start[65];
  __shared__ int cls_states[kCtcMaxS];
  __shared__ float nll_s;

  int off = 0;
  for (int i = 0; i < b; ++i) off += label_lens[i];
  const int L = label_lens[b];
  int T = act_lens[b];
  if (T > t_max) T = t_max;
  if (T < 0) T = 0;
  const int S = 2 * L + 1;
  const int* lab_g = labels + off;
  for (int i = tid; i < L; i += blockDim.x) lab_s[i] = lab_g[i];
  if (tid < 64) cls_count[tid] = 0;
  __syncthreads();

  // class -> state lists (deterministic order: by state index)
  if (tid == 0) {
    for (int s = 0; s < S; ++s) cls_count[label_at(lab_s, s, blank)]++;
    int acc = 0;
    for (int k = 0; k < c; ++k) {
      cls_start[k] = acc;
      acc += cls_count[k];
    }
    cls_start[c] = acc;
    for (int k = 0; k < c; ++k) cls_count[k] = 0;
    for (int s = 0; s < S; ++s) {
      int k = label_at(lab_s, s, blank);
      cls_states[cls_start[k] + cls_count[k]++] = s;
    }
  }

  float* lp = lp_ws + (int64_t)b * t_max * c;
  float* alpha = alpha_ws + (int64_t)b * t_max * s_max;

  // log-softmax of every valid frame (one thread per frame, C is small).
  for (int t = tid; t < T; t += blockDim.x) {
    const float* a = acts + ((int64_t)t * n + b) * c;
    float m = -INFINITY;
    for (int k = 0; k < c; ++k) m = fmaxf(m, a[k]);
    float sum = 0.f;
    for (int k = 0; k < c; ++k) sum += expf(a[k] - m);
    float lse = m + logf(sum);
    for (int k = 0; k < c; ++k) lp[(int64_t)t * c + k] = a[k] - lse;
  }
  __syncthreads();

  // ---- alpha -------------------------------------------------------------
  float* cur = row_a;
  float* prv = row_b;
  if (T > 0) {
    for (int s = tid; s < S; s += blockDim.x) {
      float v = -INFINITY;
      if (s == 0) v = lp[blank];
      else if (s == 1) v = lp[label_at(lab_s, 1, blank)];
      cur[s] = v;
      alpha[s] = v;
    }
  }
  __syncthreads();
  for (int t = 1; t < T; ++t) {
    float* tmp = prv; prv = cur; cur = tmp;
    const float* lpt = lp + (int64_t)t * c;
    for (int s = tid; s < S; s += blockDim.x) {
      const int ls = label_at(lab_s, s, blank);
      float v = prv[s];
      if (s >= 1) v = log_add(v, prv[s - 1]);
      if (s >= 2 && ls != blank && ls != label_at(lab_s, s - 2, blank)) v = log_add(v, prv[s - 2]);
      v = (v == -INFINITY) ? -INFINITY : v + lpt[ls];
      cur[s] = v;
      alpha[(int64_t)t * s_max + s] = v;
    }
    __syncthreads();
  }
  if (tid == 0) {
    float ll;
    if (T == 0) ll = (L == 0) ? 0.f : -INFINITY;
    else {
      ll = cur[S - 1];
      if (S >= 2) ll = log_add(ll, cur[S - 2]);
    }
    nll_s = -ll;
  }
  __syncthreads();
  const float nll = nll_s;
  const bool feasible = (nll != INFINITY) && (nll == nll);
  if (tid == 0) costs[b] = feasible ? nll : (zero_infinity ? 0.f : INFINITY);

  if (grads == nullptr) return;
  // zero rows outside [0, T) and every row of an infeasible utterance
  for (int i = tid; i < t_max * c; i += blockDim.x) {
    const int t = i / c;
    if (t >= T || !feasible) grads[((int64_t)t * n + b) * c + (i - t * c)] = 0.f;
  }
  if (!feasible || T == 0) return;

  // ---- beta + gradient ---------------------------------------------------
  // reuse row_a/row_b as beta rows; e = exp(alpha + beta + nll) per state.
  float* bcur = row_a;
  float* bprv = row_b;
  for (int t = T - 1; t >= 0; --t) {
    const float* lpt = lp + (int64_t)t * c;
    for (int s = tid; s < S; s += blockDim.x) {
      const int ls = label_at(lab_s, s, blank);
      float v;
      if (t == T - 1) {
        v = (s == S - 1 || s == S - 2) ? lpt[ls] : -INFINITY;
      } else {
        v = bprv[s];
        if (s + 1 < S) v = log_add(v, bprv[s + 1]);
        if (s + 2 < S && ls != blank && ls != label_at(lab_s, s + 2, blank))
          v = log_add(v, bprv[s + 2]);
        v = (v == -INFINITY) ? -INFINITY : v + lpt[ls];
      }
      bcur[s] = v;
    }
    __syncthreads();
    // gradient row t: thread k < c walks the states of class k
    for (int k = tid; k < c; k += blockDim.x) {
      const float lpk = lpt[k];
      float acc = 0.f;
      for (int i = cls_start[k]; i < cls_start[k + 1]; ++i) {
        const int s = cls_states[i];
        const float ab = alpha[(int64_t)t * s_max + s] + bcur[s];
        if (ab != -INFINITY) acc += expf(ab + nll - lpk);
      }
      grads[((int64_t)t * n + b) * c + k] = expf(lpk) - acc;
    }
    __syncthreads();
    float* tmp = bprv; bprv = bcur; bcur = tmp;
  }
}

// ---------------------------------------------------------------------------
__global__ void greedy_kernel(const float* __restrict__ probs, int n, int t_max, int c,
                              int64_t stride_n, int64_t stride_t, const int* __restrict__ sizes,
                              int blank, int* __restrict__ out_ids, int* __restrict__ out_offsets,
                              int* __restrict__ out_counts, int* __restrict__ argmax_out) {
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (wave >= n) return;
  int size = sizes != nullptr ? sizes[wave] : t_max;
  if (size > t_max) size = t_max;
  if (size < 0) size = 0;
  const float* p = probs + (int64_t)wave * stride_n;
  int prev_last = -1;  // idx of frame (chunk_start - 1)
  int count = 0;
  for (int t0 = 0; t0 < t_max; t0 += 64) {
    const int t = t0 + lane;
    int idx = -1;
    if (t < t_max) {
      const float* row = p + (int64_t)t * stride_t;
      float best = row[0];
      idx = 0;
      for (int k = 1; k < c; ++k) {
        const float v = row[k];
        // torch.max semantics: first maximum; NaN counts as the maximum.
        if (best == best && (v > best || v != v)) {
          best = v;
          idx = k;
        }
      }
      if (argmax_out != nullptr) argmax_out[(int64_t)wave * t_max + t] = idx;
    }
    int prev = __shfl_up(idx, 1, 64);
    if (lane == 0) prev = prev_last;
    const bool emit = (t < size) && (idx != blank) && !(t > 0 && idx == prev);
    const unsigned long long mask = __ballot(emit);
    const int rank = __builtin_amdgcn_mbcnt_hi(static_cast<unsigned>(mask >> 32),
                                               __builtin_amdgcn_mbcnt_lo(static_cast<unsigned>(mask), 0));
    if (emit) {
      out_ids[(int64_t)wave * t_max + count + rank] = idx;
      out_offsets[(int64_t)wave * t_max + count + rank] = t;
    }
    count += __popcll(mask);
    prev_last = __shfl(idx, 63, 64);
  }
  if (lane == 0) out_counts[wave] = count;
}

}  // namespace ds2

using namespace ds2;

extern "C" {

size_t ds2_ctc_workspace_size(int t_max, int n, int max_label_len) {
  const int64_t s_max = 2 * (int64_t)max_label_len + 1;
  // lp uses c <= 64 classes; size for 64 to keep the query independent of c.
  return (size_t)n * t_max * 64 * sizeof(float) + (size_t)n * t_max * s_max * sizeof(float) + 256;
}

ds2_status_t ds2_ctc_loss(const float* acts, int t_max, int n, int c, const int* labels,
                          const int* label_lens, const int* act_lens, int max_label_len,
                          int blank, int zero_infinity, float* costs, float* grads, void* ws,
                          size_t ws_bytes, ds2_stream_t stream) {
  if (t_max < 0 || n < 0 || c < 1 || c > 64 || blank < 0 || blank >= c) return DS2_INVALID_VALUE;
  if (max_label_len < 0 || max_label_len > 1024) return DS2_UNSUPPORTED_SHAPE;
  if (n == 0) return DS2_OK;
  if (ws == nullptr || ws_bytes < ds2_ctc_workspace_size(t_max, n, max_label_len))
    return DS2_WORKSPACE_TOO_SMALL;
  const int s_max = 2 * max_label_len + 1;
  float* lp = static_cast<float*>(ws);
  float* alpha = lp + (size_t)n * t_max * 64;
  hipLaunchKernelGGL(ctc_kernel, dim3(n), dim3(kCtcThreads), 0, as_stream(stream), acts, t_max,
                     n, c, labels, label_lens, act_lens, blank, zero_infinity, costs, grads, lp,
                     alpha, s_max);
  return launch_status("ds2_ctc_loss");
}

ds2_status_t ds2_greedy_decode(const float* probs, int n, int t_max, int c, int64_t stride_n,
                               int64_t stride_t, const int* sizes, int blank, int* out_ids,
                               int* out_offsets, int* out_counts, int* argmax_out,
                               ds2_stream_t stream) {
  if (n < 0 || t_max < 0 || c < 1 || blank < 0 || blank >= c) return DS2_INVALID_VALUE;
  if (n == 0) return DS2_OK;
  hipLaunchKernelGGL(greedy_kernel, dim3(cdiv(n, 4)), dim3(256), 0, as_stream(stream), probs, n,
                     t_max, c, stride_n, stride_t, sizes, blank, out_ids, out_offsets, out_counts,
                     argmax_out);
  return launch_status("ds2_greedy_decode");
}

}  // extern "C"
