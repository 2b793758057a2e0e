// Waveform augmentations ahead of the STFT: the arithmetic of data/audio_aug.py's Shift
// (:26-44), AudioDistort (:47-60, clip :177-178) and AddNoise (:78-107) as per-utterance
// op lists executed on the device.  The host draws every random number in the
// reference's order (ds2amd/audio_aug.py) and records what each transform does; this
// kernel replays the records:
//   SHIFT   (shift, limit): y[i] = x[i - shift] for shift <= i < shift + len, else 0;
//           len += limit                                  (np.zeros(len + limit) fill)
//   DISTORT (alpha):        y = clip(f32(alpha) * x, 0, max(x))     (float32 numpy math)
//   NOISE   (row, alpha):   y = (x + alpha * noise[row][i]) / (1 + alpha)  in float64
//           (the noise slice noise[pos : pos + len] is cut on the host; float64 like
//           np.random.normal's draws)
// Between ops the samples are kept in fp32 (the STFT input type).  One workgroup per
// utterance: DISTORT needs the utterance's max before any output sample.
#include "common.h"

namespace ds2 {

constexpr int WAV_T = 1024;
enum { WAV_END = 0, WAV_SHIFT = 1, WAV_DISTORT = 2, WAV_NOISE = 3 };

__global__ __launch_bounds__(WAV_T) void wave_aug_kernel(
    const float* __restrict__ in, int64_t in_stride, const int* __restrict__ in_lens,
    const int* __restrict__ op_i, const double* __restrict__ op_f, int max_ops,
    const double* __restrict__ noise, int64_t noise_stride, float* __restrict__ buf, int64_t cap,
    float* __restrict__ out, int64_t out_stride, const int* __restrict__ out_lens,
    int* __restrict__ err) {
  __shared__ float red[WAV_T / kWave];
  const int n = blockIdx.x;
  const int tid = threadIdx.x;
  int64_t len = in_lens[n];
  const float* src = in + (int64_t)n * in_stride;
  float* pp[2] = {buf + (int64_t)(2 * n) * cap, buf + (int64_t)(2 * n + 1) * cap};
  int which = 0;
  for (int o = 0; o < max_ops; ++o) {
    const int* rec = op_i + ((int64_t)n * max_ops + o) * 4;
    const int kind = rec[0];
    if (kind == WAV_END) break;
    float* dst = pp[which];
    if (kind == WAV_SHIFT) {
      const int64_t shift = rec[1], nl = len + rec[2];
      if (nl > cap || shift < 0 || shift > rec[2]) {
        if (tid == 0) atomicOr(err, 1);
        return;
      }
      for (int64_t i = tid; i < nl; i += WAV_T)
        dst[i] = (i >= shift && i < shift + len) ? src[i - shift] : 0.f;
      len = nl;
    } else if (kind == WAV_DISTORT) {
      float m = -INFINITY;
      for (int64_t i = tid; i < len; i += WAV_T) m = fmaxf(m, src[i]);
      m = wave_max(m);
      if ((tid & 63) == 0) red[tid >> 6] = m;
      __syncthreads();
      m = red[0];
#pragma unroll
      for (int w = 1; w < WAV_T / kWave; ++w) m = fmaxf(m, red[w]);
      const float alpha = static_cast<float>(op_f[(int64_t)n * max_ops + o]);
      // np.clip(v, 0, m) = minimum(maximum(v, 0), m)
      for (int64_t i = tid; i < len; i += WAV_T) dst[i] = fminf(fmaxf(alpha * src[i], 0.f), m);
    } else if (kind == WAV_NOISE) {
      const double alpha = op_f[(int64_t)n * max_ops + o];
      const double* nz = noise + (int64_t)rec[1] * noise_stride;
      for (int64_t i = tid; i < len; i += WAV_T)
        dst[i] = static_cast<float>(((double)src[i] + alpha * nz[i]) / (1.0 + alpha));
    } else {
      if (tid == 0) atomicOr(err, 2);
      return;
    }
    __syncthreads();
    src = dst;
    which ^= 1;
  }
  if (len != out_lens[n]) {
    if (tid == 0) atomicOr(err, 4);
    return;
  }
  float* y = out + (int64_t)n * out_stride;
  for (int64_t i = tid; i < out_stride; i += WAV_T) y[i] = i < len ? src[i] : 0.f;
}

}  // namespace ds2

using namespace ds2;

extern "C" {

size_t ds2_wave_aug_workspace_size(int n, int64_t cap) {
  return n > 0 && cap > 0 ? (size_t)2 * n * cap * sizeof(float) + 256 : 256;
}

ds2_status_t ds2_wave_aug(const float* in, int64_t in_stride, const int* in_lens, int n,
                          const int* op_i, const double* op_f, int max_ops, const double* noise,
                          int64_t noise_stride, float* out, int64_t out_stride,
                          const int* out_lens, int64_t cap, int* err, void* ws, size_t ws_bytes,
                          ds2_stream_t stream) {
  if (n < 0 || max_ops < 0 || in_stride < 0 || out_stride < 0 || cap < 0) return DS2_INVALID_VALUE;
  if (n == 0) return DS2_OK;
  if (in == nullptr || in_lens == nullptr || out == nullptr || out_lens == nullptr ||
      err == nullptr || (max_ops > 0 && (op_i == nullptr || op_f == nullptr)))
    return DS2_INVALID_VALUE;
  if (ws == nullptr || ws_bytes < ds2_wave_aug_workspace_size(n, cap)) return DS2_WORKSPACE_TOO_SMALL;
  hipLaunchKernelGGL(wave_aug_kernel, dim3(n), dim3(WAV_T), 0, as_stream(stream), in, in_stride,
                     in_lens, op_i, op_f, max_ops, noise, noise_stride, static_cast<float*>(ws),
                     cap, out, out_stride, out_lens, err);
  return launch_status("ds2_wave_aug");
}

}  // extern "C"
