// Waveform effects of the reference's augmentations that librosa computes:
//   ChangeAudioSpeed  -> librosa.effects.time_stretch(wav, rate)      (data/audio_aug.py:7-23)
//   PitchShift        -> librosa.effects.pitch_shift(wav, sr, n)      (:63-75) = time_stretch
//                        by 2^(-n/12), then resample sr / rate -> sr
//   resampling a file -> librosa.resample(y, sr_file, sr)             (data_loader_aug.py:668)
// restated from librosa 0.8 / resampy 0.2 (oracle/librosa_effects.py is the CPU checker):
//
// time stretch = STFT (n_fft 2048, hop 512, periodic Hann, reflect pad 1024; fp64 radix-2
// FFT in LDS, stored complex64 like librosa's stft matrix) -> phase vocoder (one thread per
// bin walks the output frames: magnitude interpolation, float32 phase accumulator, the
// numpy dtype of every intermediate kept) -> ISTFT (fp64 inverse FFT of the Hermitian
// spectrum x window per frame, then per output sample the overlap-add of its <= 4 frames in
// frame order with float32 rounding after every add, as numpy's float32 `y[...] += ytmp`,
// divided by the float32 window sum of squares).
//
// resample = resampy's resample_f with the 'kaiser_best' table (host-computed, fp64): one
// thread per output sample, the two filter wings in resampy's loop order, every tap
// accumulated into a float32 like numba's `y[t] += weight * x[n - i]`; products and sums
// in fp64 without FMA contraction (explicit __dmul_rn / __dadd_rn), the time register
// accumulated sequentially (one add per output sample, as resampy) by a serial pass.
//
// Rates, lengths and frame counts are per utterance (host-computed with the reference's
// Python / numpy formulas and passed in), so one launch serves a ragged batch.
#include "common.h"

namespace ds2 {

constexpr int FX_N = 2048;          // n_fft
constexpr int FX_HOP = 512;         // n_fft / 4
constexpr int FX_BINS = FX_N / 2 + 1;
constexpr int FX_T = 256;

struct cd {
  double re, im;
};

__device__ __forceinline__ int fx_reflect(int i, int n) {
  // numpy 'reflect' (edge sample not repeated), periodic for pads longer than the signal
  if (n == 1) return 0;
  const int period = 2 * (n - 1);
  i %= period;
  if (i < 0) i += period;
  return i < n ? i : period - i;
}

__device__ __forceinline__ int bitrev11(int i) { return (int)(__builtin_bitreverse32((unsigned)i) >> 21); }

// In-place radix-2 FFT of FX_N points in LDS (input already in bit-reversed order).
// sign -1: forward (e^{-2 pi i k n / N}); +1: inverse (unnormalised).
__device__ void lds_fft(cd* a, const cd* tw, int sign) {
  for (int len = 2; len <= FX_N; len <<= 1) {
    const int half = len >> 1;
    const int tstep = FX_N / len;
    for (int b = threadIdx.x; b < FX_N / 2; b += blockDim.x) {
      const int grp = b / half;
      const int pos = b - grp * half;
      const int i = grp * len + pos;
      const int j = i + half;
      cd w = tw[pos * tstep];
      if (sign > 0) w.im = -w.im;
      const cd u = a[i], v = a[j];
      const double vr = v.re * w.re - v.im * w.im;
      const double vi = v.re * w.im + v.im * w.re;
      a[i] = cd{u.re + vr, u.im + vi};
      a[j] = cd{u.re - vr, u.im - vi};
    }
    __syncthreads();
  }
}

__device__ __forceinline__ void twiddles(cd* tw) {
  for (int k = threadIdx.x; k < FX_N / 2; k += blockDim.x) {
    double s, c;
    sincospi(-2.0 * k / FX_N, &s, &c);
    tw[k] = cd{c, s};
  }
}

// STFT frames: grid (max frames, n); D[b][f][FX_BINS] complex64 (float2)
__global__ __launch_bounds__(FX_T) void fx_stft_kernel(const float* __restrict__ x, int64_t x_stride,
                                                       const int* __restrict__ lens,
                                                       const double* __restrict__ window,
                                                       float2* __restrict__ D, int max_frames) {
  __shared__ cd a[FX_N];
  __shared__ cd tw[FX_N / 2];
  const int b = blockIdx.y, f = blockIdx.x;
  const int len = lens[b];
  const int frames = 1 + len / FX_HOP;
  if (f >= frames) return;
  twiddles(tw);
  const float* y = x + (int64_t)b * x_stride;
  for (int m = threadIdx.x; m < FX_N; m += blockDim.x) {
    // librosa: window (float64) * padded float32 frame
    const double v = window[m] * (double)y[fx_reflect(f * FX_HOP + m - FX_N / 2, len)];
    a[bitrev11(m)] = cd{v, 0.0};
  }
  __syncthreads();
  lds_fft(a, tw, -1);
  float2* out = D + ((int64_t)b * max_frames + f) * FX_BINS;
  for (int k = threadIdx.x; k < FX_BINS; k += blockDim.x)
    out[k] = make_float2(static_cast<float>(a[k].re), static_cast<float>(a[k].im));
}

// np.abs / np.angle of a complex64: libm hypotf / atan2f, which evaluate in double and round
// once -- the same here, so the float32 phase chain below sees the same bits as numpy's
__device__ __forceinline__ float fx_absf(float2 c) {
  return static_cast<float>(sqrt(__dadd_rn(__dmul_rn((double)c.x, (double)c.x),
                                           __dmul_rn((double)c.y, (double)c.y))));
}
__device__ __forceinline__ float fx_anglef(float2 c) {
  return static_cast<float>(atan2((double)c.y, (double)c.x));
}

// Phase vocoder: grid (ceil(FX_BINS / 64), n), block 64; thread = bin k of utterance b.
// librosa.phase_vocoder with numpy 1.x's dtypes for a complex64 D: |.| and angle() in
// float32, alpha and dphase in float64, mag in float32, exp(1j * phase_acc) in complex64, the
// float32 phase accumulator rounded after every step.
__global__ __launch_bounds__(64) void fx_vocoder_kernel(const float2* __restrict__ D, int max_in,
                                                        const int* __restrict__ lens,
                                                        const double* __restrict__ rate,
                                                        const int* __restrict__ out_frames,
                                                        float2* __restrict__ Ds, int max_out) {
  const int b = blockIdx.y;
  const int k = blockIdx.x * 64 + threadIdx.x;
  if (k >= FX_BINS) return;
  const int n_in = 1 + lens[b] / FX_HOP;
  const int n_out = out_frames[b];
  const double r = rate[b];
  // np.linspace(0, pi * hop, FX_BINS): k * step, the last element exactly pi * hop
  const double phi = (k == FX_BINS - 1) ? M_PI * FX_HOP
                                        : __dmul_rn((double)k, (M_PI * FX_HOP) / (FX_BINS - 1));
  const float2* col = D + (int64_t)b * max_in * FX_BINS + k;
  float phase_acc = fx_anglef(col[0]);
  float2* o = Ds + (int64_t)b * max_out * FX_BINS + k;
  for (int t = 0; t < n_out; ++t) {
    const double step = __dmul_rn((double)t, r);          // np.arange: start + i * delta
    const int i0 = static_cast<int>(step);
    const float2 c0 = i0 < n_in ? col[(int64_t)i0 * FX_BINS] : make_float2(0.f, 0.f);
    const float2 c1 = i0 + 1 < n_in ? col[(int64_t)(i0 + 1) * FX_BINS] : make_float2(0.f, 0.f);
    const double alpha = step - floor(step);               // np.mod(step, 1.0)
    const float m0 = fx_absf(c0), m1 = fx_absf(c1);
    // numpy 1.x value-based casting: the float64 scalars meet float32 arrays in float32
    const float mag = __fadd_rn(__fmul_rn(static_cast<float>(1.0 - alpha), m0),
                                __fmul_rn(static_cast<float>(alpha), m1));
    double snd, csd;
    sincos((double)phase_acc, &snd, &csd);    // libm cosf / sinf: correctly rounded
    const float sn = static_cast<float>(snd), cs = static_cast<float>(csd);
    o[(int64_t)t * FX_BINS] = make_float2(__fmul_rn(mag, cs), __fmul_rn(mag, sn));
    const float a1 = fx_anglef(c1), a0 = fx_anglef(c0);
    double dphase = __dsub_rn((double)(a1 - a0), phi);
    dphase = __dsub_rn(dphase, __dmul_rn(2.0 * M_PI, rint(dphase / (2.0 * M_PI))));
    phase_acc = static_cast<float>(__dadd_rn((double)phase_acc, __dadd_rn(phi, dphase)));
  }
}

// ISTFT frames: grid (max used frames, n); frames[b][f][FX_N] = window * irfft(Ds[b][f]) (fp64)
__global__ __launch_bounds__(FX_T) void fx_istft_frame_kernel(const float2* __restrict__ Ds, int max_out,
                                                              const int* __restrict__ used,
                                                              const double* __restrict__ window,
                                                              double* __restrict__ frames) {
  __shared__ cd a[FX_N];
  __shared__ cd tw[FX_N / 2];
  const int b = blockIdx.y, f = blockIdx.x;
  if (f >= used[b]) return;
  twiddles(tw);
  const float2* X = Ds + ((int64_t)b * max_out + f) * FX_BINS;
  // Hermitian extension; numpy's irfft takes the real parts of the DC and Nyquist bins
  for (int k = threadIdx.x; k < FX_N; k += blockDim.x) {
    cd v;
    if (k == 0 || k == FX_N / 2) {
      v = cd{(double)X[k].x, 0.0};
    } else if (k < FX_N / 2) {
      v = cd{(double)X[k].x, (double)X[k].y};
    } else {
      const float2 c = X[FX_N - k];
      v = cd{(double)c.x, -(double)c.y};
    }
    a[bitrev11(k)] = v;
  }
  __syncthreads();
  lds_fft(a, tw, +1);
  double* o = frames + ((int64_t)b * max_out + f) * FX_N;
  for (int m = threadIdx.x; m < FX_N; m += blockDim.x) o[m] = window[m] * (a[m].re / FX_N);
}

// Overlap-add + window-sum normalisation + center trim + fix_length:
// grid (ceil(out_stride / FX_T), n); out[b][i], i < out_len[b]
__global__ __launch_bounds__(FX_T) void fx_ola_kernel(const double* __restrict__ frames, int max_out,
                                                      const int* __restrict__ used,
                                                      const int* __restrict__ out_len,
                                                      const double* __restrict__ window,
                                                      float* __restrict__ out, int64_t out_stride) {
  const int b = blockIdx.y;
  const int64_t i = (int64_t)blockIdx.x * FX_T + threadIdx.x;
  if (i >= out_stride) return;
  float* o = out + (int64_t)b * out_stride;
  const int nf = used[b];
  const int64_t s = i + FX_N / 2;
  const int64_t total = FX_N + (int64_t)FX_HOP * (nf - 1);
  if (i >= out_len[b] || s >= total) {
    o[i] = 0.f;
    return;
  }
  const int64_t q = s - FX_N;                                 // first frame: 512 f + 2048 > s
  const int f0 = q < 0 ? 0 : static_cast<int>(q / FX_HOP + 1);
  int f1 = static_cast<int>(s / FX_HOP);
  if (f1 > nf - 1) f1 = nf - 1;
  const double* fb = frames + (int64_t)b * max_out * FX_N;
  float y = 0.f, w = 0.f;
  for (int f = f0; f <= f1; ++f) {
    const int m = static_cast<int>(s - (int64_t)f * FX_HOP);
    y = static_cast<float>(__dadd_rn((double)y, fb[(int64_t)f * FX_N + m]));
    const double wm = window[m];
    w = static_cast<float>(__dadd_rn((double)w, __dmul_rn(wm, wm)));
  }
  o[i] = (w > 1.17549435e-38f) ? y / w : y;
}

// resampy: the sequential time register, one serial thread per utterance
__global__ void fx_treg_kernel(const double* __restrict__ ratio, const int* __restrict__ n_valid,
                               int n, double* __restrict__ treg, int64_t stride) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= n) return;
  const double inc = 1.0 / ratio[b];
  double tr = 0.0;
  double* o = treg + (int64_t)b * stride;
  const int cnt = n_valid[b];
  for (int t = 0; t < cnt; ++t) {
    o[t] = tr;
    tr = __dadd_rn(tr, inc);
  }
}

__device__ __forceinline__ double fx_win(const double* win, int j, double ratio) {
  return ratio < 1.0 ? __dmul_rn(win[j], ratio) : win[j];
}

// grid (ceil(out_stride / FX_T), n)
__global__ __launch_bounds__(FX_T) void fx_resample_kernel(const float* __restrict__ x, int64_t x_stride,
                                                           const int* __restrict__ in_lens,
                                                           const double* __restrict__ ratio_p,
                                                           const int* __restrict__ n_valid,
                                                           const double* __restrict__ treg,
                                                           int64_t treg_stride,
                                                           const double* __restrict__ win, int nwin,
                                                           int num_table, float* __restrict__ out,
                                                           int64_t out_stride) {
  const int b = blockIdx.y;
  const int64_t t = (int64_t)blockIdx.x * FX_T + threadIdx.x;
  if (t >= out_stride) return;
  float* o = out + (int64_t)b * out_stride;
  if (t >= n_valid[b]) {
    o[t] = 0.f;
    return;
  }
  const double ratio = ratio_p[b];
  const double scale = ratio < 1.0 ? ratio : 1.0;
  const int index_step = static_cast<int>(__dmul_rn(scale, (double)num_table));
  const int n_orig = in_lens[b];
  const float* xb = x + (int64_t)b * x_stride;
  const double tr = treg[(int64_t)b * treg_stride + t];
  const int n = static_cast<int>(tr);
  float acc = 0.f;
  for (int wing = 0; wing < 2; ++wing) {
    double frac = __dmul_rn(scale, __dsub_rn(tr, (double)n));
    if (wing) frac = __dsub_rn(scale, frac);
    const double index_frac = __dmul_rn(frac, (double)num_table);
    const int offset = static_cast<int>(index_frac);
    const double eta = __dsub_rn(index_frac, (double)offset);
    const int lim = (nwin - offset) / index_step;
    const int cnt = wing == 0 ? min(n + 1, lim) : min(n_orig - n - 1, lim);
    for (int i = 0; i < cnt; ++i) {
      const int j = offset + i * index_step;
      const double wj = fx_win(win, j, ratio);
      const double dj = j + 1 < nwin ? __dsub_rn(fx_win(win, j + 1, ratio), wj) : 0.0;
      const double weight = __dadd_rn(wj, __dmul_rn(eta, dj));
      const float xv = wing == 0 ? xb[n - i] : xb[n + i + 1];
      acc = static_cast<float>(__dadd_rn((double)acc, __dmul_rn(weight, (double)xv)));
    }
  }
  o[t] = acc;
}

}  // namespace ds2

using namespace ds2;

extern "C" {

static inline size_t fx_al(size_t v) { return (v + 255) & ~(size_t)255; }

size_t ds2_time_stretch_workspace_size(int n, int max_in_frames, int max_out_frames) {
  if (n <= 0) return 256;
  return fx_al((size_t)n * max_in_frames * FX_BINS * sizeof(float2)) +
         fx_al((size_t)n * max_out_frames * FX_BINS * sizeof(float2)) +
         fx_al((size_t)n * max_out_frames * FX_N * sizeof(double)) + 256;
}

ds2_status_t ds2_time_stretch(const float* x, int64_t x_stride, const int* in_lens, int n,
                              const double* rate, const int* out_frames, const int* used_frames,
                              const int* out_lens, const double* window, float* out,
                              int64_t out_stride, int max_in_frames, int max_out_frames, void* ws,
                              size_t ws_bytes, ds2_stream_t stream) {
  if (n < 0 || x_stride < 0 || out_stride < 0 || max_in_frames < 0 || max_out_frames < 0)
    return DS2_INVALID_VALUE;
  if (n == 0) return DS2_OK;
  if (x == nullptr || in_lens == nullptr || rate == nullptr || out_frames == nullptr ||
      used_frames == nullptr || out_lens == nullptr || window == nullptr || out == nullptr)
    return DS2_INVALID_VALUE;
  if (ws == nullptr || ws_bytes < ds2_time_stretch_workspace_size(n, max_in_frames, max_out_frames))
    return DS2_WORKSPACE_TOO_SMALL;
  hipStream_t st = as_stream(stream);
  char* p = static_cast<char*>(ws);
  float2* D = reinterpret_cast<float2*>(p);
  p += fx_al((size_t)n * max_in_frames * FX_BINS * sizeof(float2));
  float2* Ds = reinterpret_cast<float2*>(p);
  p += fx_al((size_t)n * max_out_frames * FX_BINS * sizeof(float2));
  double* frames = reinterpret_cast<double*>(p);
  if (max_in_frames > 0)
    hipLaunchKernelGGL(fx_stft_kernel, dim3(max_in_frames, n), dim3(FX_T), 0, st, x, x_stride,
                       in_lens, window, D, max_in_frames);
  hipLaunchKernelGGL(fx_vocoder_kernel, dim3(cdiv(FX_BINS, 64), n), dim3(64), 0, st, D,
                     max_in_frames, in_lens, rate, out_frames, Ds, max_out_frames);
  if (max_out_frames > 0)
    hipLaunchKernelGGL(fx_istft_frame_kernel, dim3(max_out_frames, n), dim3(FX_T), 0, st, Ds,
                       max_out_frames, used_frames, window, frames);
  if (out_stride > 0)
    hipLaunchKernelGGL(fx_ola_kernel, dim3(cdiv(out_stride, FX_T), n), dim3(FX_T), 0, st, frames,
                       max_out_frames, used_frames, out_lens, window, out, out_stride);
  return launch_status("ds2_time_stretch");
}

size_t ds2_resample_workspace_size(int n, int64_t max_out) {
  return n > 0 && max_out > 0 ? fx_al((size_t)n * max_out * sizeof(double)) + 256 : 256;
}

ds2_status_t ds2_resample(const float* x, int64_t x_stride, const int* in_lens, int n,
                          const double* ratio, const int* n_valid, const double* win, int nwin,
                          int num_table, float* out, int64_t out_stride, void* ws,
                          size_t ws_bytes, ds2_stream_t stream) {
  if (n < 0 || x_stride < 0 || out_stride < 0 || nwin < 2 || num_table < 1) return DS2_INVALID_VALUE;
  if (n == 0 || out_stride == 0) return DS2_OK;
  if (x == nullptr || in_lens == nullptr || ratio == nullptr || n_valid == nullptr ||
      win == nullptr || out == nullptr)
    return DS2_INVALID_VALUE;
  if (ws == nullptr || ws_bytes < ds2_resample_workspace_size(n, out_stride))
    return DS2_WORKSPACE_TOO_SMALL;
  hipStream_t st = as_stream(stream);
  double* treg = static_cast<double*>(ws);
  hipLaunchKernelGGL(fx_treg_kernel, dim3(cdiv(n, 64)), dim3(64), 0, st, ratio, n_valid, n, treg,
                     out_stride);
  hipLaunchKernelGGL(fx_resample_kernel, dim3(cdiv(out_stride, FX_T), n), dim3(FX_T), 0, st, x,
                     x_stride, in_lens, ratio, n_valid, treg, out_stride, win, nwin, num_table,
                     out, out_stride);
  return launch_status("ds2_resample");
}

}  // extern "C"
