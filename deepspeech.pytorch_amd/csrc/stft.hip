// Spectrogram front-end: SpectrogramParser.audio_to_stft + normalize_audio.
// ref data/data_loader.py:201-220,245-284 (legacy, cited by north_star) and
// data/data_loader_aug.py:220-249,274-313 (the one train.py imports).
//
// librosa.stft semantics restated (librosa < 0.10, implied by the positional API
// used in data/audio_aug.py:20,74): center=True with reflect padding of n_fft/2,
// frames of n_fft every hop, window = the caller's n_fft taps (scipy hamming,
// symmetric), real FFT evaluated in float64, stored complex64, |.| in float32.
// normalize_audio modes (data_loader_aug.py:274-313): 0 'none' log1p(S); 1 'max_frame'
// log1p(S*2^20) - mean_t(gauss20(mean_f)); 2 'mean' log1p(S) - mean; 3 'norm' (log1p(S) -
// mean) / mean_t(std_f, unbiased); 4 'frame' log1p(S) - mean_t(gauss50(mean_f)).  The stft
// kernel writes every frame's mean (and, for 'norm', its std) over the 161 rows; one block
// per utterance turns them into an offset (and scale) that a last pass applies.
// The DFT is evaluated directly in fp64 (161 bins x 320 taps per frame,
// twiddles from an LDS table indexed by (k*m) mod n_fft): ~13 GFLOP of fp64 for
// a 32 x 10 s batch, far below the fp64 roof, and bit-for-bit free of the
// float32 round-off a fp32 DFT would add to near-silent bins after the x2^20
// gain of 'max_frame'.
#include "common.h"

namespace ds2 {

constexpr int SF = 8;          // frames per workgroup
constexpr int SMAXN = 1024;    // max n_fft
constexpr int kRows = 161;     // rows of the returned spectrogram (data_loader_aug.py:234-249)
constexpr int kMaskInts = 9;   // per utterance: f_lo0 f_hi0 f_lo1 f_hi1 t_lo0 t_hi0 t_lo1 t_hi1 f_cut

__device__ __forceinline__ int reflect_idx(int i, int n) {
  // numpy 'reflect' (edge sample not repeated); assumes n > 1
  const int period = 2 * (n - 1);
  i = i % period;
  if (i < 0) i += period;
  return i < n ? i : period - i;
}

__device__ __forceinline__ int scipy_reflect(int i, int n) {
  // scipy.ndimage mode='reflect' (half-sample symmetric): d c b a | a b c d
  const int period = 2 * n;
  i = i % period;
  if (i < 0) i += period;
  return i < n ? i : period - 1 - i;
}

// grid (ceil(max_frames / SF), batch); block 256 (thread = frequency bin)
__global__ __launch_bounds__(256) void stft_kernel(const float* __restrict__ pcm,
                                                   const int* __restrict__ n_samples,
                                                   int max_samples, int n_fft, int hop,
                                                   const double* __restrict__ window,
                                                   int normalize, float* __restrict__ out,
                                                   int max_frames, float* __restrict__ frame_mean,
                                                   float* __restrict__ frame_std,
                                                   const int* __restrict__ masks,
                                                   float* __restrict__ raw) {
  __shared__ double cs[SMAXN], sn[SMAXN];
  __shared__ double fr[SF][SMAXN];
  __shared__ double red[SF][4], red2[SF][4];
  const int b = blockIdx.y;
  const int t0 = blockIdx.x * SF;
  const int nb = n_samples[b];
  const int T = 1 + nb / hop;
  const int F = n_fft / 2 + 1;
  // bins computed: the 161 returned rows when F >= 161 (spect[:161], :249); all F bins in
  // the raw mode (F < 161: the mirror-fill layout is built from them by remap_kernel)
  const int R = raw != nullptr ? F : (F < kRows ? F : kRows);
  const int pad = n_fft / 2;
  const float* y = pcm + (int64_t)b * max_samples;
  for (int m = threadIdx.x; m < n_fft; m += blockDim.x) {
    double s, c;
    sincospi(2.0 * m / n_fft, &s, &c);
    cs[m] = c;
    sn[m] = s;
  }
  for (int i = threadIdx.x; i < SF * n_fft; i += blockDim.x) {
    const int f = i / n_fft;
    const int m = i - f * n_fft;
    const int t = t0 + f;
    double v = 0.0;
    if (t < T) v = window[m] * (double)y[reflect_idx(t * hop + m - pad, nb)];
    fr[f][m] = v;
  }
  __syncthreads();
  const int k = threadIdx.x;
  // spectrogram augmentation masks of this utterance (kMaskInts per utterance, see the
  // entry point): frequency bands, time bands and the 8 kHz cut, applied to |D| before
  // the log like data_loader_aug.py:236-248 does
  int fm[4] = {0, 0, 0, 0}, tm[4] = {0, 0, 0, 0}, fcut = F;
  if (masks != nullptr) {
    const int* mk = masks + b * kMaskInts;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      fm[i] = mk[i];
      tm[i] = mk[4 + i];
    }
    fcut = mk[8];
  }
  const bool fmasked = (k >= fm[0] && k < fm[1]) || (k >= fm[2] && k < fm[3]) || k >= fcut;
  double lsum[SF];
#pragma unroll
  for (int f = 0; f < SF; ++f) lsum[f] = 0.0;
  const float gain = normalize == 1 ? 1048576.0f : 1.0f;
  if (k < R) {
    double re[SF], im[SF];
#pragma unroll
    for (int f = 0; f < SF; ++f) { re[f] = 0.0; im[f] = 0.0; }
    int idx = 0;   // (k * m) mod n_fft
    for (int m = 0; m < n_fft; ++m) {
      const double c = cs[idx], s = sn[idx];
#pragma unroll
      for (int f = 0; f < SF; ++f) {
        const double v = fr[f][m];
        re[f] = fma(v, c, re[f]);
        im[f] = fma(-v, s, im[f]);
      }
      idx += k;
      if (idx >= n_fft) idx -= n_fft;
    }
    if (raw != nullptr) {     // |D| frame-major, the memory order of librosa's stft matrix
#pragma unroll
      for (int f = 0; f < SF; ++f) {
        const int t = t0 + f;
        if (t < T && t < max_frames)
          raw[((int64_t)b * max_frames + t) * F + k] =
              hypotf(static_cast<float>(re[f]), static_cast<float>(im[f]));
      }
      return;
    }
#pragma unroll
    for (int f = 0; f < SF; ++f) {
      const int t = t0 + f;
      if (t >= max_frames) continue;
      float val = 0.f;
      if (t < T) {
        const bool masked =
            fmasked || (t >= tm[0] && t < tm[1]) || (t >= tm[2] && t < tm[3]);
        const float mag =
            masked ? 0.f : hypotf(static_cast<float>(re[f]), static_cast<float>(im[f]));
        val = log1pf(mag * gain);
        lsum[f] = val;
      }
      out[((int64_t)b * R + k) * max_frames + t] = val;
    }
  }
  if (raw != nullptr) return;
  // mean over the F bins of every frame (torch spect.mean(dim=0)); 'norm' also the sum of
  // squares for the frame's unbiased std (spect.std(dim=0))
#pragma unroll
  for (int f = 0; f < SF; ++f) {
    double v = wave_sum_d(lsum[f]);
    if ((threadIdx.x & 63) == 0) red[f][threadIdx.x >> 6] = v;
  }
  if (frame_std != nullptr) {
#pragma unroll
    for (int f = 0; f < SF; ++f) {
      double v = wave_sum_d(lsum[f] * lsum[f]);
      if ((threadIdx.x & 63) == 0) red2[f][threadIdx.x >> 6] = v;
    }
  }
  __syncthreads();
  if (threadIdx.x < SF) {
    const int f = threadIdx.x;
    const int t = t0 + f;
    if (t < T && t < max_frames) {
      const double s = red[f][0] + red[f][1] + red[f][2] + red[f][3];
      frame_mean[(int64_t)b * max_frames + t] = static_cast<float>(s / R);
      if (frame_std != nullptr) {
        const double q = red2[f][0] + red2[f][1] + red2[f][2] + red2[f][3];
        const double var = (q - s * s / R) / (R - 1);
        frame_std[(int64_t)b * max_frames + t] = static_cast<float>(sqrt(var > 0.0 ? var : 0.0));
      }
    }
  }
}

// F < 161 bins (sample rates below 16 kHz): data_loader_aug.py:234-238
//   spect.resize((161, T)); spect[81:] = spect[80:0:-1]
// on librosa's stft matrix, which is Fortran-ordered (frame-major memory), so ndarray.resize
// keeps the first 161 T values of that memory in column-major order and zero-fills the rest:
// row r <= 80 of column t holds flat value 161 t + r (bin (161 t + r) % F of frame
// (161 t + r) / F), rows 81..160 mirror rows 80..1.  Then the spectrogram masks, the 8 kHz
// cut, log1p and the per-column mean, as in the fused kernel.  One wave per column.
__global__ __launch_bounds__(256) void remap_kernel(const float* __restrict__ raw,
                                                    const int* __restrict__ n_samples, int hop,
                                                    int F, int normalize, int max_frames,
                                                    const int* __restrict__ masks,
                                                    float* __restrict__ out,
                                                    float* __restrict__ frame_mean,
                                                    float* __restrict__ frame_std) {
  const int b = blockIdx.y;
  const int t = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (t >= max_frames) return;
  const int T = 1 + n_samples[b] / hop;
  int fm[4] = {0, 0, 0, 0}, tm[4] = {0, 0, 0, 0}, fcut = kRows;
  if (masks != nullptr) {
    const int* mk = masks + b * kMaskInts;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      fm[i] = mk[i];
      tm[i] = mk[4 + i];
    }
    fcut = mk[8];
  }
  const bool tmasked = (t >= tm[0] && t < tm[1]) || (t >= tm[2] && t < tm[3]);
  const float* rb = raw + (int64_t)b * max_frames * F;
  const int64_t valid = (int64_t)F * (T < max_frames ? T : max_frames);
  double lsum = 0.0, lsq = 0.0;
  const float gain = normalize == 1 ? 1048576.0f : 1.0f;
  for (int r = lane; r < kRows; r += 64) {
    float val = 0.f;
    if (t < T) {
      const int rs = r <= 80 ? r : kRows - r;
      const int64_t kf = (int64_t)kRows * t + rs;
      const bool masked = tmasked || (r >= fm[0] && r < fm[1]) || (r >= fm[2] && r < fm[3]) ||
                          r >= fcut;
      const float mag = (masked || kf >= valid) ? 0.f : rb[kf];
      val = log1pf(mag * gain);
      lsum += val;
      lsq += (double)val * val;
    }
    out[((int64_t)b * kRows + r) * max_frames + t] = val;
  }
  lsum = wave_sum_d(lsum);
  lsq = wave_sum_d(lsq);
  if (lane == 0 && t < T) {
    frame_mean[(int64_t)b * max_frames + t] = static_cast<float>(lsum / kRows);
    if (frame_std != nullptr) {
      const double var = (lsq - lsum * lsum / kRows) / (kRows - 1);
      frame_std[(int64_t)b * max_frames + t] = static_cast<float>(sqrt(var > 0.0 ? var : 0.0));
    }
  }
}

// One block per utterance.  taps != nullptr ('max_frame', 'frame'): offset =
// mean_t(gaussian_filter1d(frame_mean, sigma)); else ('mean', 'norm') offset = the mean over
// all 161 x T values = mean_t(frame_mean), and with frame_std ('norm') scale = mean_t(std).
__global__ void maxframe_offset_kernel(const int* __restrict__ n_samples, int hop,
                                       int max_frames, const float* __restrict__ frame_mean,
                                       const float* __restrict__ frame_std,
                                       const float* __restrict__ taps, int radius,
                                       float* __restrict__ offset, float* __restrict__ scale) {
  const int b = blockIdx.x;
  int T = 1 + n_samples[b] / hop;
  if (T > max_frames) T = max_frames;
  const float* m = frame_mean + (int64_t)b * max_frames;
  double acc = 0.0, acc2 = 0.0;
  for (int t = threadIdx.x; t < T; t += blockDim.x) {
    if (taps != nullptr) {
      double s = 0.0;
      for (int j = -radius; j <= radius; ++j) s += (double)taps[j + radius] * m[scipy_reflect(t + j, T)];
      acc += (double)static_cast<float>(s);   // scipy writes the float32 filtered signal
    } else {
      acc += (double)m[t];
      if (frame_std != nullptr) acc2 += (double)frame_std[(int64_t)b * max_frames + t];
    }
  }
  __shared__ double red[4], red2[4];
  acc = wave_sum_d(acc);
  acc2 = wave_sum_d(acc2);
  if ((threadIdx.x & 63) == 0) {
    red[threadIdx.x >> 6] = acc;
    red2[threadIdx.x >> 6] = acc2;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    offset[b] = static_cast<float>((red[0] + red[1] + red[2] + red[3]) / T);
    if (scale != nullptr) scale[b] = static_cast<float>((red2[0] + red2[1] + red2[2] + red2[3]) / T);
  }
}

__global__ void subtract_offset_kernel(const int* __restrict__ n_samples, int hop, int F,
                                       int max_frames, const float* __restrict__ offset,
                                       const float* __restrict__ scale,
                                       float* __restrict__ out) {
  const int b = blockIdx.y;
  int T = 1 + n_samples[b] / hop;
  if (T > max_frames) T = max_frames;
  const float o = offset[b];
  const float sc = scale != nullptr ? scale[b] : 1.0f;
  const int64_t total = (int64_t)F * max_frames;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int t = static_cast<int>(i % max_frames);
    if (t < T) {
      const float v = out[(int64_t)b * total + i] - o;     // spect.add_(-mean)
      out[(int64_t)b * total + i] = scale != nullptr ? v / sc : v;   // spect.div_(std.mean())
    }
  }
}

}  // namespace ds2

using namespace ds2;

extern "C" {

// frame_mean, frame_std [batch][max_frames]; offset, scale [batch]
static size_t stft_base_ws(int batch, int max_frames) {
  return 2 * (size_t)batch * max_frames * sizeof(float) + 2 * (size_t)batch * sizeof(float) + 512;
}

size_t ds2_stft_workspace_size(int batch, int max_frames, int n_fft) {
  const int F = n_fft / 2 + 1;
  size_t bytes = stft_base_ws(batch, max_frames);
  if (F < kRows) bytes += (size_t)batch * max_frames * F * sizeof(float) + 256;
  return bytes;
}

ds2_status_t ds2_stft_logmag_masked(const float* pcm, const int* n_samples, int batch,
                                    int max_samples, int n_fft, int hop, const double* window,
                                    int normalize, const float* gauss_taps, int gauss_radius,
                                    const int* masks, float* out, int max_frames, void* ws,
                                    size_t ws_bytes, ds2_stream_t stream) {
  if (batch < 0 || n_fft < 2 || n_fft > SMAXN || hop < 1 || max_frames < 1) return DS2_INVALID_VALUE;
  if (n_fft / 2 + 1 > 256) return DS2_UNSUPPORTED_SHAPE;
  if (normalize < 0 || normalize > 4) return DS2_INVALID_VALUE;
  const bool smooth = normalize == 1 || normalize == 4;
  if (smooth && (gauss_taps == nullptr || gauss_radius < 0)) return DS2_INVALID_VALUE;
  if (batch == 0) return DS2_OK;
  if (ws == nullptr || ws_bytes < ds2_stft_workspace_size(batch, max_frames, n_fft))
    return DS2_WORKSPACE_TOO_SMALL;
  hipStream_t st = as_stream(stream);
  float* frame_mean = static_cast<float*>(ws);
  float* frame_std = frame_mean + (size_t)batch * max_frames;
  float* offset = frame_std + (size_t)batch * max_frames;
  float* scale = offset + batch;
  float* fstd = normalize == 3 ? frame_std : nullptr;
  const int F = n_fft / 2 + 1;
  if (F < kRows) {
    float* raw = reinterpret_cast<float*>(
        static_cast<char*>(ws) + ((stft_base_ws(batch, max_frames) + 255) & ~(size_t)255));
    hipLaunchKernelGGL(stft_kernel, dim3(cdiv(max_frames, SF), batch), dim3(256), 0, st, pcm,
                       n_samples, max_samples, n_fft, hop, window, normalize, out, max_frames,
                       frame_mean, nullptr, masks, raw);
    hipLaunchKernelGGL(remap_kernel, dim3(cdiv(max_frames, 4), batch), dim3(256), 0, st, raw,
                       n_samples, hop, F, normalize, max_frames, masks, out, frame_mean, fstd);
  } else {
    hipLaunchKernelGGL(stft_kernel, dim3(cdiv(max_frames, SF), batch), dim3(256), 0, st, pcm,
                       n_samples, max_samples, n_fft, hop, window, normalize, out, max_frames,
                       frame_mean, fstd, masks, nullptr);
  }
  if (normalize != 0) {
    hipLaunchKernelGGL(maxframe_offset_kernel, dim3(batch), dim3(256), 0, st, n_samples, hop,
                       max_frames, frame_mean, fstd, smooth ? gauss_taps : nullptr, gauss_radius,
                       offset, normalize == 3 ? scale : nullptr);
    int g = cdiv((int64_t)kRows * max_frames, 256);
    if (g > 512) g = 512;
    hipLaunchKernelGGL(subtract_offset_kernel, dim3(g, batch), dim3(256), 0, st, n_samples, hop,
                       kRows, max_frames, offset, normalize == 3 ? scale : nullptr, out);
  }
  return launch_status("ds2_stft_logmag");
}

ds2_status_t ds2_stft_logmag(const float* pcm, const int* n_samples, int batch, int max_samples,
                             int n_fft, int hop, const double* window, int normalize,
                             const float* gauss_taps, int gauss_radius, float* out,
                             int max_frames, void* ws, size_t ws_bytes, ds2_stream_t stream) {
  return ds2_stft_logmag_masked(pcm, n_samples, batch, max_samples, n_fft, hop, window,
                                normalize, gauss_taps, gauss_radius, nullptr, out, max_frames, ws,
                                ws_bytes, stream);
}

}  // extern "C"
