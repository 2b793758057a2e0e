/*
 * libds2hip — MI355X-native (gfx950 / CDNA4) DeepSpeech2 hot path, C ABI.
 *
 * The reference (vadimkantorov/deepspeech.pytorch) has no C ABI of its own: its
 * pluggable seams are Python objects whose kernels come from third-party
 * libraries (librosa FFT, cuDNN conv/BN/RNN, cuBLAS, warp-ctc, ATen argmax).
 * Every entry point below replaces one of those implicit kernels; the comment
 * above each names the reference call site (file:line) it stands in for.
 *
 * Conventions:
 *   - every function returns ds2_status_t; no exception crosses the ABI;
 *   - all buffers are caller-owned device pointers (fp32 unless noted, int32
 *     for lengths/labels), dense row-major unless a leading dimension is given;
 *   - work is enqueued on `stream` (a hipStream_t, NULL = legacy default);
 *     nothing synchronises the device, allocates, or touches host memory;
 *   - scratch memory comes in through (ws, ws_bytes); query the size with the
 *     matching *_workspace_size() function.
 */
#ifndef DS2HIP_H
#define DS2HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum ds2_status_t {
  DS2_OK = 0,
  DS2_INVALID_VALUE = 1,
  DS2_UNSUPPORTED_SHAPE = 2,
  DS2_HIP_ERROR = 3,
  DS2_RCCL_ERROR = 4,
  DS2_WORKSPACE_TOO_SMALL = 5
} ds2_status_t;

typedef void* ds2_stream_t; /* hipStream_t */

const char* ds2_status_string(ds2_status_t status);
const char* ds2_last_error(void);  /* text of the last HIP error seen (thread-local) */
const char* ds2_version(void);

/* ------------------------------------------------------------------------ */
/* Features: SpectrogramParser.audio_to_stft + normalize_audio('max_frame') */
/* ref data/data_loader.py:201-220,276-284; data/data_loader_aug.py:220-249,297-307 */
/* pcm:  [batch][max_samples] float32, utterance b has n_samples[b] valid samples   */
/* out:  [batch][161][max_frames], frames t >= 1 + n_samples[b]/hop are zero: the     */
/*       reference always returns 161 rows (data_loader_aug.py:234-249): the first   */
/*       161 bins when n_fft/2+1 >= 161, else its mirror-fill of ndarray.resize on    */
/*       librosa's (Fortran-ordered) stft matrix -- see stft.hip remap_kernel.         */
/* window: n_fft doubles (symmetric Hamming in the reference).                     */
/* normalize (normalize_audio, data_loader_aug.py:274-313): 0 = 'none' log1p(|X|),        */
/*   1 = 'max_frame' log1p(|X|*2^20) - mean_t(gauss20(mean_f)), 2 = 'mean' log1p(|X|) - mean, */
/*   3 = 'norm' (log1p(|X|) - mean) / mean_t(std_f), 4 = 'frame' log1p(|X|) -               */
/*   mean_t(gauss50(mean_f)); gauss_taps (2 radius + 1 scipy correlation weights) for 1, 4.  */
size_t ds2_stft_workspace_size(int batch, int max_frames, int n_fft);
ds2_status_t ds2_stft_logmag(const float* pcm, const int* n_samples, int batch, int max_samples,
                             int n_fft, int hop, const double* window, int normalize,
                             const float* gauss_taps, int gauss_radius,
                             float* out, int max_frames, void* ws, size_t ws_bytes,
                             ds2_stream_t stream);
/* The same with the spectrogram augmentations of data/data_loader_aug.py:236-248
 * (FrequencyMask / TimeMask via SOneOf, data/spectrogram_aug.py:64-117, and the
 * aug_prob_8khz cut) applied to |X| before the log, as the reference does.  masks: NULL
 * or [batch][9] int32 = {f_lo0, f_hi0, f_lo1, f_hi1, t_lo0, t_hi0, t_lo1, t_hi1, f_cut}:
 * bins in [f_lo, f_hi), frames in [t_lo, t_hi) and bins >= f_cut are zeroed (empty when
 * lo >= hi; f_cut = 161 for none), rows of the 161-row output.  The random draws stay on the host
 * (ds2amd/spect_aug.py) so they follow the reference's `random` call sequence. */
ds2_status_t ds2_stft_logmag_masked(const float* pcm, const int* n_samples, int batch,
                                    int max_samples, int n_fft, int hop, const double* window,
                                    int normalize, const float* gauss_taps, int gauss_radius,
                                    const int* masks, float* out, int max_frames, void* ws,
                                    size_t ws_bytes, ds2_stream_t stream);

/* Waveform augmentations before the STFT: replays per-utterance op records drawn on the
 * host by ds2amd/audio_aug.py in the reference's `random` / `np.random` order —
 * Shift (data/audio_aug.py:26-44), AudioDistort (:47-60,177-178), AddNoise (:78-107).
 * in: [n][in_stride] fp32 PCM with in_lens; op_i [n][max_ops][4] = {kind, a, b, 0}
 * (kind 0 end, 1 shift (a = shift, b = limit), 2 distort, 3 noise (a = noise row)),
 * op_f [n][max_ops] = alpha; noise [rows][noise_stride] float64 slices; out:
 * [n][out_stride] zero padded, out_lens = the lengths the host expects (mismatch, a bad
 * record or cap too small sets *err).  cap = the longest intermediate length.  Replaces
 * the numpy arithmetic of load_randomly_augmented_audio (data_loader_aug.py:660-699). */
size_t ds2_wave_aug_workspace_size(int n, int64_t cap);
ds2_status_t ds2_wave_aug(const float* in, int64_t in_stride, const int* in_lens, int n,
                          const int* op_i, const double* op_f, int max_ops, const double* noise,
                          int64_t noise_stride, float* out, int64_t out_stride,
                          const int* out_lens, int64_t cap, int* err, void* ws, size_t ws_bytes,
                          ds2_stream_t stream);

/* librosa.effects.time_stretch(y, rate[b]) per utterance (ChangeAudioSpeed, data/audio_aug.py:7-23;
 * the stretch half of PitchShift, :63-75): STFT (n_fft 2048, hop 512, periodic Hann `window`
 * [2048] doubles, reflect pad) -> phase vocoder -> ISTFT, librosa 0.8 semantics (csrc/effects.hip,
 * oracle/librosa_effects.py).  x: [n][x_stride] fp32 with in_lens; per utterance, host-computed:
 * out_frames = ceil((1 + in_len / 512) / rate) (np.arange), used_frames = min(out_frames,
 * ceil((out_len + 2048) / 512)) (istft's `length`), out_lens = round(in_len / rate).  out:
 * [n][out_stride], zero past out_lens.  max_*_frames bound the per-utterance counts. */
size_t ds2_time_stretch_workspace_size(int n, int max_in_frames, int max_out_frames);
ds2_status_t ds2_time_stretch(const float* x, int64_t x_stride, const int* in_lens, int n,
                              const double* rate, const int* out_frames, const int* used_frames,
                              const int* out_lens, const double* window, float* out,
                              int64_t out_stride, int max_in_frames, int max_out_frames, void* ws,
                              size_t ws_bytes, ds2_stream_t stream);
/* resampy.resample(x, sr_orig, sr_new, filter='kaiser_best') per utterance (librosa.resample,
 * data_loader_aug.py:668; the resample half of PitchShift): ratio[b] = sr_new / sr_orig,
 * n_valid[b] = int(in_len * ratio) output samples, zero up to out_stride (librosa's fix_length).
 * win: the filter's right wing (nwin doubles, num_table samples per zero crossing). */
size_t ds2_resample_workspace_size(int n, int64_t max_out);
ds2_status_t ds2_resample(const float* x, int64_t x_stride, const int* in_lens, int n,
                          const double* ratio, const int* n_valid, const double* win, int nwin,
                          int num_table, float* out, int64_t out_stride, void* ws,
                          size_t ws_bytes, ds2_stream_t stream);

/* ------------------------------------------------------------------------ */
/* Dense fp32 GEMM on MFMA (v_mfma_f32_16x16x4_f32 / 32x32x2_f32), strided-batched, row-major.
 * C[b] = alpha * op(A[b]) @ op(B[b]) + beta * C[b] (+ bias[n] if bias != NULL)
 * trans_a = 0: A is [m][lda];  1: A is stored [k][lda] (A^T)
 * trans_b = 0: B is [k][ldb];  1: B is stored [n][ldb] (B^T)
 * Replaces cuBLAS behind cuDNN's RNN input projection / BPTT weight gradients
 * (ref model.py:90-91,104 nn.GRU) and nn.Linear (ref model.py:337).          */
ds2_status_t ds2_sgemm(int trans_a, int trans_b, int m, int n, int k, float alpha,
                       const float* a, int64_t lda, int64_t stride_a,
                       const float* b, int64_t ldb, int64_t stride_b, float beta,
                       float* c, int64_t ldc, int64_t stride_c, int batch,
                       const float* bias, ds2_stream_t stream);
/* Same with a workspace: when the output grid cannot fill the chip and K is long
 * (weight gradients: M = 3H, N = In, K = T*N), K is split across workgroups and
 * the fp32 partials are reduced in a fixed order (deterministic).           */
size_t ds2_sgemm_workspace_size(int m, int n, int k, int batch);
ds2_status_t ds2_sgemm_ws(int trans_a, int trans_b, int m, int n, int k, float alpha,
                          const float* a, int64_t lda, int64_t stride_a,
                          const float* b, int64_t ldb, int64_t stride_b, float beta,
                          float* c, int64_t ldc, int64_t stride_c, int batch,
                          const float* bias, void* ws, size_t ws_bytes, ds2_stream_t stream);
/* fp16x3 operand scales: row_amax[r] / col_amax[c] = the float bits of max |x| over row r /
 * column c of x [rows][ld] (either output NULL: not computed; non-negative float bits order
 * as unsigned).  16-B aligned x, cols and ld multiples of 4, else DS2_UNSUPPORTED_SHAPE.  One
 * pass over x.  A NaN is skipped (max of the other elements), an inf gives inf.            */
ds2_status_t ds2_amax(const float* x, int rows, int cols, int64_t ld, unsigned* row_amax,
                      unsigned* col_amax, ds2_stream_t stream);
/* ds2_sgemm_ws (batch 1) with the fp16x3 scales of the logical operand rows supplied by the
 * caller: a_amax[m] = max over k of |op(A)[m][k]|, b_amax[n] = max over k of |op(B)[k][n]|
 * (ds2_amax bits; an upper bound is valid and costs only precision below 2^-17 of it); NULL
 * = computed here.  Ignored unless the fp16x3 kernel runs.                               */
ds2_status_t ds2_sgemm_amax_ws(int trans_a, int trans_b, int m, int n, int k, float alpha,
                               const float* a, int64_t lda, const float* b, int64_t ldb,
                               float beta, float* c, int64_t ldc, const float* bias,
                               const unsigned* a_amax, const unsigned* b_amax, void* ws,
                               size_t ws_bytes, ds2_stream_t stream);
/* bf16-operand variant (BASELINE cfg4 "bf16 MFMA RNN GEMMs", opt-in): same contract, A and
 * B rounded to bf16 (nearest even) as they are staged, v_mfma_f32_16x16x32_bf16, fp32
 * accumulation and fp32 C.  Needs float4-aligned operands (16-B aligned pointers, ld and
 * the contiguous extent multiples of 4): DS2_UNSUPPORTED_SHAPE otherwise. */
size_t ds2_sgemm_bf16_workspace_size(int m, int n, int k, int batch);
ds2_status_t ds2_sgemm_bf16_ws(int trans_a, int trans_b, int m, int n, int k, float alpha,
                               const float* a, int64_t lda, int64_t stride_a,
                               const float* b, int64_t ldb, int64_t stride_b, float beta,
                               float* c, int64_t ldc, int64_t stride_c, int batch,
                               const float* bias, void* ws, size_t ws_bytes,
                               ds2_stream_t stream);

/* ------------------------------------------------------------------------ */
/* Conv2d, NCHW fp32, on MFMA. ref model.py:209,212 (nn.Conv2d via cuDNN), masked
 * by MaskConv model.py:63-79 when out_lens != NULL: output columns w >= out_lens[n]
 * are written as 0.  Width-stride-1 convolutions (conv2) run as direct
 * convolutions from LDS input patches and need the workspace (re-laid-out
 * filter taps); others (conv1) run as an implicit GEMM and ignore it.        */
size_t ds2_conv2d_workspace_size(int n, int c_in, int h_in, int w_in, int c_out, int kh, int kw,
                                 int sh, int sw, int ph, int pw);
ds2_status_t ds2_conv2d_fwd(const float* x, const float* w, const float* bias, float* y,
                            int n, int c_in, int h_in, int w_in, int c_out, int kh, int kw,
                            int sh, int sw, int ph, int pw, const int* out_lens, void* ws,
                            size_t ws_bytes, ds2_stream_t stream);
ds2_status_t ds2_conv2d_dgrad(const float* dy, const float* w, float* dx,
                              int n, int c_in, int h_in, int w_in, int c_out, int kh, int kw,
                              int sh, int sw, int ph, int pw, void* ws, size_t ws_bytes,
                              ds2_stream_t stream);
size_t ds2_conv2d_wgrad_workspace_size(int n, int c_in, int h_in, int w_in, int c_out, int kh,
                                       int kw, int sh, int sw, int ph, int pw);
/* dw = sum over (n, ho, wo) of dy * im2col(x); dbias = sum of dy (if dbias != NULL). */
ds2_status_t ds2_conv2d_wgrad(const float* dy, const float* x, float* dw, float* dbias,
                              int n, int c_in, int h_in, int w_in, int c_out, int kh, int kw,
                              int sh, int sw, int ph, int pw, void* ws, size_t ws_bytes,
                              ds2_stream_t stream);

/* ------------------------------------------------------------------------ */
/* BatchNorm (training statistics), x viewed as [outer][c][inner].
 * ref model.py:210,213 (BatchNorm2d), model.py:89,336 (SequenceWise BatchNorm1d).
 * Batch statistics include padded (zeroed) positions, as in the reference.
 * Computes save_mean / save_invstd and updates the running stats in place
 * (running_var uses the unbiased variance, momentum as in torch).            */
size_t ds2_bn_workspace_size(int outer, int c, int inner);
ds2_status_t ds2_bn_train_stats(const float* x, int outer, int c, int inner, float eps,
                                float momentum, float* save_mean, float* save_invstd,
                                float* running_mean, float* running_var, void* ws,
                                size_t ws_bytes, ds2_stream_t stream);
ds2_status_t ds2_bn_eval_stats(const float* running_mean, const float* running_var, int c,
                               float eps, float* save_mean, float* save_invstd,
                               ds2_stream_t stream);
/* y = gamma * (x - mean) * invstd + beta over [outer][c][inner]. */
ds2_status_t ds2_bn_apply(const float* x, int outer, int c, int inner, const float* mean,
                          const float* invstd, const float* gamma, const float* beta, float* y,
                          ds2_stream_t stream);
/* ds2_bn_apply over [rows][c] (inner 1) that also writes the fp16x3 GEMM scales of y: the
 * float bits of max |y| per row (row_amax[rows]) and per column (col_amax[c]), the next
 * input projection's A-row and dW_ih's B-column maxima (ds2_sgemm_amax_ws).  Needs c % 4 == 0,
 * c <= 2048 and 16-B aligned x / y / mean / invstd / gamma / beta (DS2_UNSUPPORTED_SHAPE
 * otherwise).  Replaces the same SequenceWise BatchNorm1d as ds2_bn_apply (model.py:89). */
ds2_status_t ds2_bn_apply_amax(const float* x, int rows, int c, const float* mean,
                               const float* invstd, const float* gamma, const float* beta,
                               float* y, unsigned* row_amax, unsigned* col_amax,
                               ds2_stream_t stream);
/* Conv-block epilogue (MaskConv, model.py:69-78): x is [n][c][d][t];
 * y = mask(hardtanh(mask(bn(x)), lo, hi)) where mask zeroes t >= lens[n].
 * out_layout 0: y is [n][c][d][t];  1: y is [t][n][c*d] (the TxNxH collapse of
 * model.py:360-362, fused).                                                   */
ds2_status_t ds2_bn_apply_mask_htanh(const float* x, int n, int c, int d, int t,
                                     const float* mean, const float* invstd, const float* gamma,
                                     const float* beta, const int* lens, float lo, float hi,
                                     float* y, int out_layout, ds2_stream_t stream);
/* Backward of bn_apply (masked == 0, x viewed [outer][c][d*t]) or of
 * bn_apply_mask_htanh (masked != 0, x is [outer=n][c][d][t], lens/lo/hi as in
 * the forward).  dy has the layout of the forward output (dy_layout as
 * out_layout above; layout 1 only with masked != 0).  Writes dx
 * ([outer][c][d][t]), dgamma, dbeta (overwritten) and, if dbias_in != NULL, the
 * gradient of the per-channel bias added before the masked BN (the conv bias;
 * exact closed form, see bn.hip).  dx may not alias dy.                      */
ds2_status_t ds2_bn_backward(const float* dy, int dy_layout, const float* x, int outer, int c,
                             int d, int t, const float* mean, const float* invstd,
                             const float* gamma, const float* beta, int masked,
                             const int* lens, float lo, float hi, float* dx, float* dgamma,
                             float* dbeta, float* dbias_in, void* ws, size_t ws_bytes,
                             ds2_stream_t stream);

/* ------------------------------------------------------------------------ */
/* Bidirectional GRU recurrence (torch gate order r, z, n), packed-sequence
 * semantics: direction 0 runs t = 0..len-1, direction 1 runs t = len-1..0,
 * both from h = 0; outputs at t >= len are 0.  ref model.py:97-109 (BatchRNN
 * pack -> nn.GRU -> pad), model.py:16 (supported_rnns['gru']).
 *   xproj : [T][N][D][3H]  x @ W_ih^T + b_ih for each direction
 *   h_all : [T][N][D][H]   per-direction hidden states (output)
 *   gates : the backward cache, or NULL: ds2_gru_cache_floats(T, N, H, D) floats =
 *           [T][N][D][4H] (r, z, n, W_hn h + b_hn)
 * num_dirs = 1 or 2; w_hh_r / b_hh_r ignored when num_dirs == 1.
 * err_out: NULL, or a caller-owned device status word; the persistent
 * (one-launch-per-layer) kernels OR their hand-off status into it after the
 * launch (DS2_RNN_ERR_HANDOFF_TIMEOUT: a workgroup waited past the spin bound,
 * its outputs from that step on are NaN).  The word is never cleared by the
 * library, so one word can collect a whole training step; the caller reads
 * it whenever it synchronises anyway (same convention for ds2_gru_bwd and
 * ds2_lstm_fwd / ds2_lstm_bwd).                                               */
#define DS2_RNN_ERR_HANDOFF_TIMEOUT 1u
size_t ds2_gru_cache_floats(int t_max, int n, int h, int num_dirs);
size_t ds2_gru_fwd_workspace_size(int n, int h, int num_dirs);
ds2_status_t ds2_gru_fwd(int t_max, int n, int h, int num_dirs, const float* xproj,
                         const float* w_hh_f, const float* w_hh_r, const float* b_hh_f,
                         const float* b_hh_r, const int* lens, float* h_all, float* gates,
                         unsigned* err_out, void* ws, size_t ws_bytes, ds2_stream_t stream);
size_t ds2_gru_bwd_workspace_size(int n, int h, int num_dirs);
/* dy: [T][N][dy_dirs][H]; dy_dirs = 1: gradient of the direction-summed output
 * (model.py:107), dy_dirs = num_dirs: per-direction output gradient.
 * dgates_x: [T][N][D][3H] grad wrt xproj;  dgates_h: [T][N][D][3H] grad wrt
 * W_hh h + b_hh.  Weight gradients are then plain GEMMs (see ds2amd/ops.py). */
ds2_status_t ds2_gru_bwd(int t_max, int n, int h, int num_dirs, const float* dy, int dy_dirs,
                         const float* w_hh_f, const float* w_hh_r, const float* h_all,
                         const float* gates, const int* lens, float* dgates_x, float* dgates_h,
                         unsigned* err_out, void* ws, size_t ws_bytes, ds2_stream_t stream);
/* Workgroups the persistent backward recurrence holds at once for this shape (one per
 * CU, all resident together: they spin on each other's hand-offs; an upper bound when the
 * launch may fall back to another persistent kernel), 0 when the shape runs the per-step
 * kernels.  What a concurrent collective must leave free (DESIGN.md §6;
 * optim.GradAllReducer.guard_cooperative).                                     */
int ds2_gru_bwd_grid(int n, int h, int num_dirs);
int ds2_lstm_bwd_grid(int n, int h, int num_dirs);
/* ds2_gru_bwd plus the bias gradients of the layer (replaces the column sums of the
 * reference's autograd over bias_ih_l* / bias_hh_l*, nn.GRU via model.py:97-109):
 * db_ih_{f,r} [3H] = sum over rows of dgates_x, db_hh_{f,r} [3H] = sum over rows of
 * dgates_h.  The direct-operand backward sums them while it runs (fp64, fixed order);
 * other recurrence paths sum dgates_x / dgates_h afterwards.  db_ih_f == NULL: same as
 * ds2_gru_bwd; with num_dirs == 1 the _r pointers may be NULL.                 */
ds2_status_t ds2_gru_bwd_bias(int t_max, int n, int h, int num_dirs, const float* dy, int dy_dirs,
                              const float* w_hh_f, const float* w_hh_r, const float* h_all,
                              const float* gates, const int* lens, float* dgates_x,
                              float* dgates_h, float* db_ih_f, float* db_hh_f, float* db_ih_r,
                              float* db_hh_r, unsigned* err_out, void* ws, size_t ws_bytes,
                              ds2_stream_t stream);
/* ds2_gru_bwd_bias plus the column maxima of the gate gradients for the fp16x3 GEMMs that
 * follow (ds2_sgemm_amax_ws: dW_ih, dW_hh): col_amax[0, D 3H) = max over rows of |dgates_x|,
 * [D 3H, 2 D 3H) = the same of dgates_h, as float bits (ds2_amax's format).  The fp16x3
 * recurrence keeps them as it goes; any other kernel is followed by a column pass. */
ds2_status_t ds2_gru_bwd_bias_amax(int t_max, int n, int h, int num_dirs, const float* dy,
                                   int dy_dirs, const float* w_hh_f, const float* w_hh_r,
                                   const float* h_all, const float* gates, const int* lens,
                                   float* dgates_x, float* dgates_h, float* db_ih_f,
                                   float* db_hh_f, float* db_ih_r, float* db_hh_r,
                                   unsigned* col_amax, unsigned* err_out, void* ws,
                                   size_t ws_bytes, ds2_stream_t stream);

/* ------------------------------------------------------------------------ */
/* (Bi)directional LSTM recurrence (torch gate order i, f, g, o), same packed-
 * sequence semantics as the GRU.  ref model.py:14 (supported_rnns['lstm'] =
 * nn.LSTM) inside BatchRNN model.py:97-109.
 *   xproj : [T][N][D][4H]  x @ W_ih^T + b_ih for each direction
 *   h_all : [T][N][D][H]   hidden states (output)
 *   c_all : [T][N][D][H]   cell states (backward cache, or NULL)
 *   gates : [T][N][D][4H]  activated (i, f, g, o) cache for backward, or NULL  */
size_t ds2_lstm_fwd_workspace_size(int n, int h, int num_dirs);
ds2_status_t ds2_lstm_fwd(int t_max, int n, int h, int num_dirs, const float* xproj,
                          const float* w_hh_f, const float* w_hh_r, const float* b_hh_f,
                          const float* b_hh_r, const int* lens, float* h_all, float* c_all,
                          float* gates, unsigned* err_out, void* ws, size_t ws_bytes,
                          ds2_stream_t stream);
size_t ds2_lstm_bwd_workspace_size(int n, int h, int num_dirs);
/* dy as for ds2_gru_bwd.  dgates: [T][N][D][4H] gradient wrt the gate
 * pre-activations (= wrt xproj and wrt W_hh h + b_hh).                       */
ds2_status_t ds2_lstm_bwd(int t_max, int n, int h, int num_dirs, const float* dy, int dy_dirs,
                          const float* w_hh_f, const float* w_hh_r, const float* c_all,
                          const float* gates, const int* lens, float* dgates, unsigned* err_out,
                          void* ws, size_t ws_bytes, ds2_stream_t stream);
/* ds2_lstm_bwd for BASELINE cfg4's opt-in bf16 mode (rnn_gemm_precision='bf16'): the W_hh^T
 * product of the backward recurrence on ONE fp16 term per operand (per-row scaled gate
 * gradients, per-column scaled W_hh^T: 11 significant bits each), so a workgroup takes 32
 * samples and cfg4's batch 64 runs as one launch.  Same arguments and workspace as
 * ds2_lstm_bwd, which it falls back to where it declines the shape.
 * ds2_lstm_bwd_half_grid: workgroups that launch holds at once.                          */
int ds2_lstm_bwd_half_grid(int n, int h, int num_dirs);
ds2_status_t ds2_lstm_bwd_half(int t_max, int n, int h, int num_dirs, const float* dy, int dy_dirs,
                               const float* w_hh_f, const float* w_hh_r, const float* c_all,
                               const float* gates, const int* lens, float* dgates,
                               unsigned* err_out, void* ws, size_t ws_bytes, ds2_stream_t stream);

/* ------------------------------------------------------------------------ */
/* Lookahead convolution, ref model.py:140-177 (Lookahead.forward), optionally
 * fused with the Hardtanh that follows it (model.py:329-333):
 *   y[t][n][h] = sum_{j=0..context} w[h][j] * x[t+j][n][h]  (0 past T)
 *   clamp != 0: y = min(max(y, lo), hi).   x, y: [T][N][H]; w: [H][context+1];
 *   context + 1 <= 32.                                                       */
ds2_status_t ds2_lookahead_fwd(const float* x, int t, int n, int h, const float* w, int context,
                               int clamp, float lo, float hi, float* y, ds2_stream_t stream);
/* Backward: y = the clamped forward output (or NULL when not clamped: dz = dy,
 * else dz = dy where lo < y < hi).  dx (or NULL) overwritten; dw (or NULL)
 * overwritten, deterministic.                                                 */
size_t ds2_lookahead_bwd_workspace_size(int t, int n, int h, int context);
ds2_status_t ds2_lookahead_bwd(const float* dy, const float* y, float lo, float hi,
                               const float* x, int t, int n, int h, const float* w, int context,
                               float* dx, float* dw, void* ws, size_t ws_bytes,
                               ds2_stream_t stream);

/* y[t][n][j] = sum_d h_all[t][n][d][j]   (model.py:107 view(T,N,2,H).sum(2)) */
ds2_status_t ds2_dirsum(const float* h_all, int rows, int num_dirs, int h, float* y,
                        ds2_stream_t stream);
/* out[j] (+)= sum_i x[i*ld + j]  for i < rows, j < cols (bias gradients). */
size_t ds2_colsum_workspace_size(int rows, int cols);
ds2_status_t ds2_colsum(const float* x, int rows, int cols, int64_t ld, float* out,
                        int accumulate, void* ws, size_t ws_bytes, ds2_stream_t stream);

/* ------------------------------------------------------------------------ */
/* Softmax over C of logits stored [T][N][C] -> probs [N][T][C] (model.py:375-377). */
ds2_status_t ds2_softmax_tnc(const float* logits, int t_max, int n, int c, float* probs,
                             ds2_stream_t stream);
/* Backward of ds2_softmax_tnc: dlogits[T][N][C] (+)= y * (dy - sum(y*dy)). */
ds2_status_t ds2_softmax_tnc_bwd(const float* probs, const float* dprobs, int t_max, int n,
                                 int c, float* dlogits, int accumulate, ds2_stream_t stream);

/* ------------------------------------------------------------------------ */
/* CTC loss, warp-ctc semantics (ref train.py:12,600-602 warpctc_pytorch.CTCLoss):
 * softmax is applied internally to acts [T][N][C]; costs[b] = -log p(l_b | x_b);
 * grads [T][N][C] = d cost_b / d acts (softmax - posterior), zero for t >= len.
 * labels: concatenated int32 targets; label_lens[b] their lengths.
 * Infeasible samples (L + repeats > act_len) get cost +inf and zero gradient,
 * or cost 0 when zero_infinity != 0.                                          */
size_t ds2_ctc_workspace_size(int t_max, int n, int max_label_len);
ds2_status_t ds2_ctc_loss(const float* acts, int t_max, int n, int c, const int* labels,
                          const int* label_lens, const int* act_lens, int max_label_len,
                          int blank, int zero_infinity, float* costs, float* grads, void* ws,
                          size_t ws_bytes, ds2_stream_t stream);

/* ------------------------------------------------------------------------ */
/* GreedyDecoder.decode (ref decoder.py:182-197, process_string :165-180):
 * argmax over C (first maximum) of probs[n][t][c] (strides in elements), then
 * drop blanks and frames equal to the previous frame.  Emits compacted label
 * ids and their frame offsets per utterance plus counts[n].                   */
ds2_status_t ds2_greedy_decode(const float* probs, int n, int t_max, int c, int64_t stride_n,
                               int64_t stride_t, const int* sizes, int blank, int* out_ids,
                               int* out_offsets, int* out_counts, int* argmax_out,
                               ds2_stream_t stream);

/* CTC prefix beam search without a language model: BeamCTCDecoder.decode
 * (decoder.py:90-143, ctcdecode.CTCBeamDecoder with lm_path=None; opts.py beam
 * defaults).  probs as for ds2_greedy_decode; per utterance the top_paths best
 * prefixes (best first): out_ids / out_offsets [n][top_paths][t_max] (char ids and
 * the frame of each char), out_lens [n][top_paths], out_scores [n][top_paths]
 * (log prob).  cutoff_top_n / cutoff_prob prune the vocabulary per frame as
 * ctcdecode does.  beam_width <= 32 with c <= 64, or beam_width <= 128 with
 * c <= 32 (the reference default beam_width = 100 over its 29 labels).        */
/* Batched CER / WER edit distances (data/utils.py:47-57 get_cer_wer, decoder.py
 * Decoder.cer / .wer) over id sequences: a = decoded ids [n][a_stride] with a_lens,
 * b = reference ids flat with b_offsets / b_lens.  out[4*i .. 4*i+3] = {word
 * distance, char distance (spaces removed), max(#reference words, 1),
 * max(#reference non-space chars, 1)}.  Sequences longer than 2048 ids / 1024 words
 * set *err != 0 and distance -1 (err must be zeroed by the caller).           */
ds2_status_t ds2_edit_distance(const int* a_ids, int64_t a_stride, const int* a_lens,
                               const int* b_ids, const int* b_offsets, const int* b_lens, int n,
                               int space_id, int* out, int* err, ds2_stream_t stream);

size_t ds2_ctc_beam_workspace_size(int n, int t_max, int beam_width);
ds2_status_t ds2_ctc_beam_decode(const float* probs, int n, int t_max, int c, int64_t stride_n,
                                 int64_t stride_t, const int* sizes, int blank, int beam_width,
                                 int cutoff_top_n, double cutoff_prob, int top_paths,
                                 int* out_ids, int* out_offsets, int* out_lens,
                                 float* out_scores, void* ws, size_t ws_bytes,
                                 ds2_stream_t stream);

/* The same search with a word n-gram language model: BeamCTCDecoder(labels, lm_path,
 * alpha, beta, ...) (decoder.py:90-99 -> ctcdecode's KenLM Scorer; opts.py:6-10
 * --lm-path / --alpha / --beta).  A space extension adds float(alpha * ln p(word |
 * preceding order-1 words, "<s>" padded)) and beta; extensions follow the vocabulary
 * trie; once the beam is full a (prefix, char) below worst + log p_blank - max(0, beta)
 * is skipped; the last partial word is scored after the final frame
 * (oracle/ctc_beam_lm.py restates it).  Tables (device memory, ds2amd/lm.py builds them
 * from an ARPA file): dict_next int32 [dict_states][c] trie arcs (-1 none; state 0 =
 * start, dict_states-1 = after a word's space), dict_mask uint64 [dict_states] the arcs
 * as char bits, dict_word int32 [dict_states] the word id a state spells (-1 none);
 * lm_table int32 [lm_slots][8] {w0..w5 (-1 padded), log10 prob bits, log10 backoff
 * bits}, w0 = -1 marks an empty slot, FNV-1a over w0..w5 + avalanche, linear probing,
 * lm_slots a power of two.  lm_order <= 6; start_id = the id of "<s>" (< lm_vocab, the
 * LM's word count); dict_cols = the label count dict_next was built for (must equal c);
 * an arc past dict_states is treated as leading to the post-space state; c <= 64.
 * Same outputs and workspace as ds2_ctc_beam_decode (scores include the LM terms). */
ds2_status_t ds2_ctc_beam_decode_lm(const float* probs, int n, int t_max, int c, int64_t stride_n,
                                    int64_t stride_t, const int* sizes, int blank, int beam_width,
                                    int cutoff_top_n, double cutoff_prob, int top_paths,
                                    int space_id, int lm_order, int start_id, int lm_vocab,
                                    double alpha, double beta, const int* dict_next,
                                    const void* dict_mask, const int* dict_word, int dict_states,
                                    int dict_cols, const int* lm_table, int64_t lm_slots,
                                    int* out_ids, int* out_offsets, int* out_lens,
                                    float* out_scores, void* ws, size_t ws_bytes,
                                    ds2_stream_t stream);

/* bf16 GEMM on bf16 operands (BASELINE cfg4's bf16 MFMA RNN GEMMs; csrc/bgemm.hip):
 * C[m x n] (fp32, ldc) = alpha * A . B^T + beta * C + bias, A [m][lda] and B [n][ldb] bf16
 * (raw 16-bit words, k-contiguous), fp32 accumulation.  A and B 16-B aligned, k, lda, ldb
 * multiples of 8, each operand < 2 GiB, else DS2_UNSUPPORTED_SHAPE.  Workspace for the
 * split-K tail: ds2_bgemm_workspace_size (NULL / too small: no split).
 * ds2_cvt_bf16: fp32 [rows][ld_src] -> bf16 (round to nearest even) as [rows][ld_dst], or
 * with transpose != 0 as [cols][ld_dst] (the k-contiguous copy of an m- or n-contiguous
 * operand).                                                                    */
size_t ds2_bgemm_workspace_size(int m, int n, int k);
ds2_status_t ds2_bgemm_nt(int m, int n, int k, float alpha, const void* a, int64_t lda,
                          const void* b, int64_t ldb, float beta, float* c, int64_t ldc,
                          const float* bias, void* ws, size_t ws_bytes, ds2_stream_t stream);
ds2_status_t ds2_cvt_bf16(const float* src, int rows, int cols, int64_t ld_src, void* dst,
                          int64_t ld_dst, int transpose, ds2_stream_t stream);

/* ------------------------------------------------------------------------ */
/* Vanilla tanh RNN recurrence (supported_rnns['rnn'] = nn.RNN, model.py:15; csrc/rnn.hip):
 * h_t = tanh(xproj_t + b_hh + W_hh h_{t-1}) over packed lengths, xproj / h_all / dy / dgates
 * laid out as for ds2_gru_fwd / ds2_gru_bwd with one gate ([T][N][D][H]); dgates = the
 * gradient wrt the pre-activation (= dgx = dgh of the GEMMs).  One launch per step.      */
ds2_status_t ds2_rnn_fwd(int t_max, int n, int h, int num_dirs, const float* xproj,
                         const float* w_hh_f, const float* w_hh_r, const float* b_hh_f,
                         const float* b_hh_r, const int* lens, float* h_all,
                         ds2_stream_t stream);
ds2_status_t ds2_rnn_bwd(int t_max, int n, int h, int num_dirs, const float* dy, int dy_dirs,
                         const float* w_hh_f, const float* w_hh_r, const float* h_all,
                         const int* lens, float* dgates, ds2_stream_t stream);
/* The same recurrences on the GRU's persistent machinery (one launch per layer and pass: the
 * one-gate fp16x3 instantiations of the GRU kernels, csrc/gru_split.hip), with the per-step
 * kernels above as the fallback for shapes they decline (H % 16 != 0, a grid past the CUs)
 * and DS2_RNN_PERSISTENT=0.  err_out as for ds2_gru_fwd.  col_amax (nullable): [D H] column
 * maxima of |dgates| as float bits (ds2_amax's format) for the fp16x3 weight-gradient GEMMs.
 * ds2_rnn_bwd_grid: workgroups the persistent backward holds at once (0: per-step kernels). */
size_t ds2_rnn_fwd_workspace_size(int n, int h, int num_dirs);
ds2_status_t ds2_rnn_fwd_ws(int t_max, int n, int h, int num_dirs, const float* xproj,
                            const float* w_hh_f, const float* w_hh_r, const float* b_hh_f,
                            const float* b_hh_r, const int* lens, float* h_all, unsigned* err_out,
                            void* ws, size_t ws_bytes, ds2_stream_t stream);
size_t ds2_rnn_bwd_workspace_size(int n, int h, int num_dirs);
int ds2_rnn_bwd_grid(int n, int h, int num_dirs);
ds2_status_t ds2_rnn_bwd_ws(int t_max, int n, int h, int num_dirs, const float* dy, int dy_dirs,
                            const float* w_hh_f, const float* w_hh_r, const float* h_all,
                            const int* lens, float* dgates, unsigned* col_amax, unsigned* err_out,
                            void* ws, size_t ws_bytes, ds2_stream_t stream);

/* ------------------------------------------------------------------------ */
/* Data-parallel gradient exchange over RCCL (SURVEY §8b allreduce_bucket /
 * ds2_comm_t; replaces DistributedDataParallel's bucketed all-reduce, train.py:947-951).
 * Rank 0 makes an id (ds2_comm_id_bytes() bytes), the caller carries it to every
 * rank (torch.distributed or a file), each rank creates its communicator on its GPU;
 * ds2_allreduce_bucket sums one contiguous fp32 bucket in place across the ranks,
 * enqueued on `stream` (no averaging: the caller scales once after the last bucket).
 * RCCL is loaded at run time (librccl.so.1); DS2_RCCL_ERROR with ds2_last_error()
 * when it is missing or a collective fails.                                      */
typedef struct ds2_comm* ds2_comm_t;
size_t ds2_comm_id_bytes(void);
ds2_status_t ds2_comm_get_unique_id(void* id_out);
ds2_status_t ds2_comm_init(ds2_comm_t* comm, const void* id, int nranks, int rank, int device);
ds2_status_t ds2_allreduce_bucket(ds2_comm_t comm, float* bucket, int64_t count,
                                  ds2_stream_t stream);
ds2_status_t ds2_comm_destroy(ds2_comm_t comm);

/* ------------------------------------------------------------------------ */
/* Training-step tail (ref train.py:595-632): clip_grad_norm_(max_norm) then
 * SGD(momentum, nesterov) on flat fp32 buffers.  The global L2 norm is reduced
 * on device (fp64), nothing returns to the host.  If skip_flag != NULL and
 * *skip_flag != 0 the step is skipped (NaN guard, train.py:625-630).          */
size_t ds2_optim_workspace_size(int64_t numel);
ds2_status_t ds2_grad_norm(const float* grads, int64_t numel, float* out_norm, void* ws,
                           size_t ws_bytes, ds2_stream_t stream);
ds2_status_t ds2_clip_sgd_nesterov(float* params, const float* grads, float* momentum_buf,
                                   int64_t numel, float lr, float momentum, float max_norm,
                                   const float* norm, const int* skip_flag,
                                   ds2_stream_t stream);
/* *flag = 1 if any x is NaN (flag must be zeroed by the caller first);
 * if zero_nans, NaNs are replaced by 0 in place (train.py:595-598); mask
 * (nullable, one byte per element) records where the NaNs were.              */
ds2_status_t ds2_nan_guard(float* x, int64_t numel, int zero_nans, int* flag,
                           unsigned char* mask, ds2_stream_t stream);
/* Gradient of that in-place zeroing (autograd's index_put, train.py:598):
 * x[i] = 0 where mask[i]; a no-op when flag is non-NULL and *flag == 0.      */
ds2_status_t ds2_zero_masked(float* x, const unsigned char* mask, int64_t numel, const int* flag,
                             ds2_stream_t stream);
/* x[i] *= *scalar (device scalar, e.g. autograd's grad_output). */
ds2_status_t ds2_scale_by_device_scalar(float* x, int64_t numel, const float* scalar,
                                        ds2_stream_t stream);

#ifdef __cplusplus
}
#endif

#endif /* DS2HIP_H */
