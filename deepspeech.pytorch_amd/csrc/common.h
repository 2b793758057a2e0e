// Shared helpers for the libds2hip kernels (gfx950 / CDNA4 only).
//
// Conventions (see include/ds2hip.h):
//   * every entry point is extern "C", returns ds2_status_t, enqueues work on
//     the caller's stream and never allocates, synchronises or throws;
//   * device buffers are caller-owned; scratch comes in through (ws, ws_bytes).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>

#include "../../include/ds2hip.h"

namespace ds2 {

// Wave width is fixed at 64 on CDNA; never use warpSize-derived 32 idioms.
constexpr int kWave = 64;

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

inline hipStream_t as_stream(ds2_stream_t s) { return reinterpret_cast<hipStream_t>(s); }

// Records the last HIP error string for ds2_last_error().
void set_last_error(const char* where, hipError_t e);
void set_last_error_text(const char* where, const char* what);

inline ds2_status_t launch_status(const char* where) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_last_error(where, e);
    return DS2_HIP_ERROR;
  }
  return DS2_OK;
}

inline int cdiv(int64_t a, int64_t b) { return static_cast<int>((a + b - 1) / b); }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, 64));
  return v;
}

// log(exp(a) + exp(b)) with -inf handling (CTC recursions).
__device__ __forceinline__ float log_add(float a, float b) {
  if (a == -INFINITY) return b;
  if (b == -INFINITY) return a;
  float m = fmaxf(a, b);
  return m + log1pf(expf(-fabsf(a - b)));
}

// log(exp(a) + exp(b)) on the hardware v_exp_f32 / v_log_f32 (about 1 ulp each): the CTC
// alpha/beta recursions are a dependent chain of these, and log1pf/expf cost ~10x the
// instructions.  log(1 + x) for x = exp(-|a - b|) <= 1 loses only terms below ulp(m).
__device__ __forceinline__ float log_add_fast(float a, float b) {
  if (a == -INFINITY) return b;
  if (b == -INFINITY) return a;
  const float m = fmaxf(a, b);
  return m + __logf(1.0f + __expf(-fabsf(a - b)));
}

__device__ __forceinline__ float sigmoidf_(float x) { return 1.0f / (1.0f + expf(-x)); }

// Gate nonlinearities on v_exp_f32 / v_rcp_f32 (absolute error ~1e-7) for the recurrences'
// per-step critical path; tanh(x) = 1 - 2 / (1 + e^{2x}) saturates correctly at +-inf.
__device__ __forceinline__ float sigmoid_fast(float x) {
  return __builtin_amdgcn_rcpf(1.0f + __expf(-x));
}
__device__ __forceinline__ float tanh_fast(float x) {
  return 1.0f - 2.0f * __builtin_amdgcn_rcpf(1.0f + __expf(2.0f * x));
}

// fp16x3 row scales.  amax: the bit pattern of max |x| over a logical row (non-negative floats
// order as unsigned).  The row is staged as x 2^e, e = 14 - floor(log2 amax), so its largest
// element lies in [2^14, 2^15) (fp16 max 65504) and its fp16 (hi, lo) split keeps 22 bits for
// every element within 2^17 of the row max; a zero, inf or NaN row max keeps e = 0.
__device__ __forceinline__ int h3_exp(unsigned amax) {
  const int E = (int)(amax >> 23);                 // biased exponent (sign bit is 0)
  if (amax == 0u || E >= 255) return 0;
  int e = 14 - ((E == 0 ? 1 : E) - 127);
  return e > 127 ? 127 : e;                        // 2^e stays a normal float
}
__device__ __forceinline__ float h3_scale(int e) { return __builtin_bit_cast(float, (e + 127) << 23); }

}  // namespace ds2
