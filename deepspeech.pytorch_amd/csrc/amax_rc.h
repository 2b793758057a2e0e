// Row AND column maxima of |v| over a [rows][c] fp32 matrix (c <= 2048), one wave per row:
// the fp16x3 GEMM scales (float bits, ds2_amax's format).  APPLY: v = the BatchNorm affine of
// x, written to y (ds2_bn_apply_amax: the same expression as bn.hip's apply_rows_kernel), else
// v = x (ds2_amax of a narrow matrix).  Lane l holds the float4 columns l + 64 j (j < CPL) --
// with APPLY their gamma / mean / invstd / beta -- in registers; two rows per pass; a block
// covers `rpb` rows with 4 waves, writes each row's maximum (a wave reduction, no atomics),
// folds the waves' column maxima through LDS and leaves them with one unsigned atomic max per
// column (cmax zeroed first).
#pragma once
#include "common.h"

namespace ds2 {

template <int CPL, bool APPLY>
__global__ __launch_bounds__(256) void rows_amax_kernel(
    const float* __restrict__ x, int R, int C, int64_t ld, const float* __restrict__ mean,
    const float* __restrict__ invstd, const float* __restrict__ gamma,
    const float* __restrict__ beta, float* __restrict__ y, int rpb, unsigned* __restrict__ rmax,
    unsigned* __restrict__ cmax) {
  __shared__ float cm[4][CPL * 256];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int C4 = C / 4;
  const int r0 = blockIdx.x * rpb, r1 = min(R, r0 + rpb);
  const float4 z = float4{0.f, 0.f, 0.f, 0.f};
  float4 ga[CPL], me[CPL], is[CPL], be[CPL], cx[CPL];
#pragma unroll
  for (int j = 0; j < CPL; ++j) {
    const int c4 = lane + 64 * j;
    const bool in = APPLY && c4 < C4;
    ga[j] = in ? reinterpret_cast<const float4*>(gamma)[c4] : z;
    me[j] = in ? reinterpret_cast<const float4*>(mean)[c4] : z;
    is[j] = in ? reinterpret_cast<const float4*>(invstd)[c4] : z;
    be[j] = in ? reinterpret_cast<const float4*>(beta)[c4] : z;
    cx[j] = z;
  }
  auto bn = [&](float4 v, int j) __attribute__((always_inline)) {
    if (APPLY) {
      v.x = ga[j].x * ((v.x - me[j].x) * is[j].x) + be[j].x;
      v.y = ga[j].y * ((v.y - me[j].y) * is[j].y) + be[j].y;
      v.z = ga[j].z * ((v.z - me[j].z) * is[j].z) + be[j].z;
      v.w = ga[j].w * ((v.w - me[j].w) * is[j].w) + be[j].w;
    }
    return v;
  };
  auto vmax = [](float4 v) __attribute__((always_inline)) {
    return fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w)));
  };
  auto cfold = [&](float4 v, int j) __attribute__((always_inline)) {
    cx[j].x = fmaxf(cx[j].x, fabsf(v.x));
    cx[j].y = fmaxf(cx[j].y, fabsf(v.y));
    cx[j].z = fmaxf(cx[j].z, fabsf(v.z));
    cx[j].w = fmaxf(cx[j].w, fabsf(v.w));
  };
  for (int r = r0 + w; r < r1; r += 8) {
    const bool two = r + 4 < r1;
    const float4* xa = reinterpret_cast<const float4*>(x + (int64_t)r * ld);
    const float4* xb = reinterpret_cast<const float4*>(x + (int64_t)(two ? r + 4 : r) * ld);
    float4 va[CPL], vb[CPL];
#pragma unroll
    for (int j = 0; j < CPL; ++j) {
      const int c4 = lane + 64 * j;
      if (c4 < C4) {
        va[j] = xa[c4];
        vb[j] = xb[c4];
      }
    }
    float ma = 0.f, mb = 0.f;
#pragma unroll
    for (int j = 0; j < CPL; ++j) {
      const int c4 = lane + 64 * j;
      if (c4 < C4) {
        const float4 a = bn(va[j], j);
        if (APPLY) reinterpret_cast<float4*>(y + (int64_t)r * C)[c4] = a;
        ma = fmaxf(ma, vmax(a));
        cfold(a, j);
        if (two) {
          const float4 b = bn(vb[j], j);
          if (APPLY) reinterpret_cast<float4*>(y + (int64_t)(r + 4) * C)[c4] = b;
          mb = fmaxf(mb, vmax(b));
          cfold(b, j);
        }
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      ma = fmaxf(ma, __shfl_xor(ma, o));
      mb = fmaxf(mb, __shfl_xor(mb, o));
    }
    if (lane == 0) {
      rmax[r] = __float_as_uint(ma);
      if (two) rmax[r + 4] = __float_as_uint(mb);
    }
  }
#pragma unroll
  for (int j = 0; j < CPL; ++j) {
    float* d = &cm[w][(lane + 64 * j) * 4];
    d[0] = cx[j].x;
    d[1] = cx[j].y;
    d[2] = cx[j].z;
    d[3] = cx[j].w;
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += 256) {
    const float m = fmaxf(fmaxf(cm[0][c], cm[1][c]), fmaxf(cm[2][c], cm[3][c]));
    if (m > 0.f) atomicMax(cmax + c, __float_as_uint(m));
  }
}

// rows_amax_kernel's launch for c <= 2048 (the columns-per-lane instantiation by width)
template <bool APPLY>
inline void launch_rows_amax(const float* x, int rows, int c, int64_t ld, const float* mean,
                             const float* invstd, const float* gamma, const float* beta, float* y,
                             unsigned* rmax, unsigned* cmax, hipStream_t st) {
  constexpr int rpb = 64;
  const dim3 grid((rows + rpb - 1) / rpb);
  const int c4 = c / 4;
#define DS2_RA(CPL_)                                                                          \
  hipLaunchKernelGGL((rows_amax_kernel<CPL_, APPLY>), grid, dim3(256), 0, st, x, rows, c, ld, \
                     mean, invstd, gamma, beta, y, rpb, rmax, cmax)
  if (c4 <= 64) DS2_RA(1);
  else if (c4 <= 128) DS2_RA(2);
  else if (c4 <= 256) DS2_RA(4);
  else DS2_RA(8);
#undef DS2_RA
}

}  // namespace ds2
