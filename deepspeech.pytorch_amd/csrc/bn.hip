// BatchNorm (training + eval), fused MaskConv epilogue (mask + Hardtanh + the
// NCDT -> T,N,(C*D) collapse) and their backward passes.  HBM-bound.
//
// Reductions accumulate in fp64 per workgroup and combine the partials in a
// fixed order (deterministic; no atomics).  The backward re-sums x beside g and g*x,
// so its coefficients use the batch mean exactly (the forward keeps only the
// fp32-rounded mean): sum(g*xhat) = invstd*(sum(g*x) - mean*sum(g)), and the
// apply dx = k1*g - k2 - k3*xhat runs in fp64 with xhat from that mean.  With the
// fp32 mean, every dx of a channel carried the same -k3*invstd*(mean32 - mean)
// shift, which the next layer's per-channel sums (the conv biases' BatchNorm
// gradients) add up 1.3 M times.  Two reduction shapes:
//   rows   : x is [R][C] (SequenceWise BatchNorm1d, model.py:28-43,89,336)
//            block = 64 columns x 4 row groups, grid = column blocks x row chunks
//   planes : x is [outer][C][D][T] (BatchNorm2d, model.py:210,213)
//            block = one (outer, channel) plane slice, threads stride along T
#include "common.h"
#include "amax_rc.h"

namespace ds2 {

constexpr int kRowChunks = 256;   // row chunks for the [R][C] reduction (>= 4 workgroups per CU)
constexpr int kPlaneSplit = 4;    // slices per (outer, channel) plane

enum RedMode { RED_STATS = 0, RED_BWD = 1 };
// doubles per (part, channel) partial: stats (sum x, sum x^2, -), backward
// (sum g, sum g*x, sum x)
constexpr int kParts = 3;
// doubles per channel of backward coefficients: k1, k2, k3, exact mean
constexpr int kCoef = 4;

struct BnBwdArgs {
  const float* mean;
  const float* invstd;
  const float* gamma;
  const float* beta;
  const int* lens;
  float lo, hi;
  int masked;
};

// g (the upstream gradient after the mask/hardtanh backward) at one element.
__device__ __forceinline__ float bwd_g(float dy, float x, int c, int t, int len,
                                       const BnBwdArgs& a, float* xhat_out) {
  const float xhat = (x - a.mean[c]) * a.invstd[c];
  *xhat_out = xhat;
  if (!a.masked) return dy;
  if (t >= len) return 0.f;
  const float y2 = a.gamma[c] * xhat + a.beta[c];
  // torch hardtanh_backward: pass where min_val < x < max_val (strict)
  return (y2 > a.lo && y2 < a.hi) ? dy : 0.f;
}

// ---- rows reduction ---------------------------------------------------------
template <int MODE>
__global__ __launch_bounds__(256) void reduce_rows_kernel(const float* __restrict__ x,
                                                          const float* __restrict__ dy, int R,
                                                          int C, BnBwdArgs a,
                                                          double* __restrict__ partial) {
  __shared__ double s0[4][64], s1[4][64], s2[4][64];
  const int lane = threadIdx.x & 63;
  const int grp = threadIdx.x >> 6;
  const int col = blockIdx.x * 64 + lane;
  const int chunk = blockIdx.y;
  const int per = (R + gridDim.y - 1) / gridDim.y;
  const int r0 = chunk * per;
  const int r1 = min(R, r0 + per);
  double acc0 = 0.0, acc1 = 0.0, acc2 = 0.0;
  if (col < C) {
    for (int r = r0 + grp; r < r1; r += 4) {
      const float v = x[(int64_t)r * C + col];
      if (MODE == RED_STATS) {
        acc0 += v;
        acc1 += (double)v * v;
      } else {
        float xhat;
        const float g = bwd_g(dy[(int64_t)r * C + col], v, col, 0, 1, a, &xhat);
        acc0 += g;
        acc1 += (double)g * v;
        acc2 += v;
      }
    }
  }
  s0[grp][lane] = acc0;
  s1[grp][lane] = acc1;
  s2[grp][lane] = acc2;
  __syncthreads();
  if (grp == 0 && col < C) {
    double* pp = partial + ((int64_t)chunk * C + col) * kParts;
    pp[0] = s0[0][lane] + s0[1][lane] + s0[2][lane] + s0[3][lane];
    pp[1] = s1[0][lane] + s1[1][lane] + s1[2][lane] + s1[3][lane];
    pp[2] = s2[0][lane] + s2[1][lane] + s2[2][lane] + s2[3][lane];
  }
}

// Vector variant (C % 4 == 0, 16-B aligned rows): each lane owns 4 adjacent columns
// (float4 loads, two rows in flight per row group), per-column BN parameters held in
// registers; same partial layout as reduce_rows_kernel.
template <int MODE>
__global__ __launch_bounds__(256) void reduce_rows4_kernel(const float* __restrict__ x,
                                                           const float* __restrict__ dy, int R,
                                                           int C, BnBwdArgs a,
                                                           double* __restrict__ partial) {
  __shared__ double sh[4][256];   // one sum at a time (8 KB: occupancy of this HBM-bound pass)
  const int lane = threadIdx.x & 63;
  const int grp = threadIdx.x >> 6;
  const int col = blockIdx.x * 256 + lane * 4;
  const int chunk = blockIdx.y;
  const int per = (R + gridDim.y - 1) / gridDim.y;
  const int r0 = chunk * per;
  const int r1 = min(R, r0 + per);
  double acc0[4] = {0.0, 0.0, 0.0, 0.0}, acc1[4] = {0.0, 0.0, 0.0, 0.0};
  double acc2[4] = {0.0, 0.0, 0.0, 0.0};
  if (col < C) {
    float mu[4] = {0.f, 0.f, 0.f, 0.f}, is[4] = {0.f, 0.f, 0.f, 0.f};
    float ga[4] = {0.f, 0.f, 0.f, 0.f}, be[4] = {0.f, 0.f, 0.f, 0.f};
    if (MODE == RED_BWD) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        mu[e] = a.mean[col + e];
        is[e] = a.invstd[col + e];
        if (a.masked) {
          ga[e] = a.gamma[col + e];
          be[e] = a.beta[col + e];
        }
      }
    }
    auto add = [&](int r) {
      const float4 v = *reinterpret_cast<const float4*>(x + (int64_t)r * C + col);
      const float vv[4] = {v.x, v.y, v.z, v.w};
      if (MODE == RED_STATS) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          acc0[e] += vv[e];
          acc1[e] += (double)vv[e] * vv[e];
        }
      } else {
        const float4 d = *reinterpret_cast<const float4*>(dy + (int64_t)r * C + col);
        const float dd[4] = {d.x, d.y, d.z, d.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float xhat = (vv[e] - mu[e]) * is[e];
          float g = dd[e];
          if (a.masked) {
            const float y2 = ga[e] * xhat + be[e];
            g = (y2 > a.lo && y2 < a.hi) ? g : 0.f;
          }
          acc0[e] += g;
          acc1[e] += (double)g * vv[e];
          acc2[e] += vv[e];
        }
      }
    };
    int r = r0 + grp;
    for (; r + 4 < r1; r += 8) {
      add(r);
      add(r + 4);
    }
    if (r < r1) add(r);
  }
  const int c = blockIdx.x * 256 + threadIdx.x;
  const int t = threadIdx.x;
  double* pp = partial + ((int64_t)chunk * C + c) * kParts;
#pragma unroll
  for (int k = 0; k < (MODE == RED_BWD ? 3 : 2); ++k) {
    const double* a = k == 0 ? acc0 : (k == 1 ? acc1 : acc2);
#pragma unroll
    for (int e = 0; e < 4; ++e) sh[grp][lane * 4 + e] = a[e];
    __syncthreads();
    if (c < C) pp[k] = sh[0][t] + sh[1][t] + sh[2][t] + sh[3][t];
    __syncthreads();
  }
}

static inline bool rows_vec(const float* x, const float* dy, int c) {
  return (c % 4) == 0 &&
         ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(dy)) & 15) == 0;
}

// ---- planes reduction -------------------------------------------------------
// grid (C, outer, kPlaneSplit); the plane [D][T] is split by D-rows.
template <int MODE>
__global__ __launch_bounds__(256) void reduce_planes_kernel(const float* __restrict__ x,
                                                            const float* __restrict__ dy, int C,
                                                            int D, int T, BnBwdArgs a,
                                                            double* __restrict__ partial) {
  const int c = blockIdx.x;
  const int o = blockIdx.y;
  const int sl = blockIdx.z;
  // slices of the plane: D rows split over gridDim.z, or (D == 1: the statistics pass over a
  // whole [H x W] plane) the row itself -- split by rows alone, one slice held the plane and the
  // other three idled (61 us for 84 MB)
  int d0, d1, t0 = 0, t1 = T;
  if (D == 1) {
    const int perT = (T + gridDim.z - 1) / gridDim.z;
    t0 = min(T, sl * perT);
    t1 = min(T, t0 + perT);
    d0 = 0;
    d1 = 1;
  } else {
    const int per = (D + gridDim.z - 1) / gridDim.z;
    d0 = sl * per;
    d1 = min(D, d0 + per);
  }
  const int64_t base = ((int64_t)o * C + c) * D * T;
  const int len = (MODE == RED_BWD && a.masked) ? a.lens[o] : T;
  // statistics: two independent fp64 chains per sum (elements t and t + blockDim of a pass) --
  // the adds' latency, not the loads, bounded one chain (39 -> 24 us per 84-MB plane pass)
  double p0[2] = {0.0, 0.0}, p1[2] = {0.0, 0.0}, p2[2] = {0.0, 0.0};
  auto add = [&](int j, int64_t rb, int t) __attribute__((always_inline)) {
    const float v = x[rb + t];
    if (MODE == RED_STATS) {
      p0[j] += v;
      p1[j] += (double)v * v;
    } else {
      float xhat;
      const float g = bwd_g(dy[rb + t], v, c, t, len, a, &xhat);
      p0[j] += g;
      p1[j] += (double)g * v;
      p2[j] += v;
    }
  };
  const int bd = blockDim.x;
  if constexpr (MODE == RED_STATS) {
    for (int d = d0; d < d1; ++d) {
      const int64_t rb = base + (int64_t)d * T;
      int t = t0 + threadIdx.x;
#pragma unroll 2
      for (; t + bd < t1; t += 2 * bd) {
        add(0, rb, t);
        add(1, rb, t + bd);
      }
      if (t < t1) add(0, rb, t);
    }
  } else {
    // the backward: the two chains take rows d and d + 1 at the same columns (the same mask
    // position t); two columns of one row per pass measured slower (57 -> 70 us)
    int d = d0;
    for (; d + 1 < d1; d += 2) {
      const int64_t rb = base + (int64_t)d * T;
      for (int t = t0 + threadIdx.x; t < t1; t += bd) {
        add(0, rb, t);
        add(1, rb + T, t);
      }
    }
    if (d < d1)
      for (int t = t0 + threadIdx.x; t < t1; t += bd) add(0, base + (int64_t)d * T, t);
  }
  double acc0 = p0[0] + p0[1], acc1 = p1[0] + p1[1], acc2 = p2[0] + p2[1];
  __shared__ double r0[4], r1[4], r2[4];
  acc0 = wave_sum_d(acc0);
  acc1 = wave_sum_d(acc1);
  acc2 = wave_sum_d(acc2);
  if ((threadIdx.x & 63) == 0) {
    r0[threadIdx.x >> 6] = acc0;
    r1[threadIdx.x >> 6] = acc1;
    r2[threadIdx.x >> 6] = acc2;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const int64_t pidx = ((int64_t)o * gridDim.z + sl) * C + c;
    partial[pidx * kParts + 0] = r0[0] + r0[1] + r0[2] + r0[3];
    partial[pidx * kParts + 1] = r1[0] + r1[1] + r1[2] + r1[3];
    partial[pidx * kParts + 2] = r2[0] + r2[1] + r2[2] + r2[3];
  }
}

// ---- finalize ---------------------------------------------------------------
// Fixed-order sum of the kParts-wide partials of column c = blockIdx.x * 64 + lane:
// the 4 waves of a 256-thread block sum interleaved part subsets, wave 0 combines.
// Returns false for the threads that do not finish a column.
template <int K>
__device__ __forceinline__ bool sum_parts(const double* __restrict__ partial, int nparts, int C,
                                          int& c, double (&out)[K]) {
  __shared__ double red[K][4][64];
  const int lane = threadIdx.x & 63;
  const int grp = threadIdx.x >> 6;
  c = blockIdx.x * 64 + lane;
  double acc[K];
#pragma unroll
  for (int k = 0; k < K; ++k) acc[k] = 0.0;
  // unrolled so that 8 partials' loads are in flight at once (the sums keep their order):
  // one dependent load per iteration made these finals latency-bound (~18 us each)
  if (c < C) {
#pragma unroll 8
    for (int p = grp; p < nparts; p += 4) {
#pragma unroll
      for (int k = 0; k < K; ++k) acc[k] += partial[((int64_t)p * C + c) * kParts + k];
    }
  }
#pragma unroll
  for (int k = 0; k < K; ++k) red[k][grp][lane] = acc[k];
  __syncthreads();
  if (grp != 0 || c >= C) return false;
#pragma unroll
  for (int k = 0; k < K; ++k)
    out[k] = (red[k][0][lane] + red[k][1][lane]) + (red[k][2][lane] + red[k][3][lane]);
  return true;
}

__global__ __launch_bounds__(256) void stats_final_kernel(
    const double* __restrict__ partial, int nparts, int C, double count, float eps,
    float momentum, float* __restrict__ save_mean, float* __restrict__ save_invstd,
    float* __restrict__ running_mean, float* __restrict__ running_var) {
  int c;
  double sum[2];
  if (!sum_parts<2>(partial, nparts, C, c, sum)) return;
  const double s = sum[0], ss = sum[1];
  const double mean = s / count;
  double var = ss / count - mean * mean;
  if (var < 0.0) var = 0.0;
  save_mean[c] = static_cast<float>(mean);
  save_invstd[c] = static_cast<float>(1.0 / sqrt(var + (double)eps));
  if (running_mean != nullptr) {
    const double unbiased = count > 1.0 ? var * count / (count - 1.0) : var;
    running_mean[c] = static_cast<float>((1.0 - momentum) * running_mean[c] + momentum * mean);
    running_var[c] = static_cast<float>((1.0 - momentum) * running_var[c] + momentum * unbiased);
  }
}

__global__ void eval_stats_kernel(const float* __restrict__ rm, const float* __restrict__ rv,
                                  int C, float eps, float* __restrict__ mean,
                                  float* __restrict__ invstd) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  mean[c] = rm[c];
  invstd[c] = static_cast<float>(1.0 / sqrt((double)rv[c] + (double)eps));
}

// sums -> per-channel coefficients for the backward apply (fp64):
//   dx = k1 * g - k2 - k3 * xhat  with k1 = gamma*invstd, k2 = k1*mean(g),
//   k3 = k1*mean(g*xhat), xhat = (x - mean)*invstd with the exact batch mean
//   sum(x)/count; also dgamma = sum(g*xhat), dbeta = sum(g) and the closed-form
//   bias gradient (see ds2_bn_backward).
__global__ __launch_bounds__(256) void bwd_final_kernel(
    const double* __restrict__ partial, int nparts, int C, double count, BnBwdArgs a,
    int n_outer, int D, int T, double* __restrict__ coef, float* __restrict__ dgamma,
    float* __restrict__ dbeta, float* __restrict__ dbias) {
  int c;
  double sum[3];
  if (!sum_parts<3>(partial, nparts, C, c, sum)) return;
  const double sg = sum[0];
  const double mean = sum[2] / count;
  const double is = (double)a.invstd[c];
  const double sgx = is * (sum[1] - mean * sg);     // sum(g * xhat)
  const double gbar = sg / count;
  const double gxbar = sgx / count;
  const double k1 = (double)a.gamma[c] * is;
  coef[c * kCoef + 0] = k1;
  coef[c * kCoef + 1] = k1 * gbar;
  coef[c * kCoef + 2] = k1 * gxbar;
  coef[c * kCoef + 3] = mean;
  if (dgamma != nullptr) dgamma[c] = static_cast<float>(sgx);
  if (dbeta != nullptr) dbeta[c] = static_cast<float>(sg);
  if (dbias != nullptr) {
    // d bias = sum over unmasked positions of d x1
    //        = gamma*invstd*(M - cnt_u)*(gbar - gxbar*invstd*mean)
    double cnt_u = 0.0;
    if (a.masked) {
      for (int o = 0; o < n_outer; ++o) cnt_u += (double)max(0, min(a.lens[o], T)) * D;
    } else {
      cnt_u = count;
    }
    const double v = k1 * (count - cnt_u) * (gbar - gxbar * is * mean);
    dbias[c] = static_cast<float>(v);
  }
}

// ---- apply ------------------------------------------------------------------
__global__ void apply_rows_kernel(const float* __restrict__ x, int64_t R, int C,
                                  const float* __restrict__ mean, const float* __restrict__ invstd,
                                  const float* __restrict__ gamma, const float* __restrict__ beta,
                                  float* __restrict__ y) {
  // vectorised: C % 4 == 0
  const int64_t total4 = R * C / 4;
  const int C4 = C / 4;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total4;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int c = static_cast<int>(i % C4) * 4;
    float4 v = reinterpret_cast<const float4*>(x)[i];
    v.x = gamma[c + 0] * ((v.x - mean[c + 0]) * invstd[c + 0]) + beta[c + 0];
    v.y = gamma[c + 1] * ((v.y - mean[c + 1]) * invstd[c + 1]) + beta[c + 1];
    v.z = gamma[c + 2] * ((v.z - mean[c + 2]) * invstd[c + 2]) + beta[c + 2];
    v.w = gamma[c + 3] * ((v.w - mean[c + 3]) * invstd[c + 3]) + beta[c + 3];
    reinterpret_cast<float4*>(y)[i] = v;
  }
}

__global__ void apply_generic_kernel(const float* __restrict__ x, int64_t total, int C,
                                     int64_t inner, const float* __restrict__ mean,
                                     const float* __restrict__ invstd,
                                     const float* __restrict__ gamma,
                                     const float* __restrict__ beta, float* __restrict__ y) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int c = static_cast<int>((i / inner) % C);
    y[i] = gamma[c] * ((x[i] - mean[c]) * invstd[c]) + beta[c];
  }
}

// MaskConv epilogue, NCDT output.  grid (ceil(T/256), ceil(D/BA_ROWS), N*C): a thread takes
// BA_ROWS rows of one column, loads first
constexpr int BA_ROWS_F = 4;
__global__ void apply_mask_htanh_ncdt_kernel(const float* __restrict__ x, int N, int C, int D,
                                             int T, const float* __restrict__ mean,
                                             const float* __restrict__ invstd,
                                             const float* __restrict__ gamma,
                                             const float* __restrict__ beta,
                                             const int* __restrict__ lens, float lo, float hi,
                                             float* __restrict__ y) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  const int d0 = blockIdx.y * BA_ROWS_F;
  const int nc = blockIdx.z;
  const int n = nc / C;
  const int c = nc - n * C;
  if (t >= T) return;
  const int len = lens != nullptr ? lens[n] : T;
  float xv[BA_ROWS_F];
#pragma unroll
  for (int r = 0; r < BA_ROWS_F; ++r)
    xv[r] = x[((int64_t)nc * D + (d0 + r < D ? d0 + r : D - 1)) * T + t];
  const float mu = mean[c], is = invstd[c], ga = gamma[c], be = beta[c];
#pragma unroll
  for (int r = 0; r < BA_ROWS_F; ++r) {
    if (d0 + r >= D) break;
    float v = ga * ((xv[r] - mu) * is) + be;
    if (t >= len) v = 0.f;
    v = fminf(fmaxf(v, lo), hi);
    if (t >= len) v = 0.f;
    y[((int64_t)nc * D + d0 + r) * T + t] = v;
  }
}

// MaskConv epilogue with the TxNx(C*D) collapse.  64(f) x 64(t) LDS tile.
// grid (ceil(T/64), ceil(F/64), N) with F = C*D, block 256.
__global__ __launch_bounds__(256) void apply_mask_htanh_tnf_kernel(
    const float* __restrict__ x, int N, int C, int D, int T, const float* __restrict__ mean,
    const float* __restrict__ invstd, const float* __restrict__ gamma,
    const float* __restrict__ beta, const int* __restrict__ lens, float lo, float hi,
    float* __restrict__ y) {
  __shared__ float tile[64][65];
  const int t0 = blockIdx.x * 64;
  const int f0 = blockIdx.y * 64;
  const int n = blockIdx.z;
  const int F = C * D;
  const int len = lens != nullptr ? lens[n] : T;
  const int tl = threadIdx.x & 63;
  const int q = threadIdx.x >> 6;
#pragma unroll 4
  for (int i = 0; i < 16; ++i) {
    const int fl = i * 4 + q;
    const int f = f0 + fl;
    const int t = t0 + tl;
    float v = 0.f;
    if (f < F && t < T) {
      const int c = f / D;
      v = gamma[c] * ((x[((int64_t)n * F + f) * T + t] - mean[c]) * invstd[c]) + beta[c];
      if (t >= len) v = 0.f;
      v = fminf(fmaxf(v, lo), hi);
      if (t >= len) v = 0.f;
    }
    tile[fl][tl] = v;
  }
  __syncthreads();
#pragma unroll 4
  for (int i = 0; i < 16; ++i) {
    const int tt = i * 4 + q;
    const int t = t0 + tt;
    const int f = f0 + tl;
    if (t < T && f < F) y[((int64_t)t * N + n) * F + f] = tile[tl][tt];
  }
}

// dst[n][f][t] = src[t][n][f]  (inverse of the collapse), 64x64 tiles.
__global__ __launch_bounds__(256) void tnf_to_nft_kernel(const float* __restrict__ src, int N,
                                                         int F, int T, float* __restrict__ dst) {
  __shared__ float tile[64][65];
  const int t0 = blockIdx.x * 64;
  const int f0 = blockIdx.y * 64;
  const int n = blockIdx.z;
  const int l = threadIdx.x & 63;
  const int q = threadIdx.x >> 6;
#pragma unroll 4
  for (int i = 0; i < 16; ++i) {
    const int tt = i * 4 + q;
    const int t = t0 + tt;
    const int f = f0 + l;
    tile[tt][l] = (t < T && f < F) ? src[((int64_t)t * N + n) * F + f] : 0.f;
  }
  __syncthreads();
#pragma unroll 4
  for (int i = 0; i < 16; ++i) {
    const int fl = i * 4 + q;
    const int f = f0 + fl;
    const int t = t0 + l;
    if (t < T && f < F) dst[((int64_t)n * F + f) * T + t] = tile[l][fl];
  }
}

// backward apply over [outer][C][D][T] (rows case: D = T = 1 -> inner = 1).  grid
// (ceil(T / 256), ceil(D / BA_ROWS), outer * C): a thread takes BA_ROWS rows d of one column
// t, all loads issued before the math (one element per thread ran at ~2.8 TB/s)
constexpr int BA_ROWS = 4;
__global__ void bwd_apply_planes_kernel(const float* __restrict__ dy, const float* __restrict__ x,
                                        int C, int D, int T, BnBwdArgs a,
                                        const double* __restrict__ coef, float* __restrict__ dx) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  const int d0 = blockIdx.y * BA_ROWS;
  const int oc = blockIdx.z;
  const int o = oc / C;
  const int c = oc - o * C;
  if (t >= T) return;
  const int len = a.masked ? a.lens[o] : T;
  const double* k = coef + c * kCoef;
  float dv[BA_ROWS], xv[BA_ROWS];
#pragma unroll
  for (int r = 0; r < BA_ROWS; ++r) {
    const int64_t idx = ((int64_t)oc * D + (d0 + r < D ? d0 + r : D - 1)) * T + t;
    dv[r] = dy[idx];
    xv[r] = x[idx];
  }
#pragma unroll
  for (int r = 0; r < BA_ROWS; ++r) {
    if (d0 + r >= D) break;
    const int64_t idx = ((int64_t)oc * D + d0 + r) * T + t;
    float xhat32;
    const float g = bwd_g(dv[r], xv[r], c, t, len, a, &xhat32);   // mask as the forward's
    const double xhat = ((double)xv[r] - k[3]) * (double)a.invstd[c];
    float v = static_cast<float>(k[0] * g - k[1] - k[2] * xhat);
    if (a.masked && t >= len) v = 0.f;
    dx[idx] = v;
  }
}

__global__ void bwd_apply_rows_kernel(const float* __restrict__ dy, const float* __restrict__ x,
                                      int64_t R, int C, BnBwdArgs a,
                                      const double* __restrict__ coef, float* __restrict__ dx) {
  const int64_t total = R * C;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int c = static_cast<int>(i % C);
    const double* k = coef + c * kCoef;
    const double xhat = ((double)x[i] - k[3]) * (double)a.invstd[c];
    dx[i] = static_cast<float>(k[0] * dy[i] - k[1] - k[2] * xhat);
  }
}

static inline int grid_cap(int64_t work, int block) {
  int64_t g = (work + block - 1) / block;
  return static_cast<int>(g > 2048 ? 2048 : (g < 1 ? 1 : g));
}

static inline size_t partial_parts(int outer, int c, int inner) {
  (void)c;
  if (inner == 1) return kRowChunks;
  return (size_t)outer * kPlaneSplit;
}

}  // namespace ds2

using namespace ds2;

extern "C" {

size_t ds2_bn_workspace_size(int outer, int c, int inner) {
  return partial_parts(outer, c, inner) * (size_t)c * kParts * sizeof(double) +
         (size_t)c * kCoef * sizeof(double) + 256;
}

ds2_status_t ds2_bn_train_stats(const float* x, int outer, int c, int inner, float eps,
                                float momentum, float* save_mean, float* save_invstd,
                                float* running_mean, float* running_var, void* ws,
                                size_t ws_bytes, ds2_stream_t stream) {
  if (outer < 1 || c < 1 || inner < 1) return DS2_INVALID_VALUE;
  if (ws == nullptr || ws_bytes < ds2_bn_workspace_size(outer, c, inner))
    return DS2_WORKSPACE_TOO_SMALL;
  hipStream_t st = as_stream(stream);
  double* partial = static_cast<double*>(ws);
  BnBwdArgs a{};
  int nparts;
  if (inner == 1) {
    nparts = kRowChunks;
    if (rows_vec(x, nullptr, c))
      hipLaunchKernelGGL(reduce_rows4_kernel<RED_STATS>, dim3(cdiv(c, 256), kRowChunks),
                         dim3(256), 0, st, x, nullptr, outer, c, a, partial);
    else
      hipLaunchKernelGGL(reduce_rows_kernel<RED_STATS>, dim3(cdiv(c, 64), kRowChunks),
                         dim3(256), 0, st, x, nullptr, outer, c, a, partial);
  } else {
    nparts = outer * kPlaneSplit;
    hipLaunchKernelGGL(reduce_planes_kernel<RED_STATS>, dim3(c, outer, kPlaneSplit), dim3(256), 0,
                       st, x, nullptr, c, 1, inner, a, partial);
  }
  hipLaunchKernelGGL(stats_final_kernel, dim3(cdiv(c, 64)), dim3(256), 0, st, partial, nparts, c,
                     (double)outer * inner, eps, momentum, save_mean, save_invstd, running_mean,
                     running_var);
  return launch_status("ds2_bn_train_stats");
}

ds2_status_t ds2_bn_eval_stats(const float* running_mean, const float* running_var, int c,
                               float eps, float* save_mean, float* save_invstd,
                               ds2_stream_t stream) {
  if (c < 1) return DS2_INVALID_VALUE;
  hipLaunchKernelGGL(eval_stats_kernel, dim3(cdiv(c, 256)), dim3(256), 0, as_stream(stream),
                     running_mean, running_var, c, eps, save_mean, save_invstd);
  return launch_status("ds2_bn_eval_stats");
}

ds2_status_t ds2_bn_apply(const float* x, int outer, int c, int inner, const float* mean,
                          const float* invstd, const float* gamma, const float* beta, float* y,
                          ds2_stream_t stream) {
  if (outer < 0 || c < 1 || inner < 1) return DS2_INVALID_VALUE;
  const int64_t total = (int64_t)outer * c * inner;
  if (total == 0) return DS2_OK;
  hipStream_t st = as_stream(stream);
  const bool vec = inner == 1 && (c % 4 == 0) &&
                   ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(y)) & 15) == 0;
  if (vec)
    hipLaunchKernelGGL(apply_rows_kernel, dim3(grid_cap(total / 4, 256)), dim3(256), 0, st, x,
                       (int64_t)outer, c, mean, invstd, gamma, beta, y);
  else
    hipLaunchKernelGGL(apply_generic_kernel, dim3(grid_cap(total, 256)), dim3(256), 0, st, x,
                       total, c, (int64_t)inner, mean, invstd, gamma, beta, y);
  return launch_status("ds2_bn_apply");
}

ds2_status_t ds2_bn_apply_amax(const float* x, int rows, int c, const float* mean,
                               const float* invstd, const float* gamma, const float* beta,
                               float* y, unsigned* row_amax, unsigned* col_amax,
                               ds2_stream_t stream) {
  if (rows < 0 || c < 1 || row_amax == nullptr || col_amax == nullptr) return DS2_INVALID_VALUE;
  if (rows == 0) return DS2_OK;
  const uintptr_t al = reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(y) |
                       reinterpret_cast<uintptr_t>(mean) | reinterpret_cast<uintptr_t>(invstd) |
                       reinterpret_cast<uintptr_t>(gamma) | reinterpret_cast<uintptr_t>(beta);
  if ((c % 4) != 0 || (al & 15) != 0 || c > 2048) return DS2_UNSUPPORTED_SHAPE;
  hipStream_t st = as_stream(stream);
  (void)hipMemsetAsync(col_amax, 0, (size_t)c * 4, st);
  launch_rows_amax<true>(x, rows, c, c, mean, invstd, gamma, beta, y, row_amax, col_amax, st);
  return launch_status("ds2_bn_apply_amax");
}

ds2_status_t ds2_bn_apply_mask_htanh(const float* x, int n, int c, int d, int t,
                                     const float* mean, const float* invstd, const float* gamma,
                                     const float* beta, const int* lens, float lo, float hi,
                                     float* y, int out_layout, ds2_stream_t stream) {
  if (n < 0 || c < 1 || d < 1 || t < 0) return DS2_INVALID_VALUE;
  if ((int64_t)n * c * d * t == 0) return DS2_OK;
  hipStream_t st = as_stream(stream);
  if (out_layout == 0) {
    hipLaunchKernelGGL(apply_mask_htanh_ncdt_kernel, dim3(cdiv(t, 256), cdiv(d, BA_ROWS_F), n * c),
                       dim3(256), 0,
                       st, x, n, c, d, t, mean, invstd, gamma, beta, lens, lo, hi, y);
  } else if (out_layout == 1) {
    hipLaunchKernelGGL(apply_mask_htanh_tnf_kernel, dim3(cdiv(t, 64), cdiv(c * d, 64), n),
                       dim3(256), 0, st, x, n, c, d, t, mean, invstd, gamma, beta, lens, lo, hi,
                       y);
  } else {
    return DS2_INVALID_VALUE;
  }
  return launch_status("ds2_bn_apply_mask_htanh");
}

ds2_status_t ds2_bn_backward(const float* dy, int dy_layout, const float* x, int outer, int c,
                             int d, int t, const float* mean, const float* invstd,
                             const float* gamma, const float* beta, int masked,
                             const int* lens, float lo, float hi, float* dx, float* dgamma,
                             float* dbeta, float* dbias_in, void* ws, size_t ws_bytes,
                             ds2_stream_t stream) {
  if (outer < 1 || c < 1 || d < 1 || t < 1) return DS2_INVALID_VALUE;
  if (dy_layout == 1 && !masked) return DS2_INVALID_VALUE;
  if (masked && lens == nullptr) return DS2_INVALID_VALUE;
  const int inner = d * t;
  if (ws == nullptr || ws_bytes < ds2_bn_workspace_size(outer, c, inner))
    return DS2_WORKSPACE_TOO_SMALL;
  hipStream_t st = as_stream(stream);
  const size_t nparts = partial_parts(outer, c, inner);
  double* partial = static_cast<double*>(ws);
  double* coef = partial + nparts * c * kParts;
  BnBwdArgs a{mean, invstd, gamma, beta, lens, lo, hi, masked};

  const float* g_src = dy;
  if (dy_layout == 1) {
    // bring dy into the [n][c*d][t] layout of x, inside dx (same size)
    hipLaunchKernelGGL(tnf_to_nft_kernel, dim3(cdiv(t, 64), cdiv(c * d, 64), outer), dim3(256),
                       0, st, dy, outer, c * d, t, dx);
    g_src = dx;
  }
  if (inner == 1) {
    if (rows_vec(x, g_src, c))
      hipLaunchKernelGGL(reduce_rows4_kernel<RED_BWD>, dim3(cdiv(c, 256), kRowChunks),
                         dim3(256), 0, st, x, g_src, outer, c, a, partial);
    else
      hipLaunchKernelGGL(reduce_rows_kernel<RED_BWD>, dim3(cdiv(c, 64), kRowChunks),
                         dim3(256), 0, st, x, g_src, outer, c, a, partial);
  } else {
    hipLaunchKernelGGL(reduce_planes_kernel<RED_BWD>, dim3(c, outer, kPlaneSplit), dim3(256), 0,
                       st, x, g_src, c, d, t, a, partial);
  }
  hipLaunchKernelGGL(bwd_final_kernel, dim3(cdiv(c, 64)), dim3(256), 0, st, partial,
                     (int)nparts, c, (double)outer * inner, a, outer, d, t, coef, dgamma, dbeta,
                     dbias_in);
  if (inner == 1) {
    hipLaunchKernelGGL(bwd_apply_rows_kernel, dim3(grid_cap((int64_t)outer * c, 256)), dim3(256),
                       0, st, g_src, x, (int64_t)outer, c, a, coef, dx);
  } else {
    // elementwise and position-local: safe in place when g_src == dx
    hipLaunchKernelGGL(bwd_apply_planes_kernel, dim3(cdiv(t, 256), cdiv(d, BA_ROWS), outer * c),
                       dim3(256), 0,
                       st, g_src, x, c, d, t, a, coef, dx);
  }
  return launch_status("ds2_bn_backward");
}

}  // extern "C"
