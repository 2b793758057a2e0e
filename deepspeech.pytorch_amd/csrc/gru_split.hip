// GRU recurrences with the W_hh contraction on the bf16 matrix cores at fp32 accuracy.
//
// The fp32 MFMA (v_mfma_f32_16x16x4_f32) runs at 1/16 of the bf16 rate, and at cfg2 (H 800,
// one workgroup per (16 units, direction, 16 samples)) it was ~2.2 us of every 5.6 us
// recurrence step.  Here every fp32 operand x is split into three bf16 terms,
//   hi = bf16(x), mid = bf16(x - hi), lo = bf16(x - hi - mid)     (x = hi + mid + lo exactly
//   up to the last bit of lo: 8 + 8 + 8 significant bits),
// and a product a.b is formed from the six terms that carry fp32 weight:
//   hi.hi + hi.mid + mid.hi + hi.lo + lo.hi + mid.mid
// (dropped: mid.lo, lo.mid, lo.lo, all below 2^-24 relative).  Each bf16 product is exact in
// the fp32 accumulator, so the result has fp32 accuracy (a 501-step GRU at H 800 drifts
// 1.9e-7 from fp64, plain fp32 2.2e-7); six v_mfma_f32_16x16x32_bf16 (16 cycles each) per 32
// k replace eight v_mfma_f32_16x16x4_f32 (32 cycles each): 2.7x fewer matrix cycles.
//
// W_hh is split once at kernel start and stays in registers for all T steps (3 terms x 8 bf16
// per 32 k); the handed-off h (forward) / gate gradients (backward) are split by the
// consumer after their loads.  Workgroups of 256 threads: 4 waves, ONE per SIMD with the
// whole 512-entry register file (the split W needs 1.5x the fp32 fragment registers), each
// wave owning a contiguous range of 32-k pairs of the hand-off tiles; the MFMA k slot j of
// lane (r, q) holds tile 2p + (j >> 2), k = 4q + (j & 3) -- exactly the 16 bytes that lane
// loads from each 1-KB tile, so the hand-off tiles, ring layout and protocols are those of
// gru_fwd_dop_kernel / gru_bwd_dop_kernel (gru.hip) unchanged.
#include "rnn_common.h"

namespace ds2 {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int XW = 4;            // waves per workgroup, one per SIMD
constexpr int kXTraceS0 = 100, kXTraceSteps = 16;   // = gru.hip's DS2_GRU_STAMPS=2 window
constexpr int XT = XW * 64;      // 256 threads = 16 samples x 16 units

struct Tri {
  bf16x8 hi, mid, lo;
};

// 8 fp32 values (k slots 0..3 from a, 4..7 from b) -> three bf16 terms (RNE splits; each
// residual is exact in fp32)
__device__ __forceinline__ Tri split3(const f32x4 a, const f32x4 b) {
  Tri t;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float v = j < 4 ? a[j] : b[j - 4];
    const __bf16 h = (__bf16)v;
    const float r1 = v - (float)h;
    const __bf16 m = (__bf16)r1;
    const float r2 = r1 - (float)m;
    t.hi[j] = h;
    t.mid[j] = m;
    t.lo[j] = (__bf16)r2;
  }
  return t;
}

// c += a.b to fp32 accuracy (small terms first)
__device__ __forceinline__ f32x4 mma6(const Tri& a, const Tri& b, f32x4 c) {
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.mid, b.mid, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.lo, b.hi, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.hi, b.lo, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.mid, b.hi, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.hi, b.mid, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.hi, b.hi, c, 0, 0, 0);
  return c;
}

typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));

// 4 fp32 -> their (hi, mid) bf16 terms packed as one 16-B run {hi01, hi23, mid01, mid23} and
// their lo terms as one 8-B run (v_cvt_pk_bf16_f32, RNE: the terms split3 forms)
__device__ __forceinline__ void split_pk4(const f32x4 v, u32x4& hm, u32x2& lo) {
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const float x0 = v[2 * q], x1 = v[2 * q + 1];
    const unsigned h = __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2{x0, x1}, bf16x2v));
    const float r0 = x0 - __builtin_bit_cast(float, h << 16);
    const float r1 = x1 - __builtin_bit_cast(float, h & 0xffff0000u);
    const unsigned m = __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2{r0, r1}, bf16x2v));
    const float l0 = r0 - __builtin_bit_cast(float, m << 16);
    const float l1 = r1 - __builtin_bit_cast(float, m & 0xffff0000u);
    hm[q] = h;
    hm[2 + q] = m;
    lo[q] = __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2{l0, l1}, bf16x2v));
  }
}

// the Tri of a 32-k pair from two pre-split tiles' runs (slots 0..3 tile a, 4..7 tile b)
__device__ __forceinline__ Tri tri_of(const u32x4 ha, const u32x2 la, const u32x4 hb, const u32x2 lb) {
  Tri t;
  t.hi = __builtin_bit_cast(bf16x8, u32x4{ha[0], ha[1], hb[0], hb[1]});
  t.mid = __builtin_bit_cast(bf16x8, u32x4{ha[2], ha[3], hb[2], hb[3]});
  t.lo = __builtin_bit_cast(bf16x8, u32x4{la[0], la[1], lb[0], lb[1]});
  return t;
}

// wave's contiguous share [p0, p0 + np) of `pairs` 32-k pairs
__device__ __forceinline__ void pair_split(int pairs, int wave, int& p0, int& np) {
  p0 = (pairs * wave) / XW;
  np = (pairs * (wave + 1)) / XW - p0;
}

// ---------------------------------------------------------------------------------------
// forward: gh[16 samples x 48] = h_{t-1}[16 x H] . W_hh[r, z, n rows of 16 units]^T, with
// the sentinel-ring hand-off of gru_fwd_dop_kernel (the data is the flag).
// NG = 1: the one-gate instantiation for supported_rnns['rnn'] (nn.RNN, tanh; model.py:15):
// gh[16 x 16] = h_{t-1} . W_hh[16 units]^T and h_t = tanh(xproj_t + gh + b_hh), no gate cache.
template <int NP, bool H3 = false, int NG = 3>
__global__ __launch_bounds__(XT) __attribute__((amdgpu_waves_per_eu(1, 1))) void gru_fwd_x6_kernel(
    int T, int N, int H, int D, int UB, int BT, const float* __restrict__ xproj,
    const float* __restrict__ w_f, const float* __restrict__ w_r, const float* __restrict__ b_f,
    const float* __restrict__ b_r, const int* __restrict__ lens, float* __restrict__ h_all,
    float* __restrict__ gates, float* __restrict__ hx, unsigned* __restrict__ counters,
    unsigned* __restrict__ err, unsigned long long* __restrict__ stamps, int xmode) {
  static_assert(2 * NP <= 64, "tsame holds a wave's tiles");
  static_assert(NG == 3 || (NG == 1 && H3), "the one-gate form is fp16x3 only");
  constexpr int RP = NG * GU + 1;
  constexpr int NSLOT = kRingSlots;
  __shared__ float red[XW * GB * RP];
  __shared__ __attribute__((aligned(16))) float tile[GB * GU];
  __shared__ int failed;
  int ub, d, bt;
  // xmode: same-XCD groups as in the backward -- every tile and its sentinel refill also
  // stored plainly into a second ring (slots NSLOT..2 NSLOT-1), from which the consumers on
  // the producer's XCD read it
  const bool xg = xmode != 0;
  if (xg ? !map_work_xgrp(UB, BT, D, ub, d, bt) : !map_work(UB * D, BT, UB, ub, d, bt)) return;
  unsigned* xtab = counters + (D * BT + 1) + D * BT * 64 + (d * BT + bt) * 64;
  const unsigned my_xcc = xcc_id() + 1u;
  if (xg && threadIdx.x == 0)
    __hip_atomic_store(xtab + ub, my_xcc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  uint64_t tsame = 0;           // bit i: this wave's tile t_first + i comes from this XCD
  const int n0 = bt * GB;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  int p0, np;
  pair_split((UB + 1) >> 1, wave, p0, np);          // host guarantees np <= NP
  const int t_first = 2 * p0;                       // first hand-off tile of this wave
  const int slot_floats = D * BT * UB * 256;
  const __amdgpu_buffer_rsrc_t x_rs = __builtin_amdgcn_make_buffer_rsrc(
      hx, (short)0, (xg ? 2 * NSLOT : NSLOT) * slot_floats * 4, 0x00020000);
  const int grp_off = (d * BT + bt) * UB * 256;
  const int aoff = NSLOT * slot_floats * 4;   // the plain-store ring (xmode)
  if (threadIdx.x == 0) failed = 0;
  __syncthreads();
  // diagnostic timeline (DS2_GRU_STAMPS=2, scripts/trace_gru.py): s_memrealtime at step
  // start / wait done / products done / reduction done / published, for kXTraceSteps steps
  const bool tracing = stamps != nullptr && threadIdx.x == 0;
  auto trace_at = [&](int s, int p) {
    if (tracing && s >= kXTraceS0 && s < kXTraceS0 + kXTraceSteps)
      stamps[((int64_t)(s - kXTraceS0) * gridDim.x + blockIdx.x) * 5 + p] =
          __builtin_amdgcn_s_memrealtime();
  };

  // W_hh split fragments: pair p, gate g, k slot j -> W[g H + 16 ub + (lane & 15)]
  //   [16 (t_first + 2p + (j >> 2)) + 4 (lane >> 4) + (j & 3)]
  using WT = typename std::conditional<H3, Duo, Tri>::type;
  WT w[NG][NP];
  // fp16x3: 2^-(e(g, unit) + 14) undoes the row scale of W_hh and the fixed 2^14 of h; the
  // owner thread's unit u = threadIdx.x & 15
  float unscale[NG];
#pragma unroll
  for (int g = 0; g < NG; ++g) unscale[g] = 1.f;
  {
    const float* W = d == 0 ? w_f : w_r;
    const float* wr = W + (int64_t)(ub * GU + (lane & 15)) * H + 4 * (lane >> 4);
    auto frag = [&](int p, int g, f32x4& a, f32x4& b) {
      const int ta = t_first + 2 * p, tb = ta + 1;
      const float* wg = wr + (int64_t)g * H * H;
      const f32x4 z4 = f32x4{0.f, 0.f, 0.f, 0.f};
      a = (p < np && ta < UB) ? *reinterpret_cast<const f32x4*>(wg + 16 * ta) : z4;
      b = (p < np && tb < UB) ? *reinterpret_cast<const f32x4*>(wg + 16 * tb) : z4;
    };
    if constexpr (H3) {
      // max |W| of each (gate, unit) row over the whole K: the lane's share, the 4 lanes
      // of its unit, then the workgroup's waves (LDS, reusing `red`)
      float mx[NG];
#pragma unroll
      for (int g = 0; g < NG; ++g) mx[g] = 0.f;
#pragma unroll
      for (int p = 0; p < NP; ++p)
#pragma unroll
        for (int g = 0; g < NG; ++g) {
          f32x4 a, b;
          frag(p, g, a, b);
#pragma unroll
          for (int j = 0; j < 4; ++j) mx[g] = fmaxf(mx[g], fmaxf(fabsf(a[j]), fabsf(b[j])));
        }
#pragma unroll
      for (int g = 0; g < NG; ++g) {
        mx[g] = fmaxf(mx[g], __shfl_xor(mx[g], 16));
        mx[g] = fmaxf(mx[g], __shfl_xor(mx[g], 32));
        if (lane < 16) red[(wave * NG + g) * 16 + lane] = mx[g];
      }
      __syncthreads();
      int eg[NG];
#pragma unroll
      for (int g = 0; g < NG; ++g) {
        float m = 0.f;
#pragma unroll
        for (int w8 = 0; w8 < XW; ++w8) m = fmaxf(m, red[(w8 * NG + g) * 16 + (lane & 15)]);
        eg[g] = h3_row_exp(m);
        // the owner thread's unit is threadIdx.x & 15 = lane & 15: the same row
        unscale[g] = __builtin_ldexpf(1.f, -(eg[g] + 14));
      }
      __syncthreads();
#pragma unroll
      for (int p = 0; p < NP; ++p)
#pragma unroll
        for (int g = 0; g < NG; ++g) {
          f32x4 a, b;
          frag(p, g, a, b);
          w[g][p] = split2h(a, b, __builtin_ldexpf(1.f, eg[g]));
        }
    } else {
#pragma unroll
      for (int p = 0; p < NP; ++p)
#pragma unroll
        for (int g = 0; g < 3; ++g) {
          f32x4 a, b;
          frag(p, g, a, b);
          w[g][p] = split3(a, b);
        }
    }
  }
  const float* bh = d == 0 ? b_f : b_r;
  const int m = threadIdx.x >> 4;
  const int u = threadIdx.x & 15;
  const int n = n0 + m;
  const int j = ub * GU + u;
  const bool owner = n < N;
  float bias_r = 0.f, bias_z = 0.f, bias_n = 0.f;
  int len = 0;
  if (owner) {
    bias_r = bh[j];
    if constexpr (NG == 3) {
      bias_z = bh[H + j];
      bias_n = bh[2 * H + j];
    }
    len = lens[n];
  }
  settle(bias_r);
  settle(bias_z);
  settle(bias_n);
  settle(len);
  const int tpos = ((u >> 2) * GB + m) * 4 + (u & 3);
  float g_r = 0.f, g_z = 0.f, g_n = 0.f, g_hn = 0.f, h_own = 0.f;
  int64_t g_row = -1;
  for (int s = 0; s < T; ++s) {
    const int t = d == 0 ? s : T - 1 - s;
    const int64_t row = ((int64_t)t * N + n) * D + d;
    float xr = 0.f, xz = 0.f, xn = 0.f;
    if (owner && t < len) {
      const float* xp = xproj + row * NG * H;
      xr = xp[j];
      if constexpr (NG == 3) {
        xz = xp[H + j];
        xn = xp[2 * H + j];
      }
    }
    f32x4 acc[NG];
#pragma unroll
    for (int g = 0; g < NG; ++g) acc[g] = f32x4{0.f, 0.f, 0.f, 0.f};
    trace_at(s, 0);
    if (s > 0) {
      trace_at(s, 1);
      if (xg && s == 1) {   // which producers share this XCD (ids published at their start)
        unsigned v = 0;
        for (unsigned spins = 0;; ++spins) {
          v = lane < UB ? __hip_atomic_load(xtab + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                        : 1u;
          if (__ballot(v == 0u) == 0ull || spins > g_spin_limit) break;
          __builtin_amdgcn_s_sleep(1);
        }
        const unsigned long long same = __ballot(v == my_xcc);   // an id never seen: no bit
#pragma unroll
        for (int i = 0; i < 2 * NP; ++i)
          if (t_first + i < UB && ((same >> (t_first + i)) & 1ull)) tsame |= 1ull << i;
      }
      const int base = (((s - 1) % NSLOT) * slot_floats + grp_off + t_first * 256 + lane * 4) * 4;
      sleep_units(g_rnn_tune[1]);
      f32x4 hv[2 * NP];
#pragma unroll
      for (int i = 0; i < 2 * NP; ++i) {
        const int off = (i < 2 * np && t_first + i < UB)
                            ? base + i * 1024 + (((tsame >> i) & 1ull) ? aoff : 0) : 0x7ffffff0;
        hv[i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(x_rs, off, 0, kSc1));
      }
      asm volatile("" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      // per-pair partials summed in a fixed order afterwards: pairs are multiplied in
      // arrival order (one re-load round trip per pass), the result is deterministic
      f32x4 pacc[NP][NG];
#pragma unroll
      for (int p = 0; p < NP; ++p)
#pragma unroll
        for (int g = 0; g < NG; ++g) pacc[p][g] = f32x4{0.f, 0.f, 0.f, 0.f};
      unsigned pend = (1u << np) - 1u;
      for (unsigned spins = 0;; ++spins) {
#pragma unroll
        for (int p = 0; p < NP; ++p) {
          if (((pend >> p) & 1u) && wave_ready(hv[2 * p]) && wave_ready(hv[2 * p + 1])) {
            if constexpr (H3) {
              const Duo a = split2h(hv[2 * p], hv[2 * p + 1], 16384.f);
#pragma unroll
              for (int g = 0; g < NG; ++g) pacc[p][g] = mma3h(a, w[g][p], pacc[p][g]);
            } else {
              const Tri a = split3(hv[2 * p], hv[2 * p + 1]);
#pragma unroll
              for (int g = 0; g < NG; ++g) pacc[p][g] = mma6(a, w[g][p], pacc[p][g]);
            }
            pend &= ~(1u << p);
          }
        }
        if (pend == 0u && g_spin_limit != 0) break;
        if (spins > g_spin_limit || g_spin_limit == 0) {
          if (lane == 0) __hip_atomic_fetch_or(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          failed = 1;
          break;
        }
        sleep_units(g_rnn_tune[0]);
        asm volatile("" ::: "memory");
#pragma unroll
        for (int i = 0; i < 2 * NP; ++i)
          if (((pend >> (i >> 1)) & 1u) && t_first + i < UB)
            hv[i] = __builtin_bit_cast(
                f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                           x_rs, base + i * 1024 + (((tsame >> i) & 1ull) ? aoff : 0), 0, kSc1));
      }
#pragma unroll
      for (int g = 0; g < NG; ++g) {
        acc[g] = pacc[0][g];
#pragma unroll
        for (int p = 1; p < NP; ++p) acc[g] += pacc[p][g];
      }
      trace_at(s, 2);
    }
#pragma unroll
    for (int g = 0; g < NG; ++g)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        red[(wave * GB + (lane >> 4) * 4 + r) * RP + g * GU + (lane & 15)] = acc[g][r];
    settle(xr);
    settle(xz);
    settle(xn);
    __syncthreads();
    if (failed) {
      poison_rest(h_all, s, T, d != 0, N, D, n, d, H, j, H, 1, owner);
      return;
    }
    trace_at(s, 3);
    float hout = 0.f;
    if constexpr (NG == 1) {
      if (owner) {
        float v = 0.f;
#pragma unroll
        for (int w8 = 0; w8 < XW; ++w8) v += red[(w8 * GB + m) * RP + u];
        if (t < len) hout = tanh_fast(xr + (v * unscale[0] + bias_r));
        h_own = hout;
      }
    } else if (owner) {
      float gh[NG];
#pragma unroll
      for (int g = 0; g < NG; ++g) {
        float v = 0.f;
#pragma unroll
        for (int w8 = 0; w8 < XW; ++w8) v += red[(w8 * GB + m) * RP + g * GU + u];
        gh[g] = H3 ? v * unscale[g] : v;
      }
      const float ghr = gh[0] + bias_r;
      const float ghz = gh[1] + bias_z;
      float ghn = gh[2] + bias_n;
      float r = 0.f, z = 0.f, nn = 0.f;
      if (t < len) {
        r = sigmoid_fast(ghr + xr);
        z = sigmoid_fast(ghz + xz);
        nn = tanh_fast(xn + r * ghn);
        hout = (h_own - nn) * z + nn;
      } else {
        ghn = 0.f;
      }
      h_own = hout;
      g_r = r; g_z = z; g_n = nn; g_hn = ghn; g_row = row;
    }
    tile[tpos] = hout;
    __syncthreads();
    if (wave == 0) {
      const int toff = (grp_off + ub * 256 + lane * 4) * 4;
      const u32x4 v = desentinel(*reinterpret_cast<const u32x4*>(tile + lane * 4));
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // last step's sentinel store first
      __builtin_amdgcn_raw_buffer_store_b128(v, x_rs, (s % NSLOT) * slot_floats * 4 + toff, 0, kSc1);
      const u32x4 sv = u32x4{kSentinel, kSentinel, kSentinel, kSentinel};
      __builtin_amdgcn_raw_buffer_store_b128(sv, x_rs, ((s + 2) % NSLOT) * slot_floats * 4 + toff,
                                             0, kSc1);
      if (xg) {   // plain copies for the same-XCD consumers (kept in this XCD's L2)
        __builtin_amdgcn_raw_buffer_store_b128(v, x_rs, aoff + (s % NSLOT) * slot_floats * 4 + toff,
                                               0, 0);
        __builtin_amdgcn_raw_buffer_store_b128(
            sv, x_rs, aoff + ((s + 2) % NSLOT) * slot_floats * 4 + toff, 0, 0);
      }
    }
    trace_at(s, 4);
    if (owner) {
      h_all[row * H + j] = h_own;
      if (NG == 3 && gates != nullptr) {
        float* gp = gates + g_row * 4 * H;
        gp[j] = g_r;
        gp[H + j] = g_z;
        gp[2 * H + j] = g_n;
        gp[3 * H + j] = g_hn;
      }
    }
  }
}

// ---------------------------------------------------------------------------------------
// backward: rec[16 samples x 16 units] = dG[16 x 3H] . W_hh[3H rows, 16 units], dG = the
// (dar, daz, dghn) gate gradients of the step after (tiles g UB + ub of the ring, as in
// gru_bwd_dop_kernel).  8 waves per workgroup, two per SIMD (256 registers each).  The
// producers publish their gate-gradient tiles PRE-SPLIT (per lane a 16-B {hi, mid} run and an
// 8-B lo run: 1.5 KB per tile instead of 1 KB of fp32), so the consumer loads ready MFMA
// operands and does no split VALU; the runs stream through a window of LWP pairs per wave;
// per-producer flag hand-off (MI355X_MICROARCH "Valid forms" row 1).  Measured and removed in
// round 4's pruning: consumer-side splits of fp32 tiles (6.5 vs 6.2 us per step), one wave
// per SIMD with every run in flight (7.1), a sentinel ring over the runs (9.2: each stale pass
// re-issues the window).  dbp (nullable): per-unit bias-gradient partials as
// gru_bwd_dop_kernel's.
constexpr int BW = 8;            // waves per backward workgroup
template <int NP>
__global__ __launch_bounds__(BW * 64) __attribute__((amdgpu_waves_per_eu(2, 2))) void gru_bwd_x6_kernel(
    int T, int N, int H, int D, int UB, int BT, const float* __restrict__ dy, int dyd,
    const float* __restrict__ w_f, const float* __restrict__ w_r,
    const float* __restrict__ h_all, const float* __restrict__ gates,
    const int* __restrict__ lens, float* __restrict__ dgx, float* __restrict__ dgh,
    float* __restrict__ gx, unsigned* __restrict__ counters, unsigned* __restrict__ err,
    unsigned long long* __restrict__ stamps, double* __restrict__ dbp, int xmode) {
  static_assert(2 * NP <= 64, "tsame holds a wave's tiles");
  constexpr int RP = GU + 1;
  constexpr int TF = 384;                       // ring floats per pre-split tile
  // pairs of runs in flight per wave: with the same-XCD groups 4 (or 3) beat 5 (5.41 -> 5.34
  // us per step, 6: 5.47; profiles/r3lw_bwd_window.txt)
  constexpr int LWP = NP < 4 ? NP : 4;
  constexpr int RED = BW * GB * RP > 8 * GB * GU ? BW * GB * RP : 8 * GB * GU;
  __shared__ __attribute__((aligned(8))) float red[RED];
  __shared__ __attribute__((aligned(16))) float tile[3 * GB * GU];
  __shared__ int flag;
  int ub, d, bt;
  // xmode: same-XCD groups -- every tile is also stored plainly into ring slots 2-3 (kept in
  // the producer's L2) and a consumer loads the tiles of the producers that share its XCD
  // from there
  const bool xg = xmode != 0;
  if (xg ? !map_work_xgrp(UB, BT, D, ub, d, bt) : !map_work(UB * D, BT, UB, ub, d, bt)) return;
  const int n0 = bt * GB;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int H3 = 3 * H;
  const int NB3 = 3 * UB;
  unsigned* xtab = counters + (D * BT + 1) + D * BT * 64 + (d * BT + bt) * 64;
  const unsigned my_xcc = xcc_id() + 1u;
  if (xg && threadIdx.x == 0)   // published by the step-0 flag (wave 0 drains before it)
    __hip_atomic_store(xtab + ub, my_xcc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  uint64_t tsame = 0;           // bit i: this wave's tile t_first + i comes from this XCD
  const int pairs = (NB3 + 1) >> 1;
  const int p0 = (pairs * wave) / BW;
  const int np = (pairs * (wave + 1)) / BW - p0;   // host guarantees np <= NP
  const int t_first = 2 * p0;
  const unsigned* gflags = counters + (D * BT + 1) + (d * BT + bt) * UB;
  unsigned* myflag = counters + (D * BT + 1) + (d * BT + bt) * UB + ub;
  const int slot_floats = D * BT * NB3 * TF;
  const __amdgpu_buffer_rsrc_t x_rs = __builtin_amdgcn_make_buffer_rsrc(
      gx, (short)0, (xg ? 4 : 2) * slot_floats * 4, 0x00020000);
  const int grp_off = (d * BT + bt) * NB3 * TF;
  const int aoff = 2 * slot_floats * 4;   // the plain-store copies (xmode)
  // diagnostic timeline (DS2_GRU_STAMPS=2, scripts/trace_gru.py): s_memrealtime at step
  // start / wait done / products done / reduction done / published, for kXTraceSteps steps
  const bool tracing = stamps != nullptr && threadIdx.x == 0;
  auto trace_at = [&](int s, int p) {
    if (tracing && s >= kXTraceS0 && s < kXTraceS0 + kXTraceSteps)
      stamps[((int64_t)(s - kXTraceS0) * gridDim.x + blockIdx.x) * 5 + p] =
          __builtin_amdgcn_s_memrealtime();
  };

  // W_hh^T split fragments: pair p, k slot j -> W_hh[16 (t_first + 2p + (j >> 2)) +
  //   4 (lane >> 4) + (j & 3)][16 ub + (lane & 15)]
  Tri w[NP];
  {
    const float* W = d == 0 ? w_f : w_r;
    const float* wc = W + (int64_t)(4 * (lane >> 4)) * H + ub * GU + (lane & 15);
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      const int ta = t_first + 2 * p, tb = ta + 1;
      f32x4 a = f32x4{0.f, 0.f, 0.f, 0.f}, b = a;
      if (p < np && ta < NB3)
#pragma unroll
        for (int c = 0; c < 4; ++c) a[c] = wc[(int64_t)(16 * ta + c) * H];
      if (p < np && tb < NB3)
#pragma unroll
        for (int c = 0; c < 4; ++c) b[c] = wc[(int64_t)(16 * tb + c) * H];
      w[p] = split3(a, b);
    }
  }
  const int m = (threadIdx.x >> 4) & 15;
  const int u = threadIdx.x & 15;
  const int n = n0 + m;
  const int j = ub * GU + u;
  const bool gate_thread = threadIdx.x < GB * GU;
  const bool owner = gate_thread && n < N;
  int len = owner ? lens[n] : 0;
  settle(len);
  const int tpos = ((u >> 2) * GB + m) * 4 + (u & 3);
  float dh_prev = 0.f, z_prev = 0.f;
  float px_dar = 0.f, px_daz = 0.f, px_dan = 0.f, px_dghn = 0.f;
  int64_t px_row = -1;
  double sb_r = 0.0, sb_z = 0.0, sb_n = 0.0, sb_hn = 0.0;
  for (int s = 0; s < T; ++s) {
    const int t = d == 0 ? T - 1 - s : s;
    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
    float dyv = 0.f, g_r = 0.f, g_z = 0.f, g_n = 0.f, g_hn = 0.f, hp = 0.f;
    const int64_t row = ((int64_t)t * N + n) * D + d;
    if (owner && t < len) {
      dyv = dy[(((int64_t)t * N + n) * dyd + (dyd > 1 ? d : 0)) * H + j];
      const float* gp = gates + row * 4 * H;
      g_r = gp[j];
      g_z = gp[H + j];
      g_n = gp[2 * H + j];
      g_hn = gp[3 * H + j];
      const int tp = d == 0 ? t - 1 : t + 1;
      if (tp >= 0 && tp < T) hp = h_all[(((int64_t)tp * N + n) * D + d) * H + j];
    }
    trace_at(s, 0);
    if (s > 0) {
      if (!flags_wait(gflags, UB, (unsigned)s, err, &flag)) {
        poison_rest(dgx, s, T, d == 0, N, D, n, d, H, j, H3, 3, owner);
        return;
      }
      trace_at(s, 1);
      if (xg && s == 1) {   // which producers share this XCD (their ids came with step 0)
        const unsigned v = lane < UB ? __hip_atomic_load(xtab + lane, __ATOMIC_RELAXED,
                                                         __HIP_MEMORY_SCOPE_AGENT) : 0u;
        const unsigned long long same = __ballot(v == my_xcc);
#pragma unroll
        for (int i = 0; i < 2 * NP; ++i)
          if ((same >> ((t_first + i) % UB)) & 1ull) tsame |= 1ull << i;
      }
      // LWP pairs' runs in flight, the next pair's issued as each pair is multiplied
      const int tb0 = (((s - 1) & 1) * slot_floats + grp_off + t_first * TF) * 4;
      u32x4 hm[2 * NP];
      u32x2 lo[2 * NP];
      auto load_run = [&](int i) {
        const bool ok = i < 2 * np && t_first + i < NB3;
        const int to = tb0 + i * TF * 4 + (((tsame >> i) & 1ull) ? aoff : 0);
        hm[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                              x_rs, ok ? to + lane * 16 : 0x7ffffff0, 0, kSc1));
        lo[i] = __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(
                                              x_rs, ok ? to + 1024 + lane * 8 : 0x7ffffff0, 0, kSc1));
      };
#pragma unroll
      for (int i = 0; i < 2 * LWP; ++i) load_run(i);
      asm volatile("" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int p = 0; p < NP; ++p) {
        if (p + LWP < NP) {
          load_run(2 * (p + LWP));
          load_run(2 * (p + LWP) + 1);
        }
        acc = mma6(tri_of(hm[2 * p], lo[2 * p], hm[2 * p + 1], lo[2 * p + 1]), w[p], acc);
      }
      trace_at(s, 2);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r)
      red[(wave * GB + (lane >> 4) * 4 + r) * RP + (lane & 15)] = acc[r];
    settle(dyv);
    settle(g_r);
    settle(g_z);
    settle(g_n);
    settle(g_hn);
    settle(hp);
    __syncthreads();
    trace_at(s, 3);
    float dar = 0.f, daz = 0.f, dan = 0.f, dghn = 0.f;
    if (owner) {
      float dh = 0.f, zc = 0.f;
      if (t < len) {
        float carry = 0.f;
        if (s > 0) {
          float rec = 0.f;
#pragma unroll
          for (int w8 = 0; w8 < BW; ++w8) rec += red[(w8 * GB + m) * RP + u];
          carry = dh_prev * z_prev + rec;
        }
        dh = dyv + carry;
        zc = g_z;
        dan = dh * (1.f - zc) * (1.f - g_n * g_n);
        daz = dh * (hp - g_n) * zc * (1.f - zc);
        dar = dan * g_hn * g_r * (1.f - g_r);
        dghn = dan * g_r;
      }
      dh_prev = dh;
      z_prev = zc;
      px_dar = dar; px_daz = daz; px_dan = dan; px_dghn = dghn; px_row = row;
      sb_r += dar; sb_z += daz; sb_n += dan; sb_hn += dghn;
    }
    if (gate_thread) {
      tile[tpos] = dar;
      tile[GB * GU + tpos] = daz;
      tile[2 * GB * GU + tpos] = dghn;
    }
    __syncthreads();
    if (wave == 0) {
      const int so = ((s & 1) * slot_floats + grp_off + ub * TF) * 4;
#pragma unroll
      for (int g = 0; g < 3; ++g) {
        u32x4 hmv;
        u32x2 lov;
        split_pk4(*reinterpret_cast<const f32x4*>(tile + g * GB * GU + lane * 4), hmv, lov);
        const int go = so + g * UB * TF * 4;
        __builtin_amdgcn_raw_buffer_store_b128(hmv, x_rs, go + lane * 16, 0, kSc1);
        __builtin_amdgcn_raw_buffer_store_b64(lov, x_rs, go + 1024 + lane * 8, 0, kSc1);
        if (xg) {   // plain copies: stay in this XCD's L2 for the same-XCD consumers
          __builtin_amdgcn_raw_buffer_store_b128(hmv, x_rs, aoff + go + lane * 16, 0, 0);
          __builtin_amdgcn_raw_buffer_store_b64(lov, x_rs, aoff + go + 1024 + lane * 8, 0, 0);
        }
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (lane == 0)
        __hip_atomic_store(myflag, (unsigned)s + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    trace_at(s, 4);
    if (owner) {
      float* gxr = dgx + px_row * H3;
      gxr[j] = px_dar;
      gxr[H + j] = px_daz;
      gxr[2 * H + j] = px_dan;
      float* ghr = dgh + px_row * H3;
      ghr[j] = px_dar;
      ghr[H + j] = px_daz;
      ghr[2 * H + j] = px_dghn;
    }
  }
  if (dbp == nullptr) return;
  // the workgroup's 16 samples summed per unit in sample order -> dbp[bt][d][4][H]
  double* rd = reinterpret_cast<double*>(red);
  __syncthreads();
  if (gate_thread) {
    rd[(0 * GB + m) * GU + u] = owner ? sb_r : 0.0;
    rd[(1 * GB + m) * GU + u] = owner ? sb_z : 0.0;
    rd[(2 * GB + m) * GU + u] = owner ? sb_n : 0.0;
    rd[(3 * GB + m) * GU + u] = owner ? sb_hn : 0.0;
  }
  __syncthreads();
  if (threadIdx.x < 4 * GU) {
    const int g = threadIdx.x / GU, uu = threadIdx.x - (threadIdx.x / GU) * GU;
    double a = 0.0;
#pragma unroll
    for (int mm = 0; mm < GB; ++mm) a += rd[(g * GB + mm) * GU + uu];
    dbp[(((int64_t)bt * D + d) * 4 + g) * H + ub * GU + uu] = a;
  }
}

// ---------------------------------------------------------------------------------------
// backward on fp16x3 (default since round 5; DS2_GRU_H3_BWD=0 keeps the bf16x6 kernel
// above).  The same work, groups and flag hand-off as gru_bwd_x6_kernel, but each producer
// publishes ONE record per step: its three gate-gradient tiles (dar, daz, dghn of 16
// samples x 16 units), every sample row scaled by its own 2^e (e from the row's max over
// the 48 values) and split into fp16 (hi, lo) in the consumers' MFMA operand order, plus the
// 16 row factors 2^-e:
//   [0, 1 KB)  hi of r, z: lane L = (m, q) holds r[m][4q..4q+3], z[m][4q..4q+3]
//   [1, 2 KB)  lo of r, z, same order
//   [2, 3 KB)  n: lane L holds hi n[m][4q..4q+3], lo n[m][4q..4q+3]
//   [3 KB, +64 B)  2^-e of the 16 rows
// (3.06 KB per producer and step instead of 4.5 KB of pre-split bf16 runs).  A consumer
// multiplies each producer's record with its W_hh^T fragments -- the r, z pair as three
// v_mfma_f32_16x16x32_f16, the n tile as three v_mfma_f32_16x16x16_f16, one temporary -- and
// adds the temporary into its sum row-scaled by the producer's 2^-e: the products of one
// producer share their rows' scales, so the scale applies after the MFMAs.  W_hh^T is
// scaled per column (unit) by 2^e found at kernel start and undone on the reduced sum.
// NG = 1: the one-gate instantiation for supported_rnns['rnn'] (nn.RNN, tanh): the record is
// the pre-activation gradient da = (dy + W_hh^T da_next) (1 - h^2) of 16 samples x 16 units
// in the n tile's layout, [0, 1 KB), and the 16 row factors at 1 KB (272 floats); gates = NULL,
// h_all supplies h_t; dgx receives da ([T][N][D][H]); dgh and dbp are unused.
// NG = 4: the LSTM (supported_rnns['lstm'], model.py:14; gate order i, f, g, o): the record
// holds dai, daf as the first pair and dag, dao as the second, [0, 1 KB) hi (i, f), [1, 2 KB)
// lo (i, f), [2, 3 KB) hi (g, o), [3, 4 KB) lo (g, o), row factors at 4 KB (1040 floats);
// `h_all` is c_all ([T][N][D][H] cell states), `gates` the [T][N][D][4H] activation cache,
// dgx receives dgates ([T][N][D][4H]); dgh and dbp are unused; the carried dc lives in a
// register.  n_base: the first sample of this launch (the batch runs as consecutive chunks of
// 16-sample tiles when one launch of all of them would not fit the chip).
constexpr int HBR = 784;   // floats per producer record (3 x 256 + 16)
constexpr int HBR1 = 272;  // the one-gate record (256 + 16)
constexpr int HBR4 = 1040; // the LSTM record (4 x 256 + 16)
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
template <int NPW, int NG = 3>
__global__ __launch_bounds__(BW * 64) __attribute__((amdgpu_waves_per_eu(2, 2))) void gru_bwd_h3_kernel(
    int T, int N, int H, int D, int UB, int BT, const float* __restrict__ dy, int dyd,
    const float* __restrict__ w_f, const float* __restrict__ w_r,
    const float* __restrict__ h_all, const float* __restrict__ gates,
    const int* __restrict__ lens, float* __restrict__ dgx, float* __restrict__ dgh,
    float* __restrict__ gx, unsigned* __restrict__ counters, unsigned* __restrict__ err,
    unsigned long long* __restrict__ stamps, double* __restrict__ dbp, int xmode,
    unsigned* __restrict__ camax, int n_base) {
  static_assert(NPW <= 8, "producers per wave");
  static_assert(NG == 3 || NG == 1 || NG == 4, "GRU, one-gate RNN or LSTM");
  constexpr int RP = GU + 1;
  constexpr int HB = NG == 3 ? HBR : (NG == 4 ? HBR4 : HBR1);   // record floats
  constexpr int NO = NG >= 3 ? 2048 : 0;       // byte offset of the n-layout tile (LSTM: hi (g, o))
  constexpr int SO = NG == 3 ? 3072 : (NG == 4 ? 4096 : 1024);  // ... of the row factors
  // producers' records in flight per wave: 2 (GRU at cfg2: 4.84 us per step against 4.86
  // with 1, 5.00 with 3 and 5.11 with 4 -- more loads in flight crowd the fabric the records
  // cross; profiles/r6t_gru_bwd_window.txt; the LSTM's 4-KB records: 2 fit 256 VGPRs)
  constexpr int LWP = NPW < 2 ? NPW : 2;
  constexpr int RED = BW * GB * RP > 8 * GB * GU ? BW * GB * RP : 8 * GB * GU;
  __shared__ __attribute__((aligned(8))) float red[RED];
  __shared__ __attribute__((aligned(16))) _Float16 stg[4 * 64 * 8];   // the record published
  __shared__ __attribute__((aligned(16))) float stsc[GB];
  __shared__ int flag;
  int ub, d, bt;
  // xmode bit 0: same-XCD groups (the workgroup -> (ub, d, bt) mapping and the plain copies).
  // The flags are polled by wave 0, which reaches the poll last (it publishes the record);
  // polling from the last wave, which is done first, measured slower (6.02 vs 4.99 us per
  // step, profiles/r6j_gru_bwd_poll_ab.txt): early polls only load the flag lines the
  // producers are writing.  The round-5 timing diagnostics (no store drain, no wait:
  // profiles/r6i_gru_bwd_handoff_bounds.txt) and the tagged-record hand-off (5.27-5.53 vs
  // 5.00 us per step, profiles/r6m_gru_bwd_tagged_records_ab.txt) were removed in round 6.
  const bool xgrp = (xmode & 1) != 0;
  const bool xg = xgrp;
  if (xgrp ? !map_work_xgrp(UB, BT, D, ub, d, bt) : !map_work(UB * D, BT, UB, ub, d, bt)) return;
  const int n0 = n_base + bt * GB;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int H3 = NG * H;
  unsigned* xtab = counters + (D * BT + 1) + D * BT * 64 + (d * BT + bt) * 64;
  const unsigned my_xcc = xcc_id() + 1u;
  if (xg && threadIdx.x == 0)   // published by the step-0 flag (wave 0 drains before it)
    __hip_atomic_store(xtab + ub, my_xcc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  uint32_t psame = 0;           // bit p: producer p0 + p shares this XCD
  const int p0 = (UB * wave) / BW;
  const int np = (UB * (wave + 1)) / BW - p0;      // host guarantees np <= NPW
  const unsigned* gflags = counters + (D * BT + 1) + (d * BT + bt) * UB;
  unsigned* myflag = counters + (D * BT + 1) + (d * BT + bt) * UB + ub;
  const int slot_floats = D * BT * UB * HB;
  // 2 slots (+ 2 of plain copies with xmode)
  const __amdgpu_buffer_rsrc_t x_rs = __builtin_amdgcn_make_buffer_rsrc(
      gx, (short)0, (xg ? 4 : 2) * slot_floats * 4, 0x00020000);
  const int grp_off = (d * BT + bt) * UB * HB;
  const int aoff = 2 * slot_floats * 4;   // the plain-store copies (xmode)
  const bool tracing = stamps != nullptr && threadIdx.x == 0;
  auto trace_at = [&](int s, int p) {
    if (tracing && s >= kXTraceS0 && s < kXTraceS0 + kXTraceSteps)
      stamps[((int64_t)(s - kXTraceS0) * gridDim.x + blockIdx.x) * 5 + p] =
          __builtin_amdgcn_s_memrealtime();
  };

  // W_hh^T fragments of producer p (unit block pb = p0 + p), lane (u = lane & 15, q = lane >> 4):
  // pair slot j -> W_hh[(j >> 2) H + 16 pb + 4 q + (j & 3)][16 ub + u] (gates r, z), single
  // slot j -> W_hh[2 H + 16 pb + 4 q + j][16 ub + u] (gate n); column u scaled by 2^e(u)
  Duo wrz[NPW];                 // GRU: (r, z); LSTM: (i, f)
  Duo wgo[NPW];                 // LSTM: (g, o)
  f16x4 wnh[NPW], wnl[NPW];
  float unscale = 1.f;   // 2^-e(u) of the owner's unit (threadIdx.x & 15 = lane & 15)
  {
    const float* W = d == 0 ? w_f : w_r;
    const float* wc = W + ub * GU + (lane & 15);
    const int q4 = 4 * (lane >> 4);
    auto wv = [&](int g, int p, int j) {
      return p < np ? wc[(int64_t)(g * H + 16 * (p0 + p) + q4 + j) * H] : 0.f;
    };
    float mx = 0.f;
#pragma unroll
    for (int p = 0; p < NPW; ++p)
#pragma unroll
      for (int g = 0; g < NG; ++g)
#pragma unroll
        for (int j = 0; j < 4; ++j) mx = fmaxf(mx, fabsf(wv(g, p, j)));
    mx = fmaxf(mx, __shfl_xor(mx, 16));
    mx = fmaxf(mx, __shfl_xor(mx, 32));
    if (lane < 16) red[wave * 16 + lane] = mx;
    __syncthreads();
    float m = 0.f;
#pragma unroll
    for (int w8 = 0; w8 < BW; ++w8) m = fmaxf(m, red[w8 * 16 + (lane & 15)]);
    const int eu = h3_row_exp(m);
    unscale = __builtin_ldexpf(1.f, -eu);
    const float sc = __builtin_ldexpf(1.f, eu);
    __syncthreads();
#pragma unroll
    for (int p = 0; p < NPW; ++p) {
      f32x4 a, b, c;
      if constexpr (NG == 4) {
        f32x4 e, f;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          a[j] = wv(0, p, j);
          b[j] = wv(1, p, j);
          e[j] = wv(2, p, j);
          f[j] = wv(3, p, j);
        }
        wrz[p] = split2h(a, b, sc);
        wgo[p] = split2h(e, f, sc);
        continue;
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        a[j] = NG == 3 ? wv(0, p, j) : 0.f;
        b[j] = NG == 3 ? wv(1, p, j) : 0.f;
        c[j] = wv(NG - 1, p, j);
      }
      if constexpr (NG == 3) wrz[p] = split2h(a, b, sc);
      const Duo dn = split2h(c, c, sc);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        wnh[p][j] = dn.hi[j];
        wnl[p][j] = dn.lo[j];
      }
    }
  }
  const int m = (threadIdx.x >> 4) & 15;
  const int u = threadIdx.x & 15;
  const int n = n0 + m;
  const int j = ub * GU + u;
  const bool gate_thread = threadIdx.x < GB * GU;
  const bool owner = gate_thread && n < N;
  int len = owner ? lens[n] : 0;
  settle(len);
  // this thread's slots in the staged record: consumer lane m + 16 (u >> 2), k slot u & 3
  const int sL = (m + 16 * (u >> 2)) * 8 + (u & 3);
  float dh_prev = 0.f, z_prev = 0.f;
  float dc_carry = 0.f;   // LSTM: dc_{t+1} f_{t+1}
  float g_o = 0.f, c_t = 0.f;
  float px_dar = 0.f, px_daz = 0.f, px_dan = 0.f, px_dghn = 0.f;
  int64_t px_row = -1;
  double sb_r = 0.0, sb_z = 0.0, sb_n = 0.0, sb_hn = 0.0;
  // camax: running max |.| of the unit's dar, daz, dan, dghn over the steps (the fp16x3
  // GEMMs' column scales of dgx / dgh, published at the end)
  float cm_r = 0.f, cm_z = 0.f, cm_n = 0.f, cm_hn = 0.f;
  for (int s = 0; s < T; ++s) {
    const int t = d == 0 ? T - 1 - s : s;
    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
    float dyv = 0.f, g_r = 0.f, g_z = 0.f, g_n = 0.f, g_hn = 0.f, hp = 0.f;
    const int64_t row = ((int64_t)t * N + n) * D + d;
    if (owner && t < len) {
      dyv = dy[(((int64_t)t * N + n) * dyd + (dyd > 1 ? d : 0)) * H + j];
      if constexpr (NG == 3) {
        const float* gp = gates + row * 4 * H;
        g_r = gp[j];
        g_z = gp[H + j];
        g_n = gp[2 * H + j];
        g_hn = gp[3 * H + j];
        const int tp = d == 0 ? t - 1 : t + 1;
        if (tp >= 0 && tp < T) hp = h_all[(((int64_t)tp * N + n) * D + d) * H + j];
      } else if constexpr (NG == 4) {
        const float* gp = gates + row * 4 * H;
        g_r = gp[j];                // i
        g_z = gp[H + j];            // f
        g_n = gp[2 * H + j];        // g
        g_o = gp[3 * H + j];        // o
        c_t = h_all[row * H + j];   // c_t (h_all is c_all)
        const int tp = d == 0 ? t - 1 : t + 1;
        if (tp >= 0 && tp < T) hp = h_all[(((int64_t)tp * N + n) * D + d) * H + j];   // c_{t-1}
      } else {
        g_n = h_all[row * H + j];   // h_t
      }
    }
    trace_at(s, 0);
    if (s > 0) {
      if (!flags_wait(gflags, UB, (unsigned)s, err, &flag)) {
        poison_rest(dgx, s, T, d == 0, N, D, n, d, H, j, H3, NG, owner);
        return;
      }
      trace_at(s, 1);
      if (xg && s == 1) {   // which producers share this XCD (their ids came with step 0)
        const unsigned v = lane < UB ? __hip_atomic_load(xtab + lane, __ATOMIC_RELAXED,
                                                         __HIP_MEMORY_SCOPE_AGENT) : 0u;
        const unsigned long long same = __ballot(v == my_xcc);
#pragma unroll
        for (int p = 0; p < NPW; ++p)
          if ((same >> (p0 + p)) & 1ull) psame |= 1u << p;
      }
      const int rb = ((s - 1) & 1) * slot_floats + grp_off;
      u32x4 r0[NPW], r1[NPW], r2[NPW], r3[NPW];
      f32x4 rs[NPW];
      auto load_rec = [&](int p) {
        const bool ok = p < np;
        const int base = (rb + (p0 + p) * HB) * 4 + (((psame >> p) & 1u) ? aoff : 0);
        if constexpr (NG >= 3) {
          r0[p] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                x_rs, ok ? base + lane * 16 : 0x7ffffff0, 0, kSc1));
          r1[p] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                x_rs, ok ? base + 1024 + lane * 16 : 0x7ffffff0, 0, kSc1));
        }
        if constexpr (NG == 4)
          r3[p] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                x_rs, ok ? base + 3072 + lane * 16 : 0x7ffffff0, 0, kSc1));
        r2[p] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                              x_rs, ok ? base + NO + lane * 16 : 0x7ffffff0, 0, kSc1));
        rs[p] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                              x_rs, ok ? base + SO + (lane >> 4) * 16 : 0x7ffffff0, 0, kSc1));
      };
#pragma unroll
      for (int p = 0; p < LWP; ++p) load_rec(p);
      asm volatile("" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int p = 0; p < NPW; ++p) {
        if (p + LWP < NPW) load_rec(p + LWP);
        if (p < np) {
          // big (hi.hi) and small (lo.hi + hi.lo) products in separate zero-C chains, and the
          // 16x16x16 n-gate products apart from the 16x16x32 ones (see mma3h; a 16x16x16 MFMA
          // taking a 16x16x32 result as srcC back to back also got rows 0-1 of every 4 wrong
          // on gfx950: hipcc 7.2 inserts no wait states between the two opcodes)
          const f32x4 z4 = f32x4{0.f, 0.f, 0.f, 0.f};
          f32x4 tb = z4, ts = z4;
          if constexpr (NG >= 3) {
            // runs {hi r, hi z} and {lo r, lo z}
            const f16x8 ahi = __builtin_bit_cast(f16x8, r0[p]);
            const f16x8 alo = __builtin_bit_cast(f16x8, r1[p]);
            ts = __builtin_amdgcn_mfma_f32_16x16x32_f16(alo, wrz[p].hi, ts, 0, 0, 0);
            ts = __builtin_amdgcn_mfma_f32_16x16x32_f16(ahi, wrz[p].lo, ts, 0, 0, 0);
            tb = __builtin_amdgcn_mfma_f32_16x16x32_f16(ahi, wrz[p].hi, tb, 0, 0, 0);
          }
          if constexpr (NG == 4) {
            const f16x8 bhi = __builtin_bit_cast(f16x8, r2[p]);
            const f16x8 blo = __builtin_bit_cast(f16x8, r3[p]);
            ts = __builtin_amdgcn_mfma_f32_16x16x32_f16(blo, wgo[p].hi, ts, 0, 0, 0);
            ts = __builtin_amdgcn_mfma_f32_16x16x32_f16(bhi, wgo[p].lo, ts, 0, 0, 0);
            tb = __builtin_amdgcn_mfma_f32_16x16x32_f16(bhi, wgo[p].hi, tb, 0, 0, 0);
          }
          if constexpr (NG != 4) {
            const f16x4 nh = __builtin_bit_cast(f16x4, u32x2{r2[p][0], r2[p][1]});
            const f16x4 nl = __builtin_bit_cast(f16x4, u32x2{r2[p][2], r2[p][3]});
            f32x4 ns = __builtin_amdgcn_mfma_f32_16x16x16f16(nl, wnh[p], z4, 0, 0, 0);
            ns = __builtin_amdgcn_mfma_f32_16x16x16f16(nh, wnl[p], ns, 0, 0, 0);
            const f32x4 nb = __builtin_amdgcn_mfma_f32_16x16x16f16(nh, wnh[p], z4, 0, 0, 0);
            tb += nb;
            ts += ns;
          }
          const f32x4 tmp = tb + ts;
          acc += tmp * rs[p];   // rows 4 (lane >> 4) + i: the producer's 2^-e of those rows
        }
      }
      trace_at(s, 2);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r)
      red[(wave * GB + (lane >> 4) * 4 + r) * RP + (lane & 15)] = acc[r];
    settle(dyv);
    settle(g_r);
    settle(g_z);
    settle(g_n);
    settle(g_hn);
    settle(hp);
    if constexpr (NG == 4) {
      settle(g_o);
      settle(c_t);
    }
    __syncthreads();
    trace_at(s, 3);
    float dar = 0.f, daz = 0.f, dan = 0.f, dghn = 0.f;
    if (NG == 4 && owner) {
      // the LSTM cell: (dai, daf, dag, dao) carried in (dar, daz, dan, dghn)
      if (t < len) {
        float rec = 0.f;
        if (s > 0) {
#pragma unroll
          for (int w8 = 0; w8 < BW; ++w8) rec += red[(w8 * GB + m) * RP + u];
        }
        const float tc = tanh_fast(c_t);
        const float dh = dyv + rec * unscale;
        const float dc = dc_carry + dh * g_o * (1.f - tc * tc);
        dghn = dh * tc * g_o * (1.f - g_o);
        dar = dc * g_n * g_r * (1.f - g_r);
        dan = dc * g_r * (1.f - g_n * g_n);
        daz = dc * hp * g_z * (1.f - g_z);
        dc_carry = dc * g_z;
      } else {
        dc_carry = 0.f;
      }
      px_dar = dar; px_daz = daz; px_dan = dan; px_dghn = dghn; px_row = row;
      cm_r = fmaxf(cm_r, fabsf(dar));
      cm_z = fmaxf(cm_z, fabsf(daz));
      cm_n = fmaxf(cm_n, fabsf(dan));
      cm_hn = fmaxf(cm_hn, fabsf(dghn));
    } else if (NG == 1 && owner) {
      // the one-gate cell: da = (dy + W_hh^T da_next) (1 - h_t^2), carried in dghn
      float da = 0.f;
      if (t < len) {
        float rec = 0.f;
        if (s > 0) {
#pragma unroll
          for (int w8 = 0; w8 < BW; ++w8) rec += red[(w8 * GB + m) * RP + u];
        }
        da = (dyv + rec * unscale) * (1.f - g_n * g_n);
      }
      dghn = da;
      px_dan = da;
      px_row = row;
      cm_n = fmaxf(cm_n, fabsf(da));
    } else if (owner) {
      float dh = 0.f, zc = 0.f;
      if (t < len) {
        float carry = 0.f;
        if (s > 0) {
          float rec = 0.f;
#pragma unroll
          for (int w8 = 0; w8 < BW; ++w8) rec += red[(w8 * GB + m) * RP + u];
          carry = dh_prev * z_prev + rec * unscale;
        }
        dh = dyv + carry;
        zc = g_z;
        dan = dh * (1.f - zc) * (1.f - g_n * g_n);
        daz = dh * (hp - g_n) * zc * (1.f - zc);
        dar = dan * g_hn * g_r * (1.f - g_r);
        dghn = dan * g_r;
      }
      dh_prev = dh;
      z_prev = zc;
      px_dar = dar; px_daz = daz; px_dan = dan; px_dghn = dghn; px_row = row;
      sb_r += dar; sb_z += daz; sb_n += dan; sb_hn += dghn;
      cm_r = fmaxf(cm_r, fabsf(dar));
      cm_z = fmaxf(cm_z, fabsf(daz));
      cm_n = fmaxf(cm_n, fabsf(dan));
      cm_hn = fmaxf(cm_hn, fabsf(dghn));
    }
    if (gate_thread) {
      // the row's scale: max over the sample's 16 units x 3 gates (16 consecutive lanes)
      float mx = fmaxf(fmaxf(fabsf(dar), fabsf(daz)), fabsf(dghn));
      if constexpr (NG == 4) mx = fmaxf(mx, fabsf(dan));
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
      const int e = h3_row_exp(mx);
      const float sc = __builtin_ldexpf(1.f, e);
      const float vr = dar * sc, vz = daz * sc, vn = dghn * sc;
      const _Float16 hr = (_Float16)vr, hz = (_Float16)vz, hn = (_Float16)vn;
      if constexpr (NG >= 3) {
        stg[sL] = hr;
        stg[sL + 4] = hz;
        stg[512 + sL] = (_Float16)(vr - (float)hr);
        stg[512 + sL + 4] = (_Float16)(vz - (float)hz);
      }
      if constexpr (NG == 4) {   // second pair (g, o): dan, dghn
        const float vg = dan * sc;
        const _Float16 hg = (_Float16)vg;
        stg[1024 + sL] = hg;
        stg[1024 + sL + 4] = hn;
        stg[1536 + sL] = (_Float16)(vg - (float)hg);
        stg[1536 + sL + 4] = (_Float16)(vn - (float)hn);
      } else {
        stg[NO / 2 + sL] = hn;   // the n-layout tile (fp16 offset)
        stg[NO / 2 + sL + 4] = (_Float16)(vn - (float)hn);
      }
      if (u == 0) {
        stsc[m] = __builtin_ldexpf(1.f, -e);
      }
    }
    __syncthreads();
    if (wave == 0) {
      const int so = ((s & 1) * slot_floats + grp_off + ub * HB) * 4;
      // the record's 1-KB tiles: NG 3: (rz hi, rz lo, n); NG 4: (if hi, if lo, go hi, go lo);
      // NG 1: (n)
      constexpr int NT = NG == 4 ? 4 : (NG == 3 ? 3 : 1);
#pragma unroll
      for (int k = 0; k < NT; ++k) {
        const int tk = NG == 1 ? 0 : k;          // stg / record tile index
        const u32x4 v = *reinterpret_cast<const u32x4*>(stg + tk * 512 + lane * 8);
        __builtin_amdgcn_raw_buffer_store_b128(v, x_rs, so + tk * 1024 + lane * 16, 0, kSc1);
        // plain copies: stay in this XCD's L2 for the same-XCD consumers
        if (xg) __builtin_amdgcn_raw_buffer_store_b128(v, x_rs, aoff + so + tk * 1024 + lane * 16, 0, 0);
      }
      if (lane < 4) {
        const u32x4 vs = *reinterpret_cast<const u32x4*>(stsc + lane * 4);
        __builtin_amdgcn_raw_buffer_store_b128(vs, x_rs, so + SO + lane * 16, 0, kSc1);
        if (xg) __builtin_amdgcn_raw_buffer_store_b128(vs, x_rs, aoff + so + SO + lane * 16, 0, 0);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (lane == 0)
        __hip_atomic_store(myflag, (unsigned)s + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    trace_at(s, 4);
    if (NG == 1 && owner) {
      dgx[px_row * H + j] = px_dan;
    } else if (NG == 4 && owner) {
      float* gr = dgx + px_row * H3;
      gr[j] = px_dar;
      gr[H + j] = px_daz;
      gr[2 * H + j] = px_dan;
      gr[3 * H + j] = px_dghn;
    } else if (owner) {
      float* gxr = dgx + px_row * H3;
      gxr[j] = px_dar;
      gxr[H + j] = px_daz;
      gxr[2 * H + j] = px_dan;
      float* ghr = dgh + px_row * H3;
      ghr[j] = px_dar;
      ghr[H + j] = px_daz;
      ghr[2 * H + j] = px_dghn;
    }
  }
  if constexpr (NG == 1) {
    // the one-gate cell: column maxima of da [T N][D H] into camax[0, D H)
    if (camax == nullptr) return;
    __syncthreads();
    if (gate_thread) red[m * GU + u] = cm_n;
    __syncthreads();
    if (threadIdx.x < GU) {
      float a = 0.f;
#pragma unroll
      for (int mm = 0; mm < GB; ++mm) a = fmaxf(a, red[mm * GU + threadIdx.x]);
      const unsigned bits = __float_as_uint(a);
      if (bits != 0u) atomicMax(camax + d * H + ub * GU + threadIdx.x, bits);
    }
    return;
  }
  if constexpr (NG == 4) {
    // column maxima of dgates [T N][D 4H] into camax[0, D 4H)
    if (camax == nullptr) return;
    __syncthreads();
    if (gate_thread) {
      red[(0 * GB + m) * GU + u] = cm_r;
      red[(1 * GB + m) * GU + u] = cm_z;
      red[(2 * GB + m) * GU + u] = cm_n;
      red[(3 * GB + m) * GU + u] = cm_hn;
    }
    __syncthreads();
    if (threadIdx.x < 4 * GU) {
      const int g = threadIdx.x / GU, uu = threadIdx.x - (threadIdx.x / GU) * GU;
      float a = 0.f;
#pragma unroll
      for (int mm = 0; mm < GB; ++mm) a = fmaxf(a, red[(g * GB + mm) * GU + uu]);
      const unsigned bits = __float_as_uint(a);
      if (bits != 0u) atomicMax(camax + d * H3 + g * H + ub * GU + uu, bits);
    }
    return;
  }
  if (camax != nullptr) {
    // column maxima of dgx [T N][D 3H] and dgh: the 16 samples' running maxima per unit, then
    // one unsigned atomic max per (gate, unit) into camax[0, D 3H) (dgx) and [D 3H, 2 D 3H)
    // (dgh; its r, z columns are dgx's, its n column dghn)
    __syncthreads();
    if (gate_thread) {
      red[(0 * GB + m) * GU + u] = cm_r;
      red[(1 * GB + m) * GU + u] = cm_z;
      red[(2 * GB + m) * GU + u] = cm_n;
      red[(3 * GB + m) * GU + u] = cm_hn;
    }
    __syncthreads();
    if (threadIdx.x < 4 * GU) {
      const int g = threadIdx.x / GU, uu = threadIdx.x - (threadIdx.x / GU) * GU;
      float a = 0.f;
#pragma unroll
      for (int mm = 0; mm < GB; ++mm) a = fmaxf(a, red[(g * GB + mm) * GU + uu]);
      const unsigned bits = __float_as_uint(a);
      const int col = d * H3 + ub * GU + uu;
      if (bits != 0u) {
        if (g < 2) {
          atomicMax(camax + col + g * H, bits);
          atomicMax(camax + D * H3 + col + g * H, bits);
        } else if (g == 2) {
          atomicMax(camax + col + 2 * H, bits);
        } else {
          atomicMax(camax + D * H3 + col + 2 * H, bits);
        }
      }
    }
  }
  if (dbp == nullptr) return;
  // the workgroup's 16 samples summed per unit in sample order -> dbp[bt][d][4][H]
  double* rd = reinterpret_cast<double*>(red);
  __syncthreads();
  if (gate_thread) {
    rd[(0 * GB + m) * GU + u] = owner ? sb_r : 0.0;
    rd[(1 * GB + m) * GU + u] = owner ? sb_z : 0.0;
    rd[(2 * GB + m) * GU + u] = owner ? sb_n : 0.0;
    rd[(3 * GB + m) * GU + u] = owner ? sb_hn : 0.0;
  }
  __syncthreads();
  if (threadIdx.x < 4 * GU) {
    const int g = threadIdx.x / GU, uu = threadIdx.x - (threadIdx.x / GU) * GU;
    double a = 0.0;
#pragma unroll
    for (int mm = 0; mm < GB; ++mm) a += rd[(g * GB + mm) * GU + uu];
    dbp[(((int64_t)bt * D + d) * 4 + g) * H + ub * GU + uu] = a;
  }
}

// ---------------------------------------------------------------------------------------
// LSTM backward for cfg4's bf16 mode (BASELINE cfg4: "bf16 MFMA RNN GEMMs"; opt-in, the
// model's rnn_gemm_precision='bf16'): the W_hh^T product with ONE fp16 term per operand
// (per-row scaled gate gradients, per-column scaled W_hh^T, 11 significant bits each instead of
// 22), so a producer's record per 16-sample tile is 2 KB and a workgroup takes 32 samples:
// cfg4's batch 64 runs as ONE launch of 2 x 2 x 64 = 256 workgroups instead of two 16-sample
// chunk launches.  Record per producer and step: [b][(i, f) hi 1 KB, (g, o) hi 1 KB] for the
// two 16-sample tiles b, then 32 row factors 2^-e (4224 B).  Flag hand-off and groups as
// gru_bwd_h3_kernel; `c_all` / `gates` / `dg` as ds2_lstm_bwd.
constexpr int L1B = 32;        // samples per workgroup
constexpr int HBL1 = 1056;     // floats per producer record (2 x 512 + 32)
template <int NPW>
__global__ __launch_bounds__(BW * 64) __attribute__((amdgpu_waves_per_eu(2, 2))) void lstm_bwd_h1_kernel(
    int T, int N, int H, int D, int UB, int BT, const float* __restrict__ dy, int dyd,
    const float* __restrict__ w_f, const float* __restrict__ w_r,
    const float* __restrict__ c_all, const float* __restrict__ gates,
    const int* __restrict__ lens, float* __restrict__ dg, float* __restrict__ gx,
    unsigned* __restrict__ counters, unsigned* __restrict__ err, int xmode,
    unsigned* __restrict__ camax) {
  static_assert(NPW <= 8, "producers per wave");
  static_assert(BW * 64 == L1B * GU, "one thread per (sample, unit)");
  constexpr int RP = GU + 1;
  constexpr int LWP = NPW < 2 ? NPW : 2;       // producers' records in flight per wave
  __shared__ __attribute__((aligned(8))) float red[BW * L1B * RP];
  __shared__ __attribute__((aligned(16))) _Float16 stg[4 * 512];   // the record published
  __shared__ __attribute__((aligned(16))) float stsc[L1B];
  __shared__ int flag;
  int ub, d, bt;
  const bool xg = xmode != 0;
  if (xg ? !map_work_xgrp(UB, BT, D, ub, d, bt) : !map_work(UB * D, BT, UB, ub, d, bt)) return;
  const int n0 = bt * L1B;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int H4 = 4 * H;
  unsigned* xtab = counters + (D * BT + 1) + D * BT * 64 + (d * BT + bt) * 64;
  const unsigned my_xcc = xcc_id() + 1u;
  if (xg && threadIdx.x == 0)
    __hip_atomic_store(xtab + ub, my_xcc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  uint32_t psame = 0;
  const int p0 = (UB * wave) / BW;
  const int np = (UB * (wave + 1)) / BW - p0;      // host guarantees np <= NPW
  const unsigned* gflags = counters + (D * BT + 1) + (d * BT + bt) * UB;
  unsigned* myflag = counters + (D * BT + 1) + (d * BT + bt) * UB + ub;
  const int slot_floats = D * BT * UB * HBL1;
  const __amdgpu_buffer_rsrc_t x_rs = __builtin_amdgcn_make_buffer_rsrc(
      gx, (short)0, (xg ? 4 : 2) * slot_floats * 4, 0x00020000);
  const int grp_off = (d * BT + bt) * UB * HBL1;
  const int aoff = 2 * slot_floats * 4;   // the plain-store copies (xmode)

  // W_hh^T fragments of producer p, lane (u = lane & 15, q = lane >> 4), hi terms only:
  // slot j -> W_hh[(g0 + (j >> 2)) H + 16 pb + 4 q + (j & 3)][16 ub + u], g0 = 0 (i, f) / 2 (g, o)
  f16x8 wif[NPW], wgo[NPW];
  float unscale = 1.f;   // 2^-e(u) of the owner's unit (threadIdx.x & 15 = lane & 15)
  {
    const float* W = d == 0 ? w_f : w_r;
    const float* wc = W + ub * GU + (lane & 15);
    const int q4 = 4 * (lane >> 4);
    auto wv = [&](int g, int p, int j) {
      return p < np ? wc[(int64_t)(g * H + 16 * (p0 + p) + q4 + j) * H] : 0.f;
    };
    float mx = 0.f;
#pragma unroll
    for (int p = 0; p < NPW; ++p)
#pragma unroll
      for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int j = 0; j < 4; ++j) mx = fmaxf(mx, fabsf(wv(g, p, j)));
    mx = fmaxf(mx, __shfl_xor(mx, 16));
    mx = fmaxf(mx, __shfl_xor(mx, 32));
    if (lane < 16) red[wave * 16 + lane] = mx;
    __syncthreads();
    float m = 0.f;
#pragma unroll
    for (int w8 = 0; w8 < BW; ++w8) m = fmaxf(m, red[w8 * 16 + (lane & 15)]);
    const int eu = h3_row_exp(m);
    unscale = __builtin_ldexpf(1.f, -eu);
    const float sc = __builtin_ldexpf(1.f, eu);
    __syncthreads();
#pragma unroll
    for (int p = 0; p < NPW; ++p)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        wif[p][j] = (_Float16)(wv(j >> 2, p, j & 3) * sc);
        wgo[p][j] = (_Float16)(wv(2 + (j >> 2), p, j & 3) * sc);
      }
  }
  const int m = threadIdx.x >> 4;        // sample of the workgroup (0 .. 31)
  const int u = threadIdx.x & 15;
  const int n = n0 + m;
  const int j = ub * GU + u;
  const bool owner = n < N;
  int len = owner ? lens[n] : 0;
  settle(len);
  // this thread's slots in the staged record: tile b = m >> 4, consumer lane (m & 15) + 16 (u >> 2)
  const int sL = (m >> 4) * 1024 + ((m & 15) + 16 * (u >> 2)) * 8 + (u & 3);
  float dc_carry = 0.f;
  float p_i = 0.f, p_f = 0.f, p_g = 0.f, p_o = 0.f;
  int64_t px_row = -1;
  float cm_i = 0.f, cm_f = 0.f, cm_g = 0.f, cm_o = 0.f;
  for (int s = 0; s < T; ++s) {
    const int t = d == 0 ? T - 1 - s : s;
    f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
    float dyv = 0.f, gi = 0.f, gf = 0.f, gg = 0.f, go = 0.f, ct = 0.f, cp = 0.f;
    const int64_t row = ((int64_t)t * N + n) * D + d;
    if (owner && t < len) {
      dyv = dy[(((int64_t)t * N + n) * dyd + (dyd > 1 ? d : 0)) * H + j];
      const float* gp = gates + row * 4 * H;
      gi = gp[j];
      gf = gp[H + j];
      gg = gp[2 * H + j];
      go = gp[3 * H + j];
      ct = c_all[row * H + j];
      const int tp = d == 0 ? t - 1 : t + 1;
      if (tp >= 0 && tp < T) cp = c_all[(((int64_t)tp * N + n) * D + d) * H + j];
    }
    if (s > 0) {
      if (!flags_wait(gflags, UB, (unsigned)s, err, &flag)) {
        poison_rest(dg, s, T, d == 0, N, D, n, d, H, j, H4, 4, owner);
        return;
      }
      if (xg && s == 1) {
        const unsigned v = lane < UB ? __hip_atomic_load(xtab + lane, __ATOMIC_RELAXED,
                                                         __HIP_MEMORY_SCOPE_AGENT) : 0u;
        const unsigned long long same = __ballot(v == my_xcc);
#pragma unroll
        for (int p = 0; p < NPW; ++p)
          if ((same >> (p0 + p)) & 1ull) psame |= 1u << p;
      }
      const int rb = ((s - 1) & 1) * slot_floats + grp_off;
      u32x4 ra[NPW][2], rg[NPW][2];
      f32x4 rs[NPW][2];
      auto load_rec = [&](int p) {
        const bool ok = p < np;
        const int base = (rb + (p0 + p) * HBL1) * 4 + (((psame >> p) & 1u) ? aoff : 0);
#pragma unroll
        for (int b = 0; b < 2; ++b) {
          ra[p][b] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                   x_rs, ok ? base + b * 2048 + lane * 16 : 0x7ffffff0, 0, kSc1));
          rg[p][b] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                   x_rs, ok ? base + b * 2048 + 1024 + lane * 16 : 0x7ffffff0, 0, kSc1));
          rs[p][b] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                   x_rs, ok ? base + 4096 + b * 64 + (lane >> 4) * 16 : 0x7ffffff0, 0, kSc1));
        }
      };
#pragma unroll
      for (int p = 0; p < LWP; ++p) load_rec(p);
      asm volatile("" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int p = 0; p < NPW; ++p) {
        if (p + LWP < NPW) load_rec(p + LWP);
        if (p < np) {
#pragma unroll
          for (int b = 0; b < 2; ++b) {
            f32x4 tb = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, ra[p][b]), wif[p],
                                                              f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
            tb = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, rg[p][b]), wgo[p], tb, 0, 0, 0);
            acc[b] += tb * rs[p][b];
          }
        }
      }
    }
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        red[(wave * L1B + b * GB + (lane >> 4) * 4 + r) * RP + (lane & 15)] = acc[b][r];
    settle(dyv);
    settle(gi);
    settle(gf);
    settle(gg);
    settle(go);
    settle(ct);
    settle(cp);
    __syncthreads();
    float dai = 0.f, daf = 0.f, dag = 0.f, dao = 0.f;
    if (owner) {
      if (t < len) {
        float rec = 0.f;
        if (s > 0) {
#pragma unroll
          for (int w8 = 0; w8 < BW; ++w8) rec += red[(w8 * L1B + m) * RP + u];
        }
        const float tc = tanh_fast(ct);
        const float dh = dyv + rec * unscale;
        const float dc = dc_carry + dh * go * (1.f - tc * tc);
        dao = dh * tc * go * (1.f - go);
        dai = dc * gg * gi * (1.f - gi);
        dag = dc * gi * (1.f - gg * gg);
        daf = dc * cp * gf * (1.f - gf);
        dc_carry = dc * gf;
      } else {
        dc_carry = 0.f;
      }
      p_i = dai; p_f = daf; p_g = dag; p_o = dao; px_row = row;
      cm_i = fmaxf(cm_i, fabsf(dai));
      cm_f = fmaxf(cm_f, fabsf(daf));
      cm_g = fmaxf(cm_g, fabsf(dag));
      cm_o = fmaxf(cm_o, fabsf(dao));
    }
    {
      // the row's scale: max over the sample's 16 units x 4 gates (16 consecutive lanes)
      float mx = fmaxf(fmaxf(fabsf(dai), fabsf(daf)), fmaxf(fabsf(dag), fabsf(dao)));
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
      const int e = h3_row_exp(mx);
      const float sc = __builtin_ldexpf(1.f, e);
      stg[sL] = (_Float16)(dai * sc);
      stg[sL + 4] = (_Float16)(daf * sc);
      stg[sL + 512] = (_Float16)(dag * sc);
      stg[sL + 516] = (_Float16)(dao * sc);
      if (u == 0) stsc[m] = __builtin_ldexpf(1.f, -e);
    }
    __syncthreads();
    if (wave == 0) {
      const int so = ((s & 1) * slot_floats + grp_off + ub * HBL1) * 4;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const u32x4 v = *reinterpret_cast<const u32x4*>(stg + k * 512 + lane * 8);
        __builtin_amdgcn_raw_buffer_store_b128(v, x_rs, so + k * 1024 + lane * 16, 0, kSc1);
        if (xg) __builtin_amdgcn_raw_buffer_store_b128(v, x_rs, aoff + so + k * 1024 + lane * 16, 0, 0);
      }
      if (lane < 8) {
        const u32x4 vs = *reinterpret_cast<const u32x4*>(stsc + lane * 4);
        __builtin_amdgcn_raw_buffer_store_b128(vs, x_rs, so + 4096 + lane * 16, 0, kSc1);
        if (xg) __builtin_amdgcn_raw_buffer_store_b128(vs, x_rs, aoff + so + 4096 + lane * 16, 0, 0);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (lane == 0)
        __hip_atomic_store(myflag, (unsigned)s + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (owner) {
      float* gr = dg + px_row * H4;
      gr[j] = p_i;
      gr[H + j] = p_f;
      gr[2 * H + j] = p_g;
      gr[3 * H + j] = p_o;
    }
  }
  if (camax == nullptr) return;
  // column maxima of dg [T N][D 4H]: the 32 samples' running maxima per (gate, unit)
  __syncthreads();
  red[(0 * L1B + m) * GU + u] = cm_i;
  red[(1 * L1B + m) * GU + u] = cm_f;
  red[(2 * L1B + m) * GU + u] = cm_g;
  red[(3 * L1B + m) * GU + u] = cm_o;
  __syncthreads();
  if (threadIdx.x < 4 * GU) {
    const int g = threadIdx.x / GU, uu = threadIdx.x - (threadIdx.x / GU) * GU;
    float a = 0.f;
#pragma unroll
    for (int mm = 0; mm < L1B; ++mm) a = fmaxf(a, red[(g * L1B + mm) * GU + uu]);
    const unsigned bits = __float_as_uint(a);
    if (bits != 0u) atomicMax(camax + d * H4 + g * H + ub * GU + uu, bits);
  }
}

// ---------------------------------------------------------------------------------------
// host launchers (called by ds2_gru_fwd / ds2_gru_bwd in gru.hip with their workspace
// carve-up); false = shape not covered (caller falls back to the fp32-MFMA kernels)

// on by default; DS2_GRU_X6=0 selects the fp32-MFMA kernels (gru.hip: the accuracy
// cross-check of the tests)
static inline bool x6_enabled() {
  const char* e = getenv("DS2_GRU_X6");
  return !(e != nullptr && e[0] == '0');
}

// the forward's W_hh product on fp16x3 (default since round 5; DS2_GRU_H3=0 keeps bf16x6)
static inline bool fwd_h3_enabled() {
  const char* e = getenv("DS2_GRU_H3");
  return !(e != nullptr && e[0] == '0');
}

static const void* fwd_x6_fn(int need) {
  const bool h3 = fwd_h3_enabled();
#define DS2_FX6(K)                                                                  \
  if (need <= K)                                                                    \
    return h3 ? reinterpret_cast<const void*>(gru_fwd_x6_kernel<K, true>)           \
              : reinterpret_cast<const void*>(gru_fwd_x6_kernel<K, false>);
  DS2_FX6(1) DS2_FX6(2) DS2_FX6(3) DS2_FX6(4) DS2_FX6(5) DS2_FX6(6) DS2_FX6(7)
#undef DS2_FX6
  return nullptr;
}

static const void* bwd_x6_fn(int pairs) {
  const int need = (pairs + BW - 1) / BW;
#define DS2_BP6(K) \
  if (need <= K) return reinterpret_cast<const void*>(gru_bwd_x6_kernel<K>);
  DS2_BP6(1) DS2_BP6(2) DS2_BP6(3) DS2_BP6(4) DS2_BP6(6) DS2_BP6(8) DS2_BP6(10) DS2_BP6(12)
#undef DS2_BP6
  return nullptr;
}

// same-XCD hand-off groups (rnn_common.h map_work_xgrp), default on where the groups tile the
// 8 XCDs: cfg2 backward 5.82 -> 5.43 us per step in isolation, 6.14 -> 5.69 in the training
// step; DS2_GRU_XCD=0 keeps map_work's interleaved layout (bit-identical results)
static inline bool xcd_groups(int UB, int BT, int num_dirs) {
  return xcd_groups_on() && xgrp_fits(UB, BT, num_dirs);
}

bool launch_gru_fwd_x6(int t_max, int n, int h, int num_dirs, const float* xproj,
                       const float* w_hh_f, const float* w_hh_r, const float* b_hh_f,
                       const float* b_hh_r, const int* lens, float* h_all, float* gates,
                       float* ring, unsigned* ctrs, unsigned* err, unsigned long long* stamps,
                       size_t lds_pad, hipStream_t st) {
  if (!x6_enabled() || (h % GU) != 0) return false;
  apply_spin_limit_env();     // this translation unit's copies of the device knobs
  apply_rnn_tune_env();
  const int UB = h / GU, BT = (n + GB - 1) / GB;
  const int need = ((UB + 1) / 2 + XW - 1) / XW;
  const void* fn = fwd_x6_fn(need);
  if (fn == nullptr) return false;
  int XM_ = xcd_groups(UB, BT, num_dirs) ? 1 : 0;
  const int grid = XM_ ? xgrp_grid(UB, BT, num_dirs) : mapped_grid(UB * num_dirs, BT);
  int T_ = t_max, N_ = n, H_ = h, D_ = num_dirs, UB_ = UB, BT_ = BT;
  void* args[] = {&T_, &N_, &H_, &D_, &UB_, &BT_, &xproj, &w_hh_f, &w_hh_r, &b_hh_f,
                  &b_hh_r, &lens, &h_all, &gates, &ring, &ctrs, &err, &stamps, &XM_};
  return rnn_launch(fn, dim3(grid), dim3(XT), args, lds_pad, st) == hipSuccess;
}

// grid of the x6 backward launch_gru_bwd_x6 would make, -1 if it declines the shape
int gru_bwd_x6_grid(int n, int h, int num_dirs) {
  if (!x6_enabled() || (h % GU) != 0) return -1;
  const int UB = h / GU, BT = (n + GB - 1) / GB;
  if (bwd_x6_fn((3 * UB + 1) / 2) == nullptr) return -1;
  return xcd_groups(UB, BT, num_dirs) ? xgrp_grid(UB, BT, num_dirs)
                                      : mapped_grid(UB * num_dirs, BT);
}

// the backward's W_hh^T product on fp16x3 (default since round 5; DS2_GRU_H3_BWD=0 keeps
// the bf16x6 pre-split kernel)
static inline bool bwd_h3_enabled() {
  const char* e = getenv("DS2_GRU_H3_BWD");
  return !(e != nullptr && e[0] == '0');
}

static const void* bwd_h3_fn(int UB) {
  const int need = (UB + BW - 1) / BW;
#define DS2_BH3(K) \
  if (need <= K) return reinterpret_cast<const void*>(gru_bwd_h3_kernel<K>);
  DS2_BH3(1) DS2_BH3(2) DS2_BH3(3) DS2_BH3(4) DS2_BH3(5) DS2_BH3(6) DS2_BH3(7) DS2_BH3(8)
#undef DS2_BH3
  return nullptr;
}

// camax (nullable, zeroed by the caller): the fp16x3 backward also leaves the column maxima
// of dgates_x / dgates_h there; *camax_done says whether the kernel that ran did
bool launch_gru_bwd_x6(int t_max, int n, int h, int num_dirs, const float* dy, int dy_dirs,
                       const float* w_hh_f, const float* w_hh_r, const float* h_all,
                       const float* gates, const int* lens, float* dgates_x, float* dgates_h,
                       float* ring, unsigned* ctrs, unsigned* err, unsigned long long* stamps,
                       double* dbp, size_t lds_pad, hipStream_t st, unsigned* camax,
                       bool* camax_done) {
  if (camax_done != nullptr) *camax_done = false;
  if (!x6_enabled() || (h % GU) != 0) return false;
  apply_spin_limit_env();
  apply_rnn_tune_env();
  const int UB = h / GU, BT = (n + GB - 1) / GB;
  const void* fn = bwd_h3_enabled() ? bwd_h3_fn(UB) : nullptr;
  const bool h3 = fn != nullptr;
  if (fn == nullptr) fn = bwd_x6_fn((3 * UB + 1) / 2);
  if (fn == nullptr) return false;
  int XM_ = xcd_groups(UB, BT, num_dirs) ? 1 : 0;
  const int grid = XM_ ? xgrp_grid(UB, BT, num_dirs) : mapped_grid(UB * num_dirs, BT);
  int T_ = t_max, N_ = n, H_ = h, D_ = num_dirs, UB_ = UB, BT_ = BT, DYD_ = dy_dirs, NB_ = 0;
  void* args[] = {&T_, &N_, &H_, &D_, &UB_, &BT_, &dy, &DYD_, &w_hh_f, &w_hh_r, &h_all,
                  &gates, &lens, &dgates_x, &dgates_h, &ring, &ctrs, &err, &stamps, &dbp, &XM_,
                  &camax, &NB_};
  const bool ok = rnn_launch(fn, dim3(grid), dim3(BW * 64), args, lds_pad, st) == hipSuccess;
  if (ok && h3 && camax != nullptr && camax_done != nullptr) *camax_done = true;
  return ok;
}


// ---------------------------------------------------------------------------------------
// supported_rnns['rnn'] (nn.RNN, tanh) on the same machinery: the one-gate instantiations of
// the fp16x3 forward / backward (NG = 1), same groups, hand-offs and rings (ds2_rnn_fwd_ws /
// ds2_rnn_bwd_ws in gru.hip carve the workspace).  false = not covered (caller falls back to
// the per-step kernels of rnn.hip).
static const void* rnn_fwd_fn(int need) {
#define DS2_RF(K) \
  if (need <= K) return reinterpret_cast<const void*>(gru_fwd_x6_kernel<K, true, 1>);
  DS2_RF(1) DS2_RF(2) DS2_RF(3) DS2_RF(4) DS2_RF(5) DS2_RF(6) DS2_RF(7)
#undef DS2_RF
  return nullptr;
}

static const void* rnn_bwd_fn(int UB) {
  const int need = (UB + BW - 1) / BW;
#define DS2_RB(K) \
  if (need <= K) return reinterpret_cast<const void*>(gru_bwd_h3_kernel<K, 1>);
  DS2_RB(1) DS2_RB(2) DS2_RB(3) DS2_RB(4) DS2_RB(5) DS2_RB(6) DS2_RB(7) DS2_RB(8)
#undef DS2_RB
  return nullptr;
}

bool launch_rnn_fwd_h3(int t_max, int n, int h, int num_dirs, const float* xproj,
                       const float* w_hh_f, const float* w_hh_r, const float* b_hh_f,
                       const float* b_hh_r, const int* lens, float* h_all, float* ring,
                       unsigned* ctrs, unsigned* err, unsigned long long* stamps, size_t lds_pad,
                       hipStream_t st) {
  if ((h % GU) != 0) return false;
  apply_spin_limit_env();
  apply_rnn_tune_env();
  const int UB = h / GU, BT = (n + GB - 1) / GB;
  const void* fn = rnn_fwd_fn(((UB + 1) / 2 + XW - 1) / XW);
  if (fn == nullptr) return false;
  int XM_ = xcd_groups(UB, BT, num_dirs) ? 1 : 0;
  const int grid = XM_ ? xgrp_grid(UB, BT, num_dirs) : mapped_grid(UB * num_dirs, BT);
  int T_ = t_max, N_ = n, H_ = h, D_ = num_dirs, UB_ = UB, BT_ = BT;
  float* gates = nullptr;
  void* args[] = {&T_, &N_, &H_, &D_, &UB_, &BT_, &xproj, &w_hh_f, &w_hh_r, &b_hh_f,
                  &b_hh_r, &lens, &h_all, &gates, &ring, &ctrs, &err, &stamps, &XM_};
  return rnn_launch(fn, dim3(grid), dim3(XT), args, lds_pad, st) == hipSuccess;
}

// dgates: [T][N][D][H] gradient wrt the pre-activation; camax (nullable, zeroed by the
// caller): its column maxima
bool launch_rnn_bwd_h3(int t_max, int n, int h, int num_dirs, const float* dy, int dy_dirs,
                       const float* w_hh_f, const float* w_hh_r, const float* h_all,
                       const int* lens, float* dgates, float* ring, unsigned* ctrs, unsigned* err,
                       unsigned long long* stamps, size_t lds_pad, hipStream_t st,
                       unsigned* camax) {
  if ((h % GU) != 0) return false;
  apply_spin_limit_env();
  apply_rnn_tune_env();
  const int UB = h / GU, BT = (n + GB - 1) / GB;
  const void* fn = rnn_bwd_fn(UB);
  if (fn == nullptr) return false;
  int XM_ = xcd_groups(UB, BT, num_dirs) ? 1 : 0;
  const int grid = XM_ ? xgrp_grid(UB, BT, num_dirs) : mapped_grid(UB * num_dirs, BT);
  int T_ = t_max, N_ = n, H_ = h, D_ = num_dirs, UB_ = UB, BT_ = BT, DYD_ = dy_dirs, NB_ = 0;
  const float* gates = nullptr;
  float* dgh = nullptr;
  double* dbp = nullptr;
  void* args[] = {&T_, &N_, &H_, &D_, &UB_, &BT_, &dy, &DYD_, &w_hh_f, &w_hh_r, &h_all,
                  &gates, &lens, &dgates, &dgh, &ring, &ctrs, &err, &stamps, &dbp, &XM_,
                  &camax, &NB_};
  return rnn_launch(fn, dim3(grid), dim3(BW * 64), args, lds_pad, st) == hipSuccess;
}

// grid of the one-gate launches, -1 if they decline the shape
int rnn_h3_grid(int n, int h, int num_dirs) {
  if ((h % GU) != 0) return -1;
  const int UB = h / GU, BT = (n + GB - 1) / GB;
  if (rnn_bwd_fn(UB) == nullptr || rnn_fwd_fn(((UB + 1) / 2 + XW - 1) / XW) == nullptr) return -1;
  return xcd_groups(UB, BT, num_dirs) ? xgrp_grid(UB, BT, num_dirs) : mapped_grid(UB * num_dirs, BT);
}

// supported_rnns['lstm'] backward on the same machinery (NG = 4): one launch over the
// 16-sample tiles [tile0, tile0 + BT_launch) of the batch (the caller runs consecutive chunks
// when all tiles would not fit the chip); ring and counters sized for BT_launch groups.
// camax (nullable, zeroed by the caller): column maxima of dgates over every launch.
static const void* lstm_bwd_fn(int UB) {
  const int need = (UB + BW - 1) / BW;
#define DS2_LB(K) \
  if (need <= K) return reinterpret_cast<const void*>(gru_bwd_h3_kernel<K, 4>);
  DS2_LB(1) DS2_LB(2) DS2_LB(3) DS2_LB(4) DS2_LB(5) DS2_LB(6) DS2_LB(7) DS2_LB(8)
#undef DS2_LB
  return nullptr;
}

// grid of one LSTM fp16x3 backward launch over bt_launch tiles, -1 if it declines the shape
int lstm_h3_grid(int h, int num_dirs, int bt_launch) {
  if ((h % GU) != 0) return -1;
  const int UB = h / GU;
  if (lstm_bwd_fn(UB) == nullptr) return -1;
  return xcd_groups(UB, bt_launch, num_dirs) ? xgrp_grid(UB, bt_launch, num_dirs)
                                            : mapped_grid(UB * num_dirs, bt_launch);
}

bool launch_lstm_bwd_h3(int t_max, int n, int h, int num_dirs, const float* dy, int dy_dirs,
                        const float* w_hh_f, const float* w_hh_r, const float* c_all,
                        const float* gates, const int* lens, float* dgates, float* ring,
                        unsigned* ctrs, unsigned* err, size_t lds_pad, hipStream_t st,
                        unsigned* camax, int tile0, int bt_launch) {
  if ((h % GU) != 0) return false;
  apply_spin_limit_env();
  apply_rnn_tune_env();
  const int UB = h / GU;
  const void* fn = lstm_bwd_fn(UB);
  if (fn == nullptr) return false;
  int XM_ = xcd_groups(UB, bt_launch, num_dirs) ? 1 : 0;
  const int grid = XM_ ? xgrp_grid(UB, bt_launch, num_dirs) : mapped_grid(UB * num_dirs, bt_launch);
  int T_ = t_max, N_ = n, H_ = h, D_ = num_dirs, UB_ = UB, BT_ = bt_launch, DYD_ = dy_dirs;
  int NB_ = tile0 * GB;
  float* dgh = nullptr;
  double* dbp = nullptr;
  unsigned long long* stamps = nullptr;
  void* args[] = {&T_, &N_, &H_, &D_, &UB_, &BT_, &dy, &DYD_, &w_hh_f, &w_hh_r, &c_all,
                  &gates, &lens, &dgates, &dgh, &ring, &ctrs, &err, &stamps, &dbp, &XM_,
                  &camax, &NB_};
  return rnn_launch(fn, dim3(grid), dim3(BW * 64), args, lds_pad, st) == hipSuccess;
}

// ring bytes of the fp16x3 backward records (2 slots, doubled for the same-XCD plain copies)
size_t h3_bwd_ring_bytes(int n_tiles, int h, int num_dirs, int ng) {
  const size_t UB = (h + GU - 1) / GU;
  const size_t hb = ng == 4 ? HBR4 : (ng == 3 ? HBR : HBR1);
  return 4 * (size_t)num_dirs * n_tiles * UB * hb * sizeof(float);
}

// the single-term LSTM backward (cfg4's bf16 mode): one launch over ceil(n / 32) 32-sample
// tiles; false = not covered
static const void* lstm_bwd_h1_fn(int UB) {
  const int need = (UB + BW - 1) / BW;
#define DS2_L1(K) \
  if (need <= K) return reinterpret_cast<const void*>(lstm_bwd_h1_kernel<K>);
  DS2_L1(1) DS2_L1(2) DS2_L1(4) DS2_L1(8)
#undef DS2_L1
  return nullptr;
}

int lstm_h1_grid(int n, int h, int num_dirs) {
  if ((h % GU) != 0) return -1;
  const int UB = h / GU, BT = (n + L1B - 1) / L1B;
  if (lstm_bwd_h1_fn(UB) == nullptr) return -1;
  return xcd_groups(UB, BT, num_dirs) ? xgrp_grid(UB, BT, num_dirs) : mapped_grid(UB * num_dirs, BT);
}

size_t lstm_h1_ring_bytes(int n, int h, int num_dirs) {
  const size_t UB = (h + GU - 1) / GU, BT = (n + L1B - 1) / L1B;
  return 4 * (size_t)num_dirs * BT * UB * HBL1 * sizeof(float);
}

bool launch_lstm_bwd_h1(int t_max, int n, int h, int num_dirs, const float* dy, int dy_dirs,
                        const float* w_hh_f, const float* w_hh_r, const float* c_all,
                        const float* gates, const int* lens, float* dgates, float* ring,
                        unsigned* ctrs, unsigned* err, size_t lds_pad, hipStream_t st,
                        unsigned* camax) {
  if ((h % GU) != 0) return false;
  apply_spin_limit_env();
  apply_rnn_tune_env();
  const int UB = h / GU, BT = (n + L1B - 1) / L1B;
  const void* fn = lstm_bwd_h1_fn(UB);
  if (fn == nullptr) return false;
  int XM_ = xcd_groups(UB, BT, num_dirs) ? 1 : 0;
  const int grid = XM_ ? xgrp_grid(UB, BT, num_dirs) : mapped_grid(UB * num_dirs, BT);
  int T_ = t_max, N_ = n, H_ = h, D_ = num_dirs, UB_ = UB, BT_ = BT, DYD_ = dy_dirs;
  void* args[] = {&T_, &N_, &H_, &D_, &UB_, &BT_, &dy, &DYD_, &w_hh_f, &w_hh_r, &c_all,
                  &gates, &lens, &dgates, &ring, &ctrs, &err, &XM_, &camax};
  return rnn_launch(fn, dim3(grid), dim3(BW * 64), args, lds_pad, st) == hipSuccess;
}

}  // namespace ds2
