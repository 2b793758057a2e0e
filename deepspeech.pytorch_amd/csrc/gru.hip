// Bidirectional GRU recurrence on MFMA (v_mfma_f32_16x16x4_f32), fp32.
//
// The input projection (x @ W_ih^T + b_ih, both directions) is a separate big
// GEMM; this file only runs the sequential part.  One launch per time step
// (kernel boundaries give the step-to-step ordering/visibility for free); both
// directions advance in the same launch: direction 0 processes t = s, direction
// 1 processes t = T-1-s, so a sample of length len starts its reverse pass at
// t = len-1 from h = 0 exactly like pack_padded_sequence (model.py:103-105).
//
// Work split per launch: workgroup = (16 hidden units, direction, 16 samples).
//   forward : gh[16 x 48] = h_prev[16 x H] @ W_hh[48 rows (r,z,n of the 16 units)]^T
//   backward: rec[16 x 16] = dgh[16 x 3H] @ W_hh[:, 16 units]
// The K dimension is split over the 4 waves, partial tiles reduced through LDS,
// then one thread per (sample, unit) applies the gate math.  W_hh is repacked
// once per call into MFMA-fragment order so every B-operand load of a wave is a
// single coalesced 256-byte read.
//
// Gate math follows ATen's GRU cell (gate rows ordered r, z, n):
//   r = sigmoid(hr + xr), z = sigmoid(hz + xz), n = tanh(xn + r*hn),
//   h' = (h - n) * z + n
#include "rnn_common.h"

#include <algorithm>

namespace ds2 {

constexpr int KC_FWD = 1024;   // max H staged in LDS (forward)
constexpr int KC_BWD = 2400;   // max 3H chunk staged in LDS (backward)
constexpr int kTraceS0 = 100, kTraceSteps = 16;   // DS2_GRU_STAMPS=2 trace window

// ---------------------------------------------------------------------------
// forward step.  KSW = k-steps of W prefetched into registers per wave.
template <int KSW>
__global__ __launch_bounds__(GT) void gru_fwd_step_kernel(
    int s, int T, int N, int H, int D, int UB, int BT, const float* __restrict__ xproj,
    const float* __restrict__ wp, const float* __restrict__ b_f, const float* __restrict__ b_r,
    const int* __restrict__ lens, float* __restrict__ h_all, float* __restrict__ gates) {
  constexpr int PITCH = KC_FWD + 2;
  __shared__ __attribute__((aligned(16))) float hs[GB * PITCH];
  int ub, d, bt;
  if (!map_work(UB * D, BT, UB, ub, d, bt)) return;
  const int n0 = bt * GB;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // provably uniform
  const int t = d == 0 ? s : T - 1 - s;
  const int tp = d == 0 ? t - 1 : t + 1;
  const int KS = (H + 3) / 4;
  const int per = (KS + GW - 1) / GW;
  const int a_ks = wave * per;
  const int b_ks = min(KS, a_ks + per);

  f32x4 acc[3];
#pragma unroll
  for (int g = 0; g < 3; ++g) acc[g] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (s > 0) {
    // W fragments first: every load of this wave is in flight before the h staging
    float w[3][KSW];
    const float* wpd = wp + ((int64_t)d * UB + ub) * KS * 3 * 64 + lane;
#pragma unroll
    for (int i = 0; i < KSW; ++i) {
      const int ks = a_ks + i;
#pragma unroll
      for (int g = 0; g < 3; ++g) w[g][i] = ks < b_ks ? wpd[((int64_t)ks * 3 + g) * 64] : 0.f;
    }
    const float* hprev = h_all + ((int64_t)tp * N * D + d) * H;   // row n at + n*D*H
    stage_rows(hprev, (int64_t)D * H, N, n0, 0, H, hs, PITCH);
    __syncthreads();
    const float* hrow = hs + (lane & 15) * PITCH + (lane >> 4);
#pragma unroll
    for (int i = 0; i < KSW; ++i) {
      const int ks = a_ks + i;
      if (ks < b_ks) {
        const int k = 4 * ks;
        const float a = (k + (lane >> 4) < H) ? hrow[k] : 0.f;
        acc[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, w[0][i], acc[0], 0, 0, 0);
        acc[1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, w[1][i], acc[1], 0, 0, 0);
        acc[2] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, w[2][i], acc[2], 0, 0, 0);
      }
    }
    __syncthreads();   // hs is reused as the reduction buffer below
  }
  // partial tiles -> LDS: red[wave][m][g*16+u], C/D map col = lane&15, row = (lane>>4)*4+r
  float* red = hs;
  constexpr int RP = 3 * GU + 1;
#pragma unroll
  for (int g = 0; g < 3; ++g)
#pragma unroll
    for (int r = 0; r < 4; ++r)
      red[(wave * GB + (lane >> 4) * 4 + r) * RP + g * GU + (lane & 15)] = acc[g][r];
  __syncthreads();
  if (threadIdx.x >= GB * GU) return;

  const int m = threadIdx.x >> 4;       // sample within the tile
  const int u = threadIdx.x & 15;       // unit within the block
  const int n = n0 + m;
  const int j = ub * GU + u;
  if (n >= N || j >= H) return;
  float gh[3];
#pragma unroll
  for (int g = 0; g < 3; ++g) {
    float v = 0.f;
#pragma unroll
    for (int w8 = 0; w8 < GW; ++w8) v += red[(w8 * GB + m) * RP + g * GU + u];
    gh[g] = v;
  }
  const float* bh = d == 0 ? b_f : b_r;
  const float ghr = gh[0] + bh[j];
  const float ghz = gh[1] + bh[H + j];
  float ghn = gh[2] + bh[2 * H + j];
  const int64_t row = ((int64_t)t * N + n) * D + d;
  const bool active = t < lens[n];
  float hout = 0.f, r = 0.f, z = 0.f, nn = 0.f;
  if (active) {
    const float* xp = xproj + row * 3 * H;
    const float hp = s > 0 ? h_all[(((int64_t)tp * N + n) * D + d) * H + j] : 0.f;
    r = sigmoidf_(ghr + xp[j]);
    z = sigmoidf_(ghz + xp[H + j]);
    nn = tanhf(xp[2 * H + j] + r * ghn);
    hout = (hp - nn) * z + nn;
  } else {
    ghn = 0.f;
  }
  h_all[row * H + j] = hout;
  if (gates != nullptr) {
    float* gp = gates + row * 4 * H;
    gp[j] = r;
    gp[H + j] = z;
    gp[2 * H + j] = nn;
    gp[3 * H + j] = ghn;
  }
}

// ---------------------------------------------------------------------------
// backward step (BPTT).  KSW = k-steps of W^T prefetched per wave per chunk.
template <int KSW>
__global__ __launch_bounds__(GT) void gru_bwd_step_kernel(
    int s, int T, int N, int H, int D, int UB, int BT, const float* __restrict__ dy, int dyd,
    const float* __restrict__ wpt, const float* __restrict__ h_all,
    const float* __restrict__ gates, const int* __restrict__ lens, float* __restrict__ dgx,
    float* __restrict__ dgh, float* __restrict__ dhs) {
  constexpr int PITCH = KC_BWD + 2;
  __shared__ __attribute__((aligned(16))) float hs[GB * PITCH];
  int ub, d, bt;
  if (!map_work(UB * D, BT, UB, ub, d, bt)) return;
  const int n0 = bt * GB;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // provably uniform
  const int t = d == 0 ? T - 1 - s : s;      // time processed now
  const int tq = d == 0 ? t + 1 : t - 1;     // time processed at step s-1
  const int H3 = 3 * H;
  const int KS = (H3 + 3) / 4;

  f32x4 acc0 = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 acc1 = f32x4{0.f, 0.f, 0.f, 0.f};
  if (s > 0) {
    const float* dghq = dgh + ((int64_t)tq * N * D + d) * H3;
    const float* wpd = wpt + ((int64_t)d * UB + ub) * KS * 64 + lane;
    for (int kc0 = 0; kc0 < H3; kc0 += KC_BWD) {
      const int kc1 = min(H3, kc0 + KC_BWD);
      const int ks0 = kc0 / 4;
      const int ks1 = (kc1 + 3) / 4;
      const int per = (ks1 - ks0 + GW - 1) / GW;
      const int a_ks = ks0 + wave * per;
      const int b_ks = min(ks1, a_ks + per);
      float w[KSW];
#pragma unroll
      for (int i = 0; i < KSW; ++i) {
        const int ks = a_ks + i;
        w[i] = ks < b_ks ? wpd[(int64_t)ks * 64] : 0.f;
      }
      if (kc0 > 0) __syncthreads();
      stage_rows(dghq, (int64_t)D * H3, N, n0, kc0, kc1, hs, PITCH);
      __syncthreads();
      const float* hrow = hs + (lane & 15) * PITCH + (lane >> 4) - kc0;
#pragma unroll
      for (int i = 0; i < KSW; i += 2) {
        const int ks = a_ks + i;
        if (ks < b_ks) {
          const int k = 4 * ks;
          const float a0 = (k + (lane >> 4) < kc1) ? hrow[k] : 0.f;
          acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, w[i], acc0, 0, 0, 0);
        }
        if (i + 1 < KSW && ks + 1 < b_ks) {
          const int k = 4 * (ks + 1);
          const float a1 = (k + (lane >> 4) < kc1) ? hrow[k] : 0.f;
          acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, w[i + 1], acc1, 0, 0, 0);
        }
      }
    }
    __syncthreads();
  }
  float* red = hs;
  constexpr int RP = GU + 1;
#pragma unroll
  for (int r = 0; r < 4; ++r)
    red[(wave * GB + (lane >> 4) * 4 + r) * RP + (lane & 15)] = acc0[r] + acc1[r];
  __syncthreads();
  if (threadIdx.x >= GB * GU) return;

  const int m = threadIdx.x >> 4;
  const int u = threadIdx.x & 15;
  const int n = n0 + m;
  const int j = ub * GU + u;
  if (n >= N || j >= H) return;
  const int len = lens[n];
  const int64_t row = ((int64_t)t * N + n) * D + d;
  float* dhcur = dhs + ((int64_t)(s & 1) * N * D + (int64_t)n * D + d) * H;
  const float* dhprv = dhs + ((int64_t)((s + 1) & 1) * N * D + (int64_t)n * D + d) * H;
  float dh = 0.f;
  if (t < len) {
    float carry = 0.f;
    if (s > 0) {
      float rec = 0.f;
#pragma unroll
      for (int w8 = 0; w8 < GW; ++w8) rec += red[(w8 * GB + m) * RP + u];
      const float zq = gates[(((int64_t)tq * N + n) * D + d) * 4 * H + H + j];
      carry = dhprv[j] * zq + rec;
    }
    dh = dy[(((int64_t)t * N + n) * dyd + (dyd > 1 ? d : 0)) * H + j] + carry;
  }
  float dar = 0.f, daz = 0.f, dan = 0.f, dghn = 0.f;
  if (t < len) {
    const float* gp = gates + row * 4 * H;
    const float r = gp[j], z = gp[H + j], nn = gp[2 * H + j], ghn = gp[3 * H + j];
    float hp = 0.f;
    const int tp = d == 0 ? t - 1 : t + 1;
    if (tp >= 0 && tp < T) hp = h_all[(((int64_t)tp * N + n) * D + d) * H + j];
    dan = dh * (1.f - z) * (1.f - nn * nn);
    daz = dh * (hp - nn) * z * (1.f - z);
    dar = dan * ghn * r * (1.f - r);
    dghn = dan * r;
  }
  float* gx = dgx + row * H3;
  float* gh = dgh + row * H3;
  gx[j] = dar;
  gx[H + j] = daz;
  gx[2 * H + j] = dan;
  gh[j] = dar;
  gh[H + j] = daz;
  gh[2 * H + j] = dghn;
  dhcur[j] = dh;
}

template <int KSW>
__global__ __launch_bounds__(GT) void gru_fwd_persist_kernel(
    int T, int N, int H, int D, int UB, int BT, const float* __restrict__ xproj,
    const float* __restrict__ wp, const float* __restrict__ b_f, const float* __restrict__ b_r,
    const int* __restrict__ lens, float* __restrict__ h_all, float* __restrict__ gates,
    unsigned* __restrict__ counters, unsigned* __restrict__ err,
    unsigned long long* __restrict__ stamps, int trace) {
  constexpr int PITCH = KC_FWD + 4;
  __shared__ __attribute__((aligned(16))) float hs[GB * PITCH];
  __shared__ int flag;
  int ub, d, bt;
  if (!map_work(UB * D, BT, UB, ub, d, bt)) return;
  const int n0 = bt * GB;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // provably uniform
  const int KS = (H + 3) / 4;
  const int a_ks = wave * KSW;           // host guarantees GW * KSW >= KS
  const int b_ks = min(KS, a_ks + KSW);
  unsigned* gflags = counters + (D * BT + 1) + (d * BT + bt) * UB;
  const __amdgpu_buffer_rsrc_t h_rs = __builtin_amdgcn_make_buffer_rsrc(
      h_all, (short)0, T * N * D * H * 4, 0x00020000);
  const bool stamping = stamps != nullptr && !trace && blockIdx.x == 0 && threadIdx.x == 0;
  // trace mode (DS2_GRU_STAMPS=2): every workgroup's thread 0 records s_memrealtime
  // (100 MHz) at {step start, wait done, staged, mfma+red done, arrived} for steps
  // [kTraceS0, kTraceS0 + kTraceSteps)
  const bool tracing = stamps != nullptr && trace && threadIdx.x == 0;
  auto trace_at = [&](int s, int p) {
    if (tracing && s >= kTraceS0 && s < kTraceS0 + kTraceSteps)
      stamps[((int64_t)(s - kTraceS0) * gridDim.x + blockIdx.x) * 5 + p] =
          __builtin_amdgcn_s_memrealtime();
  };
  unsigned long long acc_t[6] = {0, 0, 0, 0, 0, 0};
  unsigned long long t0 = 0, t1 = 0;

  // W_hh fragments for the whole sequence
  float w[3][KSW];
  {
    const float* wpd = wp + ((int64_t)d * UB + ub) * KS * 3 * 64 + lane;
#pragma unroll
    for (int i = 0; i < KSW; ++i) {
      const int ks = a_ks + i;
#pragma unroll
      for (int g = 0; g < 3; ++g) w[g][i] = ks < b_ks ? wpd[((int64_t)ks * 3 + g) * 64] : 0.f;
    }
  }
  const float* bh = d == 0 ? b_f : b_r;
  const int m = threadIdx.x >> 4;
  const int u = threadIdx.x & 15;
  const int n = n0 + m;
  const int j = ub * GU + u;
  const bool owner = threadIdx.x < GB * GU && n < N && j < H;
  float bias_r = 0.f, bias_z = 0.f, bias_n = 0.f;
  int len = 0;
  if (owner) {
    bias_r = bh[j];
    bias_z = bh[H + j];
    bias_n = bh[2 * H + j];
    len = lens[n];
  }
  settle(bias_r);
  settle(bias_z);
  settle(bias_n);
  settle(len);
  constexpr int RP = 3 * GU + 1;
  __shared__ float red[GW * GB * RP];
  float g_r = 0.f, g_z = 0.f, g_n = 0.f, g_hn = 0.f;   // gate cache of the previous step
  int64_t g_row = -1;
  for (int s = 0; s < T; ++s) {
    const int t = d == 0 ? s : T - 1 - s;
    const int tp = d == 0 ? t - 1 : t + 1;
    const int64_t row = ((int64_t)t * N + n) * D + d;
    // inputs of this step that do not depend on other workgroups: issue first
    float xr = 0.f, xz = 0.f, xn = 0.f;
    if (owner && t < len) {
      const float* xp = xproj + row * 3 * H;
      xr = xp[j];
      xz = xp[H + j];
      xn = xp[2 * H + j];
    }
    f32x4 acc[3];
#pragma unroll
    for (int g = 0; g < 3; ++g) acc[g] = f32x4{0.f, 0.f, 0.f, 0.f};
    float hp = 0.f;
    if (stamping) t0 = stamp_now();
    trace_at(s, 0);
    if (s > 0) {
      if (!flags_wait(gflags, UB, (unsigned)s, err, &flag)) {
        poison_rest(h_all, s, T, d != 0, N, D, n, d, H, j, H, 1, owner);
        return;
      }
      trace_at(s, 1);
      if (stamping) { t1 = stamp_now(); acc_t[0] += t1 - t0; t0 = t1; }
      const float* hprev = h_all + ((int64_t)tp * N * D + d) * H;
      stage_rows_sc1<(GB * KC_FWD / 4 + GT - 1) / GT>(hprev, D * H, N, n0, H, 4 * GW * KSW, hs,
                                                       PITCH);
      __syncthreads();
      trace_at(s, 2);
      if (stamping) { t1 = stamp_now(); acc_t[1] += t1 - t0; t0 = t1; }
      // every wave runs exactly KSW k-steps; steps past H read zero-staged columns and
      // zero W registers, so there is no branch between the LDS reads and the MFMAs
      const float* hrow = hs + (lane & 15) * PITCH + (lane >> 4) + 4 * a_ks;
#pragma unroll
      for (int i = 0; i < KSW; ++i) {
        const float a = hrow[4 * i];
        acc[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, w[0][i], acc[0], 0, 0, 0);
        acc[1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, w[1][i], acc[1], 0, 0, 0);
        acc[2] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, w[2][i], acc[2], 0, 0, 0);
      }
      if (owner) hp = hs[m * PITCH + j];
    }
#pragma unroll
    for (int g = 0; g < 3; ++g)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        red[(wave * GB + (lane >> 4) * 4 + r) * RP + g * GU + (lane & 15)] = acc[g][r];
    __syncthreads();
    trace_at(s, 3);
    if (stamping) { t1 = stamp_now(); acc_t[2] += t1 - t0; t0 = t1; }
    if (owner) {
      float gh[3];
#pragma unroll
      for (int g = 0; g < 3; ++g) {
        float v = 0.f;
#pragma unroll
        for (int w8 = 0; w8 < GW; ++w8) v += red[(w8 * GB + m) * RP + g * GU + u];
        gh[g] = v;
      }
      const float ghr = gh[0] + bias_r;
      const float ghz = gh[1] + bias_z;
      float ghn = gh[2] + bias_n;
      float hout = 0.f, r = 0.f, z = 0.f, nn = 0.f;
      if (t < len) {
        r = sigmoidf_(ghr + xr);
        z = sigmoidf_(ghz + xz);
        nn = tanhf(xn + r * ghn);
        hout = (hp - nn) * z + nn;
      } else {
        ghn = 0.f;
      }
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, hout), h_rs,
                                            static_cast<int>((row * H + j) * 4), 0, kSc1);
      g_r = r; g_z = z; g_n = nn; g_hn = ghn; g_row = row;
    }
    if (stamping) { t1 = stamp_now(); acc_t[3] += t1 - t0; t0 = t1; }
    flags_arrive(gflags + ub, (unsigned)s + 1);
    trace_at(s, 4);
    if (stamping) { t1 = stamp_now(); acc_t[4] += t1 - t0; t0 = t1; }
    // the gate cache is consumed only by the backward kernel: store it off the
    // critical path, after this step's hand-off has been signalled
    if (owner && gates != nullptr) {
      float* gp = gates + g_row * 4 * H;
      gp[j] = g_r;
      gp[H + j] = g_z;
      gp[2 * H + j] = g_n;
      gp[3 * H + j] = g_hn;
    }
  }
  if (stamping)
    for (int i = 0; i < 5; ++i) stamps[i] = acc_t[i];
}

// Direct-operand forward recurrence (H % 16 == 0, per-producer flags).
//
// Hand-off layout: besides h_all (row-major, for the GEMMs that follow), every producer
// publishes its 16 units x 16 samples of h_t as ONE 1-KB tile in a two-slot ring,
//   hx[slot = step & 1][d][bt][unit block][q][r][c]   (unit 4 q + c, sample n0 + r),
// written by wave 0 with one 16-byte sc1 store per lane after a transpose through LDS.
// The K range of W_hh h_{t-1} is split between the 8 waves in whole producer blocks
// (wave w owns blocks [b0, b0 + nb)); lane (r, q) of a wave reads its four A operands of
// block b (the k values 16 b + 4 q + 0..3 of sample r) as one 16-byte sc1 load, so each
// load instruction is one contiguous 1-KB tile -- no LDS staging of h, no barrier between
// the loads and the MFMAs.  W_hh fragments follow the same k order and are read once
// from the unpacked weight.  Wave 0 polls the producer flags (flags_wait) and releases
// the workgroup with a barrier (MI355X_MICROARCH.md "Valid forms" row 1).  A slot is
// rewritten two steps later, after every consumer of the group has published the step
// in between, i.e. after all its loads of the slot have returned.
//
// Hand-off: the sentinel ring (rnn_common.h, kRingSlots slots, no flags; the form above with
// the data as the flag): every wave spins on its own producers' tiles, so the wait, the poll
// round trip and the producer's drain-before-flag all leave the critical path (5.93 -> 5.51
// us per step).  The per-producer flag form and a hybrid (flag-polled, sentinel-validated)
// were measured slower and removed in round 4's pruning; the backward keeps the flags.
template <int NBW>
__global__ __launch_bounds__(GT) __attribute__((amdgpu_waves_per_eu(2, 2))) void gru_fwd_dop_kernel(
    int T, int N, int H, int D, int UB, int BT, const float* __restrict__ xproj,
    const float* __restrict__ w_f, const float* __restrict__ w_r, const float* __restrict__ b_f,
    const float* __restrict__ b_r, const int* __restrict__ lens, float* __restrict__ h_all,
    float* __restrict__ gates, float* __restrict__ hx, unsigned* __restrict__ counters,
    unsigned* __restrict__ err, unsigned long long* __restrict__ stamps) {
  constexpr int RP = 3 * GU + 1;
  __shared__ float red[GW * GB * RP];
  __shared__ __attribute__((aligned(16))) float tile[GB * GU];
  int ub, d, bt;
  if (!map_work(UB * D, BT, UB, ub, d, bt)) return;
  const int n0 = bt * GB;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  int b0, nb;
  simd_split(UB, wave, b0, nb);                 // host guarantees nb <= NBW
  const int slot_floats = D * BT * UB * 256;
  constexpr bool SENT = true;        // sentinel ring: tiles validate themselves
  constexpr int NSLOT = kRingSlots;
  const __amdgpu_buffer_rsrc_t x_rs =
      __builtin_amdgcn_make_buffer_rsrc(hx, (short)0, NSLOT * slot_floats * 4, 0x00020000);
  const int grp_off = (d * BT + bt) * UB * 256;            // this group's tiles in a slot
  __shared__ int failed;
  if (threadIdx.x == 0) failed = 0;
  __syncthreads();
  const bool tracing = stamps != nullptr && threadIdx.x == 0;
  auto trace_at = [&](int s, int p) {
    if (tracing && s >= kTraceS0 && s < kTraceS0 + kTraceSteps)
      stamps[((int64_t)(s - kTraceS0) * gridDim.x + blockIdx.x) * 5 + p] =
          __builtin_amdgcn_s_memrealtime();
  };

  // W_hh fragments: w[g][i][c] = W_hh[g H + ub 16 + (lane & 15)][16 (b0 + i) + 4 (lane >> 4) + c]
  f32x4 w[3][NBW];
  {
    const float* W = d == 0 ? w_f : w_r;
    const float* wr = W + (int64_t)(ub * GU + (lane & 15)) * H + 16 * b0 + 4 * (lane >> 4);
#pragma unroll
    for (int i = 0; i < NBW; ++i)
#pragma unroll
      for (int g = 0; g < 3; ++g)
        w[g][i] = i < nb ? *reinterpret_cast<const f32x4*>(wr + (int64_t)g * H * H + 16 * i)
                         : f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const float* bh = d == 0 ? b_f : b_r;
  const int m = threadIdx.x >> 4;
  const int u = threadIdx.x & 15;
  const int n = n0 + m;
  const int j = ub * GU + u;
  const bool owner = threadIdx.x < GB * GU && n < N;
  float bias_r = 0.f, bias_z = 0.f, bias_n = 0.f;
  int len = 0;
  if (owner) {
    bias_r = bh[j];
    bias_z = bh[H + j];
    bias_n = bh[2 * H + j];
    len = lens[n];
  }
  settle(bias_r);
  settle(bias_z);
  settle(bias_n);
  settle(len);
  // this thread's slot in the transposed tile: (q = u >> 2, r = m, c = u & 3)
  const int tpos = ((u >> 2) * GB + m) * 4 + (u & 3);
  float g_r = 0.f, g_z = 0.f, g_n = 0.f, g_hn = 0.f, h_own = 0.f;
  int64_t g_row = -1;
  for (int s = 0; s < T; ++s) {
    const int t = d == 0 ? s : T - 1 - s;
    const int64_t row = ((int64_t)t * N + n) * D + d;
    float xr = 0.f, xz = 0.f, xn = 0.f;
    if (owner && t < len) {
      const float* xp = xproj + row * 3 * H;
      xr = xp[j];
      xz = xp[H + j];
      xn = xp[2 * H + j];
    }
    f32x4 acc[3];
#pragma unroll
    for (int g = 0; g < 3; ++g) acc[g] = f32x4{0.f, 0.f, 0.f, 0.f};
    trace_at(s, 0);
    if (s > 0) {
      trace_at(s, 1);
      const int base = (((s - 1) % NSLOT) * slot_floats + grp_off + b0 * 256 + lane * 4) * 4;
      sleep_units(g_rnn_tune[1]);
      f32x4 hv[NBW];
#pragma unroll
      for (int i = 0; i < NBW; ++i) {
        const int off = i < nb ? base + i * 1024 : 0x7ffffff0;
        hv[i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(x_rs, off, 0, kSc1));
      }
      // all loads in flight before the first MFMA (the scheduler would otherwise
      // interleave them with the MFMAs and expose one load latency per block)
      asm volatile("" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (NBW <= 7) {
        // Per-tile partial products summed in a fixed order afterwards, so the tiles can be
        // multiplied in arrival order (SENT: a pass multiplies every ready pending tile, then
        // re-loads the still-pending ones together: one round trip per pass, not per tile).
        f32x4 pacc[NBW][3];
  #pragma unroll
        for (int i = 0; i < NBW; ++i)
  #pragma unroll
          for (int g = 0; g < 3; ++g) pacc[i][g] = f32x4{0.f, 0.f, 0.f, 0.f};
        unsigned pend = (1u << nb) - 1u;                 // wave-uniform (nb <= NBW <= 8)
        for (unsigned spins = 0;; ++spins) {
  #pragma unroll
          for (int i = 0; i < NBW; ++i) {
            if (((pend >> i) & 1u) && (!SENT || wave_ready(hv[i]))) {
  #pragma unroll
              for (int c = 0; c < 4; ++c)
  #pragma unroll
                for (int g = 0; g < 3; ++g)
                  pacc[i][g] = __builtin_amdgcn_mfma_f32_16x16x4f32(hv[i][c], w[g][i][c], pacc[i][g],
                                                                    0, 0, 0);
              pend &= ~(1u << i);
            }
          }
          if (pend == 0u && g_spin_limit != 0) break;
          if (spins > g_spin_limit || g_spin_limit == 0) {
            if (lane == 0) __hip_atomic_fetch_or(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            failed = 1;
            break;
          }
          sleep_units(g_rnn_tune[0]);
          asm volatile("" ::: "memory");   // the re-loads are not loop-invariant (no LICM)
  #pragma unroll
          for (int i = 0; i < NBW; ++i)
            if ((pend >> i) & 1u)
              hv[i] = __builtin_bit_cast(
                  f32x4, __builtin_amdgcn_raw_buffer_load_b128(x_rs, base + i * 1024, 0, kSc1));
        }
  #pragma unroll
        for (int g = 0; g < 3; ++g) {
          acc[g] = pacc[0][g];
  #pragma unroll
          for (int i = 1; i < NBW; ++i) acc[g] += pacc[i][g];
        }
      } else {
        // 8 tiles per wave (H > 896): the per-tile partials would spill (96 more VGPRs), so
        // the ready PREFIX is multiplied in tile order straight into acc (as in the backward:
        // one accumulation order for every hand-off form) and only stale tiles are re-loaded
        unsigned rdy = 0u;
        int next = 0;
        for (unsigned spins = 0;; ++spins) {
#pragma unroll
          for (int i = 0; i < NBW; ++i)
            if (i >= next && i < nb && !((rdy >> i) & 1u) && (!SENT || wave_ready(hv[i])))
              rdy |= 1u << i;
#pragma unroll
          for (int i = 0; i < NBW; ++i) {
            if (i == next && i < nb && ((rdy >> i) & 1u)) {
#pragma unroll
              for (int c = 0; c < 4; ++c)
#pragma unroll
                for (int g = 0; g < 3; ++g)
                  acc[g] = __builtin_amdgcn_mfma_f32_16x16x4f32(hv[i][c], w[g][i][c], acc[g], 0, 0, 0);
              ++next;
            }
          }
          if (next >= nb && g_spin_limit != 0) break;
          if (spins > g_spin_limit || g_spin_limit == 0) {
            if (lane == 0) __hip_atomic_fetch_or(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            failed = 1;
            break;
          }
          sleep_units(g_rnn_tune[0]);
          asm volatile("" ::: "memory");
#pragma unroll
          for (int i = 0; i < NBW; ++i)
            if (i >= next && i < nb && !((rdy >> i) & 1u))
              hv[i] = __builtin_bit_cast(
                  f32x4, __builtin_amdgcn_raw_buffer_load_b128(x_rs, base + i * 1024, 0, kSc1));
        }
      }
      trace_at(s, 2);
    }
#pragma unroll
    for (int g = 0; g < 3; ++g)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        red[(wave * GB + (lane >> 4) * 4 + r) * RP + g * GU + (lane & 15)] = acc[g][r];
    // the step's xproj loads are consumed on every path here (not at the next step's
    // re-initialisation, where the waitcnt pass would wait for the hand-off stores too)
    settle(xr);
    settle(xz);
    settle(xn);
    __syncthreads();
    if (failed) {
      poison_rest(h_all, s, T, d != 0, N, D, n, d, H, j, H, 1, owner);
      return;
    }
    trace_at(s, 3);
    if (threadIdx.x < GB * GU) {
      float hout = 0.f;
      if (owner) {
        float gh[3];
#pragma unroll
        for (int g = 0; g < 3; ++g) {
          float v = 0.f;
#pragma unroll
          for (int w8 = 0; w8 < GW; ++w8) v += red[(w8 * GB + m) * RP + g * GU + u];
          gh[g] = v;
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
    }
    __syncthreads();
    // publish: wave 0 stores the tile (one 16-B sc1 store per lane), drains, flags
    if (wave == 0) {
      const int toff = (grp_off + ub * 256 + lane * 4) * 4;
      const u32x4 v = desentinel(*reinterpret_cast<const u32x4*>(tile + lane * 4));
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // last step's sentinel store first
      __builtin_amdgcn_raw_buffer_store_b128(v, x_rs, (s % NSLOT) * slot_floats * 4 + toff, 0, kSc1);
      const u32x4 sv = u32x4{kSentinel, kSentinel, kSentinel, kSentinel};
      __builtin_amdgcn_raw_buffer_store_b128(sv, x_rs, ((s + 2) % NSLOT) * slot_floats * 4 + toff,
                                             0, kSc1);
    }
    trace_at(s, 4);
    // outputs consumed only by later kernels, off the critical path
    if (owner) {
      h_all[row * H + j] = h_own;
      if (gates != nullptr) {
        float* gp = gates + g_row * 4 * H;
        gp[j] = g_r;
        gp[H + j] = g_z;
        gp[2 * H + j] = g_n;
        gp[3 * H + j] = g_hn;
      }
    }
  }
}

template <int KSW>
__global__ __launch_bounds__(GT) void gru_bwd_persist_kernel(
    int T, int N, int H, int D, int UB, int BT, const float* __restrict__ dy, int dyd,
    const float* __restrict__ wpt, const float* __restrict__ h_all,
    const float* __restrict__ gates, const int* __restrict__ lens, float* __restrict__ dgx,
    float* __restrict__ dgh, unsigned* __restrict__ counters, unsigned* __restrict__ err,
    unsigned long long* __restrict__ stamps) {
  constexpr int PITCH = KC_BWD + 4;
  __shared__ __attribute__((aligned(16))) float hs[GB * PITCH];
  float* red = hs;                          // reduction buffer aliases the staged rows
  __shared__ int flag;
  int ub, d, bt;
  if (!map_work(UB * D, BT, UB, ub, d, bt)) return;
  const int n0 = bt * GB;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // provably uniform
  const int H3 = 3 * H;
  const int KS = (H3 + 3) / 4;             // single chunk: 32 * KSW <= KC_BWD (host-checked)
  const int a_ks = wave * KSW;
  const int b_ks = min(KS, a_ks + KSW);
  unsigned* gflags = counters + (D * BT + 1) + (d * BT + bt) * UB;
  const __amdgpu_buffer_rsrc_t g_rs = __builtin_amdgcn_make_buffer_rsrc(
      dgh, (short)0, T * N * D * H3 * 4, 0x00020000);

  float w[KSW];
  {
    const float* wpd = wpt + ((int64_t)d * UB + ub) * KS * 64 + lane;
#pragma unroll
    for (int i = 0; i < KSW; ++i) {
      const int ks = a_ks + i;
      w[i] = ks < b_ks ? wpd[(int64_t)ks * 64] : 0.f;
    }
  }
  const int m = threadIdx.x >> 4;
  const int u = threadIdx.x & 15;
  const int n = n0 + m;
  const int j = ub * GU + u;
  const bool owner = threadIdx.x < GB * GU && n < N && j < H;
  int len = owner ? lens[n] : 0;
  settle(len);
  constexpr int RP = GU + 1;
  float dh_prev = 0.f, z_prev = 0.f;        // this thread's unit, carried in registers
  // trace mode (DS2_GRU_STAMPS=2, as in the forward kernel)
  const bool tracing = stamps != nullptr && threadIdx.x == 0;
  auto trace_at = [&](int s, int p) {
    if (tracing && s >= kTraceS0 && s < kTraceS0 + kTraceSteps)
      stamps[((int64_t)(s - kTraceS0) * gridDim.x + blockIdx.x) * 5 + p] =
          __builtin_amdgcn_s_memrealtime();
  };

  float px_dar = 0.f, px_daz = 0.f, px_dan = 0.f;   // dgx of the previous step (deferred)
  int64_t px_row = -1;
  for (int s = 0; s < T; ++s) {
    const int t = d == 0 ? T - 1 - s : s;
    f32x4 acc0 = f32x4{0.f, 0.f, 0.f, 0.f};
    f32x4 acc1 = f32x4{0.f, 0.f, 0.f, 0.f};
    trace_at(s, 0);
    // this step's inputs that do not depend on other workgroups: issue before the wait
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
    if (s > 0) {
      const int tq = d == 0 ? t + 1 : t - 1;
      if (!flags_wait(gflags, UB, (unsigned)s, err, &flag)) {
        poison_rest(dgx, s, T, d == 0, N, D, n, d, H, j, H3, 3, owner);
        return;
      }
      trace_at(s, 1);
      const float* dghq = dgh + ((int64_t)tq * N * D + d) * H3;
      stage_rows_sc1<(GB * KC_BWD / 4 + GT - 1) / GT>(dghq, D * H3, N, n0, H3, 4 * GW * KSW, hs,
                                                       PITCH);
      __syncthreads();
      trace_at(s, 2);
      const float* hrow = hs + (lane & 15) * PITCH + (lane >> 4) + 4 * a_ks;
#pragma unroll
      for (int i = 0; i < KSW; i += 2) {
        acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(hrow[4 * i], w[i], acc0, 0, 0, 0);
        if (i + 1 < KSW)
          acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(hrow[4 * i + 4], w[i + 1], acc1, 0, 0, 0);
      }
      __syncthreads();                      // all reads of hs done before red overwrites it
    }
#pragma unroll
    for (int r = 0; r < 4; ++r)
      red[(wave * GB + (lane >> 4) * 4 + r) * RP + (lane & 15)] = acc0[r] + acc1[r];
    __syncthreads();
    trace_at(s, 3);
    if (owner) {
      float dh = 0.f;
      float dar = 0.f, daz = 0.f, dan = 0.f, dghn = 0.f, zc = 0.f;
      if (t < len) {
        float carry = 0.f;
        if (s > 0) {
          float rec = 0.f;
#pragma unroll
          for (int w8 = 0; w8 < GW; ++w8) rec += red[(w8 * GB + m) * RP + u];
          carry = dh_prev * z_prev + rec;
        }
        dh = dyv + carry;
        zc = g_z;
        dan = dh * (1.f - zc) * (1.f - g_n * g_n);
        daz = dh * (hp - g_n) * zc * (1.f - zc);
        dar = dan * g_hn * g_r * (1.f - g_r);
        dghn = dan * g_r;
      }
      const int go = static_cast<int>((row * H3 + j) * 4);
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, dar), g_rs, go, 0, kSc1);
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, daz), g_rs, go + 4 * H, 0,
                                            kSc1);
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, dghn), g_rs, go + 8 * H,
                                            0, kSc1);
      dh_prev = dh;
      z_prev = zc;
      px_dar = dar; px_daz = daz; px_dan = dan; px_row = row;
    }
    flags_arrive(gflags + ub, (unsigned)s + 1);
    trace_at(s, 4);
    // dgx is consumed only by later kernels: store it after the hand-off is signalled
    if (owner) {
      float* gx = dgx + px_row * H3;
      gx[j] = px_dar;
      gx[H + j] = px_daz;
      gx[2 * H + j] = px_dan;
    }
  }
}

// Direct-operand backward recurrence (H % 16 == 0, per-producer flags).  Same scheme
// as gru_fwd_dop_kernel over K = 3H: each producer publishes its gate gradients
// (dar, daz, dghn) as three 1-KB tiles, tile g * UB + ub of the ring
//   gx[slot][d][bt][3 UB blocks][q][r][c],
// whose block order is the k order of dgh; wave w owns blocks [b0, b0 + nb) of the 3 UB.
// dgh (for the weight-gradient GEMM) and dgx are stored after the flag.  (A sentinel ring
// measured slower here: 19 tiles per wave, and an early consumer pays one serial round trip
// per stale tile, 7.55 vs 6.3 us per step; removed with the hybrid form in round 4.)
template <int NBW>
__global__ __launch_bounds__(GT) __attribute__((amdgpu_waves_per_eu(2, 2))) void gru_bwd_dop_kernel(
    int T, int N, int H, int D, int UB, int BT, const float* __restrict__ dy, int dyd,
    const float* __restrict__ w_f, const float* __restrict__ w_r,
    const float* __restrict__ h_all, const float* __restrict__ gates,
    const int* __restrict__ lens, float* __restrict__ dgx, float* __restrict__ dgh,
    float* __restrict__ gx, unsigned* __restrict__ counters, unsigned* __restrict__ err,
    unsigned long long* __restrict__ stamps, double* __restrict__ dbp) {
  constexpr int RP = GU + 1;
  __shared__ __attribute__((aligned(8))) float red[GW * GB * RP];
  __shared__ __attribute__((aligned(16))) float tile[3 * GB * GU];
  __shared__ int flag;
  int ub, d, bt;
  if (!map_work(UB * D, BT, UB, ub, d, bt)) return;
  const int n0 = bt * GB;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int H3 = 3 * H;
  const int NB3 = 3 * UB;
  int b0, nb;
  simd_split(NB3, wave, b0, nb);                // host guarantees nb <= NBW
  const unsigned* gflags = counters + (D * BT + 1) + (d * BT + bt) * UB;
  unsigned* myflag = counters + (D * BT + 1) + (d * BT + bt) * UB + ub;
  const int slot_floats = D * BT * NB3 * 256;
  const __amdgpu_buffer_rsrc_t x_rs =
      __builtin_amdgcn_make_buffer_rsrc(gx, (short)0, 2 * slot_floats * 4, 0x00020000);
  const int grp_off = (d * BT + bt) * NB3 * 256;
  const bool tracing = stamps != nullptr && threadIdx.x == 0;
  auto trace_at = [&](int s, int p) {
    if (tracing && s >= kTraceS0 && s < kTraceS0 + kTraceSteps)
      stamps[((int64_t)(s - kTraceS0) * gridDim.x + blockIdx.x) * 5 + p] =
          __builtin_amdgcn_s_memrealtime();
  };

  // W_hh^T fragments: w[i][c] = W_hh[16 (b0 + i) + 4 (lane >> 4) + c][ub 16 + (lane & 15)]
  f32x4 w[NBW];
  {
    const float* W = d == 0 ? w_f : w_r;
    const float* wc = W + (int64_t)(16 * b0 + 4 * (lane >> 4)) * H + ub * GU + (lane & 15);
#pragma unroll
    for (int i = 0; i < NBW; ++i)
#pragma unroll
      for (int c = 0; c < 4; ++c) w[i][c] = i < nb ? wc[(int64_t)(16 * i + c) * H] : 0.f;
    // pending at loop entry, these loads made the in-loop zero-initialisations of the
    // step's prefetch registers wait for the previous step's hand-off stores (settle)
#pragma unroll
    for (int i = 0; i < NBW; ++i) settle(w[i]);
  }
  const int m = threadIdx.x >> 4;
  const int u = threadIdx.x & 15;
  const int n = n0 + m;
  const int j = ub * GU + u;
  const bool owner = threadIdx.x < GB * GU && n < N;
  int len = owner ? lens[n] : 0;
  settle(len);
  const int tpos = ((u >> 2) * GB + m) * 4 + (u & 3);
  float dh_prev = 0.f, z_prev = 0.f;
  float px_dar = 0.f, px_daz = 0.f, px_dan = 0.f, px_dghn = 0.f;
  int64_t px_row = -1;
  // bias-gradient sums over this thread's (sample, unit) rows in step order (dbp != null):
  // db_ih = column sums of dgx (r, z, n), db_hh's n third = column sums of dgh's n third
  double sb_r = 0.0, sb_z = 0.0, sb_n = 0.0, sb_hn = 0.0;
  for (int s = 0; s < T; ++s) {
    const int t = d == 0 ? T - 1 - s : s;
    f32x4 acc0 = f32x4{0.f, 0.f, 0.f, 0.f};
    f32x4 acc1 = f32x4{0.f, 0.f, 0.f, 0.f};
    trace_at(s, 0);
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
    if (s > 0) {
      if (!flags_wait(gflags, UB, (unsigned)s, err, &flag)) {
        poison_rest(dgx, s, T, d == 0, N, D, n, d, H, j, H3, 3, owner);
        return;
      }
      trace_at(s, 1);
      const int base = (((s - 1) & 1) * slot_floats + grp_off + b0 * 256 + lane * 4) * 4;
      f32x4 gv[NBW];
#pragma unroll
      for (int i = 0; i < NBW; ++i) {
        const int off = i < nb ? base + i * 1024 : 0x7ffffff0;
        gv[i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(x_rs, off, 0, kSc1));
      }
      asm volatile("" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < NBW; ++i) {
        acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(gv[i][0], w[i][0], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(gv[i][1], w[i][1], acc1, 0, 0, 0);
        acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(gv[i][2], w[i][2], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(gv[i][3], w[i][3], acc1, 0, 0, 0);
      }
      trace_at(s, 2);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r)
      red[(wave * GB + (lane >> 4) * 4 + r) * RP + (lane & 15)] = acc0[r] + acc1[r];
    settle(dyv);                      // consumed here on every path (see the forward)
    settle(g_r);
    settle(g_z);
    settle(g_n);
    settle(g_hn);
    settle(hp);
    __syncthreads();
    trace_at(s, 3);
    if (threadIdx.x < GB * GU) {
      float dar = 0.f, daz = 0.f, dan = 0.f, dghn = 0.f;
      if (owner) {
        float dh = 0.f, zc = 0.f;
        if (t < len) {
          float carry = 0.f;
          if (s > 0) {
            float rec = 0.f;
#pragma unroll
            for (int w8 = 0; w8 < GW; ++w8) rec += red[(w8 * GB + m) * RP + u];
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
      tile[tpos] = dar;
      tile[GB * GU + tpos] = daz;
      tile[2 * GB * GU + tpos] = dghn;
    }
    __syncthreads();
    if (wave == 0) {
      const int toff = (grp_off + ub * 256 + lane * 4) * 4;
      const int so = (s & 1) * slot_floats * 4 + toff;
#pragma unroll
      for (int g = 0; g < 3; ++g) {
        const u32x4 v = *reinterpret_cast<const u32x4*>(tile + g * GB * GU + lane * 4);
        __builtin_amdgcn_raw_buffer_store_b128(v, x_rs, so + g * UB * 1024, 0, kSc1);
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
  double* rd = reinterpret_cast<double*>(red);   // 1024 doubles fit in red
  __syncthreads();
  if (threadIdx.x < GB * GU) {
    const bool mine = owner;
    rd[(0 * GB + m) * GU + u] = mine ? sb_r : 0.0;
    rd[(1 * GB + m) * GU + u] = mine ? sb_z : 0.0;
    rd[(2 * GB + m) * GU + u] = mine ? sb_n : 0.0;
    rd[(3 * GB + m) * GU + u] = mine ? sb_hn : 0.0;
  }
  __syncthreads();
  if (threadIdx.x < 4 * GU) {
    const int g = threadIdx.x / GU, uu = threadIdx.x - (threadIdx.x / GU) * GU;
    double acc = 0.0;
#pragma unroll
    for (int mm = 0; mm < GB; ++mm) acc += rd[(g * GB + mm) * GU + uu];
    dbp[(((int64_t)bt * D + d) * 4 + g) * H + ub * GU + uu] = acc;
  }
}

// Bias gradients from dgx / dgh when the recurrence kernel did not sum them (every path
// but the direct-operand backward): one block per (direction, gate column), fixed order.
__global__ void gru_db_cols_kernel(const float* __restrict__ dgx, const float* __restrict__ dgh,
                                   int rows, int D, int H, double* __restrict__ dbp) {
  const int c = blockIdx.x;                    // (d, g, j): dbp[0][d][g][j]
  const int d = c / (4 * H), k = c - d * 4 * H;
  const int g = k / H, j = k - g * H;
  const float* src = g < 3 ? dgx + d * 3 * H + g * H + j : dgh + d * 3 * H + 2 * H + j;
  const int64_t stride = (int64_t)D * 3 * H;
  double acc = 0.0;
  for (int r = threadIdx.x; r < rows; r += blockDim.x) acc += src[r * stride];
  __shared__ double sh[256];
  sh[threadIdx.x] = acc;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) sh[threadIdx.x] += sh[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) dbp[c] = sh[0];
}

// db_ih[d] = sum over batch tiles of dbp[.][d][0..2], db_hh[d][:2H] = the same r, z sums
// (dgh's r, z columns are dgx's), db_hh[d][2H:] = the n sums of dgh
__global__ void gru_db_final_kernel(const double* __restrict__ dbp, int BT, int D, int H,
                                    float* __restrict__ dbi_f, float* __restrict__ dbh_f,
                                    float* __restrict__ dbi_r, float* __restrict__ dbh_r) {
  const int total = D * 4 * H;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int d = i / (4 * H), k = i - d * 4 * H;
    double acc = 0.0;
    for (int b = 0; b < BT; ++b) acc += dbp[(int64_t)b * total + i];
    const float v = static_cast<float>(acc);
    float* dbi = d == 0 ? dbi_f : dbi_r;
    float* dbh = d == 0 ? dbh_f : dbh_r;
    if (k < 3 * H) dbi[k] = v;
    if (k < 2 * H) dbh[k] = v;
    if (k >= 3 * H) dbh[k - H] = v;
  }
}

}  // namespace ds2

namespace ds2 {
// gru_split.hip: the same direct-operand recurrences with the W_hh contraction on the bf16
// matrix cores at fp32 accuracy (default; DS2_GRU_X6=0 selects the fp32-MFMA kernels above)
bool launch_gru_fwd_x6(int t_max, int n, int h, int num_dirs, const float* xproj,
                       const float* w_hh_f, const float* w_hh_r, const float* b_hh_f,
                       const float* b_hh_r, const int* lens, float* h_all, float* gates,
                       float* ring, unsigned* ctrs, unsigned* err, unsigned long long* stamps,
                       size_t lds_pad, hipStream_t st);
bool launch_gru_bwd_x6(int t_max, int n, int h, int num_dirs, const float* dy, int dy_dirs,
                       const float* w_hh_f, const float* w_hh_r, const float* h_all,
                       const float* gates, const int* lens, float* dgates_x, float* dgates_h,
                       float* ring, unsigned* ctrs, unsigned* err, unsigned long long* stamps,
                       double* dbp, size_t lds_pad, hipStream_t st, unsigned* camax,
                       bool* camax_done);
int gru_bwd_x6_grid(int n, int h, int num_dirs);
bool launch_rnn_fwd_h3(int t_max, int n, int h, int num_dirs, const float* xproj,
                       const float* w_hh_f, const float* w_hh_r, const float* b_hh_f,
                       const float* b_hh_r, const int* lens, float* h_all, float* ring,
                       unsigned* ctrs, unsigned* err, unsigned long long* stamps, size_t lds_pad,
                       hipStream_t st);
bool launch_rnn_bwd_h3(int t_max, int n, int h, int num_dirs, const float* dy, int dy_dirs,
                       const float* w_hh_f, const float* w_hh_r, const float* h_all,
                       const int* lens, float* dgates, float* ring, unsigned* ctrs, unsigned* err,
                       unsigned long long* stamps, size_t lds_pad, hipStream_t st,
                       unsigned* camax);
int rnn_h3_grid(int n, int h, int num_dirs);
// gru_xl.hip: the XCD-local groups (default where the shape fits: 32 units x 8 samples per
// workgroup, a group of H / 32 workgroups in one XCD)
int gru_xl_groups(int n, int h, int num_dirs);
int gru_xl_active(int n, int h, int num_dirs);
size_t gru_xl_ctr_words();
bool launch_gru_fwd_xl(int t_max, int n, int h, int num_dirs, const float* xproj,
                       const float* w_hh_f, const float* w_hh_r, const float* b_hh_f,
                       const float* b_hh_r, const int* lens, float* h_all, float* gates,
                       float* ring, unsigned* xl, unsigned* err, unsigned long long* stamps,
                       size_t lds_pad, hipStream_t st);
bool launch_gru_bwd_xl(int t_max, int n, int h, int num_dirs, const float* dy, int dy_dirs,
                       const float* w_hh_f, const float* w_hh_r, const float* h_all,
                       const float* gates, const int* lens, float* dgates_x, float* dgates_h,
                       float* ring, unsigned* xl, unsigned* err, unsigned long long* stamps,
                       double* dbp, size_t lds_pad, hipStream_t st, unsigned* camax);
}  // namespace ds2

using namespace ds2;

extern "C" {

static inline int stamp_mode() {
  const char* e = getenv("DS2_GRU_STAMPS");
  return e == nullptr ? 0 : (e[0] == '1' ? 1 : (e[0] == '2' ? 2 : 0));
}
// the dynamic LDS of the direct-operand kernels: one workgroup per CU
constexpr unsigned kDopPadLds = 80 * 1024;
// smallest instantiated blocks-per-wave >= need (extra blocks are predicated off)
static const void* bwd_dop_fn(int need) {
#define DS2_BDOP(K) \
  if (need <= K) return reinterpret_cast<const void*>(gru_bwd_dop_kernel<K>);
  DS2_BDOP(1) DS2_BDOP(2) DS2_BDOP(3) DS2_BDOP(4) DS2_BDOP(6) DS2_BDOP(8) DS2_BDOP(10)
  DS2_BDOP(13) DS2_BDOP(16) DS2_BDOP(19) DS2_BDOP(22) DS2_BDOP(24)
#undef DS2_BDOP
  return nullptr;
}
// group counters, the error word, 64 per-producer flags per group, then 64 per-producer XCC
// ids per group (the same-XCD groups of gru_split.hip); the XCD-local kernels (gru_xl.hip) use
// gru_xl_ctr_words() words after the error word instead
static inline size_t ctr_words(int n, int num_dirs) {
  const int groups = num_dirs * ((n + GB - 1) / GB);
  const size_t a = (size_t)groups * 128, b = gru_xl_ctr_words();
  return (size_t)groups + 1 + (a > b ? a : b);
}
static inline size_t counter_bytes(int n, int num_dirs) {
  const size_t trace = stamp_mode() == 2 ? (size_t)kTraceSteps * 1024 * 5 : 16;
  return align256(ctr_words(n, num_dirs) * sizeof(unsigned)) + trace * sizeof(unsigned long long);
}
static inline unsigned long long* stamp_slots(unsigned* ctrs, int n, int num_dirs) {
  if (stamp_mode() == 0) return nullptr;
  return reinterpret_cast<unsigned long long*>(reinterpret_cast<char*>(ctrs) +
                                               align256(ctr_words(n, num_dirs) * sizeof(unsigned)));
}

// ring of hand-off tiles for the direct-operand kernels (gates tiles per unit block: 1
// forward, 3 backward).  Forward: kRingSlots slots of the sentinel ring, doubled for the
// plainly stored copy the same-XCD groups read.  Backward: 2 slots of the flag hand-off plus
// the 2 slots of plain copies, tiles sized for the pre-split form (1.5 KB, gru_split.hip).
static inline size_t ring_bytes(int n, int h, int num_dirs, int tiles) {
  const size_t UB = (h + GU - 1) / GU, BT = (n + GB - 1) / GB;
  const size_t tile_floats = tiles == 3 ? 384 : 256;
  const size_t slots = tiles == 3 ? 4 : 2 * kRingSlots;
  return align256(slots * (size_t)num_dirs * BT * UB * tiles * tile_floats * sizeof(float));
}
// every word of the forward's sentinel ring starts as the sentinel
static inline hipError_t ring_reset(float* ring, int n, int h, int num_dirs, hipStream_t st) {
  return hipMemsetAsync(ring, 0xFF, ring_bytes(n, h, num_dirs, 1), st);
}

// the gate cache: [T][N][D][4H] (r, z, n, W_hn h + b_hn)
size_t ds2_gru_cache_floats(int t_max, int n, int h, int num_dirs) {
  if (t_max <= 0 || n <= 0 || h <= 0 || num_dirs <= 0) return 0;
  return (size_t)t_max * n * num_dirs * 4 * h;
}

size_t ds2_gru_fwd_workspace_size(int n, int h, int num_dirs) {
  const int64_t UB = (h + GU - 1) / GU;
  const int64_t KS = (h + 3) / 4;
  return align256((size_t)(num_dirs * UB * KS * 3 * 64) * sizeof(float)) +
         align256(counter_bytes(n, num_dirs)) + ring_bytes(n, h, num_dirs, 1) + 256;
}

#define DS2_FWD_CASE(K)                                                                    \
  case K:                                                                                  \
    hipLaunchKernelGGL(gru_fwd_step_kernel<K>, dim3(grid), dim3(GT), 0, st, s, t_max, n, h, \
                       num_dirs, UB, BT, xproj, wp, b_hh_f, b_hh_r, lens, h_all, gates);    \
    break;

static int pick_ksw(int per) {
  const int opts[] = {8, 16, 32, 48, 64, 80, 96};
  for (int k : opts)
    if (per <= k) return k;
  return -1;
}

// Kernel choice (forward and backward alike): the direct-operand persistent kernels where
// H % 16 == 0 and the grid fits the chip -- bf16x6 (gru_split.hip) by default, the fp32-MFMA
// forms with DS2_GRU_X6=0 --, else the LDS-staged persistent kernels (H % 4 == 0), else one
// launch per step (also DS2_RNN_PERSISTENT=0).
ds2_status_t ds2_gru_fwd(int t_max, int n, int h, int num_dirs, const float* xproj,
                         const float* w_hh_f, const float* w_hh_r, const float* b_hh_f,
                         const float* b_hh_r, const int* lens, float* h_all, float* gates,
                         unsigned* err_out, void* ws, size_t ws_bytes, ds2_stream_t stream) {
  if (t_max < 0 || n < 0 || h < 1 || (num_dirs != 1 && num_dirs != 2)) return DS2_INVALID_VALUE;
  if (h > KC_FWD) return DS2_UNSUPPORTED_SHAPE;
  if (t_max == 0 || n == 0) return DS2_OK;
  if (ws == nullptr || ws_bytes < ds2_gru_fwd_workspace_size(n, h, num_dirs))
    return DS2_WORKSPACE_TOO_SMALL;
  if (num_dirs == 1) {
    w_hh_r = w_hh_f;
    b_hh_r = b_hh_f;
  }
  hipStream_t st = as_stream(stream);
  apply_spin_limit_env();
  apply_rnn_tune_env();
  const int UB = (h + GU - 1) / GU;
  const int KS = (h + 3) / 4;
  const int BT = (n + GB - 1) / GB;
  const int ksw = pick_ksw((KS + GW - 1) / GW);
  if (ksw < 0) return DS2_UNSUPPORTED_SHAPE;
  float* wp = static_cast<float*>(ws);
  const int grid = mapped_grid(UB * num_dirs, BT);
  const bool persistent = persistent_enabled() && grid <= num_cus() &&
                          (int64_t)t_max * n * num_dirs * h * 4 < (1ll << 31);
  unsigned* ctrs = reinterpret_cast<unsigned*>(
      static_cast<char*>(ws) + align256((size_t)num_dirs * UB * KS * 3 * 64 * sizeof(float)));
  unsigned* err = ctrs + num_dirs * BT;
  if (persistent && (h % GU) == 0 && UB <= 8 * GW) {
    if (hipMemsetAsync(ctrs, 0, counter_bytes(n, num_dirs), st) != hipSuccess)
      return launch_status("ds2_gru counters");
    int T_ = t_max, N_ = n, H_ = h, D_ = num_dirs, UB_ = UB, BT_ = BT;
    unsigned long long* stamps = stamp_mode() == 2 ? stamp_slots(ctrs, n, num_dirs) : nullptr;
    float* ring = reinterpret_cast<float*>(reinterpret_cast<char*>(ctrs) +
                                           align256(counter_bytes(n, num_dirs)));
    void* args[] = {&T_, &N_, &H_, &D_, &UB_, &BT_, &xproj, &w_hh_f, &w_hh_r, &b_hh_f,
                    &b_hh_r, &lens, &h_all, &gates, &ring, &ctrs, &err, &stamps};
    if (ring_reset(ring, n, h, num_dirs, st) != hipSuccess) return launch_status("ds2_gru ring");
    if (launch_gru_fwd_xl(t_max, n, h, num_dirs, xproj, w_hh_f, w_hh_r, b_hh_f, b_hh_r, lens,
                          h_all, gates, ring, err + 1, err, stamps, kDopPadLds, st)) {
      fold_err(err, err_out, st);
      return launch_status("ds2_gru_fwd");
    }
    (void)hipGetLastError();
    if (launch_gru_fwd_x6(t_max, n, h, num_dirs, xproj, w_hh_f, w_hh_r, b_hh_f, b_hh_r, lens,
                          h_all, gates, ring, ctrs, err, stamps, kDopPadLds, st)) {
      fold_err(err, err_out, st);
      return launch_status("ds2_gru_fwd");
    }
    (void)hipGetLastError();
    const void* fn = nullptr;
#define DS2_FDOP(K) \
  case K: fn = reinterpret_cast<const void*>(gru_fwd_dop_kernel<K>); break;
    switch ((UB + GW - 1) / GW) {
      DS2_FDOP(1) DS2_FDOP(2) DS2_FDOP(3) DS2_FDOP(4) DS2_FDOP(5) DS2_FDOP(6) DS2_FDOP(7)
      DS2_FDOP(8)
      default: break;
    }
#undef DS2_FDOP
    // the dynamic LDS keeps one workgroup per CU (every workgroup gets a whole CU's SIMDs)
    if (fn != nullptr &&
        rnn_launch(fn, dim3(grid), dim3(GT), args, kDopPadLds, st) == hipSuccess) {
      fold_err(err, err_out, st);
      return launch_status("ds2_gru_fwd");
    }
    (void)hipGetLastError();
  }
  hipLaunchKernelGGL(pack_fwd_kernel<3>, dim3(grid_cap((int64_t)num_dirs * UB * KS * 192)),
                     dim3(256), 0, st, w_hh_f, w_hh_r, h, num_dirs, UB, KS, wp);
  if (persistent && (h % 4) == 0) {
    if (hipMemsetAsync(ctrs, 0, counter_bytes(n, num_dirs), st) != hipSuccess)
      return launch_status("ds2_gru counters");
    int T_ = t_max, N_ = n, H_ = h, D_ = num_dirs, UB_ = UB, BT_ = BT;
    unsigned long long* stamps = stamp_slots(ctrs, n, num_dirs);
    int trace_ = stamp_mode() == 2 ? 1 : 0;
    void* args[] = {&T_, &N_, &H_, &D_, &UB_, &BT_, &xproj, &wp, &b_hh_f, &b_hh_r, &lens,
                    &h_all, &gates, &ctrs, &err, &stamps, &trace_};
    const void* fn = nullptr;
    const int kp = persist_ksw((KS + GW - 1) / GW, KC_FWD);
    switch (kp) {
      case 8: fn = reinterpret_cast<const void*>(gru_fwd_persist_kernel<8>); break;
      case 16: fn = reinterpret_cast<const void*>(gru_fwd_persist_kernel<16>); break;
      case 25: fn = reinterpret_cast<const void*>(gru_fwd_persist_kernel<25>); break;
      case 32: fn = reinterpret_cast<const void*>(gru_fwd_persist_kernel<32>); break;
      default: break;
    }
    if (fn != nullptr &&
        rnn_launch(fn, dim3(grid), dim3(GT), args, 0, st) == hipSuccess) {
      fold_err(err, err_out, st);
      return launch_status("ds2_gru_fwd");
    }
    (void)hipGetLastError();   // fall back to one launch per step
  }
  for (int s = 0; s < t_max; ++s) {
    switch (ksw) {
      DS2_FWD_CASE(8) DS2_FWD_CASE(16) DS2_FWD_CASE(32) DS2_FWD_CASE(48) DS2_FWD_CASE(64)
      DS2_FWD_CASE(80) DS2_FWD_CASE(96)
    }
  }
  return launch_status("ds2_gru_fwd");
}

static size_t gru_bwd_ws_base(int n, int h, int num_dirs) {
  const int64_t UB = (h + GU - 1) / GU;
  const int64_t KS = (3 * h + 3) / 4;
  return align256((size_t)(num_dirs * UB * KS * 64) * sizeof(float)) +
         align256((size_t)2 * n * num_dirs * h * sizeof(float)) +
         align256(counter_bytes(n, num_dirs)) + ring_bytes(n, h, num_dirs, 3) + 512;
}

// bias-gradient partial sums [batch tile][direction][4][H] fp64, at the end of the workspace
// (8-sample tiles: the XCD-local kernel's; the 16-sample kernels use the first half)
static size_t gru_db_bytes(int n, int h, int num_dirs) {
  return align256((size_t)((n + 7) / 8) * num_dirs * 4 * h * sizeof(double));
}

size_t ds2_gru_bwd_workspace_size(int n, int h, int num_dirs) {
  return gru_bwd_ws_base(n, h, num_dirs) + gru_db_bytes(n, h, num_dirs);
}

#define DS2_BWD_CASE(K)                                                                     \
  case K:                                                                                   \
    hipLaunchKernelGGL(gru_bwd_step_kernel<K>, dim3(grid), dim3(GT), 0, st, s, t_max, n, h,  \
                       num_dirs, UB, BT, dy, dy_dirs, wpt, h_all, gates, lens, dgates_x,     \
                       dgates_h, dhs);                                                       \
    break;

// workgroups the persistent backward launch holds at once (gru_bwd_run's choice), 0 for the
// per-step kernels
int ds2_gru_bwd_grid(int n, int h, int num_dirs) {
  if (n < 1 || h < 1 || (num_dirs != 1 && num_dirs != 2)) return 0;
  const int UB = (h + GU - 1) / GU, BT = (n + GB - 1) / GB;
  const int grid = mapped_grid(UB * num_dirs, BT);
  if (!persistent_enabled() || grid > num_cus()) return 0;
  if ((h % GU) == 0 && UB <= 8 * GW) {
    // the XCD-local or x6 launch may decline at run time and fall back to the direct-operand
    // kernel at `grid`: report the largest so the CU guard never budgets for fewer workgroups
    // than run
    const int g = gru_bwd_x6_grid(n, h, num_dirs);
    const int x = gru_xl_active(n, h, num_dirs);
    const int m = g > x ? g : x;
    return m > grid ? m : grid;
  }
  return (3 * h <= KC_BWD && (h % 4) == 0) ? grid : 0;
}

ds2_status_t ds2_gru_bwd(int t_max, int n, int h, int num_dirs, const float* dy, int dy_dirs,
                         const float* w_hh_f, const float* w_hh_r, const float* h_all,
                         const float* gates, const int* lens, float* dgates_x, float* dgates_h,
                         unsigned* err_out, void* ws, size_t ws_bytes, ds2_stream_t stream) {
  return ds2_gru_bwd_bias(t_max, n, h, num_dirs, dy, dy_dirs, w_hh_f, w_hh_r, h_all, gates, lens,
                          dgates_x, dgates_h, nullptr, nullptr, nullptr, nullptr, err_out, ws,
                          ws_bytes, stream);
}

// the recurrence; then, with db_ih_f non-null, the bias gradients (summed by the
// direct-operand kernel itself, else from dgates_x / dgates_h)
static ds2_status_t gru_bwd_run(int t_max, int n, int h, int num_dirs, const float* dy, int dy_dirs,
                                const float* w_hh_f, const float* w_hh_r, const float* h_all,
                                const float* gates, const int* lens, float* dgates_x,
                                float* dgates_h, unsigned* err_out, void* ws, hipStream_t st,
                                double* dbp, bool& summed, unsigned* camax, bool& camax_done,
                                int& db_tiles);

static ds2_status_t gru_bwd_bias_impl(int t_max, int n, int h, int num_dirs, const float* dy,
                                      int dy_dirs, const float* w_hh_f, const float* w_hh_r,
                                      const float* h_all, const float* gates, const int* lens,
                                      float* dgates_x, float* dgates_h, float* db_ih_f,
                                      float* db_hh_f, float* db_ih_r, float* db_hh_r,
                                      unsigned* err_out, void* ws, size_t ws_bytes,
                                      unsigned* camax, ds2_stream_t stream);

ds2_status_t ds2_gru_bwd_bias(int t_max, int n, int h, int num_dirs, const float* dy, int dy_dirs,
                              const float* w_hh_f, const float* w_hh_r, const float* h_all,
                              const float* gates, const int* lens, float* dgates_x,
                              float* dgates_h, float* db_ih_f, float* db_hh_f, float* db_ih_r,
                              float* db_hh_r, unsigned* err_out, void* ws, size_t ws_bytes,
                              ds2_stream_t stream) {
  return gru_bwd_bias_impl(t_max, n, h, num_dirs, dy, dy_dirs, w_hh_f, w_hh_r, h_all, gates, lens,
                           dgates_x, dgates_h, db_ih_f, db_hh_f, db_ih_r, db_hh_r, err_out, ws,
                           ws_bytes, nullptr, stream);
}

ds2_status_t ds2_gru_bwd_bias_amax(int t_max, int n, int h, int num_dirs, const float* dy,
                                   int dy_dirs, const float* w_hh_f, const float* w_hh_r,
                                   const float* h_all, const float* gates, const int* lens,
                                   float* dgates_x, float* dgates_h, float* db_ih_f,
                                   float* db_hh_f, float* db_ih_r, float* db_hh_r,
                                   unsigned* col_amax, unsigned* err_out, void* ws,
                                   size_t ws_bytes, ds2_stream_t stream) {
  if (col_amax == nullptr) return DS2_INVALID_VALUE;
  return gru_bwd_bias_impl(t_max, n, h, num_dirs, dy, dy_dirs, w_hh_f, w_hh_r, h_all, gates, lens,
                           dgates_x, dgates_h, db_ih_f, db_hh_f, db_ih_r, db_hh_r, err_out, ws,
                           ws_bytes, col_amax, stream);
}

static ds2_status_t gru_bwd_bias_impl(int t_max, int n, int h, int num_dirs, const float* dy,
                                      int dy_dirs, const float* w_hh_f, const float* w_hh_r,
                                      const float* h_all, const float* gates, const int* lens,
                                      float* dgates_x, float* dgates_h, float* db_ih_f,
                                      float* db_hh_f, float* db_ih_r, float* db_hh_r,
                                      unsigned* err_out, void* ws, size_t ws_bytes,
                                      unsigned* camax, ds2_stream_t stream) {
  if (t_max < 0 || n < 0 || h < 1 || (num_dirs != 1 && num_dirs != 2)) return DS2_INVALID_VALUE;
  if (gates == nullptr) return DS2_INVALID_VALUE;
  if (dy_dirs != 1 && dy_dirs != num_dirs) return DS2_INVALID_VALUE;
  const bool want_db = db_ih_f != nullptr;
  if (want_db && (db_hh_f == nullptr || (num_dirs == 2 && (db_ih_r == nullptr || db_hh_r == nullptr))))
    return DS2_INVALID_VALUE;
  if (ws == nullptr || ws_bytes < ds2_gru_bwd_workspace_size(n, h, num_dirs))
    return DS2_WORKSPACE_TOO_SMALL;
  hipStream_t st = as_stream(stream);
  double* dbp = reinterpret_cast<double*>(static_cast<char*>(ws) + gru_bwd_ws_base(n, h, num_dirs));
  const size_t camax_bytes = (size_t)2 * num_dirs * 3 * h * sizeof(unsigned);
  if (camax != nullptr && hipMemsetAsync(camax, 0, camax_bytes, st) != hipSuccess)
    return launch_status("ds2_gru_bwd_bias_amax");
  if (t_max == 0 || n == 0) {
    if (!want_db) return DS2_OK;
    // no rows: zero bias gradients
    if (hipMemsetAsync(dbp, 0, gru_db_bytes(n > 0 ? n : 1, h, num_dirs), st) != hipSuccess)
      return launch_status("ds2_gru_bwd_bias");
    hipLaunchKernelGGL(gru_db_final_kernel, dim3(cdiv(num_dirs * 4 * h, 256)), dim3(256), 0, st,
                       dbp, 1, num_dirs, h, db_ih_f, db_hh_f, db_ih_r, db_hh_r);
    return launch_status("ds2_gru_bwd_bias");
  }
  bool summed = false, camax_done = false;
  int db_tiles = (n + GB - 1) / GB;
  const ds2_status_t rc = gru_bwd_run(t_max, n, h, num_dirs, dy, dy_dirs, w_hh_f, w_hh_r, h_all,
                                      gates, lens, dgates_x, dgates_h, err_out, ws, st,
                                      want_db ? dbp : nullptr, summed, camax, camax_done, db_tiles);
  if (rc != DS2_OK) return rc;
  if (camax != nullptr && !camax_done) {
    // a kernel without the fused maxima ran: one column pass over each of dgx, dgh
    const ds2_status_t ra = ds2_amax(dgates_x, t_max * n, num_dirs * 3 * h, num_dirs * 3 * h,
                                     nullptr, camax, stream);
    const ds2_status_t rb = ra != DS2_OK ? ra
        : ds2_amax(dgates_h, t_max * n, num_dirs * 3 * h, num_dirs * 3 * h, nullptr,
                   camax + num_dirs * 3 * h, stream);
    if (rb != DS2_OK) return rb;
  }
  if (!want_db) return DS2_OK;
  int bt = db_tiles;
  if (!summed) {
    hipLaunchKernelGGL(gru_db_cols_kernel, dim3(num_dirs * 4 * h), dim3(256), 0, st, dgates_x,
                       dgates_h, t_max * n, num_dirs, h, dbp);
    bt = 1;
  }
  hipLaunchKernelGGL(gru_db_final_kernel, dim3(cdiv(num_dirs * 4 * h, 256)), dim3(256), 0, st, dbp,
                     bt, num_dirs, h, db_ih_f, db_hh_f, db_ih_r, db_hh_r);
  return launch_status("ds2_gru_bwd_bias");
}

static ds2_status_t gru_bwd_run(int t_max, int n, int h, int num_dirs, const float* dy, int dy_dirs,
                                const float* w_hh_f, const float* w_hh_r, const float* h_all,
                                const float* gates, const int* lens, float* dgates_x,
                                float* dgates_h, unsigned* err_out, void* ws, hipStream_t st,
                                double* dbp, bool& summed, unsigned* camax, bool& camax_done,
                                int& db_tiles) {
  if (num_dirs == 1) w_hh_r = w_hh_f;
  apply_spin_limit_env();
  apply_rnn_tune_env();
  const int UB = (h + GU - 1) / GU;
  const int KS = (3 * h + 3) / 4;
  const int BT = (n + GB - 1) / GB;
  const int chunk_ks = (std::min(3 * h, KC_BWD) + 3) / 4;
  const int ksw = pick_ksw((chunk_ks + GW - 1) / GW + 1);
  if (ksw < 0) return DS2_UNSUPPORTED_SHAPE;
  float* wpt = static_cast<float*>(ws);
  size_t off = align256((size_t)num_dirs * UB * KS * 64 * sizeof(float));
  float* dhs = reinterpret_cast<float*>(static_cast<char*>(ws) + off);
  const int grid = mapped_grid(UB * num_dirs, BT);
  const bool persistent = persistent_enabled() && grid <= num_cus() &&
                          (int64_t)t_max * n * num_dirs * 3 * h * 4 < (1ll << 31);
  unsigned* ctrs = reinterpret_cast<unsigned*>(
      reinterpret_cast<char*>(dhs) + align256((size_t)2 * n * num_dirs * h * sizeof(float)));
  unsigned* err = ctrs + num_dirs * BT;
  if (persistent && (h % GU) == 0 && UB <= 8 * GW) {
    if (hipMemsetAsync(ctrs, 0, counter_bytes(n, num_dirs), st) != hipSuccess)
      return launch_status("ds2_gru counters");
    int T_ = t_max, N_ = n, H_ = h, D_ = num_dirs, UB_ = UB, BT_ = BT, DYD_ = dy_dirs;
    unsigned long long* stamps = stamp_mode() == 2 ? stamp_slots(ctrs, n, num_dirs) : nullptr;
    float* ring = reinterpret_cast<float*>(reinterpret_cast<char*>(ctrs) +
                                           align256(counter_bytes(n, num_dirs)));
    void* args[] = {&T_, &N_, &H_, &D_, &UB_, &BT_, &dy, &DYD_, &w_hh_f, &w_hh_r, &h_all,
                    &gates, &lens, &dgates_x, &dgates_h, &ring, &ctrs, &err, &stamps, &dbp};
    if (launch_gru_bwd_xl(t_max, n, h, num_dirs, dy, dy_dirs, w_hh_f, w_hh_r, h_all, gates,
                          lens, dgates_x, dgates_h, ring, err + 1, err, stamps, dbp, kDopPadLds,
                          st, camax)) {
      fold_err(err, err_out, st);
      summed = dbp != nullptr;
      camax_done = camax != nullptr;
      db_tiles = (n + 7) / 8;
      return launch_status("ds2_gru_bwd");
    }
    (void)hipGetLastError();
    if (launch_gru_bwd_x6(t_max, n, h, num_dirs, dy, dy_dirs, w_hh_f, w_hh_r, h_all, gates,
                          lens, dgates_x, dgates_h, ring, ctrs, err, stamps, dbp, kDopPadLds, st,
                          camax, &camax_done)) {
      fold_err(err, err_out, st);
      summed = dbp != nullptr;
      return launch_status("ds2_gru_bwd");
    }
    (void)hipGetLastError();
    const void* fn = bwd_dop_fn((3 * UB + GW - 1) / GW);
    if (fn != nullptr &&
        rnn_launch(fn, dim3(grid), dim3(GT), args, kDopPadLds, st) == hipSuccess) {
      fold_err(err, err_out, st);
      summed = dbp != nullptr;
      return launch_status("ds2_gru_bwd");
    }
    (void)hipGetLastError();
  }
  hipLaunchKernelGGL(pack_bwd_kernel<3>, dim3(grid_cap((int64_t)num_dirs * UB * KS * 64)),
                     dim3(256), 0, st, w_hh_f, w_hh_r, h, num_dirs, UB, KS, wpt);
  if (persistent && 3 * h <= KC_BWD && (h % 4) == 0) {
    if (hipMemsetAsync(ctrs, 0, counter_bytes(n, num_dirs), st) != hipSuccess)
      return launch_status("ds2_gru counters");
    int T_ = t_max, N_ = n, H_ = h, D_ = num_dirs, UB_ = UB, BT_ = BT, DYD_ = dy_dirs;
    unsigned long long* stamps = stamp_mode() == 2 ? stamp_slots(ctrs, n, num_dirs) : nullptr;
    void* args[] = {&T_, &N_, &H_, &D_, &UB_, &BT_, &dy, &DYD_, &wpt, &h_all, &gates, &lens,
                    &dgates_x, &dgates_h, &ctrs, &err, &stamps};
    const void* fn = nullptr;
    const int kp = persist_ksw((KS + GW - 1) / GW, KC_BWD);
    switch (kp) {
      case 8: fn = reinterpret_cast<const void*>(gru_bwd_persist_kernel<8>); break;
      case 16: fn = reinterpret_cast<const void*>(gru_bwd_persist_kernel<16>); break;
      case 25: fn = reinterpret_cast<const void*>(gru_bwd_persist_kernel<25>); break;
      case 32: fn = reinterpret_cast<const void*>(gru_bwd_persist_kernel<32>); break;
      case 48: fn = reinterpret_cast<const void*>(gru_bwd_persist_kernel<48>); break;
      case 64: fn = reinterpret_cast<const void*>(gru_bwd_persist_kernel<64>); break;
      case 75: fn = reinterpret_cast<const void*>(gru_bwd_persist_kernel<75>); break;
      default: break;
    }
    if (fn != nullptr &&
        rnn_launch(fn, dim3(grid), dim3(GT), args, 0, st) == hipSuccess) {
      fold_err(err, err_out, st);
      return launch_status("ds2_gru_bwd");
    }
    (void)hipGetLastError();
  }
  for (int s = 0; s < t_max; ++s) {
    switch (ksw) {
      DS2_BWD_CASE(8) DS2_BWD_CASE(16) DS2_BWD_CASE(32) DS2_BWD_CASE(48) DS2_BWD_CASE(64)
      DS2_BWD_CASE(80) DS2_BWD_CASE(96)
    }
  }
  return launch_status("ds2_gru_bwd");
}

// ---------------------------------------------------------------------------------------
// supported_rnns['rnn'] (nn.RNN, tanh; model.py:15) on the persistent machinery: the
// one-gate fp16x3 instantiations of the GRU recurrences (gru_split.hip), falling back to the
// per-step kernels of rnn.hip (ds2_rnn_fwd / ds2_rnn_bwd) where they decline the shape or
// DS2_RNN_PERSISTENT=0.  Workspace: the counters and the hand-off ring.
static bool rnn_persistent_ok(int t_max, int n, int h, int num_dirs) {
  const int g = rnn_h3_grid(n, h, num_dirs);
  return persistent_enabled() && g > 0 && g <= num_cus() &&
         (int64_t)t_max * n * num_dirs * h * 4 < (1ll << 31);
}

size_t ds2_rnn_fwd_workspace_size(int n, int h, int num_dirs) {
  if (n < 1 || h < 1 || num_dirs < 1) return 256;
  return align256(counter_bytes(n, num_dirs)) + ring_bytes(n, h, num_dirs, 1) + 256;
}

ds2_status_t ds2_rnn_fwd_ws(int t_max, int n, int h, int num_dirs, const float* xproj,
                            const float* w_hh_f, const float* w_hh_r, const float* b_hh_f,
                            const float* b_hh_r, const int* lens, float* h_all, unsigned* err_out,
                            void* ws, size_t ws_bytes, ds2_stream_t stream) {
  if (t_max < 0 || n < 0 || h < 1 || (num_dirs != 1 && num_dirs != 2)) return DS2_INVALID_VALUE;
  if (t_max == 0 || n == 0) return DS2_OK;
  if (xproj == nullptr || w_hh_f == nullptr || b_hh_f == nullptr || lens == nullptr ||
      h_all == nullptr || (num_dirs == 2 && (w_hh_r == nullptr || b_hh_r == nullptr)))
    return DS2_INVALID_VALUE;
  if (ws == nullptr || ws_bytes < ds2_rnn_fwd_workspace_size(n, h, num_dirs))
    return DS2_WORKSPACE_TOO_SMALL;
  if (num_dirs == 1) {
    w_hh_r = w_hh_f;
    b_hh_r = b_hh_f;
  }
  hipStream_t st = as_stream(stream);
  if (rnn_persistent_ok(t_max, n, h, num_dirs)) {
    unsigned* ctrs = static_cast<unsigned*>(ws);
    unsigned* err = ctrs + num_dirs * ((n + GB - 1) / GB);
    float* ring = reinterpret_cast<float*>(static_cast<char*>(ws) + align256(counter_bytes(n, num_dirs)));
    if (hipMemsetAsync(ctrs, 0, counter_bytes(n, num_dirs), st) != hipSuccess)
      return launch_status("ds2_rnn counters");
    if (ring_reset(ring, n, h, num_dirs, st) != hipSuccess) return launch_status("ds2_rnn ring");
    unsigned long long* stamps = stamp_mode() == 2 ? stamp_slots(ctrs, n, num_dirs) : nullptr;
    if (launch_rnn_fwd_h3(t_max, n, h, num_dirs, xproj, w_hh_f, w_hh_r, b_hh_f, b_hh_r, lens,
                          h_all, ring, ctrs, err, stamps, kDopPadLds, st)) {
      fold_err(err, err_out, st);
      return launch_status("ds2_rnn_fwd");
    }
    (void)hipGetLastError();
  }
  return ds2_rnn_fwd(t_max, n, h, num_dirs, xproj, w_hh_f, w_hh_r, b_hh_f, b_hh_r, lens, h_all,
                     stream);
}

size_t ds2_rnn_bwd_workspace_size(int n, int h, int num_dirs) {
  if (n < 1 || h < 1 || num_dirs < 1) return 256;
  return align256(counter_bytes(n, num_dirs)) + ring_bytes(n, h, num_dirs, 3) + 256;
}

int ds2_rnn_bwd_grid(int n, int h, int num_dirs) {
  if (n < 1 || h < 1 || (num_dirs != 1 && num_dirs != 2)) return 0;
  const int g = rnn_h3_grid(n, h, num_dirs);
  return persistent_enabled() && g > 0 && g <= num_cus() ? g : 0;
}

ds2_status_t ds2_rnn_bwd_ws(int t_max, int n, int h, int num_dirs, const float* dy, int dy_dirs,
                            const float* w_hh_f, const float* w_hh_r, const float* h_all,
                            const int* lens, float* dgates, unsigned* col_amax, unsigned* err_out,
                            void* ws, size_t ws_bytes, ds2_stream_t stream) {
  if (t_max < 0 || n < 0 || h < 1 || (num_dirs != 1 && num_dirs != 2)) return DS2_INVALID_VALUE;
  if (dy_dirs != 1 && dy_dirs != num_dirs) return DS2_INVALID_VALUE;
  if (ws == nullptr || ws_bytes < ds2_rnn_bwd_workspace_size(n, h, num_dirs))
    return DS2_WORKSPACE_TOO_SMALL;
  hipStream_t st = as_stream(stream);
  if (col_amax != nullptr &&
      hipMemsetAsync(col_amax, 0, (size_t)num_dirs * h * sizeof(unsigned), st) != hipSuccess)
    return launch_status("ds2_rnn_bwd_ws");
  if (t_max == 0 || n == 0) return DS2_OK;
  if (dy == nullptr || w_hh_f == nullptr || h_all == nullptr || lens == nullptr ||
      dgates == nullptr || (num_dirs == 2 && w_hh_r == nullptr))
    return DS2_INVALID_VALUE;
  if (num_dirs == 1) w_hh_r = w_hh_f;
  if (rnn_persistent_ok(t_max, n, h, num_dirs)) {
    unsigned* ctrs = static_cast<unsigned*>(ws);
    unsigned* err = ctrs + num_dirs * ((n + GB - 1) / GB);
    float* ring = reinterpret_cast<float*>(static_cast<char*>(ws) + align256(counter_bytes(n, num_dirs)));
    if (hipMemsetAsync(ctrs, 0, counter_bytes(n, num_dirs), st) != hipSuccess)
      return launch_status("ds2_rnn counters");
    unsigned long long* stamps = stamp_mode() == 2 ? stamp_slots(ctrs, n, num_dirs) : nullptr;
    if (launch_rnn_bwd_h3(t_max, n, h, num_dirs, dy, dy_dirs, w_hh_f, w_hh_r, h_all, lens, dgates,
                          ring, ctrs, err, stamps, kDopPadLds, st, col_amax)) {
      fold_err(err, err_out, st);
      return launch_status("ds2_rnn_bwd");
    }
    (void)hipGetLastError();
  }
  const ds2_status_t rc = ds2_rnn_bwd(t_max, n, h, num_dirs, dy, dy_dirs, w_hh_f, w_hh_r, h_all,
                                      lens, dgates, stream);
  if (rc != DS2_OK || col_amax == nullptr) return rc;
  return ds2_amax(dgates, t_max * n, num_dirs * h, num_dirs * h, nullptr, col_amax, stream);
}

}  // extern "C"
