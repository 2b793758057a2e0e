// (Bi)directional LSTM recurrence on MFMA (v_mfma_f32_16x16x4_f32), fp32 —
// SURVEY §8 row a8' (reference model.py:14 supported_rnns['lstm'] = nn.LSTM).
//
// Same structure as gru.hip: the input projection x @ W_ih^T + b_ih (both
// directions, 4H gate rows i, f, g, o) is a separate GEMM; this file runs the
// sequential part.  Workgroup = (16 hidden units, direction, 16 samples); the
// forward product is gh[16 x 64] = h_prev[16 x H] @ W_hh[64 rows (i,f,g,o of
// the 16 units)]^T, the backward one rec[16 x 16] = dg[16 x 4H] @ W_hh[:, 16
// units].  K is split over the 8 waves; partial tiles are reduced through LDS.
//
// Gate math follows ATen's LSTM cell:
//   i = sigmoid(.), f = sigmoid(.), g = tanh(.), o = sigmoid(.)
//   c' = f*c + i*g,  h' = o*tanh(c')
// Packed-sequence semantics as in gru.hip: direction 1 of a sample of length len
// starts at t = len-1 from (h, c) = 0; outputs past len are 0.
//
// Persistent variants (one cooperative launch per layer, W_hh in registers, the
// hand-off of gru.hip) run when the grid fits the chip; otherwise one launch per
// time step carries the cell state through a ping-pong buffer.
#include "rnn_common.h"

#include <algorithm>

namespace ds2 {

constexpr int LKC_FWD = 1024;   // max H staged in LDS (forward)
constexpr int LKC_BWD = 2048;   // 4H columns staged per chunk (backward)
constexpr int LRP = 4 * GU + 1; // forward reduction row pitch (4 gates x 16 units)

// ---------------------------------------------------------------------------
// shared pointwise pieces
struct LstmFwdOut {
  float i, f, g, o, c, h;
};

__device__ __forceinline__ LstmFwdOut lstm_cell(float ai, float af, float ag, float ao, float cp) {
  LstmFwdOut r;
  r.i = sigmoid_fast(ai);
  r.f = sigmoid_fast(af);
  r.g = tanh_fast(ag);
  r.o = sigmoid_fast(ao);
  r.c = r.f * cp + r.i * r.g;
  r.h = r.o * tanh_fast(r.c);
  return r;
}

// d(gate pre-activations) from dh, the carried dc (= dc_{t+1} * f_{t+1}), the cached
// activations and c_t, c_{t-1}; returns the new carry dc_t * f_t.
__device__ __forceinline__ float lstm_cell_bwd(float dh, float dc_carry, float gi, float gf,
                                               float gg, float go, float c, float cp,
                                               float& dai, float& daf, float& dag, float& dao) {
  const float tc = tanh_fast(c);
  const float dc = dc_carry + dh * go * (1.f - tc * tc);
  dao = dh * tc * go * (1.f - go);
  dai = dc * gg * gi * (1.f - gi);
  dag = dc * gi * (1.f - gg * gg);
  daf = dc * cp * gf * (1.f - gf);
  return dc * gf;
}

// ---------------------------------------------------------------------------
// forward step (one launch per time step)
template <int KSW>
__global__ __launch_bounds__(GT) void lstm_fwd_step_kernel(
    int s, int T, int N, int H, int D, int UB, int BT, const float* __restrict__ xproj,
    const float* __restrict__ wp, const float* __restrict__ b_f, const float* __restrict__ b_r,
    const int* __restrict__ lens, float* __restrict__ h_all, float* __restrict__ c_all,
    float* __restrict__ gates, float* __restrict__ cs) {
  constexpr int PITCH = LKC_FWD + 2;
  __shared__ __attribute__((aligned(16))) float hs[GB * PITCH];
  int ub, d, bt;
  if (!map_work(UB * D, BT, UB, ub, d, bt)) return;
  const int n0 = bt * GB;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int t = d == 0 ? s : T - 1 - s;
  const int tp = d == 0 ? t - 1 : t + 1;
  const int KS = (H + 3) / 4;
  const int per = (KS + GW - 1) / GW;
  const int a_ks = wave * per;
  const int b_ks = min(KS, a_ks + per);

  f32x4 acc[4];
#pragma unroll
  for (int g = 0; g < 4; ++g) acc[g] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (s > 0) {
    float w[4][KSW];
    const float* wpd = wp + ((int64_t)d * UB + ub) * KS * 4 * 64 + lane;
#pragma unroll
    for (int i = 0; i < KSW; ++i) {
      const int ks = a_ks + i;
#pragma unroll
      for (int g = 0; g < 4; ++g) w[g][i] = ks < b_ks ? wpd[((int64_t)ks * 4 + g) * 64] : 0.f;
    }
    stage_rows(h_all + ((int64_t)tp * N * D + d) * H, (int64_t)D * H, N, n0, 0, H, hs, PITCH);
    __syncthreads();
    const float* hrow = hs + (lane & 15) * PITCH + (lane >> 4);
#pragma unroll
    for (int i = 0; i < KSW; ++i) {
      const int ks = a_ks + i;
      if (ks < b_ks) {
        const int k = 4 * ks;
        const float a = (k + (lane >> 4) < H) ? hrow[k] : 0.f;
#pragma unroll
        for (int g = 0; g < 4; ++g)
          acc[g] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, w[g][i], acc[g], 0, 0, 0);
      }
    }
    __syncthreads();
  }
  float* red = hs;
#pragma unroll
  for (int g = 0; g < 4; ++g)
#pragma unroll
    for (int r = 0; r < 4; ++r)
      red[(wave * GB + (lane >> 4) * 4 + r) * LRP + g * GU + (lane & 15)] = acc[g][r];
  __syncthreads();
  if (threadIdx.x >= GB * GU) return;
  const int m = threadIdx.x >> 4;
  const int u = threadIdx.x & 15;
  const int n = n0 + m;
  const int j = ub * GU + u;
  if (n >= N || j >= H) return;
  const int64_t row = ((int64_t)t * N + n) * D + d;
  const int64_t cidx = (int64_t)n * D * H + (int64_t)d * H + j;
  const int64_t plane = (int64_t)N * D * H;
  LstmFwdOut o{0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (t < lens[n]) {
    float gh[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      float v = 0.f;
#pragma unroll
      for (int w8 = 0; w8 < GW; ++w8) v += red[(w8 * GB + m) * LRP + g * GU + u];
      gh[g] = v;
    }
    const float* bh = d == 0 ? b_f : b_r;
    const float* xp = xproj + row * 4 * H;
    const float cp = s > 0 ? cs[((s + 1) & 1) * plane + cidx] : 0.f;
    o = lstm_cell(gh[0] + bh[j] + xp[j], gh[1] + bh[H + j] + xp[H + j],
                  gh[2] + bh[2 * H + j] + xp[2 * H + j], gh[3] + bh[3 * H + j] + xp[3 * H + j],
                  cp);
  }
  cs[(s & 1) * plane + cidx] = o.c;
  h_all[row * H + j] = o.h;
  if (c_all != nullptr) c_all[row * H + j] = o.c;
  if (gates != nullptr) {
    float* gp = gates + row * 4 * H;
    gp[j] = o.i;
    gp[H + j] = o.f;
    gp[2 * H + j] = o.g;
    gp[3 * H + j] = o.o;
  }
}

// ---------------------------------------------------------------------------
// backward step (BPTT, one launch per time step)
template <int KSW>
__global__ __launch_bounds__(GT) void lstm_bwd_step_kernel(
    int s, int T, int N, int H, int D, int UB, int BT, const float* __restrict__ dy, int dyd,
    const float* __restrict__ wpt, const float* __restrict__ c_all,
    const float* __restrict__ gates, const int* __restrict__ lens, float* __restrict__ dg,
    float* __restrict__ dcs) {
  constexpr int PITCH = LKC_BWD + 2;
  __shared__ __attribute__((aligned(16))) float hs[GB * PITCH];
  int ub, d, bt;
  if (!map_work(UB * D, BT, UB, ub, d, bt)) return;
  const int n0 = bt * GB;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int t = d == 0 ? T - 1 - s : s;
  const int tq = d == 0 ? t + 1 : t - 1;
  const int H4 = 4 * H;
  const int KS = H;   // (4H + 3) / 4

  f32x4 acc0 = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 acc1 = f32x4{0.f, 0.f, 0.f, 0.f};
  if (s > 0) {
    const float* dgq = dg + ((int64_t)tq * N * D + d) * H4;
    const float* wpd = wpt + ((int64_t)d * UB + ub) * KS * 64 + lane;
    for (int kc0 = 0; kc0 < H4; kc0 += LKC_BWD) {
      const int kc1 = min(H4, kc0 + LKC_BWD);
      const int ks0 = kc0 / 4;
      const int ks1 = kc1 / 4;
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
      stage_rows(dgq, (int64_t)D * H4, N, n0, kc0, kc1, hs, PITCH);
      __syncthreads();
      const float* hrow = hs + (lane & 15) * PITCH + (lane >> 4) - kc0;
#pragma unroll
      for (int i = 0; i < KSW; i += 2) {
        const int ks = a_ks + i;
        if (ks < b_ks) acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(hrow[4 * ks], w[i], acc0, 0, 0, 0);
        if (i + 1 < KSW && ks + 1 < b_ks)
          acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(hrow[4 * ks + 4], w[i + 1], acc1, 0, 0, 0);
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
  const int64_t row = ((int64_t)t * N + n) * D + d;
  const int64_t cidx = (int64_t)n * D * H + (int64_t)d * H + j;
  const int64_t plane = (int64_t)N * D * H;
  float dai = 0.f, daf = 0.f, dag = 0.f, dao = 0.f, carry = 0.f;
  if (t < lens[n]) {
    float rec = 0.f, dcc = 0.f;
    if (s > 0) {
#pragma unroll
      for (int w8 = 0; w8 < GW; ++w8) rec += red[(w8 * GB + m) * RP + u];
      dcc = dcs[((s + 1) & 1) * plane + cidx];
    }
    const float dh = dy[(((int64_t)t * N + n) * dyd + (dyd > 1 ? d : 0)) * H + j] + rec;
    const float* gp = gates + row * 4 * H;
    const int tp = d == 0 ? t - 1 : t + 1;
    const float cp = (tp >= 0 && tp < T) ? c_all[(((int64_t)tp * N + n) * D + d) * H + j] : 0.f;
    carry = lstm_cell_bwd(dh, dcc, gp[j], gp[H + j], gp[2 * H + j], gp[3 * H + j],
                          c_all[row * H + j], cp, dai, daf, dag, dao);
  }
  dcs[(s & 1) * plane + cidx] = carry;
  float* go = dg + row * H4;
  go[j] = dai;
  go[H + j] = daf;
  go[2 * H + j] = dag;
  go[3 * H + j] = dao;
}

// ---------------------------------------------------------------------------
// persistent forward: W_hh fragments (4 gates x KSW k-steps) in registers, cell
// state in a register of the owning thread, h hand-off through sc1 stores +
// per-(direction, batch tile) arrival counters.  BTS = 16-sample tiles per workgroup:
// with BTS = 2 every wave runs its W_hh fragments over two tiles of A operands, so a
// batch whose 16-sample tiles would not fit the chip as one workgroup each (cfg4: 7 x
// BiLSTM-1024 at batch 64 = 512 workgroups) runs as ONE launch of 32-sample workgroups
// instead of two consecutive launches (the dependent steps, not the MFMAs, set the pace);
// the reduction tile then aliases the staged rows.
template <int KSW, int BTS>
__global__ __launch_bounds__(GT) void lstm_fwd_persist_kernel(
    int T, int N, int H, int D, int UB, int BT, const float* __restrict__ xproj,
    const float* __restrict__ wp, const float* __restrict__ b_f, const float* __restrict__ b_r,
    const int* __restrict__ lens, float* __restrict__ h_all, float* __restrict__ c_all,
    float* __restrict__ gates, unsigned* __restrict__ counters, unsigned* __restrict__ err,
    int n_base) {
  constexpr int PITCH = LKC_FWD + 4;
  constexpr int RB = GB * BTS;         // samples per workgroup
  constexpr int HSF = RB * PITCH, REDF = GW * RB * LRP;
  __shared__ __attribute__((aligned(16))) float hs[BTS == 1 || HSF >= REDF ? HSF : REDF];
  __shared__ float red_own[BTS == 1 ? REDF : 1];
  float* red = BTS == 1 ? red_own : hs;
  __shared__ int flag;
  int ub, d, bt;
  if (!map_work(UB * D, BT, UB, ub, d, bt)) return;
  const int n0 = n_base + bt * RB;     // samples [n_base, ...) of a batch chunk
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int KS = H / 4;                    // host guarantees H % 4 == 0, GW * KSW >= KS
  const int a_ks = wave * KSW;
  const int b_ks = min(KS, a_ks + KSW);
  unsigned* gflags = counters + (D * BT + 1) + (d * BT + bt) * UB;   // flag variant
  const __amdgpu_buffer_rsrc_t h_rs = __builtin_amdgcn_make_buffer_rsrc(
      h_all, (short)0, T * N * D * H * 4, 0x00020000);

  float w[4][KSW];
  {
    const float* wpd = wp + ((int64_t)d * UB + ub) * KS * 4 * 64 + lane;
#pragma unroll
    for (int i = 0; i < KSW; ++i) {
      const int ks = a_ks + i;
#pragma unroll
      for (int g = 0; g < 4; ++g) w[g][i] = ks < b_ks ? wpd[((int64_t)ks * 4 + g) * 64] : 0.f;
    }
  }
  const float* bh = d == 0 ? b_f : b_r;
  const int m = threadIdx.x >> 4;
  const int u = threadIdx.x & 15;
  const int n = n0 + m;
  const int j = ub * GU + u;
  const bool owner = threadIdx.x < RB * GU && n < N && j < H;
  float bias[4] = {0.f, 0.f, 0.f, 0.f};
  int len = 0;
  if (owner) {
#pragma unroll
    for (int g = 0; g < 4; ++g) bias[g] = bh[g * H + j];
    len = lens[n];
  }
#pragma unroll
  for (int g = 0; g < 4; ++g) settle(bias[g]);
  settle(len);
  float c = 0.f;
  LstmFwdOut prev{0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  int64_t prev_row = -1;
  for (int s = 0; s < T; ++s) {
    const int t = d == 0 ? s : T - 1 - s;
    const int tp = d == 0 ? t - 1 : t + 1;
    const int64_t row = ((int64_t)t * N + n) * D + d;
    float xg[4] = {0.f, 0.f, 0.f, 0.f};
    if (owner && t < len) {
      const float* xp = xproj + row * 4 * H;
#pragma unroll
      for (int g = 0; g < 4; ++g) xg[g] = xp[g * H + j];
    }
    f32x4 acc[BTS][4];
#pragma unroll
    for (int b = 0; b < BTS; ++b)
#pragma unroll
      for (int g = 0; g < 4; ++g) acc[b][g] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (s > 0) {
      if (!flags_wait(gflags, UB, (unsigned)s, err, &flag)) {
        poison_rest(h_all, s, T, d != 0, N, D, n, d, H, j, H, 1, owner);
        return;
      }
      stage_rows_sc1<(RB * LKC_FWD / 4 + GT - 1) / GT, RB>(
          h_all + ((int64_t)tp * N * D + d) * H, D * H, N, n0, H, 4 * GW * KSW, hs, PITCH);
      __syncthreads();
#pragma unroll
      for (int b = 0; b < BTS; ++b) {
        const float* hrow = hs + (b * GB + (lane & 15)) * PITCH + (lane >> 4) + 4 * a_ks;
#pragma unroll
        for (int i = 0; i < KSW; ++i) {
          const float a = hrow[4 * i];
#pragma unroll
          for (int g = 0; g < 4; ++g)
            acc[b][g] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, w[g][i], acc[b][g], 0, 0, 0);
        }
      }
      if (BTS > 1) __syncthreads();   // every wave's reads of hs done before red overwrites it
    }
#pragma unroll
    for (int b = 0; b < BTS; ++b)
#pragma unroll
      for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          red[(wave * RB + b * GB + (lane >> 4) * 4 + r) * LRP + g * GU + (lane & 15)] = acc[b][g][r];
    __syncthreads();
    if (owner) {
      LstmFwdOut o{0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      if (t < len) {
        float gh[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          float v = 0.f;
#pragma unroll
          for (int w8 = 0; w8 < GW; ++w8) v += red[(w8 * RB + m) * LRP + g * GU + u];
          gh[g] = v + bias[g] + xg[g];
        }
        o = lstm_cell(gh[0], gh[1], gh[2], gh[3], c);
      }
      c = o.c;
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, o.h), h_rs,
                                            static_cast<int>((row * H + j) * 4), 0, kSc1);
      prev = o;
      prev_row = row;
    }
    flags_arrive(gflags + ub, (unsigned)s + 1);
    // backward-only caches, off the critical path
    if (owner) {
      if (c_all != nullptr) c_all[prev_row * H + j] = prev.c;
      if (gates != nullptr) {
        float* gp = gates + prev_row * 4 * H;
        gp[j] = prev.i;
        gp[H + j] = prev.f;
        gp[2 * H + j] = prev.g;
        gp[3 * H + j] = prev.o;
      }
    }
  }
}

// persistent backward: W_hh^T fragments for NCH chunks of 4*GW*KSWC gate columns in
// registers; dc carried in a register; gate gradients handed off through sc1 stores.
// BTS as in the forward (BTS = 2 stages 32 rows per chunk: KSWC = 32 keeps them in LDS).
// XG: the same-XCD group placement of the GRU backward (rnn_common.h map_work_xgrp), each
// (direction, batch tile) group on its own 8 / G XCDs, same hand-off; bit-identical results.
// cfg4 bf16 145.8 -> 144.9 ms per step (the forward's too: 143.7).  Measured and not kept on top of it: the GRU's
// plain same-XCD copies (a two-slot ring stored write-through and plainly, consumers staging
// the same-XCD producers' pieces from the plain copy): 150.5 ms, with dg's own stores moved
// after the flag or not (profiles/r4zd_*).
template <int KSWC, int NCH, int BTS, bool XG>
__global__ __launch_bounds__(GT) void lstm_bwd_persist_kernel(
    int T, int N, int H, int D, int UB, int BT, const float* __restrict__ dy, int dyd,
    const float* __restrict__ wpt, const float* __restrict__ c_all,
    const float* __restrict__ gates, const int* __restrict__ lens, float* __restrict__ dg,
    unsigned* __restrict__ counters, unsigned* __restrict__ err, int n_base) {
  constexpr int CW = 4 * GW * KSWC;         // gate columns per chunk (<= LKC_BWD)
  constexpr int PITCH = CW + 4;
  constexpr int RB = GB * BTS;              // samples per workgroup
  __shared__ __attribute__((aligned(16))) float hs[RB * PITCH];
  float* red = hs;                          // reduction buffer aliases the staged rows
  __shared__ int flag;
  int ub, d, bt;
  if (XG ? !map_work_xgrp(UB, BT, D, ub, d, bt) : !map_work(UB * D, BT, UB, ub, d, bt)) return;
  const int n0 = n_base + bt * RB;     // samples [n_base, ...) of a batch chunk
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int H4 = 4 * H;
  const int KS = H;
  unsigned* gflags = counters + (D * BT + 1) + (d * BT + bt) * UB;   // flag variant
  const __amdgpu_buffer_rsrc_t g_rs = __builtin_amdgcn_make_buffer_rsrc(
      dg, (short)0, T * N * D * H4 * 4, 0x00020000);

  float w[NCH][KSWC];
  {
    const float* wpd = wpt + ((int64_t)d * UB + ub) * KS * 64 + lane;
#pragma unroll
    for (int c = 0; c < NCH; ++c)
#pragma unroll
      for (int i = 0; i < KSWC; ++i) {
        const int ks = c * (CW / 4) + wave * KSWC + i;
        w[c][i] = ks < KS ? wpd[(int64_t)ks * 64] : 0.f;
      }
  }
  const int m = threadIdx.x >> 4;
  const int u = threadIdx.x & 15;
  const int n = n0 + m;
  const int j = ub * GU + u;
  const bool owner = threadIdx.x < RB * GU && n < N && j < H;
  int len = owner ? lens[n] : 0;
  settle(len);
  constexpr int RP = GU + 1;
  float carry = 0.f;

  for (int s = 0; s < T; ++s) {
    const int t = d == 0 ? T - 1 - s : s;
    // inputs of this step that do not depend on other workgroups: issue first
    float dyv = 0.f, gi = 0.f, gf = 0.f, gg = 0.f, go = 0.f, cc = 0.f, cp = 0.f;
    const int64_t row = ((int64_t)t * N + n) * D + d;
    if (owner && t < len) {
      dyv = dy[(((int64_t)t * N + n) * dyd + (dyd > 1 ? d : 0)) * H + j];
      const float* gp = gates + row * 4 * H;
      gi = gp[j];
      gf = gp[H + j];
      gg = gp[2 * H + j];
      go = gp[3 * H + j];
      cc = c_all[row * H + j];
      const int tp = d == 0 ? t - 1 : t + 1;
      if (tp >= 0 && tp < T) cp = c_all[(((int64_t)tp * N + n) * D + d) * H + j];
    }
    f32x4 acc0[BTS], acc1[BTS];
#pragma unroll
    for (int b = 0; b < BTS; ++b) {
      acc0[b] = f32x4{0.f, 0.f, 0.f, 0.f};
      acc1[b] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    if (s > 0) {
      const int tq = d == 0 ? t + 1 : t - 1;
      if (!flags_wait(gflags, UB, (unsigned)s, err, &flag)) {
        poison_rest(dg, s, T, d == 0, N, D, n, d, H, j, H4, 4, owner);
        return;
      }
      const float* dgq = dg + ((int64_t)tq * N * D + d) * H4;
      // n0 opaque per step: otherwise the compiler hoists every chunk's staging offsets out
      // of the step loop (NCH x loads-per-lane registers held for all T steps), and the full
      // chunk's loads could not be in flight at once beside the W_hh^T fragments
      int n0s = n0;
      asm volatile("" : "+s"(n0s));
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
        if (c > 0) __syncthreads();
        const int c0 = c * CW;
        // one staging per chunk, all its loads in flight (16 rows x 2048 columns: 16 per lane;
        // two half-chunk stagings of 8 were 1.2 % slower at cfg4, 143.0 vs 141.6 ms per step)
        stage_rows_sc1<(RB * CW / 4 + GT - 1) / GT, RB>(dgq + c0, D * H4, N, n0s,
                                                        max(0, min(H4 - c0, CW)), CW, hs, PITCH);
        __syncthreads();
#pragma unroll
        for (int b = 0; b < BTS; ++b) {
          const float* hrow = hs + (b * GB + (lane & 15)) * PITCH + (lane >> 4) + 4 * wave * KSWC;
#pragma unroll
          for (int i = 0; i < KSWC; i += 2) {
            acc0[b] = __builtin_amdgcn_mfma_f32_16x16x4f32(hrow[4 * i], w[c][i], acc0[b], 0, 0, 0);
            if (i + 1 < KSWC)
              acc1[b] = __builtin_amdgcn_mfma_f32_16x16x4f32(hrow[4 * i + 4], w[c][i + 1], acc1[b],
                                                             0, 0, 0);
          }
        }
      }
      __syncthreads();                      // all reads of hs done before red overwrites it
    }
#pragma unroll
    for (int b = 0; b < BTS; ++b)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        red[(wave * RB + b * GB + (lane >> 4) * 4 + r) * RP + (lane & 15)] = acc0[b][r] + acc1[b][r];
    __syncthreads();
    if (owner) {
      float dai = 0.f, daf = 0.f, dag = 0.f, dao = 0.f;
      if (t < len) {
        float rec = 0.f;
#pragma unroll
        for (int w8 = 0; w8 < GW; ++w8) rec += red[(w8 * RB + m) * RP + u];
        carry = lstm_cell_bwd(dyv + rec, carry, gi, gf, gg, go, cc, cp, dai, daf, dag, dao);
      } else {
        carry = 0.f;
      }
      const int o = static_cast<int>((row * H4 + j) * 4);
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, dai), g_rs, o, 0, kSc1);
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, daf), g_rs, o + 4 * H, 0,
                                            kSc1);
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, dag), g_rs, o + 8 * H, 0,
                                            kSc1);
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, dao), g_rs, o + 12 * H, 0,
                                            kSc1);
    }
    flags_arrive(gflags + ub, (unsigned)s + 1);
  }
}

// Direct-operand persistent forward (H % 16 == 0): gru_fwd_dop_kernel's hand-off with
// the LSTM cell.  Each producer publishes its 16 units x 16 samples of h_t per batch tile
// as one 1-KB transposed tile,
//   hx[slot][d][workgroup batch tile][b < BTS][unit block][q][r][c]  (unit 4 q + c, sample r),
// stored by wave 0 with one 16-B sc1 store per lane; every consumer wave loads the tiles of
// its own producers straight into its A operands (lane (r, q): the k values 16 blk + 4 q +
// 0..3 of sample r), so no LDS staging of h and no barrier stands between the loads and
// the MFMAs.  HM: 1 the sentinel ring of gru_fwd_dop_kernel, 0 per-producer flags (the 8-tile
// shapes, H > 512: W_hh's 128 fragment registers leave no room for the sentinel spin's live
// state); BTS as in lstm_fwd_persist_kernel.  h_all, c_all and the gate cache are written after the publish.
// H3: the W_hh product on fp16x3 (rnn_common.h; default since round 5, DS2_LSTM_H3=0 keeps fp32
// MFMA): the wave's blocks are taken in pairs (one v_mfma_f32_16x16x32_f16 k-step: slots 0..3
// of lane (r, q) from block 2p, 4..7 from 2p + 1, the 16 B the lane loads from each tile),
// W_hh rows (gate, unit) scaled by their own 2^e, h (|h| < 1) by 2^14; three products per
// pair instead of sixteen v_mfma_f32_16x16x4_f32 (each 4x the cycles of one f16 product).
template <int NBW, int HM, int BTS, bool H3 = false>
__global__ __launch_bounds__(GT) __attribute__((amdgpu_waves_per_eu(2, 2))) void lstm_fwd_dop_kernel(
    int T, int N, int H, int D, int UB, int BT, const float* __restrict__ xproj,
    const float* __restrict__ w_f, const float* __restrict__ w_r, const float* __restrict__ b_f,
    const float* __restrict__ b_r, const int* __restrict__ lens, float* __restrict__ h_all,
    float* __restrict__ c_all, float* __restrict__ gates, float* __restrict__ hx,
    unsigned* __restrict__ counters, unsigned* __restrict__ err, int n_base, int xg) {
  constexpr int RB = GB * BTS;
  __shared__ float red[GW * RB * LRP];
  __shared__ __attribute__((aligned(16))) float tile[RB * GU];
  __shared__ int flag;
  __shared__ int failed;
  int ub, d, bt;
  // xg: the same-XCD group placement (as lstm_bwd_persist_kernel's XG), same hand-off
  if (xg ? !map_work_xgrp(UB, BT, D, ub, d, bt) : !map_work(UB * D, BT, UB, ub, d, bt)) return;
  const int n0 = n_base + bt * RB;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  int b0, nb;
  simd_split(UB, wave, b0, nb);                 // host guarantees nb <= NBW
  const unsigned* gflags = counters + (D * BT + 1) + (d * BT + bt) * UB;
  unsigned* myflag = counters + (D * BT + 1) + (d * BT + bt) * UB + ub;
  const int slot_floats = D * BT * BTS * UB * 256;
  static_assert(HM == 0 || HM == 1, "hand-off form");
  constexpr bool SENT = HM == 1;
  constexpr bool FLAG = HM == 0;
  constexpr int NSLOT = SENT ? kRingSlots : 2;
  const __amdgpu_buffer_rsrc_t x_rs =
      __builtin_amdgcn_make_buffer_rsrc(hx, (short)0, NSLOT * slot_floats * 4, 0x00020000);
  const int grp_off = (d * BT + bt) * BTS * UB * 256;      // this group's tiles in a slot
  if (SENT) {
    if (threadIdx.x == 0) failed = 0;
    __syncthreads();
  }

  // W_hh fragments: w[g][i][c] = W_hh[g H + ub 16 + (lane & 15)][16 (b0 + i) + 4 (lane >> 4) + c]
  // (fp32), or their fp16x3 pairs w3[g][p] (blocks 2p, 2p + 1) with the row scales undone by
  // unscale[g] (the owner thread's unit is threadIdx.x & 15 = lane & 15: the same row)
  constexpr int NW32 = H3 ? 1 : NBW;
  constexpr int NPR = H3 ? (NBW + 1) / 2 : 1;
  f32x4 w[4][NW32];
  Duo w3[4][NPR];
  float unscale[4] = {1.f, 1.f, 1.f, 1.f};
  {
    const float* W = d == 0 ? w_f : w_r;
    const float* wr = W + (int64_t)(ub * GU + (lane & 15)) * H + 16 * b0 + 4 * (lane >> 4);
    auto wblk = [&](int g, int i) {
      return i < nb ? *reinterpret_cast<const f32x4*>(wr + (int64_t)g * H * H + 16 * i)
                    : f32x4{0.f, 0.f, 0.f, 0.f};
    };
    if constexpr (H3) {
      float mx[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < NBW; ++i)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const f32x4 v = wblk(g, i);
#pragma unroll
          for (int q = 0; q < 4; ++q) mx[g] = fmaxf(mx[g], fabsf(v[q]));
        }
      // the row's max over the lane's 4 k quads, then over the 8 waves (LDS, before `red` is used)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        mx[g] = fmaxf(mx[g], __shfl_xor(mx[g], 16));
        mx[g] = fmaxf(mx[g], __shfl_xor(mx[g], 32));
        if (lane < 16) red[(wave * 4 + g) * 16 + lane] = mx[g];
      }
      __syncthreads();
      float sc[4];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        float m8 = 0.f;
#pragma unroll
        for (int w8 = 0; w8 < GW; ++w8) m8 = fmaxf(m8, red[(w8 * 4 + g) * 16 + (lane & 15)]);
        const int e = h3_row_exp(m8);
        sc[g] = __builtin_ldexpf(1.f, e);
        unscale[g] = __builtin_ldexpf(1.f, -(e + 14));
      }
      __syncthreads();
#pragma unroll
      for (int p = 0; p < NPR; ++p)
#pragma unroll
        for (int g = 0; g < 4; ++g) w3[g][p] = split2h(wblk(g, 2 * p), wblk(g, 2 * p + 1), sc[g]);
    } else {
#pragma unroll
      for (int i = 0; i < NBW; ++i)
#pragma unroll
        for (int g = 0; g < 4; ++g) w[g][i] = wblk(g, i);
#pragma unroll
      for (int i = 0; i < NBW; ++i)
#pragma unroll
        for (int g = 0; g < 4; ++g) settle(w[g][i]);
    }
  }
  const float* bh = d == 0 ? b_f : b_r;
  const int m = threadIdx.x >> 4;               // sample within the workgroup (< RB)
  const int u = threadIdx.x & 15;
  const int n = n0 + m;
  const int j = ub * GU + u;
  const bool owner = threadIdx.x < RB * GU && n < N;
  float bias[4] = {0.f, 0.f, 0.f, 0.f};
  int len = 0;
  if (owner) {
#pragma unroll
    for (int g = 0; g < 4; ++g) bias[g] = bh[g * H + j];
    len = lens[n];
  }
#pragma unroll
  for (int g = 0; g < 4; ++g) settle(bias[g]);
  settle(len);
  // this thread's slot in its batch tile's transposed tile: (q = u >> 2, r = m % 16, c = u & 3)
  const int tpos = (m >> 4) * GB * GU + ((u >> 2) * GB + (m & 15)) * 4 + (u & 3);
  float c = 0.f;
  LstmFwdOut prev{0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  int64_t prev_row = -1;
  for (int s = 0; s < T; ++s) {
    const int t = d == 0 ? s : T - 1 - s;
    const int64_t row = ((int64_t)t * N + n) * D + d;
    float xg[4] = {0.f, 0.f, 0.f, 0.f};
    if (owner && t < len) {
      const float* xp = xproj + row * 4 * H;
#pragma unroll
      for (int g = 0; g < 4; ++g) xg[g] = xp[g * H + j];
    }
    f32x4 acc[BTS][4];
#pragma unroll
    for (int b = 0; b < BTS; ++b)
#pragma unroll
      for (int g = 0; g < 4; ++g) acc[b][g] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (s > 0) {
      if (FLAG && !flags_wait(gflags, UB, (unsigned)s, err, &flag)) {
        poison_rest(h_all, s, T, d != 0, N, D, n, d, H, j, H, 1, owner);
        return;
      }
      const int base = (((s - 1) % NSLOT) * slot_floats + grp_off + b0 * 256 + lane * 4) * 4;
      f32x4 hv[BTS][NBW];
#pragma unroll
      for (int b = 0; b < BTS; ++b)
#pragma unroll
        for (int i = 0; i < NBW; ++i) {
          const int off = i < nb ? base + (b * UB + i) * 1024 : 0x7ffffff0;
          hv[b][i] = __builtin_bit_cast(f32x4,
                                        __builtin_amdgcn_raw_buffer_load_b128(x_rs, off, 0, kSc1));
        }
      asm volatile("" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int b = 0; b < BTS; ++b) {
        if constexpr (H3) {
#pragma unroll
          for (int i = 0; i < NBW; ++i)
            if (SENT && i < nb && !spin_tile(hv[b][i], x_rs, base + (b * UB + i) * 1024, err))
              failed = 1;
#pragma unroll
          for (int p = 0; p < NPR; ++p) {
            const f32x4 z4 = f32x4{0.f, 0.f, 0.f, 0.f};
            const Duo a = split2h(hv[b][2 * p], 2 * p + 1 < NBW ? hv[b][2 * p + 1] : z4, 16384.f);
#pragma unroll
            for (int g = 0; g < 4; ++g) acc[b][g] = mma3h(a, w3[g][p], acc[b][g]);
          }
        } else {
#pragma unroll
          for (int i = 0; i < NBW; ++i) {
            if (SENT && i < nb && !spin_tile(hv[b][i], x_rs, base + (b * UB + i) * 1024, err))
              failed = 1;
#pragma unroll
            for (int cc = 0; cc < 4; ++cc)
#pragma unroll
              for (int g = 0; g < 4; ++g)
                acc[b][g] = __builtin_amdgcn_mfma_f32_16x16x4f32(hv[b][i][cc], w[g][i][cc],
                                                                 acc[b][g], 0, 0, 0);
          }
        }
      }
    }
#pragma unroll
    for (int b = 0; b < BTS; ++b)
#pragma unroll
      for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          red[(wave * RB + b * GB + (lane >> 4) * 4 + r) * LRP + g * GU + (lane & 15)] = acc[b][g][r];
#pragma unroll
    for (int g = 0; g < 4; ++g) settle(xg[g]);
    __syncthreads();
    if (SENT && failed) {
      poison_rest(h_all, s, T, d != 0, N, D, n, d, H, j, H, 1, owner);
      return;
    }
    if (threadIdx.x < RB * GU) {
      float hout = 0.f;
      if (owner) {
        LstmFwdOut o{0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        if (t < len) {
          float gh[4];
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            float v = 0.f;
#pragma unroll
            for (int w8 = 0; w8 < GW; ++w8) v += red[(w8 * RB + m) * LRP + g * GU + u];
            gh[g] = (H3 ? v * unscale[g] : v) + bias[g] + xg[g];
          }
          o = lstm_cell(gh[0], gh[1], gh[2], gh[3], c);
        }
        c = o.c;
        hout = o.h;
        prev = o;
        prev_row = row;
      }
      tile[tpos] = hout;
    }
    __syncthreads();
    if (wave == 0) {
#pragma unroll
      for (int b = 0; b < BTS; ++b) {
        const int toff = (grp_off + (b * UB + ub) * 256 + lane * 4) * 4;
        if (SENT) {
          const u32x4 v = desentinel(*reinterpret_cast<const u32x4*>(tile + b * GB * GU + lane * 4));
          if (b == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // last step's sentinels
          __builtin_amdgcn_raw_buffer_store_b128(v, x_rs, (s % NSLOT) * slot_floats * 4 + toff, 0,
                                                 kSc1);
        } else {
          const u32x4 v = *reinterpret_cast<const u32x4*>(tile + b * GB * GU + lane * 4);
          __builtin_amdgcn_raw_buffer_store_b128(v, x_rs, (s & 1) * slot_floats * 4 + toff, 0, kSc1);
        }
      }
      if (SENT) {
        const u32x4 sv = u32x4{kSentinel, kSentinel, kSentinel, kSentinel};
#pragma unroll
        for (int b = 0; b < BTS; ++b) {
          const int toff = (grp_off + (b * UB + ub) * 256 + lane * 4) * 4;
          __builtin_amdgcn_raw_buffer_store_b128(sv, x_rs, ((s + 2) % NSLOT) * slot_floats * 4 + toff,
                                                 0, kSc1);
        }
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane == 0)
          __hip_atomic_store(myflag, (unsigned)s + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    // outputs consumed only by later kernels, off the critical path
    if (owner) {
      h_all[row * H + j] = prev.h;
      if (c_all != nullptr) c_all[prev_row * H + j] = prev.c;
      if (gates != nullptr) {
        float* gp = gates + prev_row * 4 * H;
        gp[j] = prev.i;
        gp[H + j] = prev.f;
        gp[2 * H + j] = prev.g;
        gp[3 * H + j] = prev.o;
      }
    }
  }
}

// per-step kernels: forward needs <= 32 (H <= 1024), backward <= 64 (2048-column chunks)
static int lstm_pick_ksw(int per) {
  const int opts[] = {8, 16, 32, 64};
  for (int k : opts)
    if (per <= k) return k;
  return -1;
}

// gru_split.hip: the fp16x3 backward with the LSTM cell (gru_bwd_h3_kernel<., 4>)
int lstm_h3_grid(int h, int num_dirs, int bt_launch);
bool launch_lstm_bwd_h3(int t_max, int n, int h, int num_dirs, const float* dy, int dy_dirs,
                        const float* w_hh_f, const float* w_hh_r, const float* c_all,
                        const float* gates, const int* lens, float* dgates, float* ring,
                        unsigned* ctrs, unsigned* err, size_t lds_pad, hipStream_t st,
                        unsigned* camax, int tile0, int bt_launch);
size_t h3_bwd_ring_bytes(int n_tiles, int h, int num_dirs, int ng);
// gru_split.hip: the single-term backward of cfg4's bf16 mode (lstm_bwd_h1_kernel)
int lstm_h1_grid(int n, int h, int num_dirs);
size_t lstm_h1_ring_bytes(int n, int h, int num_dirs);
bool launch_lstm_bwd_h1(int t_max, int n, int h, int num_dirs, const float* dy, int dy_dirs,
                        const float* w_hh_f, const float* w_hh_r, const float* c_all,
                        const float* gates, const int* lens, float* dgates, float* ring,
                        unsigned* ctrs, unsigned* err, size_t lds_pad, hipStream_t st,
                        unsigned* camax);

}  // namespace ds2

using namespace ds2;

extern "C" {

// counters (one per group) + error word + per-producer flags (64 per group)
static inline size_t lstm_counter_bytes(int n, int num_dirs) {
  const size_t groups = (size_t)num_dirs * ((n + GB - 1) / GB);
  return align256((groups + 1 + groups * 64) * sizeof(unsigned));
}

// Batch chunking of the persistent launches: the largest number of 16-sample tiles per
// launch whose grid fits the chip (one workgroup per CU); a batch with more tiles runs as
// consecutive launches over sample ranges [n_base, n_base + 16 * chunk) -- the samples'
// recurrences are independent (cfg4: 7 x BiLSTM-1024 at batch 64 = two launches of 256).
static inline int lstm_chunk_tiles(int UB, int D, int BT) {
  int c = BT;
  while (c > 1 && mapped_grid(UB * D, c) > num_cus()) --c;
  return c;
}

// 16-sample tiles per workgroup of the persistent kernels (template BTS): 2 when the
// batch's 16-sample tiles would not fit the chip one workgroup each but its 32-sample
// tiles do -- one launch per layer instead of consecutive batch chunks.
static inline int lstm_bts(int UB, int D, int BT) {
  const bool fits2 = mapped_grid(UB * D, (BT + 1) / 2) <= num_cus();
  return mapped_grid(UB * D, BT) > num_cus() && fits2 ? 2 : 1;
}

// ring of 1-KB hand-off tiles of the direct-operand forward: kRingSlots slots of
// (direction, 16-sample tile rounded up to a 32-sample workgroup, unit block)
static inline size_t lstm_ring_bytes(int n, int h, int num_dirs) {
  const size_t UB = (h + GU - 1) / GU, BT2 = 2 * (((size_t)n + 2 * GB - 1) / (2 * GB));
  return align256(kRingSlots * (size_t)num_dirs * BT2 * UB * 256 * sizeof(float));
}
constexpr unsigned kLstmDopPadLds = 80 * 1024;   // dynamic LDS: one workgroup per CU

// the recurrences' W_hh products on fp16x3 (default since round 5; DS2_LSTM_H3=0 keeps the
// fp32-MFMA kernels)
static inline bool lstm_h3_on() {
  const char* e = getenv("DS2_LSTM_H3");
  return !(e != nullptr && e[0] == '0');
}

size_t ds2_lstm_fwd_workspace_size(int n, int h, int num_dirs) {
  const int64_t UB = (h + GU - 1) / GU;
  const int64_t KS = (h + 3) / 4;
  return align256((size_t)(num_dirs * UB * KS * 4 * 64) * sizeof(float)) +
         align256((size_t)2 * n * num_dirs * h * sizeof(float)) + lstm_counter_bytes(n, num_dirs) +
         lstm_ring_bytes(n, h, num_dirs) + 256;
}

#define DS2_LFWD_CASE(K)                                                                    \
  case K:                                                                                   \
    hipLaunchKernelGGL(lstm_fwd_step_kernel<K>, dim3(grid), dim3(GT), 0, st, s, t_max, n, h, \
                       num_dirs, UB, BT, xproj, wp, b_hh_f, b_hh_r, lens, h_all, c_all, gates, \
                       cs);                                                                 \
    break;

ds2_status_t ds2_lstm_fwd(int t_max, int n, int h, int num_dirs, const float* xproj,
                          const float* w_hh_f, const float* w_hh_r, const float* b_hh_f,
                          const float* b_hh_r, const int* lens, float* h_all, float* c_all,
                          float* gates, unsigned* err_out, void* ws, size_t ws_bytes,
                          ds2_stream_t stream) {
  if (t_max < 0 || n < 0 || h < 1 || (num_dirs != 1 && num_dirs != 2)) return DS2_INVALID_VALUE;
  if (h > LKC_FWD) return DS2_UNSUPPORTED_SHAPE;
  if (t_max == 0 || n == 0) return DS2_OK;
  if (ws == nullptr || ws_bytes < ds2_lstm_fwd_workspace_size(n, h, num_dirs))
    return DS2_WORKSPACE_TOO_SMALL;
  if (num_dirs == 1) {
    w_hh_r = w_hh_f;
    b_hh_r = b_hh_f;
  }
  hipStream_t st = as_stream(stream);
  apply_spin_limit_env();
  const int UB = (h + GU - 1) / GU;
  const int KS = (h + 3) / 4;
  const int BT = (n + GB - 1) / GB;
  const int ksw = lstm_pick_ksw((KS + GW - 1) / GW);
  if (ksw < 0 || ksw > 32) return DS2_UNSUPPORTED_SHAPE;
  float* wp = static_cast<float*>(ws);
  size_t off = align256((size_t)num_dirs * UB * KS * 4 * 64 * sizeof(float));
  float* cs = reinterpret_cast<float*>(static_cast<char*>(ws) + off);
  off += align256((size_t)2 * n * num_dirs * h * sizeof(float));
  unsigned* ctrs = reinterpret_cast<unsigned*>(static_cast<char*>(ws) + off);
  float* ring = reinterpret_cast<float*>(static_cast<char*>(ws) + off +
                                         lstm_counter_bytes(n, num_dirs));
  // direct-operand persistent kernels (W_hh read unpacked; no LDS staging of h)
  if (persistent_enabled() && (h % GU) == 0 && UB <= 8 * GW &&
      (int64_t)t_max * n * num_dirs * h * 4 < (1ll << 31)) {
    int hm = 1;   // the sentinel ring
    const int bts = lstm_bts(UB, num_dirs, BT);
    const int BTW = (BT + bts - 1) / bts;
    const int ct = lstm_chunk_tiles(UB, num_dirs, BTW);
    // NBW = blocks per wave, rounded up to an instantiated 1, 2, 4 or 8 (extra blocks are
    // predicated off)
    const int need = (UB + GW - 1) / GW;
    const int nbw = need <= 1 ? 1 : need <= 2 ? 2 : need <= 4 ? 4 : 8;
    // 8 blocks per wave (H > 512): W_hh's 128 fragment registers leave no room for the
    // sentinel spin's live state (it spills), so those run the flag hand-off
    if (nbw == 8) hm = 0;
    const void* fn = nullptr;
    const bool h3 = lstm_h3_on();
#define DS2_LDOP(K, HM)                                                                       \
  case K:                                                                                     \
    if (h3)                                                                                   \
      fn = bts == 2 ? reinterpret_cast<const void*>(lstm_fwd_dop_kernel<K, HM, 2, true>)      \
                    : reinterpret_cast<const void*>(lstm_fwd_dop_kernel<K, HM, 1, true>);     \
    else                                                                                      \
      fn = bts == 2 ? reinterpret_cast<const void*>(lstm_fwd_dop_kernel<K, HM, 2>)            \
                    : reinterpret_cast<const void*>(lstm_fwd_dop_kernel<K, HM, 1>);           \
    break;
    switch (nbw) {
      DS2_LDOP(1, 1) DS2_LDOP(2, 1) DS2_LDOP(4, 1) DS2_LDOP(8, 0)
      default: break;
    }
#undef DS2_LDOP
    bool ok = fn != nullptr && mapped_grid(UB * num_dirs, ct) <= num_cus();
    bool launched = false;
    for (int b0 = 0; ok && b0 < BTW; b0 += ct) {
      int T_ = t_max, N_ = n, H_ = h, D_ = num_dirs, UB_ = UB, BT_ = std::min(ct, BTW - b0);
      int NB_ = b0 * GB * bts;
      unsigned* err = ctrs + num_dirs * BT_;
      if (hipMemsetAsync(ctrs, 0, lstm_counter_bytes(n, num_dirs), st) != hipSuccess)
        return launch_status("ds2_lstm counters");
      if (hm != 0 && hipMemsetAsync(ring, 0xFF, lstm_ring_bytes(n, h, num_dirs), st) != hipSuccess)
        return launch_status("ds2_lstm ring");
      // same-XCD groups (DS2_GRU_XCD) where they tile the XCDs: cfg4 bf16 144.9 -> 143.7 ms
      int XG_ = xcd_groups_on() && xgrp_fits(UB, BT_, num_dirs) ? 1 : 0;
      void* args[] = {&T_, &N_, &H_, &D_, &UB_, &BT_, &xproj, &w_hh_f, &w_hh_r, &b_hh_f,
                      &b_hh_r, &lens, &h_all, &c_all, &gates, &ring, &ctrs, &err, &NB_, &XG_};
      ok = rnn_launch(fn,
                      dim3(XG_ ? xgrp_grid(UB, BT_, num_dirs) : mapped_grid(UB * num_dirs, BT_)),
                      dim3(GT), args, kLstmDopPadLds, st) == hipSuccess;
      if (ok) fold_err(err, err_out, st);
      if (!ok && launched) return launch_status("ds2_lstm_fwd chunk");
      launched = launched || ok;
    }
    if (ok) return launch_status("ds2_lstm_fwd");
    (void)hipGetLastError();
  }
  hipLaunchKernelGGL(pack_fwd_kernel<4>, dim3(grid_cap((int64_t)num_dirs * UB * KS * 256)),
                     dim3(256), 0, st, w_hh_f, w_hh_r, h, num_dirs, UB, KS, wp);
  const int grid = mapped_grid(UB * num_dirs, BT);
  const int kp = persist_ksw((KS + GW - 1) / GW, LKC_FWD);
  const int bts = lstm_bts(UB, num_dirs, BT);
  const int BTW = (BT + bts - 1) / bts;                   // workgroup batch tiles
  const int ct = lstm_chunk_tiles(UB, num_dirs, BTW);
  if (persistent_enabled() && (h % 4) == 0 && mapped_grid(UB * num_dirs, ct) <= num_cus() &&
      kp > 0 && kp <= 32 && (int64_t)t_max * n * num_dirs * h * 4 < (1ll << 31)) {
    const void* fn = nullptr;
#define DS2_LFP(K)                                                                        \
  case K:                                                                                 \
    fn = bts == 2 ? reinterpret_cast<const void*>(lstm_fwd_persist_kernel<K, 2>)          \
                  : reinterpret_cast<const void*>(lstm_fwd_persist_kernel<K, 1>);         \
    break;
    switch (kp) {
      DS2_LFP(8) DS2_LFP(16) DS2_LFP(25) DS2_LFP(32)
      default: break;
    }
#undef DS2_LFP
    bool ok = fn != nullptr;
    for (int b0 = 0; ok && b0 < BTW; b0 += ct) {
      int T_ = t_max, N_ = n, H_ = h, D_ = num_dirs, UB_ = UB, BT_ = std::min(ct, BTW - b0);
      int NB_ = b0 * GB * bts;
      unsigned* err = ctrs + num_dirs * BT_;
      if (hipMemsetAsync(ctrs, 0, lstm_counter_bytes(n, num_dirs), st) != hipSuccess)
        return launch_status("ds2_lstm counters");
      void* args[] = {&T_, &N_, &H_, &D_, &UB_, &BT_, &xproj, &wp, &b_hh_f, &b_hh_r, &lens,
                      &h_all, &c_all, &gates, &ctrs, &err, &NB_};
      ok = rnn_launch(fn, dim3(mapped_grid(UB * num_dirs, BT_)), dim3(GT), args,
                                      0, st) == hipSuccess;
      if (ok) fold_err(err, err_out, st);
      if (!ok && b0 > 0) return launch_status("ds2_lstm_fwd chunk");
    }
    if (ok) return launch_status("ds2_lstm_fwd");
    (void)hipGetLastError();   // fall back to one launch per step
  }
  for (int s = 0; s < t_max; ++s) {
    switch (ksw) {
      DS2_LFWD_CASE(8) DS2_LFWD_CASE(16) DS2_LFWD_CASE(32)
    }
  }
  return launch_status("ds2_lstm_fwd");
}

// the fp16x3 backward's counters (as the GRU's: group counters, error word, 64 flags and 64
// XCC ids per group) and record ring, after the fp32 kernels' regions
static inline size_t lstm_h3_ctr_bytes(int n, int num_dirs) {
  const size_t groups = (size_t)num_dirs * ((n + GB - 1) / GB);
  return align256((groups + 1 + groups * 128) * sizeof(unsigned));
}
static size_t lstm_bwd_ws_base(int n, int h, int num_dirs) {
  const int64_t UB = (h + GU - 1) / GU;
  const int64_t KS = h;
  return align256((size_t)(num_dirs * UB * KS * 64) * sizeof(float)) +
         align256((size_t)2 * n * num_dirs * h * sizeof(float)) + lstm_counter_bytes(n, num_dirs);
}

size_t ds2_lstm_bwd_workspace_size(int n, int h, int num_dirs) {
  if (n < 1 || h < 1 || num_dirs < 1) return 256;
  const size_t r3 = h3_bwd_ring_bytes((n + GB - 1) / GB, h, num_dirs, 4);
  const size_t r1 = lstm_h1_ring_bytes(n, h, num_dirs);
  return lstm_bwd_ws_base(n, h, num_dirs) + lstm_h3_ctr_bytes(n, num_dirs) +
         align256(r3 > r1 ? r3 : r1) + 256;
}

// the single-term backward (cfg4's bf16 mode) as launched: its grid, 0 when it declines
static int lstm_h1_launch_grid(int t_max, int n, int h, int num_dirs) {
  if (!persistent_enabled() || (h % GU) != 0) return 0;
  if ((int64_t)t_max * n * num_dirs * 4 * h * 4 >= (1ll << 31)) return 0;
  const int g = lstm_h1_grid(n, h, num_dirs);
  return g > 0 && g <= num_cus() ? g : 0;
}

// ds2_lstm_bwd_half falls back to ds2_lstm_bwd when the single-term launch declines at run time
// (t_max past the 32-bit offset bound, a failed launch); that kernel's 16-sample tiles can hold
// more workgroups, so report the larger grid: the CU guard never budgets for fewer than run
int ds2_lstm_bwd_half_grid(int n, int h, int num_dirs) {
  if (n < 1 || h < 1 || (num_dirs != 1 && num_dirs != 2)) return 0;
  const int g = lstm_h1_launch_grid(1, n, h, num_dirs);
  const int f = ds2_lstm_bwd_grid(n, h, num_dirs);
  return g > f ? g : f;
}

ds2_status_t ds2_lstm_bwd_half(int t_max, int n, int h, int num_dirs, const float* dy, int dy_dirs,
                               const float* w_hh_f, const float* w_hh_r, const float* c_all,
                               const float* gates, const int* lens, float* dgates,
                               unsigned* err_out, void* ws, size_t ws_bytes, ds2_stream_t stream) {
  if (t_max < 0 || n < 0 || h < 1 || (num_dirs != 1 && num_dirs != 2)) return DS2_INVALID_VALUE;
  if (t_max == 0 || n == 0) return DS2_OK;
  if (gates == nullptr || c_all == nullptr) return DS2_INVALID_VALUE;
  if (dy_dirs != 1 && dy_dirs != num_dirs) return DS2_INVALID_VALUE;
  if (ws == nullptr || ws_bytes < ds2_lstm_bwd_workspace_size(n, h, num_dirs))
    return DS2_WORKSPACE_TOO_SMALL;
  if (lstm_h1_launch_grid(t_max, n, h, num_dirs) > 0) {
    hipStream_t st = as_stream(stream);
    apply_spin_limit_env();
    char* base3 = static_cast<char*>(ws) + lstm_bwd_ws_base(n, h, num_dirs);
    unsigned* ctrs3 = reinterpret_cast<unsigned*>(base3);
    float* ring3 = reinterpret_cast<float*>(base3 + lstm_h3_ctr_bytes(n, num_dirs));
    const int BT32 = (n + 31) / 32;
    unsigned* err = ctrs3 + num_dirs * BT32;
    if (hipMemsetAsync(ctrs3, 0, lstm_h3_ctr_bytes(n, num_dirs), st) != hipSuccess)
      return launch_status("ds2_lstm counters");
    if (launch_lstm_bwd_h1(t_max, n, h, num_dirs, dy, dy_dirs, w_hh_f,
                           num_dirs == 2 ? w_hh_r : w_hh_f, c_all, gates, lens, dgates, ring3,
                           ctrs3, err, kLstmDopPadLds, st, nullptr)) {
      fold_err(err, err_out, st);
      return launch_status("ds2_lstm_bwd_half");
    }
    (void)hipGetLastError();
  }
  return ds2_lstm_bwd(t_max, n, h, num_dirs, dy, dy_dirs, w_hh_f, w_hh_r, c_all, gates, lens,
                      dgates, err_out, ws, ws_bytes, stream);
}

// the fp16x3 backward's launch: 16-sample tiles per launch (consecutive launches cover the
// batch), 0 when it declines the shape
static int lstm_h3_tiles(int t_max, int n, int h, int num_dirs) {
  if (!lstm_h3_on() || !persistent_enabled() || (h % GU) != 0) return 0;
  if ((int64_t)t_max * n * num_dirs * 4 * h * 4 >= (1ll << 31)) return 0;
  const int UB = h / GU, BT = (n + GB - 1) / GB;
  const int ct = lstm_chunk_tiles(UB, num_dirs, BT);
  const int g = lstm_h3_grid(h, num_dirs, ct);
  return g > 0 && g <= num_cus() ? ct : 0;
}

#define DS2_LBWD_CASE(K)                                                                    \
  case K:                                                                                   \
    hipLaunchKernelGGL(lstm_bwd_step_kernel<K>, dim3(grid), dim3(GT), 0, st, s, t_max, n, h, \
                       num_dirs, UB, BT, dy, dy_dirs, wpt, c_all, gates, lens, dgates, dcs);  \
    break;

// workgroups one persistent backward launch holds at once (a batch larger than the chip
// runs as consecutive launches of at most this many), 0 for the per-step kernels
int ds2_lstm_bwd_grid(int n, int h, int num_dirs) {
  if (n < 1 || h < 1 || (num_dirs != 1 && num_dirs != 2)) return 0;
  // t_max only bounds 32-bit offsets; 1 asks about the launch shape
  const int ct = lstm_h3_tiles(1, n, h, num_dirs);
  if (ct > 0) return lstm_h3_grid(h, num_dirs, ct);
  if (!persistent_enabled() || (h % 4) != 0) return 0;
  const int UB = (h + GU - 1) / GU, BT = (n + GB - 1) / GB;
  int bts = lstm_bts(UB, num_dirs, BT);
  if (bts == 2 && 4 * h > 2 * 4 * GW * 32) bts = 1;
  const int BTW = (BT + bts - 1) / bts;
  const int g = mapped_grid(UB * num_dirs, lstm_chunk_tiles(UB, num_dirs, BTW));
  return g <= num_cus() ? g : 0;
}

ds2_status_t ds2_lstm_bwd(int t_max, int n, int h, int num_dirs, const float* dy, int dy_dirs,
                          const float* w_hh_f, const float* w_hh_r, const float* c_all,
                          const float* gates, const int* lens, float* dgates, unsigned* err_out,
                          void* ws, size_t ws_bytes, ds2_stream_t stream) {
  if (t_max < 0 || n < 0 || h < 1 || (num_dirs != 1 && num_dirs != 2)) return DS2_INVALID_VALUE;
  if (t_max == 0 || n == 0) return DS2_OK;
  if (gates == nullptr || c_all == nullptr) return DS2_INVALID_VALUE;
  if (dy_dirs != 1 && dy_dirs != num_dirs) return DS2_INVALID_VALUE;
  if (ws == nullptr || ws_bytes < ds2_lstm_bwd_workspace_size(n, h, num_dirs))
    return DS2_WORKSPACE_TOO_SMALL;
  if (num_dirs == 1) w_hh_r = w_hh_f;
  hipStream_t st = as_stream(stream);
  apply_spin_limit_env();
  const int UB = (h + GU - 1) / GU;
  const int KS = h;
  const int BT = (n + GB - 1) / GB;
  const int chunk_ks = std::min(4 * h, LKC_BWD) / 4;
  const int ksw = lstm_pick_ksw((chunk_ks + GW - 1) / GW);
  if (ksw < 0) return DS2_UNSUPPORTED_SHAPE;
  float* wpt = static_cast<float*>(ws);
  size_t off = align256((size_t)num_dirs * UB * KS * 64 * sizeof(float));
  float* dcs = reinterpret_cast<float*>(static_cast<char*>(ws) + off);
  off += align256((size_t)2 * n * num_dirs * h * sizeof(float));
  unsigned* ctrs = reinterpret_cast<unsigned*>(static_cast<char*>(ws) + off);
  // the fp16x3 backward (gru_split.hip, NG = 4): W_hh read directly, gate gradients handed
  // off as one scaled fp16 hi / lo record per producer and step
  const int ct3 = lstm_h3_tiles(t_max, n, h, num_dirs);
  if (ct3 > 0) {
    char* base3 = static_cast<char*>(ws) + lstm_bwd_ws_base(n, h, num_dirs);
    unsigned* ctrs3 = reinterpret_cast<unsigned*>(base3);
    float* ring3 = reinterpret_cast<float*>(base3 + lstm_h3_ctr_bytes(n, num_dirs));
    bool ok = true, launched = false;
    for (int b0 = 0; ok && b0 < BT; b0 += ct3) {
      const int bt = std::min(ct3, BT - b0);
      unsigned* err = ctrs3 + num_dirs * bt;
      if (hipMemsetAsync(ctrs3, 0, lstm_h3_ctr_bytes(n, num_dirs), st) != hipSuccess)
        return launch_status("ds2_lstm counters");
      ok = launch_lstm_bwd_h3(t_max, n, h, num_dirs, dy, dy_dirs, w_hh_f, w_hh_r, c_all, gates,
                              lens, dgates, ring3, ctrs3, err, kLstmDopPadLds, st, nullptr, b0, bt);
      if (ok) fold_err(err, err_out, st);
      if (!ok && launched) return launch_status("ds2_lstm_bwd chunk");
      launched = launched || ok;
    }
    if (ok) return launch_status("ds2_lstm_bwd");
    (void)hipGetLastError();
  }
  hipLaunchKernelGGL(pack_bwd_kernel<4>, dim3(grid_cap((int64_t)num_dirs * UB * KS * 64)),
                     dim3(256), 0, st, w_hh_f, w_hh_r, h, num_dirs, UB, KS, wpt);
  const int grid = mapped_grid(UB * num_dirs, BT);
  if (persistent_enabled() && (h % 4) == 0 &&
      (int64_t)t_max * n * num_dirs * 4 * h * 4 < (1ll << 31)) {
    // smallest (k-steps per wave per chunk, chunks) covering 4H gate columns
    const int opts[] = {8, 16, 25, 32, 48, 64};
    int kswc = -1, nch = -1;
    for (int c = 1; c <= 2 && kswc < 0; ++c)
      for (int k : opts)
        if (c * 4 * GW * k >= 4 * h) {
          kswc = k;
          nch = c;
          break;
        }
    // 32-sample workgroups stage chunks of at most 1024 gate columns (32 rows in LDS);
    // past two chunks (H > 512) the W_hh^T fragments and a chunk's in-flight loads exceed
    // the 256 VGPRs, so the batch runs in 16-sample chunks instead
    int bts = lstm_bts(UB, num_dirs, BT);
    if (bts == 2 && 4 * h > 2 * 4 * GW * 32) bts = 1;
    if (bts == 2) {
      kswc = 32;
      nch = (4 * h + 4 * GW * 32 - 1) / (4 * GW * 32);
    }
    const void* fn = nullptr;    // the interleaved layout
    const void* fx = nullptr;    // the same-XCD groups
#define DS2_LBP(K, C, B)                                                          \
  if (kswc == K && nch == C && bts == B) {                                        \
    fn = reinterpret_cast<const void*>(lstm_bwd_persist_kernel<K, C, B, false>);  \
    fx = reinterpret_cast<const void*>(lstm_bwd_persist_kernel<K, C, B, true>);   \
  }
    DS2_LBP(8, 1, 1) DS2_LBP(16, 1, 1) DS2_LBP(25, 1, 1) DS2_LBP(32, 1, 1) DS2_LBP(48, 1, 1)
    DS2_LBP(64, 1, 1) DS2_LBP(48, 2, 1) DS2_LBP(64, 2, 1)
    DS2_LBP(32, 1, 2) DS2_LBP(32, 2, 2)
#undef DS2_LBP
    const int BTW = (BT + bts - 1) / bts;
    const int ct = lstm_chunk_tiles(UB, num_dirs, BTW);
    bool ok = fn != nullptr && mapped_grid(UB * num_dirs, ct) <= num_cus();
    for (int b0 = 0; ok && b0 < BTW; b0 += ct) {
      int T_ = t_max, N_ = n, H_ = h, D_ = num_dirs, UB_ = UB, BT_ = std::min(ct, BTW - b0);
      int DYD_ = dy_dirs, NB_ = b0 * GB * bts;
      unsigned* err = ctrs + num_dirs * BT_;
      if (hipMemsetAsync(ctrs, 0, lstm_counter_bytes(n, num_dirs), st) != hipSuccess)
        return launch_status("ds2_lstm counters");
      // same-XCD groups (DS2_GRU_XCD, as the GRU backward's) where they tile the XCDs
      const bool xm = xcd_groups_on() && xgrp_fits(UB, BT_, num_dirs);
      void* args[] = {&T_, &N_, &H_, &D_, &UB_, &BT_, &dy, &DYD_, &wpt, &c_all, &gates, &lens,
                      &dgates, &ctrs, &err, &NB_};
      ok = rnn_launch(xm ? fx : fn,
                      dim3(xm ? xgrp_grid(UB, BT_, num_dirs) : mapped_grid(UB * num_dirs, BT_)),
                      dim3(GT), args, 0, st) == hipSuccess;
      if (ok) fold_err(err, err_out, st);
      if (!ok && b0 > 0) return launch_status("ds2_lstm_bwd chunk");
    }
    if (ok) return launch_status("ds2_lstm_bwd");
    (void)hipGetLastError();
  }
  for (int s = 0; s < t_max; ++s) {
    switch (ksw) {
      DS2_LBWD_CASE(8) DS2_LBWD_CASE(16) DS2_LBWD_CASE(32) DS2_LBWD_CASE(64)
    }
  }
  return launch_status("ds2_lstm_bwd");
}

}  // extern "C"
