// GRU backward recurrence that exchanges dh instead of the gate gradients (opt-in,
// DS2_GRU_BWD=dh; measured slower than the gate exchange, see the end of this comment).
//
// The backward step of one direction is (model.py:97-109 nn.GRU BPTT, gates r, z, n):
//   dh_t   = dy_t + z_{t+1} dh_{t+1} + sum_k dG_{t+1}[k] W_hh[k][u]        (k over the 3H gate rows)
//   dG_t   = (dar, daz, dghn)_t = dh_t x (c_r, c_z, c_hn)_t                 (rnn_common.h coefficients)
// gru_bwd_dop_kernel (gru.hip) hands the 3H-wide dG_{t+1} from its 50 producers to every
// consumer: 150 KB of write-through tiles per workgroup per step, the step's critical path.
// Here every producer publishes its 16 units of dh_t (one 1-KB tile, the forward's hand-off),
// and each consumer forms the A operands of its W_hh^T contraction itself: the dh tile of a
// unit block times the coefficient tiles of its three gate rows, which the forward wrote long
// before (coef, read with plain cached loads issued a step ahead, off the critical path).
// Per step a consumer waits for 50 KB of fresh data instead of 150 KB; the MFMA work is the
// same (16 samples x 3H x 16 units, v_mfma_f32_16x16x4_f32, fp32).
//
// Workgroup = (16 units ub, direction d, 16-sample batch tile bt), NW waves; wave w owns unit
// blocks [b0, b0 + nb) of the 50 and all three gates of each (K blocks g H + 16 v): one wave
// per SIMD with the whole register file (NW 4, default), or two balanced per SIMD (NW 8).  The owner threads (sample m, unit u) compute dh_t, write dgx / dgh
// (dh x coefficients, the same products the consumers form), sum the bias gradients, and
// publish the dh tile.  HM: 0 per-producer flags (ring of 2 slots), 1 sentinel ring (the data
// is the flag), as the direct-operand forward.
//
// Measured (cfg2, same box, alternating with the gate exchange at 6.31-6.39 us per step):
// 7.05-7.09 us with the coefficient loads issued before the flag poll, 7.53-7.55 issued after
// the MFMAs (a __syncthreads drains them at the next barrier), 8.57 with raw LDS barriers so
// they stay in flight across the reduction, publish and poll.  The coefficients are 150 KB per
// workgroup per step -- the bytes the gate exchange hands off -- and the longer they stream
// beside the hand-off, the more they slow it: the per-CU memory queue, not the freshness of
// the bytes, prices the step (MI355X_MICROARCH.md handoff-1to1 under streaming waves).
#include "rnn_common.h"

namespace ds2 {

constexpr int kDhTraceS0 = 100, kDhTraceSteps = 16;   // = gru.hip's DS2_GRU_STAMPS=2 window

// Workgroup barrier for LDS data only: waits for this wave's LDS operations, not its vector
// memory ones.  __syncthreads() carries a workgroup fence, before which hipcc drains vmcnt --
// that would stall every wave on the coefficient prefetch below at each of the step's barriers.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// flags_wait (rnn_common.h) with the raw barrier: wave 0 polls the UB producer flags (one
// sc1 load + ballot per round); the other waves load after the barrier it joins (the valid
// form's consumer rule), with their prefetches still in flight
__device__ __forceinline__ bool dh_flags_wait(const unsigned* flags, int count, unsigned target,
                                              unsigned* err, int* lds_flag) {
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    unsigned spins = 0;
    int ok = 1;
    if (g_spin_limit == 0) {   // fault injection
      if (lane == 0) __hip_atomic_fetch_or(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      ok = 0;
    }
    for (; ok;) {
      const unsigned v = lane < count ? __hip_atomic_load(flags + lane, __ATOMIC_RELAXED,
                                                          __HIP_MEMORY_SCOPE_AGENT)
                                      : target;
      if (__ballot(v < target) == 0ull) break;
      __builtin_amdgcn_s_sleep(1);
      if (++spins > g_spin_limit) {
        if (lane == 0) __hip_atomic_fetch_or(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ok = 0;
        break;
      }
    }
    if (lane == 0) *lds_flag = ok;
  }
  lds_barrier();
  return *lds_flag != 0;
}

template <int NVB, int HM, int NW>
__global__ __launch_bounds__(NW * 64) __attribute__((amdgpu_waves_per_eu(NW / 4, NW / 4))) void gru_bwd_dh_kernel(
    int T, int N, int H, int D, int UB, int BT, const float* __restrict__ dy, int dyd,
    const float* __restrict__ w_f, const float* __restrict__ w_r,
    const float* __restrict__ gates, const float* __restrict__ coef,
    const int* __restrict__ lens, float* __restrict__ dgx, float* __restrict__ dgh,
    float* __restrict__ ring, unsigned* __restrict__ counters, unsigned* __restrict__ err,
    unsigned long long* __restrict__ stamps, double* __restrict__ dbp) {
  constexpr int RP = GU + 1;
  constexpr bool SENT = HM == 1;
  constexpr int NSLOT = SENT ? kRingSlots : 2;
  __shared__ __attribute__((aligned(8))) float red[NW * GB * RP];
  __shared__ __attribute__((aligned(16))) float tile[GB * GU];
  __shared__ int flag;
  __shared__ int failed;
  int ub, d, bt;
  if (!map_work(UB * D, BT, UB, ub, d, bt)) return;
  const int n0 = bt * GB;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int H3 = 3 * H;
  int b0, nb;
  if (NW == GW) {
    simd_split(UB, wave, b0, nb);                // host guarantees nb <= NVB
  } else {                                       // one wave per SIMD
    b0 = (UB * wave) / NW;
    nb = (UB * (wave + 1)) / NW - b0;
  }
  const unsigned* gflags = counters + (D * BT + 1) + (d * BT + bt) * UB;
  unsigned* myflag = counters + (D * BT + 1) + (d * BT + bt) * UB + ub;
  const int slot_floats = D * BT * UB * 256;
  const __amdgpu_buffer_rsrc_t x_rs =
      __builtin_amdgcn_make_buffer_rsrc(ring, (short)0, NSLOT * slot_floats * 4, 0x00020000);
  const int grp_off = (d * BT + bt) * UB * 256;
  // coefficient tiles of this (direction, batch tile): [t][g][ub][256] with a t stride
  const int64_t coef_floats = (int64_t)T * D * BT * kCoefPlanes * UB * 256;
  const __amdgpu_buffer_rsrc_t c_rs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(coef), (short)0, static_cast<int>(coef_floats * 4), 0x00020000);
  if (threadIdx.x == 0) failed = 0;
  __syncthreads();
  const bool tracing = stamps != nullptr && threadIdx.x == 0;
  auto trace_at = [&](int s, int p) {
    if (tracing && s >= kDhTraceS0 && s < kDhTraceS0 + kDhTraceSteps)
      stamps[((int64_t)(s - kDhTraceS0) * gridDim.x + blockIdx.x) * 5 + p] =
          __builtin_amdgcn_s_memrealtime();
  };

  // W_hh^T fragments: w[g][i][c] = W_hh[g H + 16 (b0 + i) + 4 (lane >> 4) + c][16 ub + (lane & 15)]
  f32x4 w[3][NVB];
  {
    const float* W = d == 0 ? w_f : w_r;
    const float* wc = W + (int64_t)(4 * (lane >> 4)) * H + ub * GU + (lane & 15);
#pragma unroll
    for (int g = 0; g < 3; ++g)
#pragma unroll
      for (int i = 0; i < NVB; ++i)
#pragma unroll
        for (int c = 0; c < 4; ++c)
          w[g][i][c] = i < nb ? wc[((int64_t)g * H + 16 * (b0 + i) + c) * H] : 0.f;
#pragma unroll
    for (int g = 0; g < 3; ++g)
#pragma unroll
      for (int i = 0; i < NVB; ++i) settle(w[g][i]);
  }
  const int m = threadIdx.x >> 4;
  const int u = threadIdx.x & 15;
  const int n = n0 + m;
  const int j = ub * GU + u;
  const bool gate_thread = threadIdx.x < GB * GU;
  const bool owner = gate_thread && n < N;
  int len = owner ? lens[n] : 0;
  settle(len);
  const int tpos = ((u >> 2) * GB + m) * 4 + (u & 3);
  // byte offset of this lane's 16 B in tile (g, v) of time t's coefficients
  auto coef_off = [&](int t, int g, int v) -> int {
    return static_cast<int>((coef_tile(t, d, bt, g, v, D, BT, UB) * 256 + lane * 4) * 4);
  };
  float dh_prev = 0.f, z_prev = 0.f;
  float px_dar = 0.f, px_daz = 0.f, px_dan = 0.f, px_dghn = 0.f;
  int64_t px_row = -1;
  double sb_r = 0.0, sb_z = 0.0, sb_n = 0.0, sb_hn = 0.0;
  // the coefficients the step's consumers multiply (time of the previous step), prefetched
  f32x4 cf[3][NVB];
  for (int s = 0; s < T; ++s) {
    const int t = d == 0 ? T - 1 - s : s;
    f32x4 acc0 = f32x4{0.f, 0.f, 0.f, 0.f};
    f32x4 acc1 = f32x4{0.f, 0.f, 0.f, 0.f};
    trace_at(s, 0);
    float dyv = 0.f, g_z = 0.f, g_n = 0.f, c_r = 0.f, c_z = 0.f, c_hn = 0.f;
    const int64_t row = ((int64_t)t * N + n) * D + d;
    if (owner && t < len) {
      dyv = dy[(((int64_t)t * N + n) * dyd + (dyd > 1 ? d : 0)) * H + j];
      const float* gp = gates + row * 4 * H;
      g_z = gp[H + j];
      g_n = gp[2 * H + j];
      const float* cp = coef + coef_tile(t, d, bt, 0, ub, D, BT, UB) * 256 + tpos;
      c_r = cp[0];
      c_z = cp[(int64_t)UB * 256];
      c_hn = cp[(int64_t)2 * UB * 256];
    }
    if (s > 0) {
      if (!SENT && !dh_flags_wait(gflags, UB, (unsigned)s, err, &flag)) {
        poison_rest(dgx, s, T, d == 0, N, D, n, d, H, j, H3, 3, owner);
        return;
      }
      trace_at(s, 1);
      const int base = (((s - 1) % NSLOT) * slot_floats + grp_off + b0 * 256 + lane * 4) * 4;
      if (SENT) sleep_units(g_rnn_tune[2]);
      f32x4 hv[NVB];
#pragma unroll
      for (int i = 0; i < NVB; ++i) {
        const int off = i < nb ? base + i * 1024 : 0x7ffffff0;
        hv[i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(x_rs, off, 0, kSc1));
      }
      asm volatile("" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      auto mma_block = [&](int i) {
#pragma unroll
        for (int g = 0; g < 3; ++g) {
          const f32x4 a = hv[i] * cf[g][i];
          acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[0], w[g][i][0], acc0, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[1], w[g][i][1], acc1, 0, 0, 0);
          acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[2], w[g][i][2], acc0, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[3], w[g][i][3], acc1, 0, 0, 0);
        }
      };
      if (SENT) {
        // the ready prefix in unit-block order (one accumulation order for both forms);
        // a pass re-loads only the stale tiles
        unsigned rdy = 0u;
        int next = 0;
        for (unsigned spins = 0;; ++spins) {
#pragma unroll
          for (int i = 0; i < NVB; ++i)
            if (i >= next && i < nb && !((rdy >> i) & 1u) && wave_ready(hv[i])) rdy |= 1u << i;
#pragma unroll
          for (int i = 0; i < NVB; ++i) {
            if (i == next && i < nb && ((rdy >> i) & 1u)) {
              mma_block(i);
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
          for (int i = 0; i < NVB; ++i)
            if (i >= next && i < nb && !((rdy >> i) & 1u))
              hv[i] = __builtin_bit_cast(
                  f32x4, __builtin_amdgcn_raw_buffer_load_b128(x_rs, base + i * 1024, 0, kSc1));
        }
      } else {
#pragma unroll
        for (int i = 0; i < NVB; ++i) mma_block(i);
      }
      trace_at(s, 2);
    }
    // the coefficients step s + 1 multiplies (time t), in flight across the step's barriers
    // (lds_barrier): waves 1.. issue them now, wave 0 -- which drains vmcnt to publish and
    // then polls -- right after its flag store
    auto prefetch = [&]() {
      if (s + 1 < T) {
#pragma unroll
        for (int g = 0; g < 3; ++g)
#pragma unroll
          for (int i = 0; i < NVB; ++i)
            cf[g][i] = __builtin_bit_cast(
                f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                           c_rs, i < nb ? coef_off(t, g, b0 + i) : 0x7ffffff0, 0, 0));
      }
    };
    if (wave != 0) prefetch();
#pragma unroll
    for (int r = 0; r < 4; ++r)
      red[(wave * GB + (lane >> 4) * 4 + r) * RP + (lane & 15)] = acc0[r] + acc1[r];
    settle(dyv);
    settle(g_z);
    settle(g_n);
    settle(c_r);
    settle(c_z);
    settle(c_hn);
    lds_barrier();
    if (SENT && failed) {
      poison_rest(dgx, s, T, d == 0, N, D, n, d, H, j, H3, 3, owner);
      return;
    }
    trace_at(s, 3);
    float dh = 0.f;
    if (owner) {
      float zc = 0.f;
      float dar = 0.f, daz = 0.f, dan = 0.f, dghn = 0.f;
      if (t < len) {
        float carry = 0.f;
        if (s > 0) {
          float rec = 0.f;
#pragma unroll
          for (int w8 = 0; w8 < NW; ++w8) rec += red[(w8 * GB + m) * RP + u];
          carry = dh_prev * z_prev + rec;
        }
        dh = dyv + carry;
        zc = g_z;
        dan = dh * ((1.f - zc) * (1.f - g_n * g_n));   // c_n as the forward forms it
        dar = dh * c_r;
        daz = dh * c_z;
        dghn = dh * c_hn;
      }
      dh_prev = dh;
      z_prev = zc;
      px_dar = dar; px_daz = daz; px_dan = dan; px_dghn = dghn; px_row = row;
      sb_r += dar; sb_z += daz; sb_n += dan; sb_hn += dghn;
    }
    if (gate_thread) tile[tpos] = dh;
    lds_barrier();
    if (wave == 0) {
      const int toff = (grp_off + ub * 256 + lane * 4) * 4;
      if (SENT) {
        const u32x4 v = desentinel(*reinterpret_cast<const u32x4*>(tile + lane * 4));
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // last step's sentinel store first
        __builtin_amdgcn_raw_buffer_store_b128(v, x_rs, (s % NSLOT) * slot_floats * 4 + toff, 0, kSc1);
        const u32x4 sv = u32x4{kSentinel, kSentinel, kSentinel, kSentinel};
        __builtin_amdgcn_raw_buffer_store_b128(sv, x_rs, ((s + 2) % NSLOT) * slot_floats * 4 + toff,
                                               0, kSc1);
      } else {
        const u32x4 v = *reinterpret_cast<const u32x4*>(tile + lane * 4);
        __builtin_amdgcn_raw_buffer_store_b128(v, x_rs, (s & 1) * slot_floats * 4 + toff, 0, kSc1);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane == 0)
          __hip_atomic_store(myflag, (unsigned)s + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      prefetch();
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

// Coefficient tiles from a forward that wrote only the classic gate cache (the non-default
// forward kernels): one thread per tile element, the forward's formula (rnn_common.h).
__global__ void gru_coef_kernel(const float* __restrict__ gates, const float* __restrict__ h_all,
                                const int* __restrict__ lens, int T, int N, int H, int D, int UB,
                                int BT, float* __restrict__ coef) {
  const int64_t total = (int64_t)T * D * BT * UB * 256;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    int64_t r = i;
    const int tpos = static_cast<int>(r % 256); r /= 256;
    const int ub = static_cast<int>(r % UB); r /= UB;
    const int bt = static_cast<int>(r % BT); r /= BT;
    const int d = static_cast<int>(r % D); r /= D;
    const int t = static_cast<int>(r);
    const int m = (tpos >> 2) % GB;
    const int u = (tpos / (4 * GB)) * 4 + (tpos & 3);
    const int n = bt * GB + m, j = ub * GU + u;
    float cr = 0.f, cz = 0.f, chn = 0.f;
    if (n < N && j < H && t < lens[n]) {
      const float* gp = gates + (((int64_t)t * N + n) * D + d) * 4 * H;
      const int tp = d == 0 ? t - 1 : t + 1;
      const float hp = (tp >= 0 && tp < T) ? h_all[(((int64_t)tp * N + n) * D + d) * H + j] : 0.f;
      gru_coefs(gp[j], gp[H + j], gp[2 * H + j], gp[3 * H + j], hp, cr, cz, chn);
    }
    float* cp = coef + coef_tile(t, d, bt, 0, ub, D, BT, UB) * 256 + tpos;
    cp[0] = cr;
    cp[(int64_t)UB * 256] = cz;
    cp[(int64_t)2 * UB * 256] = chn;
  }
}

static inline bool dh_bwd_enabled() { return gru_dh_bwd_opted_in(); }

static inline int dh_handoff_mode() {
  const char* e = getenv("DS2_RNN_HANDOFF_BWD");
  if (e == nullptr || e[0] == 0) e = getenv("DS2_RNN_HANDOFF");
  if (e == nullptr || e[0] == 0) return 0;
  return e[0] == 's' ? 1 : 0;
}

// waves per workgroup: 4 (one per SIMD, 512 registers: W_hh^T, the prefetched coefficients
// and the dh tiles of 12-13 unit blocks in registers; default) or 8 (DS2_GRU_BWD_WAVES=8:
// 256 registers, 6-7 blocks per wave)
static inline int dh_waves() {
  const char* e = getenv("DS2_GRU_BWD_WAVES");
  return (e != nullptr && e[0] == '8') ? 8 : 4;
}

static const void* bwd_dh_fn(int UB, int hm, int& nw) {
  if (nw == 8 && ((UB + 3) / 4 + 1) / 2 > 4) nw = 4;
  const int need = nw == 8 ? ((UB + 3) / 4 + 1) / 2 : (UB + 3) / 4;
#define DS2_BDH(K, W)                                                                       \
  if (need <= K)                                                                            \
    return hm == 1 ? reinterpret_cast<const void*>(gru_bwd_dh_kernel<K, 1, W>)              \
                   : reinterpret_cast<const void*>(gru_bwd_dh_kernel<K, 0, W>);
  // instantiated only where nothing spills (W_hh^T, coefficients, tiles: 3 x 4 x 2 + 4 floats
  // per block and lane): 8 waves up to 4 blocks (H <= 512), 4 waves up to 13 (H <= 832);
  // larger H takes the gate-exchange kernels
  if (nw == 8) {
    DS2_BDH(2, 8) DS2_BDH(4, 8)
  }
  DS2_BDH(2, 4) DS2_BDH(4, 4) DS2_BDH(8, 4) DS2_BDH(13, 4)
#undef DS2_BDH
  return nullptr;
}

void launch_gru_coef(const float* gates, const float* h_all, const int* lens, int t_max, int n,
                     int h, int num_dirs, float* coef, hipStream_t st) {
  const int UB = (h + GU - 1) / GU, BT = (n + GB - 1) / GB;
  hipLaunchKernelGGL(gru_coef_kernel, dim3(grid_cap((int64_t)t_max * num_dirs * BT * UB * 256)),
                     dim3(256), 0, st, gates, h_all, lens, t_max, n, h, num_dirs, UB, BT, coef);
}

// false: not applicable (the caller falls back to the gate-exchange kernels)
bool launch_gru_bwd_dh(int t_max, int n, int h, int num_dirs, const float* dy, int dy_dirs,
                       const float* w_hh_f, const float* w_hh_r, const float* gates,
                       const float* coef, const int* lens, float* dgates_x, float* dgates_h,
                       float* ring, unsigned* ctrs, unsigned* err, unsigned long long* stamps,
                       double* dbp, size_t lds_pad, hipStream_t st) {
  if (!dh_bwd_enabled() || coef == nullptr || (h % GU) != 0) return false;
  const char* x6b = getenv("DS2_GRU_X6_BWD");          // the opt-in bf16x6 gate exchange
  if (x6b != nullptr && x6b[0] == '1') return false;
  if ((int64_t)gru_coef_floats(t_max, n, h, num_dirs) * 4 >= (1ll << 31)) return false;
  apply_spin_limit_env();
  apply_rnn_tune_env();
  const int UB = h / GU, BT = (n + GB - 1) / GB;
  const int hm = dh_handoff_mode();
  int nw = dh_waves();
  const void* fn = bwd_dh_fn(UB, hm, nw);
  if (fn == nullptr) return false;
  if (hm == 1 && hipMemsetAsync(ring, 0xFF,
                                align256(kRingSlots * (size_t)num_dirs * BT * UB * 256 * sizeof(float)),
                                st) != hipSuccess)
    return false;
  int T_ = t_max, N_ = n, H_ = h, D_ = num_dirs, UB_ = UB, BT_ = BT, DYD_ = dy_dirs;
  void* args[] = {&T_, &N_, &H_, &D_, &UB_, &BT_, &dy, &DYD_, &w_hh_f, &w_hh_r, &gates,
                  &coef, &lens, &dgates_x, &dgates_h, &ring, &ctrs, &err, &stamps, &dbp};
  return rnn_launch(fn, dim3(mapped_grid(UB * num_dirs, BT)), dim3(nw * 64), args,
                                    lds_pad, st) == hipSuccess;
}

}  // namespace ds2
