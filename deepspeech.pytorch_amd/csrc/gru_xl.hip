// GRU recurrences in XCD-local hand-off groups (round 6; default where the shape fits).
//
// The fp16x3 kernels of gru_split.hip tile a (direction, 16-sample) group as 50 workgroups of
// 16 units at cfg2 (H 800).  A group then spans two XCDs, and every step each consumer pulls
// 50 producer tiles (the backward: 50 x 3.06 KB = 153 KB), half of them across the fabric
// (MI355X_MICROARCH "handoff-payload": 62-70 GB/s per block cross-XCD, 104-122 same-XCD from
// plain stores).  The backward's no-synchronisation bound was 4.02 us of its 5.0 us step: the
// bytes, not the protocol, set the step.
//
// Here a workgroup owns 32 units x 8 samples, so a group is H / 32 = 25 workgroups (one XCD's
// 32 CUs) and cfg2 runs 2 directions x 4 batch tiles = 8 groups, one per XCD (200 workgroups).
// Per step a consumer pulls 25 forward tiles of 1 KB (was 50) or 25 backward records of
// 3.1 KB (was 153 KB), all from its own XCD's L2.
//
// Which XCD a workgroup runs on is never assumed: every workgroup publishes its HW_REG_XCC_ID
// at start (agent-scope atomic store) and waits for its group's ids.  If all share one XCD the
// group runs LOCAL: payloads and flags are stored plainly (they stay in that XCD's L2, the
// coherence point of its CUs) and read with sc1 loads (L1 bypassed, served by that L2).  Else
// the group runs GLOBAL: every store is sc1 (write-through) and the protocol is
// MI355X_MICROARCH "Valid forms" row 1, correct at any placement.  Blocks b with equal b % 8
// form a group, which under the observed round-robin dispatch lands on one XCD.
//
// Half-empty 16-row MFMAs are avoided by stacking: an A fragment holds the fp16 hi terms of
// the 8 samples in rows 0-7 and their lo terms in rows 8-15, so A.W_hi gives hi.W_hi (rows
// 0-7) and lo.W_hi (rows 8-15) and A.W_lo gives hi.W_lo (rows 0-7; rows 8-15 = lo.lo): the
// three fp16x3 products in two v_mfma_f32_16x16x32_f16, and the big (hi.hi) and small products
// land in different rows, i.e. in separate accumulation chains (the MFMA rounding note of
// DESIGN.md section 4).  The two halves are added when the waves' partials are reduced.
// Producers publish these stacked fragments ready-made (the forward's 1-KB tile is exactly the
// fp16 A fragment of its 8 x 32 h values), so consumers load one 16-B run per lane per tile
// and split nothing.
//
// Forward hand-off: the sentinel ring of gru_fwd_x6_kernel (4 slots, the data is the flag),
// tiles consumed in a fixed producer order (a wave multiplies tile p only after tile p - 1:
// deterministic sums).  Backward: per-producer flags (the record after a drain, then the
// flag), records multiplied in a fixed order, two in flight per wave.
#include "rnn_common.h"

namespace ds2 {

// Timing ablations (scripts/xl_ablation.sh builds them into deepspeech.pytorch_amd/ablation/;
// results wrong, never in the product library): bit 0 skips the per-step pointwise input loads
// (xproj; dy / gates / h_prev), bit 1 the per-step output stores (h_all / gates; dgx / dgh),
// bit 2 every hand-off wait (the tiles / records are read whatever they hold).
#ifndef DS2_XL_ABL
#define DS2_XL_ABL 0
#endif
constexpr bool kAblLoads = (DS2_XL_ABL & 1) != 0;
constexpr bool kAblStores = (DS2_XL_ABL & 2) != 0;
constexpr bool kAblWait = (DS2_XL_ABL & 4) != 0;
constexpr bool kAblFixT = (DS2_XL_ABL & 8) != 0;   // every step loads the rows of t = 0

constexpr int LB = 8;            // samples per workgroup
constexpr int LU = 32;           // units per workgroup
constexpr int LW = 4;            // waves per workgroup, one per SIMD (the whole register file)
constexpr int LT = LW * 64;      // 256 threads = 8 samples x 32 units, one owner each
constexpr int LSLOTS = 4;        // forward sentinel ring slots
constexpr int LRB = 784;         // floats per backward record: 3 x 1-KB fragments + 8 factors
constexpr int kXlTraceS0 = 100, kXlTraceSteps = 16;   // = gru.hip's DS2_GRU_STAMPS=2 window

// the launch's workgroup -> (group, producer index); blocks with equal b % 8 form a group
__device__ __forceinline__ bool xl_map(int G, int UBX, int& g, int& ub) {
  g = blockIdx.x & 7;
  ub = blockIdx.x >> 3;
  return g < G && ub < UBX;
}

// Every workgroup publishes its XCC id (+1) into its group's table and waits for the group's
// UBX entries; true when all equal this workgroup's (every member reaches the same answer from
// the same table).  A timeout sets the error word and answers false.  `mode` (diagnostic, read
// by scripts/trace_gru.py): OR of 1 (a member ran LOCAL) / 2 (GLOBAL) per group.
__device__ __forceinline__ bool xl_group_local(unsigned* xtab, int ub, int UBX, unsigned* err,
                                               int* lds_word, unsigned* mode, int force_global) {
  const unsigned mine = xcc_id() + 1u;
  if (threadIdx.x == 0) __hip_atomic_store(xtab + ub, mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if ((threadIdx.x >> 6) == 0) {
    const int lane = threadIdx.x & 63;
    unsigned v = mine;
    bool ok = true;
    for (unsigned spins = 0;; ++spins) {
      v = lane < UBX ? __hip_atomic_load(xtab + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                     : mine;
      if (__ballot(v == 0u) == 0ull) break;
      if (spins > g_spin_limit) {
        if (lane == 0) __hip_atomic_fetch_or(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ok = false;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    const bool loc = ok && __ballot(v != mine) == 0ull && force_global == 0;
    if (lane == 0) {
      *lds_word = loc ? 1 : 0;
      __hip_atomic_fetch_or(mode, loc ? 1u : 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  __syncthreads();
  return *lds_word != 0;
}

__device__ __forceinline__ void xl_store(u32x4 v, __amdgpu_buffer_rsrc_t rs, int off, bool local) {
  if (local)
    __builtin_amdgcn_raw_buffer_store_b128(v, rs, off, 0, 0);
  else
    __builtin_amdgcn_raw_buffer_store_b128(v, rs, off, 0, kSc1);
}

// the stacked fp16 (hi; lo) A-fragment slots of value (row m < 8, k) in a 1-KB fragment:
// lane (k >> 3) * 16 + m (hi) / + m + 8 (lo), slot k & 7
__device__ __forceinline__ int xl_frag_hi(int m, int k) { return (((k >> 3) << 4) + m) * 8 + (k & 7); }

// ---------------------------------------------------------------------------------------
// forward: gh[8 samples x 96] = h_{t-1}[8 x H] . W_hh[(r, z, n) rows of 32 units]^T.
// Wave w holds W_hh for the producers [p0, p0 + np) (k = their 32 units each): per producer and
// column tile ct = gate * 2 + unit half, the fp16 hi / lo B fragments of W_hh's rows scaled by
// 2^e(gate, unit) (the row's max over the whole K).  h (|h| < 1) takes the fixed scale 2^14.
template <int NPW>
__global__ __launch_bounds__(LT) __attribute__((amdgpu_waves_per_eu(1, 1))) void gru_fwd_xl_kernel(
    int T, int N, int H, int D, int UBX, int BTX, const float* __restrict__ xproj,
    const float* __restrict__ w_f, const float* __restrict__ w_r, const float* __restrict__ b_f,
    const float* __restrict__ b_r, const int* __restrict__ lens, float* __restrict__ h_all,
    float* __restrict__ gates, float* __restrict__ ring, unsigned* __restrict__ xl,
    unsigned* __restrict__ err, unsigned long long* __restrict__ stamps, int force_global) {
  constexpr int NCT = 6;
  constexpr int RC = 3 * LU + 1;   // reduction row pitch
  __shared__ float red[LW * 16 * RC];
  __shared__ __attribute__((aligned(16))) _Float16 stg[64 * 8];
  __shared__ float unsc[3 * LU];
  __shared__ __attribute__((aligned(16))) float pin[3 * 256];    // xproj (r, z, n) [gate][sample][unit]
  __shared__ __attribute__((aligned(16))) float pout[5 * 256];   // h, r, z, n, W_hn h + b_hn
  __shared__ int slen[LB];
  __shared__ int sh_local;
  __shared__ int failed;
  // W_hh fragments of a wave's last producer when it has NPW + 1 (cfg2: 25 = 6 + 6 + 6 + 7):
  // in LDS, read every step, instead of 48 more registers in every wave
  __shared__ u32x4 wx[LW * NCT * 2 * 64];
  const int G = D * BTX;
  int g, ub;
  if (!xl_map(G, UBX, g, ub)) return;
  const int d = g / BTX, bt = g - d * BTX;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // the wave's producers: UBX / 4 each and one more for the lowest UBX % 4 waves -- wave 0,
  // which issues none of the step's HBM traffic (the io waves below), takes the extra one
  const int p0 = wave * (UBX / LW) + min(wave, UBX % LW);
  const int np = UBX / LW + (wave < UBX % LW ? 1 : 0);   // host guarantees np <= NPW + 1
  if (threadIdx.x == 0) failed = 0;
  const bool local = xl_group_local(xl + g * 32, ub, UBX, err, &sh_local, xl + 512 + g, force_global);
  const int slot_floats = G * UBX * 256;
  const __amdgpu_buffer_rsrc_t x_rs =
      __builtin_amdgcn_make_buffer_rsrc(ring, (short)0, LSLOTS * slot_floats * 4, 0x00020000);
  const int grp_off = g * UBX * 256;
  // per-wave timeline (DS2_GRU_STAMPS=2): [step][block][wave][6] = step start, hand-off wait
  // done, products done, io done (waves 1-3), reduction barrier done, published; lane 0 of
  // every wave (scripts/trace_gru.py)
  const bool tracing = stamps != nullptr && lane == 0;
  auto trace_at = [&](int s, int p) __attribute__((always_inline)) {
    if (tracing && s >= kXlTraceS0 && s < kXlTraceS0 + kXlTraceSteps)
      stamps[(((int64_t)(s - kXlTraceS0) * gridDim.x + blockIdx.x) * LW + wave) * 6 + p] =
          __builtin_amdgcn_s_memrealtime();
  };

  // W_hh fragments: producer p, tile ct (gate gt = ct >> 1, half c = ct & 1), k slot i ->
  // W[gt H + 32 ub + 16 c + (lane & 15)][32 (p0 + p) + 8 (lane >> 4) + i]
  Duo w[NPW][NCT];
  auto wfr = [&](int p, int ct) __attribute__((always_inline)) {   // producer p's fragments (p == NPW: from LDS)
    if (p < NPW) return w[p < NPW ? p : 0][ct];
    Duo r;
    r.hi = __builtin_bit_cast(f16x8, wx[((wave * NCT + ct) * 2 + 0) * 64 + lane]);
    r.lo = __builtin_bit_cast(f16x8, wx[((wave * NCT + ct) * 2 + 1) * 64 + lane]);
    return r;
  };
  {
    const float* W = d == 0 ? w_f : w_r;
    const int q8 = 8 * (lane >> 4);
    auto frag = [&](int p, int ct, f32x4& a, f32x4& b) __attribute__((always_inline)) {
      const f32x4 z4 = f32x4{0.f, 0.f, 0.f, 0.f};
      if (p < np) {
        const float* r = W + (int64_t)((ct >> 1) * H + LU * ub + 16 * (ct & 1) + (lane & 15)) * H +
                         LU * (p0 + p) + q8;
        a = *reinterpret_cast<const f32x4*>(r);
        b = *reinterpret_cast<const f32x4*>(r + 4);
      } else {
        a = z4;
        b = z4;
      }
    };
    float mx[NCT];
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct) mx[ct] = 0.f;
#pragma unroll
    for (int p = 0; p < NPW + 1; ++p)
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct) {
        f32x4 a, b;
        frag(p, ct, a, b);
#pragma unroll
        for (int i = 0; i < 4; ++i) mx[ct] = fmaxf(mx[ct], fmaxf(fabsf(a[i]), fabsf(b[i])));
      }
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct) {
      mx[ct] = fmaxf(mx[ct], __shfl_xor(mx[ct], 16));
      mx[ct] = fmaxf(mx[ct], __shfl_xor(mx[ct], 32));
      if (lane < 16) red[wave * 96 + ct * 16 + lane] = mx[ct];
    }
    __syncthreads();
    float sc[NCT];
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct) {
      float m = 0.f;
#pragma unroll
      for (int w4 = 0; w4 < LW; ++w4) m = fmaxf(m, red[w4 * 96 + ct * 16 + (lane & 15)]);
      sc[ct] = __builtin_ldexpf(1.f, h3_row_exp(m));
    }
    if (threadIdx.x < 3 * LU) {   // (gate, unit) = threadIdx.x = ct * 16 + column
      float m = 0.f;
#pragma unroll
      for (int w4 = 0; w4 < LW; ++w4) m = fmaxf(m, red[w4 * 96 + threadIdx.x]);
      unsc[threadIdx.x] = __builtin_ldexpf(1.f, -(h3_row_exp(m) + 14));
    }
    __syncthreads();
    asm volatile("" ::: "memory");   // re-load W below (do not keep the max pass's loads live)
#pragma unroll
    for (int p = 0; p < NPW + 1; ++p)
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct) {
        f32x4 a, b;
        frag(p, ct, a, b);
        const Duo dd = split2h(a, b, sc[ct]);
        if (p < NPW) {
          w[p < NPW ? p : 0][ct] = dd;
        } else {
          wx[((wave * NCT + ct) * 2 + 0) * 64 + lane] = __builtin_bit_cast(u32x4, dd.hi);
          wx[((wave * NCT + ct) * 2 + 1) * 64 + lane] = __builtin_bit_cast(u32x4, dd.lo);
        }
      }
  }
  const float* bh = d == 0 ? b_f : b_r;
  const int m = threadIdx.x >> 5;        // sample of the tile
  const int u = threadIdx.x & 31;        // unit of the block
  const int n = bt * LB + m;
  const int j = ub * LU + u;
  const bool owner = n < N;
  float bias_r = 0.f, bias_z = 0.f, bias_n = 0.f;
  if (owner) {
    bias_r = bh[j];
    bias_z = bh[H + j];
    bias_n = bh[2 * H + j];
  }
  if (threadIdx.x < LB) slen[threadIdx.x] = bt * LB + (int)threadIdx.x < N ? lens[bt * LB + threadIdx.x] : 0;
  __syncthreads();
  const int len = slen[m];
  const float us_r = unsc[u], us_z = unsc[LU + u], us_n = unsc[2 * LU + u];
  settle(bias_r);
  settle(bias_z);
  settle(bias_n);
  const int shi = xl_frag_hi(m, u), slo = shi + 64;   // this owner's stg slots (lo: row + 8)
  // The step's HBM traffic (xproj in; h_all, gates out) goes through LDS, issued by waves 1-3
  // only: wave 0 publishes, and its drain before the publish would otherwise wait for those
  // loads and stores (vmcnt counts in order).  Inputs are loaded one step ahead, after the
  // wave's hand-off loop (so they never sit in front of its tile loads); outputs of step s are
  // stored during step s + 1.  io float4 q: sample q / 24, gate (q % 24) / 8, units 4 (q % 8).
  // Addresses are set up once: each io float4 has a fixed row pointer advanced by a fixed
  // stride per step (per-step 64-bit index arithmetic and lane-divergent branches cost ~1 us
  // of VALU latency at one wave per SIMD); masked lanes load from a valid address.
  const bool io = wave != 0;
  const int q = io ? (int)threadIdx.x - 64 : 0;
  const int qm = q / 24, qg = (q % 24) >> 3, q4 = (q & 7) * 4;
  const int qn = bt * LB + qm;
  const bool qv = io && qn < N;
  const int qlen = slen[qm];
  const float* xq = xproj + ((int64_t)qn * D + d) * 3 * H + qg * H + ub * LU + q4;
  const int64_t xstep = (int64_t)N * D * 3 * H;
  const f32x4 z4v = f32x4{0.f, 0.f, 0.f, 0.f};
  // the load (from a valid address when masked) and, separately, whether step st has a row:
  // the zero select happens when the value is staged -- a select right after the load would
  // make the wave wait for it there (vmcnt(0) at issue: the whole HBM latency)
  auto in_ok = [&](int st) __attribute__((always_inline)) {
    const int tt = d == 0 ? st : T - 1 - st;
    return !kAblLoads && qv && tt < qlen;
  };
  auto load_in = [&](int st) __attribute__((always_inline)) {
    const int tt = d == 0 ? st : T - 1 - st;
    return *reinterpret_cast<const f32x4*>(in_ok(st) ? xq + (kAblFixT ? 0 : tt) * xstep : xproj);
  };
  // outputs: float4 idx = q + 192 k (< 320): sample idx / 40, field (idx % 40) / 8 (h, r, z,
  // n, W_hn h + b_hn), units 4 (idx % 8)
  float* ob[2];
  int64_t ostr[2];
  int osrc[2];
  bool ov[2];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int idx = q + 192 * k;
    const int sm = (idx / 40) & 7, f = (idx % 40) >> 3, o4 = (idx & 7) * 4, sn = bt * LB + sm;
    ov[k] = io && idx < 320 && sn < N && (f == 0 || gates != nullptr);
    osrc[k] = f * 256 + sm * LU + o4;
    if (f == 0) {
      ob[k] = h_all + ((int64_t)sn * D + d) * H + ub * LU + o4;
      ostr[k] = (int64_t)N * D * H;
    } else {
      ob[k] = gates + ((int64_t)sn * D + d) * 4 * H + (f - 1) * H + ub * LU + o4;
      ostr[k] = (int64_t)N * D * 4 * H;
    }
  }
  auto store_out = [&](int st) __attribute__((always_inline)) {   // pout (step st) -> h_all, gates
    const int tt = d == 0 ? st : T - 1 - st;
#pragma unroll
    for (int k = 0; k < 2; ++k)
      if (ov[k])
        *reinterpret_cast<f32x4*>(ob[k] + tt * ostr[k]) = *reinterpret_cast<const f32x4*>(pout + osrc[k]);
  };
  // one step ahead (vmcnt counts in order: a load still in flight would hold back the next
  // step's tile waits whatever its own use, so a longer prefetch distance buys nothing)
  f32x4 xin = io ? load_in(0) : z4v;
  float h_own = 0.f;
  for (int s = 0; s < T; ++s) {
    const int t = d == 0 ? s : T - 1 - s;
    f32x4 acc[NCT];
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct) acc[ct] = f32x4{0.f, 0.f, 0.f, 0.f};
    trace_at(s, 0);
    // the step's inputs (loaded during the last step), staged before the tile loads: the wait
    // for them overlaps the producers' latency, and nothing HBM-bound is left in flight in
    // front of the tile loads
    if (io) *reinterpret_cast<f32x4*>(pin + qg * 256 + qm * LU + q4) = in_ok(s) ? xin : z4v;
    if (s > 0) {
      trace_at(s, 1);
      const int base = (((s - 1) % LSLOTS) * slot_floats + grp_off + p0 * 256 + lane * 4) * 4;
      sleep_units(g_rnn_tune[7]);
      u32x4 hv[NPW + 1];
#pragma unroll
      for (int p = 0; p < NPW + 1; ++p)
        hv[p] = __builtin_amdgcn_raw_buffer_load_b128(x_rs, p < np ? base + p * 1024 : 0x7ffffff0, 0, kSc1);
      asm volatile("" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      // fixed order: tile p is multiplied once it and every tile before it have arrived; a
      // stale pass re-loads every tile not yet multiplied (their round trips overlap)
      bool bad = false;   // a tile of this wave timed out: the rest are skipped
#pragma unroll
      for (int p = 0; p < NPW + 1; ++p) {
        if (p < np && !bad) {
          for (unsigned spins = 0;
               !kAblWait && (!wave_ready(__builtin_bit_cast(f32x4, hv[p])) || g_spin_limit == 0);
               ++spins) {
            if (spins > g_spin_limit || g_spin_limit == 0) {
              if (lane == 0) __hip_atomic_fetch_or(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              failed = 1;
              bad = true;
              break;
            }
            sleep_units(g_rnn_tune[0]);
            asm volatile("" ::: "memory");
#pragma unroll
            for (int q = p; q < NPW + 1; ++q)
              if (q < np && (unsigned)(q - p) < g_rnn_tune[6])
                hv[q] = __builtin_amdgcn_raw_buffer_load_b128(x_rs, base + q * 1024, 0, kSc1);
          }
          const f16x8 a = __builtin_bit_cast(f16x8, hv[p]);
#pragma unroll
          for (int ct = 0; ct < NCT; ++ct) {
            // one chain over the producers, small products first (mma3h's order).  Per-producer
            // zero-C chains joined by the VALU (the backward's form) moved the bs-32 step's
            // bias gradients by 3 % and cost 0.6 us per step: the adds wait on each MFMA
            const Duo wf = wfr(p, ct);
            acc[ct] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, wf.lo, acc[ct], 0, 0, 0);
            acc[ct] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, wf.hi, acc[ct], 0, 0, 0);
          }
        }
      }
      trace_at(s, 2);
    }
    if (io) {
      if (s + 1 < T) xin = load_in(s + 1);
      if (!kAblStores && s > 0) store_out(s - 1);
    }
    trace_at(s, 3);
    // the wave's partial: rows 4 (lane >> 4) + i (0-7 hi products, 8-15 lo products) of
    // columns ct * 16 + (lane & 15) = gate * 32 + unit
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        red[(wave * 16 + (lane >> 4) * 4 + i) * RC + ct * 16 + (lane & 15)] = acc[ct][i];
    __syncthreads();
    if (failed) {
      poison_rest(h_all, s, T, d != 0, N, D, n, d, H, j, H, 1, owner);
      return;
    }
    trace_at(s, 4);
    float gh[3];
#pragma unroll
    for (int gt = 0; gt < 3; ++gt) {
      float v = 0.f;
#pragma unroll
      for (int w4 = 0; w4 < LW; ++w4)
        v += red[(w4 * 16 + m) * RC + gt * LU + u] + red[(w4 * 16 + m + 8) * RC + gt * LU + u];
      gh[gt] = v;
    }
    const float xr = pin[m * LU + u], xz = pin[256 + m * LU + u], xn = pin[512 + m * LU + u];
    float hout = 0.f, r = 0.f, z = 0.f, nn = 0.f, ghn = 0.f;
    if (owner && t < len) {
      ghn = gh[2] * us_n + bias_n;
      r = sigmoid_fast(gh[0] * us_r + bias_r + xr);
      z = sigmoid_fast(gh[1] * us_z + bias_z + xz);
      nn = tanh_fast(xn + r * ghn);
      hout = (h_own - nn) * z + nn;
    }
    h_own = owner ? hout : 0.f;
    pout[m * LU + u] = hout;
    pout[256 + m * LU + u] = r;
    pout[512 + m * LU + u] = z;
    pout[768 + m * LU + u] = nn;
    pout[1024 + m * LU + u] = ghn;
    {
      const float v = hout * 16384.f;
      const _Float16 hi = (_Float16)v;
      stg[shi] = hi;
      stg[slo] = (_Float16)(v - (float)hi);
    }
    __syncthreads();
    if (wave == 0) {
      const int toff = (grp_off + ub * 256 + lane * 4) * 4;
      const u32x4 v = desentinel(*reinterpret_cast<const u32x4*>(stg + lane * 8));
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // last step's sentinel store first
      xl_store(v, x_rs, (s % LSLOTS) * slot_floats * 4 + toff, local);
      xl_store(u32x4{kSentinel, kSentinel, kSentinel, kSentinel}, x_rs,
               ((s + 2) % LSLOTS) * slot_floats * 4 + toff, local);
    }
    trace_at(s, 5);
  }
  __syncthreads();
  if (io && !kAblStores) store_out(T - 1);
}

// ---------------------------------------------------------------------------------------
// backward: rec[8 samples x 32 units] = dG[8 x 3H] . W_hh[3H rows, 32 units], dG = the (dar,
// daz, dghn) gate gradients of the step after.  Producer p publishes per step ONE record: per
// gate the stacked (hi; lo) fp16 A fragment of its 8 x 32 gradients, each sample row scaled by
// its own 2^e (max over the row's 96 values), then the 8 factors 2^-e.  Wave w holds W_hh^T's
// fragments for the producers [p0, p0 + np): per producer, gate and unit half, hi / lo of the
// 32 rows of that gate block in the consumer's 16 columns, each column scaled by 2^e(unit)
// (its max over the whole 3H).  Per record: 12 MFMAs from zero C, (C1 + C2) scaled per row and
// added to the wave's partial in producer order.
// Per-producer flags: the records as their own flags (the forward's sentinel ring over 3.1-KB
// records, no drain and no flag) measured 5.3-5.5 vs 3.8 us per step and was removed.
template <int NPW>
__global__ __launch_bounds__(LT) __attribute__((amdgpu_waves_per_eu(1, 1))) void gru_bwd_xl_kernel(
    int T, int N, int H, int D, int UBX, int BTX, const float* __restrict__ dy, int dyd,
    const float* __restrict__ w_f, const float* __restrict__ w_r,
    const float* __restrict__ h_all, const float* __restrict__ gates,
    const int* __restrict__ lens, float* __restrict__ dgx, float* __restrict__ dgh,
    float* __restrict__ ring, unsigned* __restrict__ xl, unsigned* __restrict__ err,
    unsigned long long* __restrict__ stamps, double* __restrict__ dbp,
    unsigned* __restrict__ camax, int force_global) {
  constexpr int RC = LU + 1;
  constexpr int LWP = 3;     // records in flight per wave beside the one multiplied
  __shared__ __attribute__((aligned(8))) float red[LW * 16 * RC > 4 * LB * LU * 2 ? LW * 16 * RC : 4 * LB * LU * 2];
  __shared__ __attribute__((aligned(16))) _Float16 stg[3 * 64 * 8];
  __shared__ __attribute__((aligned(16))) float stsc[LB];
  __shared__ float colmx[LW * LU];
  __shared__ __attribute__((aligned(16))) float pin[6 * 256];    // dy, r, z, n, W_hn h + b_hn, h_prev
  __shared__ __attribute__((aligned(16))) float pout[4 * 256];   // dar, daz, dan, dghn
  __shared__ int slen[LB];
  __shared__ int sh_local;
  __shared__ int flag;
  // W_hh^T fragments of a wave's last producer when it has NPW + 1 (as the forward's)
  __shared__ u32x4 wx[LW * 6 * 2 * 64];
  const int G = D * BTX;
  int g, ub;
  if (!xl_map(G, UBX, g, ub)) return;
  const int d = g / BTX, bt = g - d * BTX;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // the wave's producers: UBX / 4 each and one more for the lowest UBX % 4 waves -- wave 0,
  // which issues none of the step's HBM traffic (the io waves below), takes the extra one
  const int p0 = wave * (UBX / LW) + min(wave, UBX % LW);
  const int np = UBX / LW + (wave < UBX % LW ? 1 : 0);   // host guarantees np <= NPW + 1
  const int H3 = 3 * H;
  const int slot_floats = G * UBX * LRB;
  const __amdgpu_buffer_rsrc_t x_rs =
      __builtin_amdgcn_make_buffer_rsrc(ring, (short)0, 2 * slot_floats * 4, 0x00020000);
  const int grp_off = g * UBX * LRB;
  const bool local = xl_group_local(xl + g * 32, ub, UBX, err, &sh_local, xl + 512 + g, force_global);
  unsigned* flags = xl + 256 + g * 32;
  const __amdgpu_buffer_rsrc_t f_rs =
      __builtin_amdgcn_make_buffer_rsrc(xl + 256, (short)0, 8 * 32 * 4, 0x00020000);
  // per-wave timeline (DS2_GRU_STAMPS=2): [step][block][wave][6] = step start, hand-off wait
  // done, products done, io done (waves 1-3), reduction barrier done, published; lane 0 of
  // every wave (scripts/trace_gru.py)
  const bool tracing = stamps != nullptr && lane == 0;
  auto trace_at = [&](int s, int p) __attribute__((always_inline)) {
    if (tracing && s >= kXlTraceS0 && s < kXlTraceS0 + kXlTraceSteps)
      stamps[(((int64_t)(s - kXlTraceS0) * gridDim.x + blockIdx.x) * LW + wave) * 6 + p] =
          __builtin_amdgcn_s_memrealtime();
  };

  // W_hh^T fragments: producer p, gate gt, half c, k slot i ->
  //   W_hh[gt H + 32 (p0 + p) + 8 (lane >> 4) + i][32 ub + 16 c + (lane & 15)]
  Duo w[NPW][3][2];
  auto wfr = [&](int p, int gt, int c) __attribute__((always_inline)) {   // producer p's fragments (p == NPW: from LDS)
    if (p < NPW) return w[p < NPW ? p : 0][gt][c];
    Duo r;
    r.hi = __builtin_bit_cast(f16x8, wx[((wave * 6 + gt * 2 + c) * 2 + 0) * 64 + lane]);
    r.lo = __builtin_bit_cast(f16x8, wx[((wave * 6 + gt * 2 + c) * 2 + 1) * 64 + lane]);
    return r;
  };
  float unscale;   // 2^-e of the owner's unit (threadIdx.x & 31)
  {
    const float* W = d == 0 ? w_f : w_r;
    const int q8 = 8 * (lane >> 4);
    auto col = [&](int p, int gt, int c, f32x4& a, f32x4& b) __attribute__((always_inline)) {
      if (p < np) {
        const float* wc = W + (int64_t)(gt * H + LU * (p0 + p) + q8) * H + LU * ub + 16 * c + (lane & 15);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          a[i] = wc[(int64_t)i * H];
          b[i] = wc[(int64_t)(i + 4) * H];
        }
      } else {
        a = f32x4{0.f, 0.f, 0.f, 0.f};
        b = a;
      }
    };
    float mx[2] = {0.f, 0.f};
#pragma unroll
    for (int p = 0; p < NPW + 1; ++p)
#pragma unroll
      for (int gt = 0; gt < 3; ++gt)
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          f32x4 a, b;
          col(p, gt, c, a, b);
#pragma unroll
          for (int i = 0; i < 4; ++i) mx[c] = fmaxf(mx[c], fmaxf(fabsf(a[i]), fabsf(b[i])));
        }
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      mx[c] = fmaxf(mx[c], __shfl_xor(mx[c], 16));
      mx[c] = fmaxf(mx[c], __shfl_xor(mx[c], 32));
      if (lane < 16) colmx[wave * LU + 16 * c + lane] = mx[c];
    }
    __syncthreads();
    float sc[2];
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      float m = 0.f;
#pragma unroll
      for (int w4 = 0; w4 < LW; ++w4) m = fmaxf(m, colmx[w4 * LU + 16 * c + (lane & 15)]);
      sc[c] = __builtin_ldexpf(1.f, h3_row_exp(m));
    }
    {
      float m = 0.f;
#pragma unroll
      for (int w4 = 0; w4 < LW; ++w4) m = fmaxf(m, colmx[w4 * LU + (threadIdx.x & 31)]);
      unscale = __builtin_ldexpf(1.f, -h3_row_exp(m));
    }
    asm volatile("" ::: "memory");   // re-load W below (do not keep the max pass's loads live)
#pragma unroll
    for (int p = 0; p < NPW + 1; ++p)
#pragma unroll
      for (int gt = 0; gt < 3; ++gt)
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          f32x4 a, b;
          col(p, gt, c, a, b);
          const Duo dd = split2h(a, b, sc[c]);
          if (p < NPW) {
            w[p < NPW ? p : 0][gt][c] = dd;
          } else {
            wx[((wave * 6 + gt * 2 + c) * 2 + 0) * 64 + lane] = __builtin_bit_cast(u32x4, dd.hi);
            wx[((wave * 6 + gt * 2 + c) * 2 + 1) * 64 + lane] = __builtin_bit_cast(u32x4, dd.lo);
          }
        }
  }
  const int m = threadIdx.x >> 5;
  const int u = threadIdx.x & 31;
  const int n = bt * LB + m;
  const int j = ub * LU + u;
  const bool owner = n < N;
  if (threadIdx.x < LB) slen[threadIdx.x] = bt * LB + (int)threadIdx.x < N ? lens[bt * LB + threadIdx.x] : 0;
  __syncthreads();
  const int len = slen[m];
  const int shi = xl_frag_hi(m, u), slo = shi + 64;
  // The step's HBM traffic through LDS, issued by waves 1-3 only (as in the forward): wave 0
  // polls the flags and publishes, and neither its poll nor its drain may queue behind HBM
  // loads or stores (vmcnt counts in order).  Inputs one step ahead, loaded after the wave's
  // record loop; the gradients of step s stored during step s + 1.  io float4 idx = q + 192 k:
  // sample idx / 48, field (idx % 48) / 8, units 4 (idx % 8).
  // Addresses set up once (as the forward's): a fixed row pointer per io float4, advanced by
  // a fixed stride per step; masked lanes load from a valid address.
  const bool io = wave != 0;
  const int q = io ? (int)threadIdx.x - 64 : 0;
  // (32-bit element offsets: the host bounds every tensor below 2^31 bytes)
  const f32x4 z4v = f32x4{0.f, 0.f, 0.f, 0.f};
  const int ostr = N * D * H3;
  // per io float4 k (two per thread): field, sample length (-1: none), element offset of the
  // t = 0 row, stride per t, and the output offset (-1: none)
  struct IoSlot {
    const float* in;   // the input row of t = 0 (h_prev: its own t)
    float* out;        // the output row of t = 0 (nullptr: none)
    int f, len, str, pin_at, pout_at;
  };
  auto make_slot = [&](int k) __attribute__((always_inline)) {
    const int idx = q + 192 * k;
    const int sm = idx / 48, f = (idx % 48) >> 3, o4 = (idx & 7) * 4, sn = bt * LB + sm;
    IoSlot r;
    r.f = f;
    r.len = io && sn < N ? slen[sm] : -1;
    if (f == 0) {
      r.in = dy + (sn * dyd + (dyd > 1 ? d : 0)) * H + ub * LU + o4;
      r.str = N * dyd * H;
    } else if (f < 5) {
      r.in = gates + (sn * D + d) * 4 * H + (f - 1) * H + ub * LU + o4;
      r.str = N * D * 4 * H;
    } else {
      r.in = h_all + (sn * D + d) * H + ub * LU + o4;
      r.str = N * D * H;
    }
    r.out = io && sn < N ? (f < 3 ? dgx : dgh) + (sn * D + d) * H3 + (f % 3) * H + ub * LU + o4
                         : nullptr;
    r.pin_at = f * 256 + sm * LU + o4;
    r.pout_at = (f < 3 ? f : (f == 5 ? 3 : f - 3)) * 256 + sm * LU + o4;
    return r;
  };
  const IoSlot sl0 = make_slot(0), sl1 = make_slot(1);
  // the load, and separately whether step st has that row (the zero select is applied when the
  // value is staged: a select right after the load would wait for it there, as the forward's)
  auto in_ok = [&](int st, const IoSlot sl) __attribute__((always_inline)) {
    const int tt = d == 0 ? T - 1 - st : st;
    const int tr = sl.f == 5 ? (d == 0 ? tt - 1 : tt + 1) : tt;
    return !kAblLoads && tt < sl.len && tr >= 0 && tr < T;
  };
  auto load_in = [&](int st, const IoSlot sl) __attribute__((always_inline)) {
    const int tt = d == 0 ? T - 1 - st : st;
    const int tr = sl.f == 5 ? (d == 0 ? tt - 1 : tt + 1) : tt;
    return *reinterpret_cast<const f32x4*>(sl.in + (in_ok(st, sl) && !kAblFixT ? tr * sl.str : 0));
  };
  auto stage_in = [&](const f32x4 v, const IoSlot sl, int st) __attribute__((always_inline)) {
    *reinterpret_cast<f32x4*>(pin + sl.pin_at) = in_ok(st, sl) ? v : z4v;
  };
  auto store_one = [&](int tt, const IoSlot sl) __attribute__((always_inline)) {
    if (sl.out != nullptr)
      *reinterpret_cast<f32x4*>(sl.out + tt * ostr) = *reinterpret_cast<const f32x4*>(pout + sl.pout_at);
  };
  // pout (step st) -> dgx (dar, daz, dan), dgh (dar, daz, dghn)
  auto store_out = [&](int st) __attribute__((always_inline)) {
    const int tt = d == 0 ? T - 1 - st : st;
    store_one(tt, sl0);
    store_one(tt, sl1);
  };
  // one step ahead (as the forward's)
  f32x4 xin0 = io ? load_in(0, sl0) : z4v, xin1 = io ? load_in(0, sl1) : z4v;
  float dh_prev = 0.f, z_prev = 0.f;
  double sb_r = 0.0, sb_z = 0.0, sb_n = 0.0, sb_hn = 0.0;
  float cm_r = 0.f, cm_z = 0.f, cm_n = 0.f, cm_hn = 0.f;
  const int rsel = ((lane >> 4) & 1) * 16;   // this lane's 4 row factors (samples 4 (..) + i)
  // the io waves' issue point: right after a step's last record load (the records are then
  // older than these loads and stores, so the record waits never queue behind HBM: vmcnt
  // counts in order), inputs for the next step and the outputs of the previous one
  auto io_issue = [&](int st) __attribute__((always_inline)) {
    if (!io) return;
    if (st + 1 < T) {
      xin0 = load_in(st + 1, sl0);
      xin1 = load_in(st + 1, sl1);
    }
    if (!kAblStores && st > 0) store_out(st - 1);
  };
  for (int s = 0; s < T; ++s) {
    const int t = d == 0 ? T - 1 - s : s;
    f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
    trace_at(s, 0);
    if (io) {   // the step's inputs (loaded during the last step; waited for beside the poll)
      stage_in(xin0, sl0, s);
      stage_in(xin1, sl1, s);
    }
    if (s == 0) io_issue(0);
    if (s > 0) {
      if (!kAblWait && !flags_wait(flags, UBX, (unsigned)s, err, &flag)) {
        poison_rest(dgx, s, T, d == 0, N, D, n, d, H, j, H3, 3, owner);
        return;
      }
      trace_at(s, 1);
      const int rb = (((s - 1) & 1) * slot_floats + grp_off + p0 * LRB) * 4;
      u32x4 r0[NPW + 1], r1[NPW + 1], r2[NPW + 1];
      f32x4 rs[NPW + 1];
      auto load_rec = [&](int p) __attribute__((always_inline)) {
        const int base = p < np ? rb + p * LRB * 4 : 0x7ffff000;
        r0[p] = __builtin_amdgcn_raw_buffer_load_b128(x_rs, base + lane * 16, 0, kSc1);
        r1[p] = __builtin_amdgcn_raw_buffer_load_b128(x_rs, base + 1024 + lane * 16, 0, kSc1);
        r2[p] = __builtin_amdgcn_raw_buffer_load_b128(x_rs, base + 2048 + lane * 16, 0, kSc1);
        rs[p] = __builtin_bit_cast(
            f32x4, __builtin_amdgcn_raw_buffer_load_b128(x_rs, base + 3072 + rsel, 0, kSc1));
      };
#pragma unroll
      for (int p = 0; p < LWP && p < NPW + 1; ++p) load_rec(p);
      if (LWP >= NPW + 1) io_issue(s);
      asm volatile("" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int p = 0; p < NPW + 1; ++p) {
        if (p + LWP < NPW + 1) load_rec(p + LWP);
        if (p + LWP == NPW) io_issue(s);
        if (p < np) {
          const f16x8 ar = __builtin_bit_cast(f16x8, r0[p]);
          const f16x8 az = __builtin_bit_cast(f16x8, r1[p]);
          const f16x8 an = __builtin_bit_cast(f16x8, r2[p]);
#pragma unroll
          for (int c = 0; c < 2; ++c) {
            const f32x4 z4 = f32x4{0.f, 0.f, 0.f, 0.f};
            const Duo w0 = wfr(p, 0, c), w1 = wfr(p, 1, c), w2 = wfr(p, 2, c);
            f32x4 c1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(ar, w0.hi, z4, 0, 0, 0);
            f32x4 c2 = __builtin_amdgcn_mfma_f32_16x16x32_f16(ar, w0.lo, z4, 0, 0, 0);
            c1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(az, w1.hi, c1, 0, 0, 0);
            c2 = __builtin_amdgcn_mfma_f32_16x16x32_f16(az, w1.lo, c2, 0, 0, 0);
            c1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(an, w2.hi, c1, 0, 0, 0);
            c2 = __builtin_amdgcn_mfma_f32_16x16x32_f16(an, w2.lo, c2, 0, 0, 0);
            acc[c] += (c1 + c2) * rs[p];
          }
        }
      }
      trace_at(s, 2);
    }
    trace_at(s, 3);
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        red[(wave * 16 + (lane >> 4) * 4 + i) * RC + 16 * c + (lane & 15)] = acc[c][i];
    __syncthreads();
    const float dyv = pin[m * LU + u], g_r = pin[256 + m * LU + u], g_z = pin[512 + m * LU + u];
    const float g_n = pin[768 + m * LU + u], g_hn = pin[1024 + m * LU + u];
    const float hp = pin[1280 + m * LU + u];
    trace_at(s, 4);
    float dar = 0.f, daz = 0.f, dan = 0.f, dghn = 0.f;
    if (owner) {
      float dh = 0.f, zc = 0.f;
      if (t < len) {
        float carry = 0.f;
        if (s > 0) {
          float rec = 0.f;
#pragma unroll
          for (int w4 = 0; w4 < LW; ++w4)
            rec += red[(w4 * 16 + m) * RC + u] + red[(w4 * 16 + m + 8) * RC + u];
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
      sb_r += dar; sb_z += daz; sb_n += dan; sb_hn += dghn;
      cm_r = fmaxf(cm_r, fabsf(dar));
      cm_z = fmaxf(cm_z, fabsf(daz));
      cm_n = fmaxf(cm_n, fabsf(dan));
      cm_hn = fmaxf(cm_hn, fabsf(dghn));
    }
    pout[m * LU + u] = dar;
    pout[256 + m * LU + u] = daz;
    pout[512 + m * LU + u] = dan;
    pout[768 + m * LU + u] = dghn;
    {
      // the row's scale: max over the sample's 32 units x 3 gates (32 consecutive lanes)
      float mx = fmaxf(fmaxf(fabsf(dar), fabsf(daz)), fabsf(dghn));
#pragma unroll
      for (int o = 1; o < 32; o <<= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
      const int e = h3_row_exp(mx);
      const float sc = __builtin_ldexpf(1.f, e);
      const float vr = dar * sc, vz = daz * sc, vn = dghn * sc;
      const _Float16 hr = (_Float16)vr, hz = (_Float16)vz, hn = (_Float16)vn;
      stg[shi] = hr;
      stg[slo] = (_Float16)(vr - (float)hr);
      stg[512 + shi] = hz;
      stg[512 + slo] = (_Float16)(vz - (float)hz);
      stg[1024 + shi] = hn;
      stg[1024 + slo] = (_Float16)(vn - (float)hn);
      if (u == 0) stsc[m] = __builtin_ldexpf(1.f, -e);
    }
    __syncthreads();
    if (wave == 0) {
      const int so = ((s & 1) * slot_floats + grp_off + ub * LRB) * 4;
#pragma unroll
      for (int k = 0; k < 3; ++k)
        xl_store(*reinterpret_cast<const u32x4*>(stg + k * 512 + lane * 8), x_rs,
                 so + k * 1024 + lane * 16, local);
      if (lane < 2) xl_store(*reinterpret_cast<const u32x4*>(stsc + lane * 4), x_rs, so + 3072 + lane * 16, local);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (lane == 0) {
        const unsigned fv = (unsigned)s + 1;
        if (local)
          __builtin_amdgcn_raw_buffer_store_b32(fv, f_rs, (g * 32 + ub) * 4, 0, 0);
        else
          __builtin_amdgcn_raw_buffer_store_b32(fv, f_rs, (g * 32 + ub) * 4, 0, kSc1);
      }
    }
    trace_at(s, 5);
  }
  __syncthreads();
  if (io && !kAblStores) store_out(T - 1);
  if (camax != nullptr) {
    // column maxima of dgx [T N][D 3H] into camax[0, D 3H) and dgh into [D 3H, 2 D 3H): the 8
    // samples' running maxima per unit, one unsigned atomic max per (gate, unit)
    __syncthreads();
    red[(0 * LB + m) * LU + u] = cm_r;
    red[(1 * LB + m) * LU + u] = cm_z;
    red[(2 * LB + m) * LU + u] = cm_n;
    red[(3 * LB + m) * LU + u] = cm_hn;
    __syncthreads();
    if (threadIdx.x < 4 * LU) {
      const int gq = threadIdx.x / LU, uu = threadIdx.x - gq * LU;
      float a = 0.f;
#pragma unroll
      for (int mm = 0; mm < LB; ++mm) a = fmaxf(a, red[(gq * LB + mm) * LU + uu]);
      const unsigned bits = __float_as_uint(a);
      const int cl = d * H3 + ub * LU + uu;
      if (bits != 0u) {
        if (gq < 2) {
          atomicMax(camax + cl + gq * H, bits);
          atomicMax(camax + D * H3 + cl + gq * H, bits);
        } else if (gq == 2) {
          atomicMax(camax + cl + 2 * H, bits);
        } else {
          atomicMax(camax + D * H3 + cl + 2 * H, bits);
        }
      }
    }
  }
  if (dbp == nullptr) return;
  // the workgroup's 8 samples summed per unit in sample order -> dbp[bt][d][4][H]
  double* rd = reinterpret_cast<double*>(red);
  __syncthreads();
  rd[(0 * LB + m) * LU + u] = owner ? sb_r : 0.0;
  rd[(1 * LB + m) * LU + u] = owner ? sb_z : 0.0;
  rd[(2 * LB + m) * LU + u] = owner ? sb_n : 0.0;
  rd[(3 * LB + m) * LU + u] = owner ? sb_hn : 0.0;
  __syncthreads();
  if (threadIdx.x < 4 * LU) {
    const int gq = threadIdx.x / LU, uu = threadIdx.x - gq * LU;
    double a = 0.0;
#pragma unroll
    for (int mm = 0; mm < LB; ++mm) a += rd[(gq * LB + mm) * LU + uu];
    dbp[(((int64_t)bt * D + d) * 4 + gq) * H + ub * LU + uu] = a;
  }
}

// ---------------------------------------------------------------------------------------
// host side (called by ds2_gru_fwd / ds2_gru_bwd in gru.hip with their workspace carve-up)

static inline bool env_off(const char* name) {
  const char* e = getenv(name);
  return e != nullptr && e[0] == '0';
}
// DS2_GRU_XL=0 keeps the 16-unit kernels of gru_split.hip; the XCD-local kernels are fp16x3,
// so DS2_GRU_X6=0 (fp32 MFMA) and DS2_GRU_H3[_BWD]=0 (bf16x6) select the others as before.
// DS2_GRU_XL=2 (test) runs every group GLOBAL (sc1 stores), whatever the placement.
static inline bool xl_enabled() { return !env_off("DS2_GRU_XL") && !env_off("DS2_GRU_X6"); }
static inline int xl_force_global() {
  const char* e = getenv("DS2_GRU_XL");
  return (e != nullptr && e[0] == '2') ? 1 : 0;
}

// the shapes the XCD-local kernels take: H a multiple of 32 with a group (H / 32 workgroups)
// inside one XCD's 32 CUs, at most 8 groups (D x ceil(N / 8)), W_hh fragments within the
// instantiated producers per wave
int gru_xl_groups(int n, int h, int num_dirs) {
  if (!xl_enabled() || n < 1 || h < LU || (h % LU) != 0) return 0;
  const int UBX = h / LU, BTX = (n + LB - 1) / LB, G = num_dirs * BTX;
  if (UBX > 32 || G > 8 || (UBX + LW - 1) / LW > 7) return 0;
  return G;
}

// workgroups the launch holds (the blocks of unused groups return at once)
int gru_xl_active(int n, int h, int num_dirs) {
  const int G = gru_xl_groups(n, h, num_dirs);
  return G > 0 ? G * (h / LU) : 0;
}

// counter words the kernels use after the error word: 8 x 32 XCC ids, 8 x 32 flags, 8 mode words
size_t gru_xl_ctr_words() { return 520; }

// producers per wave: NPW in registers + one from LDS
static const void* fwd_xl_fn(int UBX) {
  const int need = (UBX + LW - 1) / LW;
#define DS2_FXL(K) \
  if (need <= K + 1) return reinterpret_cast<const void*>(gru_fwd_xl_kernel<K>);
  DS2_FXL(1) DS2_FXL(3) DS2_FXL(6)
#undef DS2_FXL
  return nullptr;
}

static const void* bwd_xl_fn(int UBX) {
  const int need = (UBX + LW - 1) / LW;
#define DS2_BXL(K) \
  if (need <= K + 1) return reinterpret_cast<const void*>(gru_bwd_xl_kernel<K>);
  DS2_BXL(1) DS2_BXL(3) DS2_BXL(6)
#undef DS2_BXL
  return nullptr;
}

// ring bytes: forward 4 slots of 1-KB tiles, backward 2 slots of records (both within the
// rings ds2_gru_fwd / ds2_gru_bwd carve for the 16-unit kernels)
size_t gru_xl_ring_bytes(int n, int h, int num_dirs, bool bwd) {
  const size_t UBX = h / LU, G = (size_t)num_dirs * ((n + LB - 1) / LB);
  return bwd ? 2 * G * UBX * LRB * sizeof(float) : LSLOTS * G * UBX * 256 * sizeof(float);
}

bool launch_gru_fwd_xl(int t_max, int n, int h, int num_dirs, const float* xproj,
                       const float* w_hh_f, const float* w_hh_r, const float* b_hh_f,
                       const float* b_hh_r, const int* lens, float* h_all, float* gates,
                       float* ring, unsigned* xl, unsigned* err, unsigned long long* stamps,
                       size_t lds_pad, hipStream_t st) {
  if (gru_xl_groups(n, h, num_dirs) == 0 || env_off("DS2_GRU_H3")) return false;
  apply_spin_limit_env();
  apply_rnn_tune_env();
  const int UBX = h / LU, BTX = (n + LB - 1) / LB;
  const void* fn = fwd_xl_fn(UBX);
  if (fn == nullptr) return false;
  int T_ = t_max, N_ = n, H_ = h, D_ = num_dirs, UB_ = UBX, BT_ = BTX, FG_ = xl_force_global();
  void* args[] = {&T_, &N_, &H_, &D_, &UB_, &BT_, &xproj, &w_hh_f, &w_hh_r, &b_hh_f,
                  &b_hh_r, &lens, &h_all, &gates, &ring, &xl, &err, &stamps, &FG_};
  return rnn_launch(fn, dim3(8 * UBX), dim3(LT), args, lds_pad, st) == hipSuccess;
}

// dbp: [ceil(n / 8)][D][4][H] partials (nullable); camax as launch_gru_bwd_x6's
bool launch_gru_bwd_xl(int t_max, int n, int h, int num_dirs, const float* dy, int dy_dirs,
                       const float* w_hh_f, const float* w_hh_r, const float* h_all,
                       const float* gates, const int* lens, float* dgates_x, float* dgates_h,
                       float* ring, unsigned* xl, unsigned* err, unsigned long long* stamps,
                       double* dbp, size_t lds_pad, hipStream_t st, unsigned* camax) {
  if (gru_xl_groups(n, h, num_dirs) == 0 || env_off("DS2_GRU_H3_BWD")) return false;
  apply_spin_limit_env();
  apply_rnn_tune_env();
  const int UBX = h / LU, BTX = (n + LB - 1) / LB;
  const void* fn = bwd_xl_fn(UBX);
  if (fn == nullptr) return false;
  int T_ = t_max, N_ = n, H_ = h, D_ = num_dirs, UB_ = UBX, BT_ = BTX, DYD_ = dy_dirs;
  int FG_ = xl_force_global();
  void* args[] = {&T_, &N_, &H_, &D_, &UB_, &BT_, &dy, &DYD_, &w_hh_f, &w_hh_r, &h_all,
                  &gates, &lens, &dgates_x, &dgates_h, &ring, &xl, &err, &stamps, &dbp, &camax,
                  &FG_};
  return rnn_launch(fn, dim3(8 * UBX), dim3(LT), args, lds_pad, st) == hipSuccess;
}

}  // namespace ds2
