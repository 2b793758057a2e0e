// Shared pieces of the recurrent kernels (gru.hip, lstm.hip): the workgroup
// tiling constants, W_hh repacking into MFMA-fragment order, XCD-aware work
// mapping, LDS staging, and the inter-workgroup hand-off of the persistent
// kernels (MI355X_MICROARCH.md "Valid forms" row 1).
#pragma once

#include "common.h"

#include <cstdlib>

namespace ds2 {

constexpr int GU = 16;      // hidden units per workgroup
constexpr int GB = 16;      // samples per workgroup
constexpr int GW = 8;       // waves per workgroup (K split 8 ways)
constexpr int GT = GW * 64; // threads per workgroup

// Wp[d][ub][ks][g][64] (G gates): lane l of k-step ks, gate g ->
//   W_hh_d[g*H + ub*16 + (l&15)][4*ks + (l>>4)]
template <int G>
__global__ void pack_fwd_kernel(const float* __restrict__ w_f, const float* __restrict__ w_r,
                                int H, int D, int UB, int KS, float* __restrict__ wp) {
  const int64_t total = (int64_t)D * UB * KS * G * 64;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    int64_t r = i;
    const int l = r % 64; r /= 64;
    const int g = r % G; r /= G;
    const int ks = r % KS; r /= KS;
    const int ub = r % UB; r /= UB;
    const int d = static_cast<int>(r);
    const float* w = d == 0 ? w_f : w_r;
    const int u = ub * GU + (l & 15);
    const int k = 4 * ks + (l >> 4);
    wp[i] = (u < H && k < H) ? w[(int64_t)(g * H + u) * H + k] : 0.f;
  }
}

// WpT[d][ub][ks][64] (W_hh has G*H rows): lane l of k-step ks ->
//   W_hh_d[4*ks + (l>>4)][ub*16 + (l&15)]
template <int G>
__global__ void pack_bwd_kernel(const float* __restrict__ w_f, const float* __restrict__ w_r,
                                int H, int D, int UB, int KS, float* __restrict__ wp) {
  const int64_t total = (int64_t)D * UB * KS * 64;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    int64_t r = i;
    const int l = r % 64; r /= 64;
    const int ks = r % KS; r /= KS;
    const int ub = r % UB; r /= UB;
    const int d = static_cast<int>(r);
    const float* w = d == 0 ? w_f : w_r;
    const int u = ub * GU + (l & 15);
    const int k = 4 * ks + (l >> 4);
    wp[i] = (u < H && k < G * H) ? w[(int64_t)k * H + u] : 0.f;
  }
}

// Stage rows [n0, n0+16) x cols [kc0, kc1) of a row-major matrix (row stride ld,
// valid rows < N) into hs[m][pitch], zero-filled.  8-byte accesses.
__device__ __forceinline__ void stage_rows(const float* __restrict__ src, int64_t ld, int N,
                                           int n0, int kc0, int kc1, float* __restrict__ hs,
                                           int pitch) {
  const int width = kc1 - kc0;
  const int pairs = (width + 1) >> 1;
  for (int i = threadIdx.x; i < GB * pairs; i += blockDim.x) {
    const int m = i / pairs;
    const int kp = (i - m * pairs) * 2;
    const int n = n0 + m;
    float2 v = make_float2(0.f, 0.f);
    if (n < N) {
      const float* p = src + (int64_t)n * ld + kc0 + kp;
      v.x = p[0];
      v.y = (kp + 1 < width) ? p[1] : 0.f;
    }
    *reinterpret_cast<float2*>(hs + m * pitch + kp) = v;
  }
}

// XCD-aware work mapping: the batch tiles of one (unit block, direction) pair run
// on the same XCD (blocks b and b+8 share one under the observed round-robin
// dispatch), and a pair keeps its XCD across the per-step launches, so its W_hh
// slice stays resident in that XCD's L2.  Speed only, never correctness.
__device__ __forceinline__ bool map_work(int P, int BT, int UB, int& ub, int& d, int& bt) {
  const int wg = blockIdx.x;
  const int xcd = wg & 7;
  const int slot = wg >> 3;
  const int pair = xcd + 8 * (slot / BT);
  bt = slot - (slot / BT) * BT;
  if (pair >= P) return false;
  ub = pair % UB;
  d = pair / UB;
  return true;
}

static inline int mapped_grid(int P, int BT) { return 8 * ((P + 7) / 8) * BT; }

// Same-XCD groups (DS2_GRU_XCD, the pre-split GRU backward): each of the G = D * BT hand-off
// groups on its own 8 / G XCDs, UB / (8 / G) unit blocks per XCD (cfg2: 4 groups x 2 XCDs x
// 25), so half of a consumer's producers share its XCD and the consumer reads their tiles
// from copies the producers also store plainly (kept in that XCD's L2: MI355X_MICROARCH
// "handoff-payload", 104-122 vs 66-73 GB/s per block).  Which producer shares the XCD is read
// at run time (xcc_id(), published per producer), never assumed from the placement.
static inline bool xgrp_fits(int UB, int BT, int D) {
  const int G = D * BT;
  return G >= 1 && G <= 8 && 8 % G == 0 && UB % (8 / G) == 0;
}
static inline int xgrp_grid(int UB, int BT, int D) { return 8 * (UB / (8 / (D * BT))); }
// DS2_GRU_XCD=0 keeps map_work's interleaved layout for every persistent backward
static inline bool xcd_groups_on() {
  const char* xe = getenv("DS2_GRU_XCD");
  return !(xe != nullptr && xe[0] == '0');
}
__device__ __forceinline__ bool map_work_xgrp(int UB, int BT, int D, int& ub, int& d, int& bt) {
  const int wg = blockIdx.x;
  const int xcd = wg & 7, slot = wg >> 3;
  const int G = D * BT, xpg = 8 / G, per = UB / xpg;
  const int q = xcd / xpg, part = xcd - q * xpg;
  if (slot >= per || q >= G) return false;
  ub = part * per + slot;
  d = q / BT;
  bt = q - d * BT;
  return true;
}
__device__ __forceinline__ unsigned xcc_id() {
  return __builtin_amdgcn_s_getreg(20 | (0 << 6) | ((4 - 1) << 11)) & 15u;   // HW_REG_XCC_ID
}


// ===========================================================================
// Persistent variants: one launch per layer and direction pair.  Each workgroup
// keeps its W_hh fragments in registers for all T steps; the per-step hand-off of
// the new hidden states (forward) / gate gradients (backward) between the UB
// workgroups of a (direction, batch tile) group follows the write-through form
// of MI355X_MICROARCH.md "Valid forms" row 1: payload stored sc1 (agent-scope
// relaxed atomic stores), every storing wave drains vmcnt, workgroup barrier,
// one lane stores the producer's step count to its flag (sc1); consumers poll
// the group's flags relaxed (one wave, s_sleep, bounded), barrier, then load the
// payload with sc1 loads -- or the sentinel ring below, where the data is the flag.
// Flags are zeroed by a hipMemsetAsync before every launch; a spin that exceeds its
// bound sets the error word and the workgroup leaves (no hang, results invalid).
constexpr unsigned kSpinLimit = 1u << 21;

// The bound the kernels use: kSpinLimit unless DS2_RNN_SPIN_LIMIT is set in the environment
// (checked at every recurrence entry point).  0 is fault injection: every hand-off wait fails
// as a timeout would, whether or not its data has arrived -- the test that checks the failure
// surfaces through err_out (and as Ds2Error in the Trainer) instead of going silent uses it.
static __constant__ unsigned g_spin_limit = kSpinLimit;

static void apply_spin_limit_env() {
  static unsigned applied = kSpinLimit;
  const char* e = getenv("DS2_RNN_SPIN_LIMIT");
  const unsigned v = (e == nullptr || e[0] == 0) ? kSpinLimit
                                                 : static_cast<unsigned>(strtoul(e, nullptr, 10));
  if (v == applied) return;
  // synchronous symbol write: only ever taken when a test changes the variable
  if (hipMemcpyToSymbol(HIP_SYMBOL(g_spin_limit), &v, sizeof(v)) == hipSuccess) applied = v;
}

// Polling knobs of the sentinel hand-off: [0] s_sleep(1) units between re-load passes, [1]
// units before a forward step's first load pass, [2] the same for the backward (a consumer
// that loads right after publishing mostly gets sentinels back, and those full-tile polls
// from every workgroup crowd the fabric that carries the real tiles).  Defaults from
// scripts/gru_ab.py sweeps (the forward's first-poll delay 14 -> 10 with the same-XCD groups,
// whose same-XCD tiles arrive sooner: 4.32-4.40 -> 4.26 us per step, `ftune`,
// profiles/r3fa_fwd_tune.txt; the fp16x3 forward: 10 -> 7, 3.74-3.83 -> 3.74-3.75 us,
// profiles/r6p_fwd_tune.txt); [3] s_sleep(1) units between the flag hand-off's polls.
// [4]: the flag hand-off's second poll in flight, issued this many s_sleep(1) units after the
// first (0: one poll at a time, each after the previous one returned).  [5]: s_sleep(1) units
// before the flag hand-off's first poll of a step (polls before the group's last producer can
// have published only load the flag lines that producers are writing).  [6]: tiles the
// XCD-local forward re-loads per stale pass, from the one it waits on, and [7] its first-poll
// delay (gru_xl.hip; scripts/gru_ab.py xlrepoll: every pending tile with no delay 3.38 us per
// step, one tile 3.46, every tile after 7 units 3.62).
// DS2_RNN_TUNE="a,b,c,d,e" overrides them (diagnostic; checked at every recurrence entry point).
constexpr unsigned kRepollSleep = 1u, kFirstPollDelay = 7u, kFirstPollDelayBwd = 14u,
                   kFlagPollSleep = 1u, kFlagPollGap = 0u, kFlagFirstDelay = 0u, kXlRepoll = 8u,
                   kXlFirstDelay = 0u;
constexpr int kTuneN = 8;
static __constant__ unsigned g_rnn_tune[kTuneN] = {kRepollSleep, kFirstPollDelay,
                                                   kFirstPollDelayBwd, kFlagPollSleep,
                                                   kFlagPollGap, kFlagFirstDelay, kXlRepoll,
                                                   kXlFirstDelay};

static void apply_rnn_tune_env() {
  static unsigned applied[kTuneN] = {kRepollSleep, kFirstPollDelay, kFirstPollDelayBwd,
                                     kFlagPollSleep, kFlagPollGap, kFlagFirstDelay, kXlRepoll,
                                     kXlFirstDelay};
  unsigned v[kTuneN] = {kRepollSleep, kFirstPollDelay, kFirstPollDelayBwd, kFlagPollSleep,
                        kFlagPollGap, kFlagFirstDelay, kXlRepoll, kXlFirstDelay};
  const char* e = getenv("DS2_RNN_TUNE");
  for (int i = 0; e != nullptr && e[0] != 0 && i < kTuneN; ++i) {
    char* end = nullptr;
    v[i] = static_cast<unsigned>(strtoul(e, &end, 10));
    e = (end != nullptr && *end == ',') ? end + 1 : nullptr;
  }
  bool same = true;
  for (int i = 0; i < kTuneN; ++i) same = same && v[i] == applied[i];
  if (same) return;
  if (hipMemcpyToSymbol(HIP_SYMBOL(g_rnn_tune), v, sizeof(v)) == hipSuccess)
    for (int i = 0; i < kTuneN; ++i) applied[i] = v[i];
}

__device__ __forceinline__ void sleep_units(unsigned k) {
  for (unsigned i = 0; i < k; ++i) __builtin_amdgcn_s_sleep(1);
}

// err_out (C ABI, nullable): the caller's device status word.  After a persistent launch the
// launch's own error word (in the workspace, reset before every launch) is OR-ed into it, so
// a hand-off timeout stays visible to the host after the workspace is recycled.
static __global__ void err_fold_kernel(const unsigned* __restrict__ err, unsigned* __restrict__ out) {
  if (threadIdx.x == 0) {
    const unsigned v = __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (v != 0u) __hip_atomic_fetch_or(out, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

static inline void fold_err(const unsigned* err, unsigned* err_out, hipStream_t st) {
  if (err_out != nullptr) hipLaunchKernelGGL(err_fold_kernel, dim3(1), dim3(64), 0, st, err, err_out);
}

__device__ __forceinline__ void st_sc1(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ unsigned long long ld_sc1_u64(const float* p) {
  return __hip_atomic_load(reinterpret_cast<const unsigned long long*>(p), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ float ld_sc1(const float* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Per-producer flag variant of the hand-off (same valid form, row 1: one lane of each
// storing workgroup publishes with an sc1 store; the consumer polls every shard).  The
// group's UB flags sit in one or two cache lines; wave 0 polls them with one vector sc1
// load (lane i <- producer i) and a ballot, so no atomic read-modify-write serialises
// the arrivals.  flags[i] holds the number of steps producer i has published.
// poll_wave: the wave that polls.  Its loads return in order, so any global load it issued
// before the poll (a step's dy / gate-cache loads) holds the poll's first answer back until
// that load is served; a wave that loads nothing else polls unhindered.
__device__ __forceinline__ bool flags_wait(const unsigned* flags, int count, unsigned target,
                                           unsigned* err, int* lds_flag, int poll_wave = 0) {
  if ((threadIdx.x >> 6) == poll_wave) {
    const int lane = threadIdx.x & 63;
    unsigned spins = 0;
    int ok = 1;
    if (g_spin_limit == 0) {   // fault injection
      if (lane == 0) __hip_atomic_fetch_or(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      ok = 0;
    }
    auto poll = [&]() {
      return lane < count ? __hip_atomic_load(flags + lane, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT)
                          : target;
    };
    const unsigned gap = g_rnn_tune[4];
    sleep_units(g_rnn_tune[5]);
    if (gap != 0u && ok) {
      // two polls in flight, `gap` apart: a flag set just after one poll passed the L2 is
      // seen by the other about half a round trip later instead of a full one
      unsigned a = poll();
      sleep_units(gap);
      unsigned b = poll();
      for (;;) {
        if (__ballot(a < target) == 0ull) break;
        a = poll();
        if (__ballot(b < target) == 0ull) break;
        b = poll();
        if (++spins > g_spin_limit) {
          if (lane == 0) __hip_atomic_fetch_or(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          ok = 0;
          break;
        }
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the poll left in flight
    }
    for (; ok && gap == 0u;) {
      const unsigned v = poll();
      if (__ballot(v < target) == 0ull) break;
      sleep_units(g_rnn_tune[3]);
      if (++spins > g_spin_limit) {
        if (lane == 0) __hip_atomic_fetch_or(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ok = 0;
        break;
      }
    }
    if (lane == 0) *lds_flag = ok;
  }
  __syncthreads();
  return *lds_flag != 0;
}

// After a hand-off timeout the workgroup leaves its step loop; its owning lanes first
// fill their unit's outputs for every remaining step with NaN (`groups` slices of H
// columns per row of `width` floats), so the failure reaches the loss instead of
// leaving stale memory behind.  `rev` is true when direction d walks t downwards.
__device__ __forceinline__ void poison_rest(float* out, int s, int T, bool rev, int N, int D,
                                            int n, int d, int H, int j, int width, int groups,
                                            bool owner) {
  if (!owner || out == nullptr) return;
  for (int q = s; q < T; ++q) {
    const int t = rev ? T - 1 - q : q;
    float* o = out + (((int64_t)t * N + n) * D + d) * width + j;
    for (int g = 0; g < groups; ++g) o[(int64_t)g * H] = __builtin_nanf("");
  }
}

// K split of the direct-operand kernels: `nblk` 16-wide blocks over the GW = 8 waves,
// balanced per SIMD (waves w and w + 4 share SIMD w % 4): SIMD s gets its share of the
// blocks, split between its two waves; wave w owns the contiguous blocks [b0, b0 + nb).
__device__ __forceinline__ void simd_split(int nblk, int wave, int& b0, int& nb) {
  auto simd_lo = [&](int s) { return (nblk * s) / 4; };
  auto wave_cnt = [&](int w) {
    const int s = w & 3;
    const int c = simd_lo(s + 1) - simd_lo(s);
    return w < 4 ? (c + 1) / 2 : c / 2;
  };
  int start = 0;
  for (int w = 0; w < wave; ++w) start += wave_cnt(w);
  b0 = start;
  nb = wave_cnt(wave);
}

__device__ __forceinline__ void flags_arrive(unsigned* flag, unsigned value) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every storing wave drains first
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(flag, value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr int kSc1 = 16;   // buffer-op aux bit: sc1 (write-through store / L1-bypassing load)

// Wait for a loaded value HERE, once: a loop-invariant load first used inside the step loop
// makes the waitcnt pass put a conservative vmcnt(0) at that use on EVERY iteration, which
// then also waits for the previous step's write-through hand-off stores (gru_fwd_dop_kernel:
// 1.16 us of a 5.5 us step).  "+v" forces the value into a VGPR and redefines it.
template <typename T>
__device__ __forceinline__ void settle(T& v) { asm volatile("" : "+v"(v)); }

// Sentinel-ring hand-off of the direct-operand kernels (the data is the flag; the R2 idea
// of cdna_hip_programming.md G16 without widening the payload).  Each producer tile lives
// in a ring of kRingSlots slots; a slot that will next hold step s + 2 is refilled with the
// sentinel word at step s (once the producer has consumed every producer's step s - 1
// tile, so every consumer has finished reading the slot's old step s - 2 contents).  The
// producer drains vmcnt before each data store, so the sentinel of a slot is performed
// before the tile a consumer must observe before it reads that slot again.  Consumers
// spin with sc1 loads until none of their words is the sentinel.  Every word is written
// whole by one 16-B sc1 store (R2: untorn).  A payload word equal to the sentinel (one
// NaN bit pattern) is published as the canonical quiet NaN instead.
constexpr unsigned kSentinel = 0xFFFFFFFFu;
constexpr int kRingSlots = 4;

__device__ __forceinline__ bool tile_ready(f32x4 v) {
  const u32x4 b = __builtin_bit_cast(u32x4, v);
  return (b.x != kSentinel) & (b.y != kSentinel) & (b.z != kSentinel) & (b.w != kSentinel);
}

__device__ __forceinline__ u32x4 desentinel(u32x4 v) {
  const unsigned qnan = 0x7FC00000u;
  return u32x4{v.x == kSentinel ? qnan : v.x, v.y == kSentinel ? qnan : v.y,
               v.z == kSentinel ? qnan : v.z, v.w == kSentinel ? qnan : v.w};
}

// wave-uniform "every lane's tile words are ready"
__device__ __forceinline__ bool wave_ready(f32x4 v) { return __ballot(!tile_ready(v)) == 0ull; }

// Spin until the wave's ring tile at byte offset off (already loaded into v once) holds no
// sentinel word, re-loading it alone; false (and the error word set) after g_spin_limit polls.
// The wave's later tiles stay in flight meanwhile.
__device__ __forceinline__ bool spin_tile(f32x4& v, __amdgpu_buffer_rsrc_t rs, int off,
                                          unsigned* err) {
  for (unsigned spins = 0; g_spin_limit == 0 || !wave_ready(v); ++spins) {
    if (spins > g_spin_limit || g_spin_limit == 0) {
      if ((threadIdx.x & 63) == 0)
        __hip_atomic_fetch_or(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
    asm volatile("" ::: "memory");   // the re-load is not loop-invariant (no LICM)
    v = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, kSc1));
  }
  return true;
}

// Stage rows [n0, n0+ROWS) x [0, cols) of a row-major slab (row stride ld floats, N
// valid rows, `width` valid columns) into hs[m][pitch] with 16-byte sc1 buffer loads.
// Rows >= N and columns >= width read as zero (out-of-range buffer offsets return
// 0), so the MFMA loop needs no bounds checks.  All MAXI loads of a thread are
// issued before the first LDS store.  width, cols and ld are multiples of 4.
template <int MAXI, int ROWS = GB>
__device__ __forceinline__ void stage_rows_sc1(const float* src, int ld, int N, int n0,
                                               int width, int cols, float* __restrict__ hs,
                                               int pitch) {
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(src), (short)0, N * ld * 4, 0x00020000);
  const int q = cols >> 2;
  const int total = ROWS * q;
  u32x4 v[MAXI];
#pragma unroll
  for (int r = 0; r < MAXI; ++r) {
    const int i = threadIdx.x + r * GT;
    int off = 0x7ffffff0;
    if (i < total) {
      const int m = i / q;
      const int k = (i - m * q) * 4;
      if (k < width) off = ((n0 + m) * ld + k) * 4;
    }
    v[r] = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, kSc1);
  }
#pragma unroll
  for (int r = 0; r < MAXI; ++r) {
    const int i = threadIdx.x + r * GT;
    if (i < total) {
      const int m = i / q;
      const int k = (i - m * q) * 4;
      *reinterpret_cast<u32x4*>(hs + m * pitch + k) = v[r];
    }
  }
}

// phase stamps (diagnostic, DS2_GRU_STAMPS=1): workgroup 0, thread 0 accumulates
// s_memtime deltas per phase into stamps[0..7] (units: shader clocks)
__device__ __forceinline__ unsigned long long stamp_now() { return __builtin_amdgcn_s_memtime(); }

static int g_num_cus = -1;
static int num_cus() {
  if (g_num_cus < 0) {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess) dev = 0;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) v = 0;
    g_num_cus = v;
  }
  return g_num_cus;
}

// smallest instantiated k-steps-per-wave >= per whose zero-padded span fits the LDS pitch
static int persist_ksw(int per, int kc) {
  const int opts[] = {8, 16, 25, 32, 48, 64, 75};
  for (int k : opts)
    if (per <= k && 4 * GW * k <= kc) return k;
  return -1;
}

static bool persistent_enabled() {
  const char* e = getenv("DS2_RNN_PERSISTENT");
  return !(e != nullptr && e[0] == '0');
}

// Launch of a persistent recurrence kernel: a plain launch.  The host has already sized the
// grid to the chip (grid <= CUs, one workgroup per CU through its LDS footprint), so a
// cooperative launch would add only the runtime's occupancy check (and 15-20 us of host time
// per launch; residency is the same for plain and cooperative launches, MI355X_MICROARCH.md
// "Residency and cooperative launch").  Cooperative launches were also the cause of round 2's
// rocprofv3 exit SIGSEGV (scripts/prof_exit_probe2.sh) and were removed.  What a concurrent
// collective may take is budgeted by optim.GradAllReducer.guard_cooperative
// (tests/test_gpu_residency.py).
// `lds` is a dynamic-LDS pad that keeps one workgroup per CU; a kernel whose static LDS
// already takes more than half the CU's LDS gets less pad, so static + pad never exceeds the
// per-workgroup limit (a dispatch over it faulted: the pre-split sentinel backward's 94 KB of
// static LDS + the 80 KB pad; pinned by ds2_test_rnn_launch_lds).
static inline hipError_t rnn_launch(const void* fn, dim3 grid, dim3 block, void** args,
                                    size_t lds, hipStream_t st) {
  constexpr size_t max_lds = 160 * 1024;   // gfx950: LDS per CU = per workgroup maximum
  hipFuncAttributes fa;
  if (hipFuncGetAttributes(&fa, fn) != hipSuccess) return hipErrorInvalidDeviceFunction;
  const size_t stat = fa.sharedSizeBytes;
  if (stat > max_lds) return hipErrorInvalidValue;
  if (stat + lds > max_lds) lds = max_lds - stat;
  return hipLaunchKernel(fn, grid, block, args, lds, st);
}

static inline int grid_cap(int64_t work) {
  int64_t g = (work + 255) / 256;
  return static_cast<int>(g > 2048 ? 2048 : (g < 1 ? 1 : g));
}

static inline size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

// fp16x3 (the recurrences' default since round 5): a value x of a row scaled by 2^e into
// [2^14, 2^15) splits into hi = f16(x 2^e) and lo = f16(x 2^e - hi) (22 significant bits
// kept for every element within 2^17 of the row's max), and a.b takes three products
// lo.hi + hi.lo + hi.hi on v_mfma_f32_16x16x32_f16 (each exact in fp32): half the MFMAs of
// the bf16x6 form and two operand planes instead of three.  h (|h| <= 1) takes the fixed
// scale 2^14; each W_hh row (gate, unit) its own, found at kernel start.
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2h __attribute__((ext_vector_type(2)));
struct Duo {
  f16x8 hi, lo;
};

// 8 fp32 values (k slots 0..3 from a, 4..7 from b) times sc -> fp16 (hi, lo)
__device__ __forceinline__ Duo split2h(const f32x4 a, const f32x4 b, float sc) {
  typedef float f32x2v __attribute__((ext_vector_type(2)));
  Duo t;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const f32x2v x = (j < 2 ? f32x2v{a[2 * j], a[2 * j + 1]} : f32x2v{b[2 * j - 4], b[2 * j - 3]}) * sc;
    const f16x2h h = __builtin_convertvector(x, f16x2h);
    const f16x2h l = __builtin_convertvector(x - __builtin_convertvector(h, f32x2v), f16x2h);
    t.hi[2 * j] = h[0];
    t.hi[2 * j + 1] = h[1];
    t.lo[2 * j] = l[0];
    t.lo[2 * j + 1] = l[1];
  }
  return t;
}

// c += a.b from the fp16 terms in one MFMA chain (small terms first): the forward
// recurrences' form.  The matrix cores floor an addend's bits below ~2^-31 of the largest
// operand of one instruction, C included (scripts/mfma_rounding.hip), so the small products
// chained beside hi.hi lose their lowest bits downward: ~1e-7 relative per result, which the
// forward's state update does not sum up (the backward kernels, whose gate gradients feed the
// bias-gradient sums, keep the small products in a chain of their own).  Splitting the chains
// here cost the GRU forward 1.95 -> 2.32 ms per launch (the join is a VALU add on the
// critical path of every hand-off step).
__device__ __forceinline__ f32x4 mma3h(const Duo& a, const Duo& b, f32x4 c) {
  c = __builtin_amdgcn_mfma_f32_16x16x32_f16(a.lo, b.hi, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_f16(a.hi, b.lo, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_f16(a.hi, b.hi, c, 0, 0, 0);
  return c;
}

// 2^e scale of a row whose max |x| is m (m > 0 finite: m 2^e in [2^14, 2^15); else 1)
__device__ __forceinline__ int h3_row_exp(float m) {
  const unsigned u = __float_as_uint(m);
  const int E = (int)(u >> 23);
  if (u == 0u || E >= 255) return 0;
  const int e = 14 - ((E == 0 ? 1 : E) - 127);
  return e > 127 ? 127 : e;
}

}  // namespace ds2
