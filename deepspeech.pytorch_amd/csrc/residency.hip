// Residency of the persistent recurrences beside a collective, made testable on
// one GPU.  The recurrences are plain launches sized to one workgroup per CU whose workgroups
// spin on each other's hand-offs, so they finish only if every workgroup is resident at once;
// at world > 1 an RCCL all-reduce overlapping the backward holds up to NCCL_MAX_NCHANNELS CUs
// (optim.GradAllReducer.guard_cooperative budgets for it).  These entry points let a one-GPU
// test hold CUs the way a collective's CTAs would and order the events on the device clock:
//   ds2_test_occupy     -- `ctas` workgroups, each alone on its CU (an LDS footprint no
//                          recurrence workgroup fits beside), each spinning on s_memrealtime for
//                          max_us (bounded: every wave exits by itself), recording
//                          [start, end, xcc id, hw id] per workgroup;
//   ds2_test_timestamp  -- one s_memrealtime stamp on a stream (orders kernels on it);
//   ds2_test_ring_traffic -- a ring all-reduce's local HBM traffic (read-only on the bucket),
//                          paced at a bus bandwidth, on `ctas` CUs: the interference of a
//                          bucket all-reduce with the recurrences, measured on one GPU;
//   ds2_test_rnn_launch_lds -- the same occupier with 94 KB of STATIC LDS launched through
//                          rnn_launch with the recurrences' 80 KB pad: the clamp that fixed round
//                          3's dispatch fault (static + pad over the 160 KB per workgroup) must
//                          shrink the pad so the launch runs.
#include "rnn_common.h"
#include "../../include/ds2hip_test.h"

namespace ds2 {

constexpr unsigned long long kRealtimeHz = 100000000ull;   // s_memrealtime: 100 MHz

__device__ __forceinline__ void occupy_body(int max_us, unsigned long long* __restrict__ rec,
                                            bool bad = false) {
  if (threadIdx.x != 0) return;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  const unsigned long long lim = (unsigned long long)max_us * (kRealtimeHz / 1000000ull);
  unsigned long long t = t0;
  while (t - t0 < lim) {
    __builtin_amdgcn_s_sleep(127);
    t = __builtin_amdgcn_s_memrealtime();
  }
  unsigned long long* r = rec + (size_t)blockIdx.x * 4;
  r[0] = t0;
  r[1] = t;
  r[2] = bad ? ~0ull : (unsigned long long)xcc_id();
  r[3] = __builtin_amdgcn_s_getreg(4 | (0 << 6) | ((32 - 1) << 11));   // HW_REG_HW_ID
}

__global__ __launch_bounds__(64) void occupy_kernel(int max_us, unsigned long long* rec) {
  extern __shared__ float pad[];   // dynamic LDS: holds the CU's LDS
  if (threadIdx.x == 0) pad[0] = 0.f;
  occupy_body(max_us, rec);
}

constexpr int kStaticLdsFloats = 94 * 1024 / 4;
__global__ __launch_bounds__(64) void occupy_static_kernel(int max_us, unsigned long long* rec) {
  __shared__ float big[kStaticLdsFloats];
  volatile float* vb = big;
  vb[threadIdx.x * 367] = (float)threadIdx.x;   // keep the static array (and its size)
  __syncthreads();
  occupy_body(max_us, rec, vb[63 * 367] != 63.f);
}

// A ring all-reduce's local HBM traffic on ONE GPU (ds2_test_ring_traffic): the
// 2 (W - 1) phases over W ranks each read one S / W chunk of the bucket and the scratch chunk
// a peer would have landed here, and write the reduced chunk back to scratch (what is sent
// on).  Phase p starts no earlier than p * phase_ticks after the workgroup's start (the link
// pace; 0 = as fast as the CTAs go).  The bucket is only read.
__global__ __launch_bounds__(256) void ring_traffic_kernel(const float4* __restrict__ bucket,
                                                           int64_t count4, int world,
                                                           float4* __restrict__ scratch,
                                                           int64_t chunk4, long long phase_ticks) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  const int phases = 2 * (world - 1);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int p = 0; p < phases; ++p) {
    if (phase_ticks > 0) {
      const unsigned long long due = t0 + (unsigned long long)p * phase_ticks;
      // bounded: at most 2^20 sleeps (~80 ms) per phase whatever the clock says
      for (int i = 0; i < (1 << 20) && __builtin_amdgcn_s_memrealtime() < due; ++i)
        __builtin_amdgcn_s_sleep(8);
    }
    const int64_t base = (int64_t)(p % world) * chunk4;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < chunk4; i += stride) {
      const int64_t j = base + i;
      const float4 a = j < count4 ? bucket[j] : make_float4(0.f, 0.f, 0.f, 0.f);
      float4 b = scratch[i];
      b.x += a.x; b.y += a.y; b.z += a.z; b.w += a.w;
      scratch[i] = b;
    }
  }
}

__global__ void timestamp_kernel(unsigned long long* out) {
  if (threadIdx.x == 0) *out = __builtin_amdgcn_s_memrealtime();
}

}  // namespace ds2

using namespace ds2;

extern "C" {

ds2_status_t ds2_test_occupy(int ctas, int lds_kb, int max_us, unsigned long long* rec,
                             ds2_stream_t stream) {
  if (ctas < 1 || ctas > 4096 || lds_kb < 0 || lds_kb > 160 || max_us < 0 || max_us > 5000000 ||
      rec == nullptr)
    return DS2_INVALID_VALUE;
  hipLaunchKernelGGL(occupy_kernel, dim3(ctas), dim3(64), (size_t)lds_kb * 1024,
                     as_stream(stream), max_us, rec);
  return launch_status("ds2_test_occupy");
}

ds2_status_t ds2_test_rnn_launch_lds(int ctas, int max_us, unsigned long long* rec,
                                     ds2_stream_t stream) {
  if (ctas < 1 || ctas > 4096 || max_us < 0 || max_us > 5000000 || rec == nullptr)
    return DS2_INVALID_VALUE;
  int mu = max_us;
  void* args[] = {&mu, &rec};
  // the recurrences' one-workgroup-per-CU pad (gru.hip kDopPadLds)
  if (rnn_launch(reinterpret_cast<const void*>(occupy_static_kernel), dim3(ctas), dim3(64), args,
                 80 * 1024, as_stream(stream)) != hipSuccess)
    return launch_status("ds2_test_rnn_launch_lds");
  return launch_status("ds2_test_rnn_launch_lds");
}

ds2_status_t ds2_test_ring_traffic(const float* bucket, int64_t count, int world, float* scratch,
                                   int ctas, double busbw_gbps, ds2_stream_t stream) {
  if (bucket == nullptr || scratch == nullptr || count < 0 || world < 2 || world > 64 ||
      ctas < 1 || ctas > 1024 || busbw_gbps < 0 || (reinterpret_cast<uintptr_t>(bucket) & 15) ||
      (reinterpret_cast<uintptr_t>(scratch) & 15))
    return DS2_INVALID_VALUE;
  if (count == 0) return DS2_OK;
  const int64_t count4 = count / 4;                       // a partial float4 is not streamed
  const int64_t chunk4 = (count4 + world - 1) / world;
  // one phase moves chunk bytes over the link: (S / W) / busbw seconds, 100 MHz ticks
  const long long ticks =
      busbw_gbps > 0 ? (long long)((double)chunk4 * 16.0 / (busbw_gbps * 1e9) * 1e8) : 0;
  hipLaunchKernelGGL(ring_traffic_kernel, dim3(ctas), dim3(256), 0, as_stream(stream),
                     reinterpret_cast<const float4*>(bucket), count4, world,
                     reinterpret_cast<float4*>(scratch), chunk4, ticks);
  return launch_status("ds2_test_ring_traffic");
}

ds2_status_t ds2_test_timestamp(unsigned long long* out, ds2_stream_t stream) {
  if (out == nullptr) return DS2_INVALID_VALUE;
  hipLaunchKernelGGL(timestamp_kernel, dim3(1), dim3(64), 0, as_stream(stream), out);
  return launch_status("ds2_test_timestamp");
}

}  // extern "C"
