// MFMA ceiling probe: the rate a bare MFMA loop reaches at the GEMM
// kernel's own wave tile and product count, on random operands, at the clock the chip holds
// under that load.  No global memory in the loop.  Modes:
//   x6   : 6 v_mfma_f32_16x16x32_bf16 per (A, B) fragment pair (the bf16x6 products)
//   h3   : 3 v_mfma_f32_16x16x32_f16 per pair (an fp16 two-term split, 3 products)
//   b1   : 1 v_mfma_f32_16x16x32_bf16 per pair (plain bf16)
// Wave tile WMT x WNT 16x16 tiles (sxgemm2 M16: 4 x 4 at TBN 128, 2 x 10 at TBN 160), 8 waves
// per workgroup (two per SIMD), one workgroup per CU (LDS pad), grid = CUs.  With lds=1 every
// k-step re-reads the fragments from LDS (ds_read_b128 per plane), as the GEMM does.
// Each workgroup stamps s_memtime / s_memrealtime around its loop: the in-kernel clock.
// build: hipcc -O3 --offload-arch=gfx950 -o scripts/mfma_ceiling scripts/mfma_ceiling.hip
// run:   scripts/mfma_ceiling [seconds]   -> one JSON line per configuration
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include <algorithm>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1); } } while (0)

__device__ __forceinline__ unsigned hash32(unsigned x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return x;
}
// a random finite value of moderate magnitude in [-2, 2)
__device__ __forceinline__ float rnd(unsigned s) {
  return (float)(int)(hash32(s) & 0xffffff) * (1.0f / 4194304.0f) - 2.0f;
}

template <int MODE, int WMT, int WNT, bool LDS>
__global__ __launch_bounds__(512, 1) void ceiling_kernel(int iters, float* out,
                                                         unsigned long long* stamps) {
  constexpr int NPL = MODE == 0 ? 3 : (MODE == 1 ? 2 : 1);
  __shared__ __attribute__((aligned(16))) unsigned short lds[2][NPL][WMT + WNT][64 * 8];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const unsigned seed = blockIdx.x * 1000003u + threadIdx.x * 7919u;
  // operand fragments: planes of random values (hi / mid / lo magnitudes)
  bf16x8 ab[WMT + WNT][NPL];
  f16x8 ah[WMT + WNT][NPL];
#pragma unroll
  for (int f = 0; f < WMT + WNT; ++f)
#pragma unroll
    for (int p = 0; p < NPL; ++p)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float v = rnd(seed + 131u * (f * 8 + p) + j) * (p == 0 ? 1.f : p == 1 ? 0x1p-9f : 0x1p-18f);
        ab[f][p][j] = (__bf16)v;
        ah[f][p][j] = (_Float16)v;
      }
  if (LDS) {
#pragma unroll
    for (int f = 0; f < WMT + WNT; ++f)
#pragma unroll
      for (int p = 0; p < NPL; ++p) {
        if (wave == 0) {
          if (MODE == 1) *reinterpret_cast<f16x8*>(&lds[0][p][f][lane * 8]) = ah[f][p];
          else *reinterpret_cast<bf16x8*>(&lds[0][p][f][lane * 8]) = ab[f][p];
        }
        if (wave == 1) {
          if (MODE == 1) *reinterpret_cast<f16x8*>(&lds[1][p][f][lane * 8]) = ah[f][p];
          else *reinterpret_cast<bf16x8*>(&lds[1][p][f][lane * 8]) = ab[f][p];
        }
      }
    __syncthreads();
  }
  f32x4 acc[WMT][WNT];
#pragma unroll
  for (int i = 0; i < WMT; ++i)
#pragma unroll
    for (int j = 0; j < WNT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  unsigned long long c0 = 0, r0 = 0;
  if (threadIdx.x == 0) { c0 = __builtin_amdgcn_s_memtime(); r0 = __builtin_amdgcn_s_memrealtime(); }
  for (int it = 0; it < iters; ++it) {
    if (LDS) {
      asm volatile("" ::: "memory");   // re-read every k-step (no hoisting)
      const int b = it & 1;
#pragma unroll
      for (int f = 0; f < WMT + WNT; ++f)
#pragma unroll
        for (int p = 0; p < NPL; ++p) {
          if (MODE == 1) ah[f][p] = *reinterpret_cast<const f16x8*>(&lds[b][p][f][lane * 8]);
          else ab[f][p] = *reinterpret_cast<const bf16x8*>(&lds[b][p][f][lane * 8]);
        }
    }
#pragma unroll
    for (int j = 0; j < WNT; ++j)
#pragma unroll
      for (int i = 0; i < WMT; ++i) {
        f32x4 c = acc[i][j];
        if constexpr (MODE == 0) {
          const bf16x8* a = ab[i];
          const bf16x8* bb = ab[WMT + j];
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], bb[1], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[2], bb[0], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], bb[2], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], bb[0], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], bb[1], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], bb[0], c, 0, 0, 0);
        } else if constexpr (MODE == 1) {
          const f16x8* a = ah[i];
          const f16x8* bb = ah[WMT + j];
          c = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[1], bb[0], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[0], bb[1], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[0], bb[0], c, 0, 0, 0);
        } else {
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ab[i][0], ab[WMT + j][0], c, 0, 0, 0);
        }
        acc[i][j] = c;
      }
  }
  if (threadIdx.x == 0) {
    const unsigned long long c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    stamps[blockIdx.x * 2] = c1 - c0;
    stamps[blockIdx.x * 2 + 1] = r1 - r0;
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < WMT; ++i)
#pragma unroll
    for (int j = 0; j < WNT; ++j) s += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
  out[blockIdx.x * 512 + threadIdx.x] = s;
}

template <int MODE, int WMT, int WNT, bool LDS>
void run(const char* name, double seconds, int cus) {
  const int iters = 2000;
  float* out;
  unsigned long long* st;
  CHECK(hipMalloc(&out, (size_t)cus * 512 * 4));
  CHECK(hipMalloc(&st, (size_t)cus * 16));
  auto k = ceiling_kernel<MODE, WMT, WNT, LDS>;
  // one workgroup per CU: pad the LDS footprint past half the CU's 160 KB
  hipFuncAttributes fa;
  CHECK(hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(k)));
  const size_t pad = fa.sharedSizeBytes >= 84 * 1024 ? 0 : 84 * 1024 - fa.sharedSizeBytes;
  CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(k),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)pad));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  // warm-up until the clock settles (>= 1 s), then time back-to-back launches
  float ms = 0.f;
  int launches = 0;
  for (int phase = 0; phase < 2; ++phase) {
    CHECK(hipEventRecord(e0));
    launches = 0;
    do {
      for (int r = 0; r < 10; ++r) hipLaunchKernelGGL(k, dim3(cus), dim3(512), pad, 0, iters, out, st);
      launches += 10;
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      CHECK(hipEventElapsedTime(&ms, e0, e1));
    } while (ms < (phase == 0 ? 1000.0 : seconds * 1000.0));
  }
  std::vector<unsigned long long> h(cus * 2);
  CHECK(hipMemcpy(h.data(), st, cus * 16, hipMemcpyDeviceToHost));
  std::vector<double> clk(cus);
  for (int i = 0; i < cus; ++i) clk[i] = (double)h[2 * i] / (double)h[2 * i + 1] * 100.0;   // MHz
  std::sort(clk.begin(), clk.end());
  constexpr int per_pair = MODE == 0 ? 6 : (MODE == 1 ? 3 : 1);
  const double mfma = (double)launches * cus * 8 * iters * WMT * WNT * per_pair;
  const double flop = mfma * 16 * 16 * 32 * 2;
  const double tf = flop / (ms * 1e-3) / 1e12;
  const double useful = tf / per_pair;   // fp32-equivalent (x6, h3) or bf16 (b1)
  printf("{\"probe\": \"%s\", \"mode\": \"%s\", \"wave_tile\": [%d, %d], \"lds_reads\": %s, "
         "\"mfma_tflops\": %.1f, \"useful_tflops\": %.1f, \"clock_mhz_median\": %.0f, "
         "\"clock_mhz_min\": %.0f, \"ms\": %.1f, \"launches\": %d}\n",
         name, MODE == 0 ? "x6" : (MODE == 1 ? "h3" : "b1"), WMT, WNT, LDS ? "true" : "false",
         tf, useful, clk[cus / 2], clk[0], ms, launches);
  fflush(stdout);
  CHECK(hipFree(out));
  CHECK(hipFree(st));
}

int main(int argc, char** argv) {
  const double sec = argc > 1 ? atof(argv[1]) : 2.0;
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  const int cus = p.multiProcessorCount;
  run<0, 4, 4, false>("x6 regs 4x4 (TBN 128)", sec, cus);
  run<0, 4, 4, true>("x6 lds 4x4 (TBN 128)", sec, cus);
  run<0, 2, 10, false>("x6 regs 2x10 (TBN 160)", sec, cus);
  run<0, 2, 10, true>("x6 lds 2x10 (TBN 160)", sec, cus);
  run<1, 4, 4, false>("h3 regs 4x4", sec, cus);
  run<1, 4, 4, true>("h3 lds 4x4", sec, cus);
  run<1, 2, 10, true>("h3 lds 2x10", sec, cus);
  run<2, 4, 4, false>("b1 regs 4x4", sec, cus);
  return 0;
}
