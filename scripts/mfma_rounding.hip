// MFMA accumulation rounding probe: how the fp32 result of one MFMA is rounded when the
// exact value C + sum(a b) is not representable, for the instructions the fp32-accurate
// split kernels use (f16 / bf16 16x16x32, 32x32x16) and the fp32 one (16x16x4f32).
// Case "tie+": C = 2^24, products sum to 1.5 (exact 2^24 + 1.5): RNE 2^24 + 2, RZ / RD 2^24.
// Case "tie-": the same negated: RNE -(2^24 + 2), RZ / RU -2^24.
// Case "sum": C = 0, products 2^24, 1, 1 in one instruction: exact 2^24 + 2 (one rounding of
// the exact sum) vs 2^24 (sequential fp32 adds, each tie to even).
// build: hipcc -O3 --offload-arch=gfx950 -o scripts/mfma_rounding scripts/mfma_rounding.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

// lane 0..15 hold row i = lane, k = 0..7 (16x16x32: k = 8 (lane / 16) + j); products placed at
// k = 0, 1, 2 of row/column 0 only
__global__ void probe(float* out) {
  const int lane = threadIdx.x;
  const int cases = 3;
  for (int cs = 0; cs < cases; ++cs) {
    float pa[3] = {0.f, 0.f, 0.f}, c0 = 0.f;
    if (cs == 0) { pa[0] = 1.5f; c0 = 16777216.f; }
    if (cs == 1) { pa[0] = -1.5f; c0 = -16777216.f; }
    if (cs == 2) { pa[0] = 16777216.f; pa[1] = 1.f; pa[2] = 1.f; c0 = 0.f; }
    // f16 16x16x32: a = value (f16 holds 2^24? no: max 65504) -> use a = v / 2^12, b = 2^12
    {
      f16x8 a = {}, b = {};
      if (lane == 0)
        for (int j = 0; j < 3; ++j) { a[j] = (_Float16)(pa[j] / 4096.f); b[j] = (_Float16)4096.f; }
      f32x4 c = {c0, c0, c0, c0};
      c = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
      if (lane == 0) out[cs * 8 + 0] = c[0];
    }
    {
      bf16x8 a = {}, b = {};
      if (lane == 0)
        for (int j = 0; j < 3; ++j) { a[j] = (__bf16)(pa[j] / 4096.f); b[j] = (__bf16)4096.f; }
      f32x4 c = {c0, c0, c0, c0};
      c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
      if (lane == 0) out[cs * 8 + 1] = c[0];
    }
    {
      // 32x32x16 bf16: lane L holds row L % 32, k = 8 (L / 32) + j
      bf16x8 a = {}, b = {};
      if (lane == 0)
        for (int j = 0; j < 3; ++j) { a[j] = (__bf16)(pa[j] / 4096.f); b[j] = (__bf16)4096.f; }
      f32x16 c;
      for (int r = 0; r < 16; ++r) c[r] = c0;
      c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
      if (lane == 0) out[cs * 8 + 2] = c[0];
    }
    {
      f16x8 a = {}, b = {};
      if (lane == 0)
        for (int j = 0; j < 3; ++j) { a[j] = (_Float16)(pa[j] / 4096.f); b[j] = (_Float16)4096.f; }
      f32x16 c;
      for (int r = 0; r < 16; ++r) c[r] = c0;
      c = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
      if (lane == 0) out[cs * 8 + 3] = c[0];
    }
    {
      // 16x16x4 f32: lane L holds row L % 16, k = L / 16: three MFMAs, one product each
      // (k = 0 only), so this is three sequential accumulations
      f32x4 c = {c0, c0, c0, c0};
      for (int j = 0; j < 3; ++j) {
        const float a = lane == 0 ? pa[j] : 0.f, b = lane == 0 ? 1.f : 0.f;
        c = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
      }
      if (lane == 0) out[cs * 8 + 4] = c[0];
    }
  }
}

// Width of the exact window: C = 2^20 (even lsb, ulp 2^-3) or 2^20 + 2^-3 (odd lsb); products
// {2^-4 (half an ulp: a tie), +-2^(-4-d)} in ONE instruction.  T1 (C even, +tiny): exact
// rounds UP (+2^-3); tiny dropped -> tie -> even (+0).  T2 (C odd, -tiny): exact rounds DOWN
// (+2^-3 kept); tiny dropped toward zero -> tie -> even (+2^-2); floor-truncated -> down (+2^-3).
__global__ void window(float* out) {
  const int lane = threadIdx.x;
  for (int d = 0; d < 8; ++d) {
    const int dd = 2 + 3 * d;                         // tiny = 2^(-4 - dd)
    const float tiny = ldexpf(1.f, -4 - dd);
    for (int t = 0; t < 2; ++t) {
      const float c0 = t == 0 ? 1048576.f : 1048576.f + 0.125f;
      const float p1 = t == 0 ? tiny : -tiny;
      {
        f16x8 a = {}, b = {};
        if (lane == 0) {
          a[0] = (_Float16)0.25f; b[0] = (_Float16)0.25f;                 // 2^-4
          a[1] = (_Float16)ldexpf(p1, (4 + dd) / 2); b[1] = (_Float16)ldexpf(1.f, -(4 + dd) + (4 + dd) / 2);
        }
        f32x4 c = {c0, c0, c0, c0};
        c = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
        if (lane == 0) out[(d * 2 + t) * 4 + 0] = c[0] - 1048576.f;
      }
      {
        bf16x8 a = {}, b = {};
        if (lane == 0) {
          a[0] = (__bf16)0.25f; b[0] = (__bf16)0.25f;
          a[1] = (__bf16)p1; b[1] = (__bf16)1.f;
        }
        f32x4 c = {c0, c0, c0, c0};
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
        if (lane == 0) out[(d * 2 + t) * 4 + 1] = c[0] - 1048576.f;
      }
      {
        bf16x8 a = {}, b = {};
        if (lane == 0) {
          a[0] = (__bf16)0.25f; b[0] = (__bf16)0.25f;
          a[1] = (__bf16)p1; b[1] = (__bf16)1.f;
        }
        f32x16 c;
        for (int r = 0; r < 16; ++r) c[r] = c0;
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
        if (lane == 0) out[(d * 2 + t) * 4 + 2] = c[0] - 1048576.f;
      }
      {
        f16x8 a = {}, b = {};
        if (lane == 0) {
          a[0] = (_Float16)0.25f; b[0] = (_Float16)0.25f;
          a[1] = (_Float16)ldexpf(p1, (4 + dd) / 2); b[1] = (_Float16)ldexpf(1.f, -(4 + dd) + (4 + dd) / 2);
        }
        f32x16 c;
        for (int r = 0; r < 16; ++r) c[r] = c0;
        c = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
        if (lane == 0) out[(d * 2 + t) * 4 + 3] = c[0] - 1048576.f;
      }
    }
  }
}

// Conversion rounding of the split code's packed converts (v_cvt_pk_f16_f32 /
// v_cvt_pk_bf16_f32 via __builtin_convertvector) and the scalar casts: x = 1 + 0.75 ulp
// (RNE: up, RZ / RD: down) and its negation, for fp16 (ulp 2^-10 at 1) and bf16 (ulp 2^-7)
typedef float cvf2 __attribute__((ext_vector_type(2)));
typedef _Float16 cvh2 __attribute__((ext_vector_type(2)));
typedef __bf16 cvb2 __attribute__((ext_vector_type(2)));
__global__ void convs(const float* in, float* out) {
  if (threadIdx.x != 0) return;
  const float xh = in[0], xb = in[1];
  const cvh2 ph = __builtin_convertvector(cvf2{xh, -xh}, cvh2);
  const cvb2 pb = __builtin_convertvector(cvf2{xb, -xb}, cvb2);
  out[0] = (float)ph[0]; out[1] = (float)ph[1];
  out[2] = (float)pb[0]; out[3] = (float)pb[1];
  out[4] = (float)(_Float16)xh; out[5] = (float)(_Float16)(-xh);
  out[6] = (float)(__bf16)xb; out[7] = (float)(__bf16)(-xb);
}

int main() {
  float* d;
  hipMalloc(&d, 64 * sizeof(float));
  hipMemset(d, 0, 64 * sizeof(float));
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d);
  float h[64];
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  const char* names[5] = {"f16 16x16x32", "bf16 16x16x32", "bf16 32x32x16", "f16 32x32x16",
                          "f32 16x16x4 (3 MFMAs)"};
  const char* cases[3] = {"tie+ (2^24 + 1.5: RNE +2, RZ +0)", "tie- (-(2^24 + 1.5): RNE -2, RZ -0)",
                          "sum (2^24 + 1 + 1 in one MFMA: exact +2, sequential +0)"};
  for (int cs = 0; cs < 3; ++cs)
    for (int i = 0; i < 5; ++i) {
      const double base = cs == 1 ? -16777216.0 : 16777216.0;
      printf("{\"instr\": \"%s\", \"case\": \"%s\", \"result_minus_2^24\": %.1f}\n", names[i],
             cases[cs], (double)h[cs * 8 + i] - base);
    }
  float* w;
  hipMalloc(&w, 128 * sizeof(float));
  hipMemset(w, 0, 128 * sizeof(float));
  hipLaunchKernelGGL(window, dim3(1), dim3(64), 0, 0, w);
  float hw[128];
  hipMemcpy(hw, w, sizeof(hw), hipMemcpyDeviceToHost);
  const char* wn[4] = {"f16 16x16x32", "bf16 16x16x32", "bf16 32x32x16", "f16 32x32x16"};
  for (int dd = 0; dd < 8; ++dd)
    for (int i = 0; i < 4; ++i)
      printf("{\"instr\": \"%s\", \"tiny_rel_to_C\": \"2^-%d\", \"T1_even_plus\": %.4f, "
             "\"T2_odd_minus\": %.4f}\n", wn[i], 24 + 2 + 3 * dd, (double)hw[(dd * 2) * 4 + i],
             (double)hw[(dd * 2 + 1) * 4 + i]);
  printf("T1: 0.125 = tiny kept (exact RNE), 0 = tiny dropped; T2: 0.125 = exact or floor, "
         "0.25 = tiny dropped toward zero\n");
  hipFree(w);
  {
    float hin[2] = {1.f + 0.75f * 0x1p-10f, 1.f + 0.75f * 0x1p-7f}, *din, *dout, hout[8];
    hipMalloc(&din, sizeof(hin));
    hipMalloc(&dout, sizeof(hout));
    hipMemcpy(din, hin, sizeof(hin), hipMemcpyHostToDevice);
    hipLaunchKernelGGL(convs, dim3(1), dim3(64), 0, 0, din, dout);
    hipMemcpy(hout, dout, sizeof(hout), hipMemcpyDeviceToHost);
    const char* cn[8] = {"pk f16 +", "pk f16 -", "pk bf16 +", "pk bf16 -", "cast f16 +",
                         "cast f16 -", "cast bf16 +", "cast bf16 -"};
    for (int i = 0; i < 8; ++i) {
      const double ulp = i % 4 < 2 ? 0x1p-10 : 0x1p-7;
      const double got = (i & 1) ? -(double)hout[i] : (double)hout[i];
      printf("{\"convert\": \"%s\", \"|result| - 1 in ulps\": %.2f, \"RNE\": 1, \"RZ\": 0}\n",
             cn[i], (got - 1.0) / ulp);
    }
    hipFree(din);
    hipFree(dout);
  }
  hipFree(d);
  return 0;
}
