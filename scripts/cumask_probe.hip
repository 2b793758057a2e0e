// Probe: which (XCC, SE, CU) a kernel's workgroups land on under hipExtStreamCreateWithCUMask
// masks -- to learn how mask bits map to XCDs before restricting a side stream to the CUs a
// persistent recurrence leaves idle.  Build: hipcc --offload-arch=gfx950 -O2 cumask_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <set>
#include <vector>

__global__ void where(unsigned* out, int spin) {
  if (threadIdx.x == 0) {
    const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_REG_HW_ID
    const unsigned xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // HW_REG_XCC_ID
    out[blockIdx.x] = ((xcc & 0xf) << 16) | (hw & 0xffff);
    // keep the workgroup resident a little so the grid spreads over the CUs
    const long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < spin) {}
  }
}

static void run(const char* name, hipStream_t st, int grid) {
  unsigned* d = nullptr;
  hipMalloc(&d, grid * 4);
  hipLaunchKernelGGL(where, dim3(grid), dim3(64), 0, st, d, 2000);
  hipStreamSynchronize(st);
  std::vector<unsigned> h(grid);
  hipMemcpy(h.data(), d, grid * 4, hipMemcpyDeviceToHost);
  hipFree(d);
  std::set<unsigned> cus;
  int per_xcc[8] = {0};
  std::set<unsigned> xcc_cus[8];
  for (unsigned v : h) {
    const unsigned xcc = v >> 16, cu = (v >> 8) & 0xf, sh = (v >> 12) & 1, se = (v >> 13) & 7;
    const unsigned key = (xcc << 8) | (se << 5) | (sh << 4) | cu;
    cus.insert(key);
    if (xcc < 8) xcc_cus[xcc].insert(key);
  }
  for (int x = 0; x < 8; ++x) per_xcc[x] = (int)xcc_cus[x].size();
  printf("%-34s distinct CUs %3zu | per XCC:", name, cus.size());
  for (int x = 0; x < 8; ++x) printf(" %2d", per_xcc[x]);
  printf(" | wg0..15 xcc:");
  for (int i = 0; i < 16 && i < grid; ++i) printf(" %u", h[i] >> 16);
  printf("\n");
}

int main() {
  int ncu = 0;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  printf("CUs %d\n", ncu);
  run("default stream", 0, 4096);
  const int words = (ncu + 31) / 32;
  auto mk = [&](const char* name, auto pred) {
    std::vector<uint32_t> m(words, 0);
    int n = 0;
    for (int i = 0; i < ncu; ++i)
      if (pred(i)) { m[i / 32] |= 1u << (i % 32); ++n; }
    hipStream_t st;
    if (hipExtStreamCreateWithCUMask(&st, words, m.data()) != hipSuccess) {
      printf("%s: create failed\n", name);
      return;
    }
    char buf[96];
    snprintf(buf, sizeof buf, "%s (%d bits)", name, n);
    run(buf, st, 4096);
    hipStreamDestroy(st);
  };
  mk("bits 0..199", [](int i) { return i < 200; });
  mk("bits 200..255", [](int i) { return i >= 200; });
  mk("i % 32 < 25", [](int i) { return i % 32 < 25; });
  mk("i % 32 >= 25", [](int i) { return i % 32 >= 25; });
  mk("i / 8 < 25", [](int i) { return i / 8 < 25; });
  mk("bits 0..31", [](int i) { return i < 32; });
  mk("even bits", [](int i) { return i % 2 == 0; });
  return 0;
}
