// Which SIMD does wave w of a workgroup land on?  The common-mode kernel's median phases keep 3
// of its 4 waves busy (176 row segments, 48 columns x 4 lanes); if wave 3 of every 256-thread
// workgroup sits on the same SIMD of its CU, a quarter of the CU's VALU issue slots idle through
// the medians.  Same launch shape as the production kernel (256 threads, 40 KiB dynamic LDS,
// 8192 workgroups); each wave records its HW_ID (SIMD_ID bits 5:4, CU_ID 11:8, SE_ID 15:13).
//   hipcc -O3 --offload-arch=gfx950 tools/simd_probe.hip -o simd_probe && ./simd_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <map>
#include <vector>

__global__ __launch_bounds__(256) void probe_kernel(unsigned* out, int spin) {
  extern __shared__ float lds[];
  const unsigned hw = __builtin_amdgcn_s_getreg(4 | (31 << 11));
  lds[threadIdx.x] = (float)threadIdx.x;
  float acc = lds[(threadIdx.x + 1) & 255];
  for (int i = 0; i < spin; ++i) acc = acc * 1.0001f + 0.5f;   // keep the workgroup resident a while
  if ((threadIdx.x & 63) == 0) out[blockIdx.x * 4 + (threadIdx.x >> 6)] = hw ^ (acc == -1.0f ? 1u : 0u);
}

int main() {
  const int nwg = 8192;
  unsigned* d = nullptr;
  if (hipMalloc(&d, nwg * 4 * sizeof(unsigned)) != hipSuccess) return 1;
  (void)hipFuncSetAttribute((const void*)probe_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 40 * 1024);
  hipLaunchKernelGGL(probe_kernel, dim3(nwg), dim3(256), 40 * 1024, 0, d, 20000);
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  std::vector<unsigned> h(nwg * 4);
  (void)hipMemcpy(h.data(), d, h.size() * sizeof(unsigned), hipMemcpyDeviceToHost);
  int hist[4][4] = {};
  std::map<int, int> rel;   // (simd(w) - simd(0)) pattern of a workgroup
  int same_cu = 0;
  for (int b = 0; b < nwg; ++b) {
    int pat = 0;
    const unsigned s0 = (h[b * 4] >> 4) & 3;
    bool cu_same = true;
    for (int w = 0; w < 4; ++w) {
      const unsigned hw = h[b * 4 + w];
      const unsigned s = (hw >> 4) & 3;
      hist[w][s]++;
      pat = pat * 4 + (int)((s - s0) & 3);
      cu_same &= ((hw >> 8) & 0xF) == ((h[b * 4] >> 8) & 0xF) && ((hw >> 13) & 7) == ((h[b * 4] >> 13) & 7);
    }
    rel[pat]++;
    same_cu += cu_same;
  }
  printf("{\"workgroups\": %d, \"waves_on_one_cu\": %d, \"wave_simd_hist\": [", nwg, same_cu);
  for (int w = 0; w < 4; ++w)
    printf("%s[%d, %d, %d, %d]", w ? ", " : "", hist[w][0], hist[w][1], hist[w][2], hist[w][3]);
  printf("], \"relative_patterns\": {");
  bool first = true;
  for (auto& kv : rel) {
    printf("%s\"%d%d%d%d\": %d", first ? "" : ", ", (kv.first >> 6) & 3, (kv.first >> 4) & 3, (kv.first >> 2) & 3,
           kv.first & 3, kv.second);
    first = false;
  }
  printf("}}\n");
  (void)hipFree(d);
  return 0;
}
