// VALU issue rate of one SIMD with 1..8 resident waves (the common-mode kernel's bound).
//
// Every wave runs ITERS x 16 independent v_maximum3_f32-class ops (8 independent chains of
// min/max pairs, the median networks' instruction mix) or v_fma_f32; the grid is one workgroup of
// W waves per CU (W / 4 waves per SIMD), so kernel time / (instructions per SIMD) = cycles per
// wave64 VALU at the SIMD level.  Prints, per (waves per SIMD, op): us, and the shader clock from
// s_memtime over the kernel so cycles are in the chip's actual clock.
//   hipcc -O3 --offload-arch=gfx950 tools/valu_rate.hip -o /tmp/valu_rate && /tmp/valu_rate
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#define PR_V16(OPS)                                                                               \
  asm volatile(OPS " %0, %0, %16, %0\n\t" OPS " %1, %1, %16, %1\n\t" OPS " %2, %2, %16, %2\n\t" OPS \
               " %3, %3, %16, %3\n\t" OPS " %4, %4, %16, %4\n\t" OPS " %5, %5, %16, %5\n\t" OPS         \
               " %6, %6, %16, %6\n\t" OPS " %7, %7, %16, %7\n\t" OPS " %8, %8, %16, %8\n\t" OPS         \
               " %9, %9, %16, %9\n\t" OPS " %10, %10, %16, %10\n\t" OPS " %11, %11, %16, %11\n\t" OPS   \
               " %12, %12, %16, %12\n\t" OPS " %13, %13, %16, %13\n\t" OPS " %14, %14, %16, %14\n\t" OPS \
               " %15, %15, %16, %15"                                                                       \
               : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]),        \
                 "+v"(r[7]), "+v"(r[8]), "+v"(r[9]), "+v"(r[10]), "+v"(r[11]), "+v"(r[12]), "+v"(r[13]),    \
                 "+v"(r[14]), "+v"(r[15])                                                                   \
               : "v"(k))

// OP 0: v_maximum3_f32 (the networks' comparator half), 1: v_fma_f32; 16 independent chains, exactly
// 16 VALU per iteration (inline asm: no compiler moves)
template <int OP>
__global__ void valu_kernel(float* out, unsigned long long* clk, int iters) {
  float r[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) r[q] = (float)threadIdx.x * 1e-3f + q;
  const float k = 0.5f + (float)(threadIdx.x & 1);
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
    if constexpr (OP == 0) PR_V16("v_maximum3_f32");
    else PR_V16("v_fma_f32");
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float z = 0.f;
#pragma unroll
  for (int q = 0; q < 16; ++q) z += r[q];
  if (z == -12345.f) out[threadIdx.x] = z;
  if (threadIdx.x == 0 && blockIdx.x == 0) clk[0] = t1 - t0;
}

int main() {
  int dev = 0, cus = 0;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  float* out = nullptr;
  unsigned long long* clk = nullptr;
  (void)hipMalloc(&out, 4096 * sizeof(float));
  (void)hipMalloc(&clk, sizeof(unsigned long long));
  const int iters = 4000;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int op = 0; op < 2; ++op) {
    for (int wps : {1, 2, 3, 4, 6, 8}) {
      const int threads = 64 * 4 * wps;   // one workgroup per CU, wps waves per SIMD
      auto k = op == 0 ? valu_kernel<0> : valu_kernel<1>;
      std::vector<float> ts;
      unsigned long long c = 0;
      for (int r = 0; r < 5; ++r) {
        (void)hipEventRecord(e0, 0);
        hipLaunchKernelGGL(k, dim3(cus), dim3(threads), 0, 0, out, clk, iters);
        (void)hipEventRecord(e1, 0);
        (void)hipEventSynchronize(e1);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        ts.push_back(ms);
        (void)hipMemcpy(&c, clk, sizeof(c), hipMemcpyDeviceToHost);
      }
      std::sort(ts.begin(), ts.end());
      const double us = ts[2] * 1e3;
      const double instr_per_wave = (double)iters * 16;   // 16 VALU per iteration
      const double sclk_ghz = (double)c / (us * 1e3);     // shader cycles of wave 0 / wall us (approx)
      const double cyc_per_simd_instr = (us * 1e3 * sclk_ghz) / (instr_per_wave * wps);
      printf("{\"op\": \"%s\", \"waves_per_simd\": %d, \"us\": %.1f, \"sclk_ghz\": %.3f, \"cycles_per_wave_instr_at_simd\": %.2f}\n",
             op == 0 ? "maximum3" : "fma", wps, us, sclk_ghz, cyc_per_simd_instr);
    }
  }
  return 0;
}
