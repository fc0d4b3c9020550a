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
#include <cstdlib>
#include <cstdio>
#include <vector>

// 16 independent chains of one instruction form: "%r" is the chain register, "%k" a constant VGPR
#define PR_CHAIN(FMT) FMT
#define PR_ASM16(T)                                                                                     \
  asm volatile(T(0) "\n\t" T(1) "\n\t" T(2) "\n\t" T(3) "\n\t" T(4) "\n\t" T(5) "\n\t" T(6) "\n\t" T(7)  \
               "\n\t" T(8) "\n\t" T(9) "\n\t" T(10) "\n\t" T(11) "\n\t" T(12) "\n\t" T(13) "\n\t" T(14)  \
               "\n\t" T(15)                                                                             \
               : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]),    \
                 "+v"(r[7]), "+v"(r[8]), "+v"(r[9]), "+v"(r[10]), "+v"(r[11]), "+v"(r[12]), "+v"(r[13]), \
                 "+v"(r[14]), "+v"(r[15])                                                               \
               : "v"(k), "s"(ks), "s"(km))
#define S_(x) #x
#define R_(i) "%" S_(i)
#define T_MAXIMUM3(i) "v_maximum3_f32 " R_(i) ", " R_(i) ", %16, " R_(i)
#define T_MAX3(i) "v_max3_f32 " R_(i) ", " R_(i) ", %16, " R_(i)
#define T_MAX_E32(i) "v_max_f32_e32 " R_(i) ", %16, " R_(i)
#define T_MAX_E64(i) "v_max_f32_e64 " R_(i) ", " R_(i) ", %16"
#define T_FMA(i) "v_fma_f32 " R_(i) ", " R_(i) ", %16, " R_(i)
#define T_ADD(i) "v_add_f32_e32 " R_(i) ", %16, " R_(i)
#define T_MED3(i) "v_med3_f32 " R_(i) ", " R_(i) ", %16, " R_(i)
#define T_MINIMUM3(i) "v_minimum3_f32 " R_(i) ", " R_(i) ", %16, " R_(i)
#define T_BFI(i) "v_bfi_b32 " R_(i) ", " R_(i) ", %16, " R_(i)
#define T_PKMAX16(i) "v_pk_max_f16 " R_(i) ", " R_(i) ", %16"
#define T_CVT(i) "v_cvt_f32_u32 " R_(i) ", " R_(i)
#define T_BFE(i) "v_bfe_u32 " R_(i) ", " R_(i) ", 3, 14"
#define T_ANDOR(i) "v_and_or_b32 " R_(i) ", " R_(i) ", %16, " R_(i)
#define T_CNDMASK(i) "v_cndmask_b32 " R_(i) ", " R_(i) ", %16, vcc"
#define T_MUL(i) "v_mul_f32 " R_(i) ", %16, " R_(i)
#define T_MOV(i) "v_mov_b32 " R_(i) ", %16"
#define T_XOR(i) "v_xor_b32 " R_(i) ", %16, " R_(i)
#define T_SUB(i) "v_sub_f32 " R_(i) ", %16, " R_(i)
#define T_PERM(i) "v_perm_b32 " R_(i) ", " R_(i) ", %16, %16"
#define T_MAXDPP(i) "v_max_f32_dpp " R_(i) ", %16, " R_(i) " quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf"
#define T_MAXI32(i) "v_max_i32 " R_(i) ", %16, " R_(i)
#define T_MINU32(i) "v_min_u32 " R_(i) ", %16, " R_(i)
#define T_MAX3I32(i) "v_max3_i32 " R_(i) ", " R_(i) ", %16, " R_(i)
#define T_MED3I32(i) "v_med3_i32 " R_(i) ", " R_(i) ", %16, " R_(i)
#define T_ADDU32(i) "v_add_u32 " R_(i) ", %16, " R_(i)
#define T_PKMAXI16(i) "v_pk_max_i16 " R_(i) ", " R_(i) ", %16"
#define T_MINF32(i) "v_min_f32_e32 " R_(i) ", %16, " R_(i)
#define T_CND64(i) "v_cndmask_b32_e64 " R_(i) ", " R_(i) ", %16, %18"
#define T_MAXS(i) "v_max_f32_e64 " R_(i) ", " R_(i) ", %17"
#define T_ADDS(i) "v_add_f32_e64 " R_(i) ", " R_(i) ", %17"
#define T_CMPCND(i) "v_cmp_lt_f32_e64 s[40:41], " R_(i) ", %16\n\tv_cndmask_b32_e64 " R_(i) ", " R_(i) ", %16, s[40:41]"

constexpr int kOps = 31;
static const char* kOpNames[kOps] = {"v_maximum3_f32", "v_minimum3_f32", "v_max3_f32", "v_med3_f32", "v_max_f32_e32",
                                     "v_max_f32_e64", "v_max_f32_dpp", "v_fma_f32", "v_add_f32", "v_bfi_b32",
                                     "v_pk_max_f16", "v_cvt_f32_u32", "v_bfe_u32", "v_and_or_b32", "v_cndmask_b32",
                                     "v_mul_f32", "v_mov_b32", "v_xor_b32", "v_sub_f32", "v_perm_b32",
                                     "v_max_i32", "v_min_u32", "v_max3_i32", "v_med3_i32", "v_add_u32",
                                     "v_pk_max_i16", "v_min_f32_e32", "v_cndmask_b32_e64_sgpr_mask",
                                     "v_max_f32_e64_sgpr_operand", "v_add_f32_e64_sgpr_operand",
                                     "v_cmp_lt_f32+v_cndmask (pair, per 2 instr)"};

template <int OP>
__global__ void valu_kernel(float* out, unsigned long long* clk, int iters) {
  float r[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) r[q] = (float)threadIdx.x * 1e-3f + q;
  const float k = 0.5f + (float)(threadIdx.x & 1);
  // wave-uniform operands for the SGPR-operand forms
  const float ks = __builtin_amdgcn_readfirstlane(__float_as_int(k)) == 0 ? 1.0f : 0.75f;
  const unsigned long long km = (unsigned long long)__builtin_amdgcn_read_exec() & 0x5555555555555555ull;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
    if constexpr (OP == 0) PR_ASM16(T_MAXIMUM3);
    else if constexpr (OP == 1) PR_ASM16(T_MINIMUM3);
    else if constexpr (OP == 2) PR_ASM16(T_MAX3);
    else if constexpr (OP == 3) PR_ASM16(T_MED3);
    else if constexpr (OP == 4) PR_ASM16(T_MAX_E32);
    else if constexpr (OP == 5) PR_ASM16(T_MAX_E64);
    else if constexpr (OP == 6) PR_ASM16(T_MAXDPP);
    else if constexpr (OP == 7) PR_ASM16(T_FMA);
    else if constexpr (OP == 8) PR_ASM16(T_ADD);
    else if constexpr (OP == 9) PR_ASM16(T_BFI);
    else if constexpr (OP == 10) PR_ASM16(T_PKMAX16);
    else if constexpr (OP == 11) PR_ASM16(T_CVT);
    else if constexpr (OP == 12) PR_ASM16(T_BFE);
    else if constexpr (OP == 13) PR_ASM16(T_ANDOR);
    else if constexpr (OP == 14) PR_ASM16(T_CNDMASK);
    else if constexpr (OP == 15) PR_ASM16(T_MUL);
    else if constexpr (OP == 16) PR_ASM16(T_MOV);
    else if constexpr (OP == 17) PR_ASM16(T_XOR);
    else if constexpr (OP == 18) PR_ASM16(T_SUB);
    else if constexpr (OP == 19) PR_ASM16(T_PERM);
    else if constexpr (OP == 20) PR_ASM16(T_MAXI32);
    else if constexpr (OP == 21) PR_ASM16(T_MINU32);
    else if constexpr (OP == 22) PR_ASM16(T_MAX3I32);
    else if constexpr (OP == 23) PR_ASM16(T_MED3I32);
    else if constexpr (OP == 24) PR_ASM16(T_ADDU32);
    else if constexpr (OP == 25) PR_ASM16(T_PKMAXI16);
    else if constexpr (OP == 26) PR_ASM16(T_MINF32);
    else if constexpr (OP == 27) PR_ASM16(T_CND64);
    else if constexpr (OP == 28) PR_ASM16(T_MAXS);
    else if constexpr (OP == 29) PR_ASM16(T_ADDS);
    else PR_ASM16(T_CMPCND);
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float z = 0.f;
#pragma unroll
  for (int q = 0; q < 16; ++q) z += r[q];
  if (z == -12345.f) out[threadIdx.x] = z;
  if (threadIdx.x == 0 && blockIdx.x == 0) clk[0] = t1 - t0;
}

template <int OP>
static void run_op(int cus, float* out, unsigned long long* clk, int iters, hipEvent_t e0, hipEvent_t e1) {
  double us1 = 0;
  for (int wps : {1, 2, 3, 4}) {
    const int threads = 64 * 4 * wps;   // one workgroup per CU, wps waves per SIMD
    std::vector<float> ts;
    unsigned long long c = 0;
    for (int r = 0; r < 5; ++r) {
      (void)hipEventRecord(e0, 0);
      hipLaunchKernelGGL(valu_kernel<OP>, dim3(cus), dim3(threads), 0, 0, out, clk, iters);
      (void)hipEventRecord(e1, 0);
      (void)hipEventSynchronize(e1);
      float ms = 0;
      (void)hipEventElapsedTime(&ms, e0, e1);
      ts.push_back(ms);
      (void)hipMemcpy(&c, clk, sizeof(c), hipMemcpyDeviceToHost);
    }
    if (hipGetLastError() != hipSuccess) {
      printf("{\"op\": \"%s\", \"error\": true}\n", kOpNames[OP]);
      return;
    }
    std::sort(ts.begin(), ts.end());
    const double us = ts[2] * 1e3;
    if (wps == 1) us1 = us;
    // SIMD-level throughput relative to one wave alone: wps waves x the same work in `us`
    printf("{\"op\": \"%s\", \"waves_per_simd\": %d, \"us\": %.1f, \"wave0_cycles_per_instr\": %.2f, "
           "\"simd_throughput_vs_one_wave\": %.2f}\n",
           kOpNames[OP], wps, us, (double)c / ((double)iters * 16), wps * us1 / us);
  }
}

int main(int argc, char** argv) {
  const int first = argc > 1 ? atoi(argv[1]) : 0;   // run ops [first, kOps)
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
  if (0 >= first) run_op<0>(cus, out, clk, iters, e0, e1);
  if (1 >= first) run_op<1>(cus, out, clk, iters, e0, e1);
  if (2 >= first) run_op<2>(cus, out, clk, iters, e0, e1);
  if (3 >= first) run_op<3>(cus, out, clk, iters, e0, e1);
  if (4 >= first) run_op<4>(cus, out, clk, iters, e0, e1);
  if (5 >= first) run_op<5>(cus, out, clk, iters, e0, e1);
  if (6 >= first) run_op<6>(cus, out, clk, iters, e0, e1);
  if (7 >= first) run_op<7>(cus, out, clk, iters, e0, e1);
  if (8 >= first) run_op<8>(cus, out, clk, iters, e0, e1);
  if (9 >= first) run_op<9>(cus, out, clk, iters, e0, e1);
  if (10 >= first) run_op<10>(cus, out, clk, iters, e0, e1);
  if (11 >= first) run_op<11>(cus, out, clk, iters, e0, e1);
  if (12 >= first) run_op<12>(cus, out, clk, iters, e0, e1);
  if (13 >= first) run_op<13>(cus, out, clk, iters, e0, e1);
  if (14 >= first) run_op<14>(cus, out, clk, iters, e0, e1);
  if (15 >= first) run_op<15>(cus, out, clk, iters, e0, e1);
  if (16 >= first) run_op<16>(cus, out, clk, iters, e0, e1);
  if (17 >= first) run_op<17>(cus, out, clk, iters, e0, e1);
  if (18 >= first) run_op<18>(cus, out, clk, iters, e0, e1);
  if (19 >= first) run_op<19>(cus, out, clk, iters, e0, e1);
  if (20 >= first) run_op<20>(cus, out, clk, iters, e0, e1);
  if (21 >= first) run_op<21>(cus, out, clk, iters, e0, e1);
  if (22 >= first) run_op<22>(cus, out, clk, iters, e0, e1);
  if (23 >= first) run_op<23>(cus, out, clk, iters, e0, e1);
  if (24 >= first) run_op<24>(cus, out, clk, iters, e0, e1);
  if (25 >= first) run_op<25>(cus, out, clk, iters, e0, e1);
  if (26 >= first) run_op<26>(cus, out, clk, iters, e0, e1);
  if (27 >= first) run_op<27>(cus, out, clk, iters, e0, e1);
  if (28 >= first) run_op<28>(cus, out, clk, iters, e0, e1);
  if (29 >= first) run_op<29>(cus, out, clk, iters, e0, e1);
  if (30 >= first) run_op<30>(cus, out, clk, iters, e0, e1);
  return 0;
}
