// Streaming-read ceiling on one MI355X for the peak finder's access pattern: 32 epix10k2M float32
// frames (8.65 MB each, separate allocations as in the queue ring) read once per launch.  Varies the
// loads in flight per lane (U float4), workgroups per CU, the work split (grid-stride vs contiguous
// range per workgroup) and the load flavour (plain / non-temporal).  Prints one JSON line.
//   hipcc -O3 --offload-arch=gfx950 tools/read_probe.hip -o /tmp/read_probe && /tmp/read_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      std::exit(1);                                                            \
    }                                                                          \
  } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));
constexpr int kFrames = 32;
constexpr long kN4 = 16L * 352 * 384 / 4;   // float4 per frame

struct Ptrs {
  const f4* p[kFrames];
};

template <int U, bool NT, bool RANGE>
__global__ __launch_bounds__(256) void rd(Ptrs fp, float* sink) {
  const long chunk = 256L * U;                       // float4 per chunk
  const long cpf = (kN4 + chunk - 1) / chunk;
  const long T = cpf * kFrames;
  long g0, g1, gs;
  if (RANGE) {
    g0 = T * blockIdx.x / gridDim.x;
    g1 = T * (blockIdx.x + 1) / gridDim.x;
    gs = 1;
  } else {
    g0 = blockIdx.x;
    g1 = T;
    gs = gridDim.x;
  }
  float acc = 0.f;
  for (long g = g0; g < g1; g += gs) {
    const int f = (int)(g / cpf);
    const long q0 = (g - (long)f * cpf) * chunk + threadIdx.x;
    f4 v[U];
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const long q = q0 + 256L * k;
      if (q < kN4) v[k] = NT ? __builtin_nontemporal_load(fp.p[f] + q) : fp.p[f][q];
      else v[k] = f4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int k = 0; k < U; ++k) acc += v[k].x + v[k].y + v[k].z + v[k].w;
  }
  if (acc == 1234.5f) sink[0] = acc;
}

template <int U, bool NT, bool RANGE>
static double run(const Ptrs& fp, float* sink, int blocks) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((rd<U, NT, RANGE>), dim3(blocks), dim3(256), 0, 0, fp, sink);
  CK(hipDeviceSynchronize());
  std::vector<float> t;
  for (int r = 0; r < 9; ++r) {
    CK(hipEventRecord(a));
    for (int i = 0; i < 8; ++i) hipLaunchKernelGGL((rd<U, NT, RANGE>), dim3(blocks), dim3(256), 0, 0, fp, sink);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    t.push_back(ms / 8);
  }
  std::sort(t.begin(), t.end());
  const double ms = t[t.size() / 2];
  return (double)kFrames * kN4 * 16 / (ms * 1e-3) / 1e12;   // TB/s
}

int main() {
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  Ptrs fp;
  for (int f = 0; f < kFrames; ++f) {
    f4* p;
    CK(hipMalloc(&p, kN4 * 16));
    CK(hipMemset(p, 0, kN4 * 16));
    fp.p[f] = p;
  }
  // flush the Infinity Cache between configurations: one 1-GB read
  float* sink;
  CK(hipMalloc(&sink, 64));
  std::printf("{\"cus\": %d", cus);
#define R(U, NT, RANGE, M)                                                                        \
  std::printf(", \"U%d_%s_%s_x%d\": %.2f", U, NT ? "nt" : "plain", RANGE ? "range" : "stride", M, \
              run<U, NT, RANGE>(fp, sink, cus * M))
  R(4, false, true, 4);
  R(4, false, true, 8);
  R(4, true, true, 4);
  R(4, true, true, 8);
  R(2, false, true, 8);
  R(8, false, true, 4);
  R(8, true, true, 4);
  R(4, false, false, 4);
  R(4, false, false, 8);
  R(4, false, false, 16);
  R(4, true, false, 8);
  R(8, true, false, 8);
  R(2, true, false, 16);
  std::printf("}\n");
  return 0;
}
