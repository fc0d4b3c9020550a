// Memory ceiling of the calibration store pattern on one MI355X: per pixel read 2 B raw +
// 4 B pedestal + 4 B gain factor (tables shared by every frame), write 4 B float -- the bytes the
// fused common-mode kernel must move with its medians removed.  Times several orders of the same
// work (frame-major, table-major with all frames of a pixel block in one workgroup) so the CM kernel
// can be priced against a measured ceiling, not a datasheet number.
//
//   hipcc -O3 --offload-arch=gfx950 tools/bw_ceiling.hip -o /tmp/bw_ceiling && /tmp/bw_ceiling
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e = (x);                                                         \
    if (e != hipSuccess) {                                                      \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      std::exit(1);                                                             \
    }                                                                           \
  } while (0)

typedef unsigned u4v __attribute__((ext_vector_type(4)));
typedef float f4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 ldnt(const void* p) {
  const u4v v = __builtin_nontemporal_load(reinterpret_cast<const u4v*>(p));
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void stnt(void* p, float4 o) {
  f4v v = {o.x, o.y, o.z, o.w};
  __builtin_nontemporal_store(v, reinterpret_cast<f4v*>(p));
}

constexpr int kNpix = 16 * 352 * 384;   // epix10k2M
constexpr int kGroups = kNpix / 8;

template <bool NTL = true, bool NTS = true>
__device__ __forceinline__ void work(const uint16_t* raw, const float* ped, const float* gf, float* out, int g) {
  const uint4 rw = NTL ? ldnt(reinterpret_cast<const uint4*>(raw) + g) : reinterpret_cast<const uint4*>(raw)[g];
  const float4 p0 = reinterpret_cast<const float4*>(ped)[2 * g], p1 = reinterpret_cast<const float4*>(ped)[2 * g + 1];
  const float4 g0 = reinterpret_cast<const float4*>(gf)[2 * g], g1 = reinterpret_cast<const float4*>(gf)[2 * g + 1];
  const float a[8] = {(float)(rw.x & 0x3fff), (float)((rw.x >> 16) & 0x3fff), (float)(rw.y & 0x3fff),
                      (float)((rw.y >> 16) & 0x3fff), (float)(rw.z & 0x3fff), (float)((rw.z >> 16) & 0x3fff),
                      (float)(rw.w & 0x3fff), (float)((rw.w >> 16) & 0x3fff)};
  float4 o0 = make_float4((a[0] - p0.x) * g0.x, (a[1] - p0.y) * g0.y, (a[2] - p0.z) * g0.z, (a[3] - p0.w) * g0.w);
  float4 o1 = make_float4((a[4] - p1.x) * g1.x, (a[5] - p1.y) * g1.y, (a[6] - p1.z) * g1.z, (a[7] - p1.w) * g1.w);
  if (NTS) {
    stnt(reinterpret_cast<float4*>(out) + 2 * g, o0);
    stnt(reinterpret_cast<float4*>(out) + 2 * g + 1, o1);
  } else {
    reinterpret_cast<float4*>(out)[2 * g] = o0;
    reinterpret_cast<float4*>(out)[2 * g + 1] = o1;
  }
}

// frame-major: block b handles 256 groups of frame b / blocks_per_frame
__global__ __launch_bounds__(256) void k_frame_major(const uint16_t* raw, const float* ped, const float* gf, float* out,
                                                     int nframes) {
  const int bpf = kGroups / 256;
  const int f = blockIdx.x / bpf, g = (blockIdx.x % bpf) * 256 + threadIdx.x;
  work(raw + (size_t)f * kNpix, ped, gf, out + (size_t)f * kNpix, g);
}

template <bool NTL, bool NTS>
__global__ __launch_bounds__(256) void k_fm(const uint16_t* raw, const float* ped, const float* gf, float* out,
                                            int nframes) {
  const int bpf = kGroups / 256;
  const int f = blockIdx.x / bpf, g = (blockIdx.x % bpf) * 256 + threadIdx.x;
  work<NTL, NTS>(raw + (size_t)f * kNpix, ped, gf, out + (size_t)f * kNpix, g);
}
template <bool NTL, bool NTS>
__global__ __launch_bounds__(256) void k_tm(const uint16_t* raw, const float* ped, const float* gf, float* out,
                                            int nframes) {
  const int f = blockIdx.x % nframes, g = (blockIdx.x / nframes) * 256 + threadIdx.x;
  work<NTL, NTS>(raw + (size_t)f * kNpix, ped, gf, out + (size_t)f * kNpix, g);
}

// 4 pixels per lane: 8-B raw load, one 16-B store, consecutive lanes on consecutive 16 B
template <bool TABLES>
__global__ __launch_bounds__(256) void k_fm4(const uint16_t* raw, const float* ped, const float* gf, float* out,
                                             int nframes) {
  const int bpf = kNpix / 4 / 256;
  const int f = blockIdx.x / bpf, q = (blockIdx.x % bpf) * 256 + threadIdx.x;
  const uint2 r = *reinterpret_cast<const uint2*>(raw + (size_t)f * kNpix + 4 * (size_t)q);
  float4 p = make_float4(0.f, 0.f, 0.f, 0.f), g = make_float4(1.f, 1.f, 1.f, 1.f);
  if (TABLES) {
    p = reinterpret_cast<const float4*>(ped)[q];
    g = reinterpret_cast<const float4*>(gf)[q];
  }
  const float4 o = make_float4(((float)(r.x & 0x3fff) - p.x) * g.x, ((float)(r.x >> 16 & 0x3fff) - p.y) * g.y,
                               ((float)(r.y & 0x3fff) - p.z) * g.z, ((float)(r.y >> 16 & 0x3fff) - p.w) * g.w);
  reinterpret_cast<float4*>(out + (size_t)f * kNpix)[q] = o;
}
// 8 pixels per lane, but the two 16-B stores of a wave each cover 1 KiB contiguous (lane l holds
// pixels 4l..4l+3 and 256+4l..256+4l+3 of the wave's 512-pixel span)
__global__ __launch_bounds__(256) void k_fm8c(const uint16_t* raw, const float* ped, const float* gf, float* out,
                                              int nframes) {
  const int bpf = kGroups / 256;
  const int f = blockIdx.x / bpf;
  const int w = (blockIdx.x % bpf) * 4 + (threadIdx.x >> 6), l = threadIdx.x & 63;
  const size_t base = (size_t)w * 512;
  float4 o[2];
  for (int h = 0; h < 2; ++h) {
    const size_t px = base + 256 * h + 4 * l;
    const uint2 r = *reinterpret_cast<const uint2*>(raw + (size_t)f * kNpix + px);
    const float4 p = *reinterpret_cast<const float4*>(ped + px), g = *reinterpret_cast<const float4*>(gf + px);
    o[h] = make_float4(((float)(r.x & 0x3fff) - p.x) * g.x, ((float)(r.x >> 16 & 0x3fff) - p.y) * g.y,
                       ((float)(r.y & 0x3fff) - p.z) * g.z, ((float)(r.y >> 16 & 0x3fff) - p.w) * g.w);
  }
  for (int h = 0; h < 2; ++h) *reinterpret_cast<float4*>(out + (size_t)f * kNpix + base + 256 * h + 4 * l) = o[h];
}

// table-major: consecutive blocks = the same pixels of consecutive frames (the CM kernel's order)
__global__ __launch_bounds__(256) void k_table_major(const uint16_t* raw, const float* ped, const float* gf, float* out,
                                                     int nframes) {
  const int f = blockIdx.x % nframes, g = (blockIdx.x / nframes) * 256 + threadIdx.x;
  work(raw + (size_t)f * kNpix, ped, gf, out + (size_t)f * kNpix, g);
}

// one workgroup walks all frames of its pixel block (tables once from HBM, then L1/L2)
__global__ __launch_bounds__(256) void k_frames_inner(const uint16_t* raw, const float* ped, const float* gf, float* out,
                                                      int nframes) {
  const int g = blockIdx.x * 256 + threadIdx.x;
  for (int f = 0; f < nframes; ++f) work(raw + (size_t)f * kNpix, ped, gf, out + (size_t)f * kNpix, g);
}

// raw read + float write only (tables skipped): the unavoidable bytes
__global__ __launch_bounds__(256) void k_no_tables(const uint16_t* raw, const float* ped, const float* gf, float* out,
                                                   int nframes) {
  const int bpf = kGroups / 256;
  const int f = blockIdx.x / bpf, g = (blockIdx.x % bpf) * 256 + threadIdx.x;
  const uint4 rw = ldnt(reinterpret_cast<const uint4*>(raw + (size_t)f * kNpix) + g);
  float* o = out + (size_t)f * kNpix;
  stnt(reinterpret_cast<float4*>(o) + 2 * g, make_float4((float)rw.x, (float)rw.y, 0.f, 0.f));
  stnt(reinterpret_cast<float4*>(o) + 2 * g + 1, make_float4((float)rw.z, (float)rw.w, 0.f, 0.f));
}

// the same with ordinary (cached) stores
__global__ __launch_bounds__(256) void k_no_tables_plain(const uint16_t* raw, const float* ped, const float* gf,
                                                         float* out, int nframes) {
  const int bpf = kGroups / 256;
  const int f = blockIdx.x / bpf, g = (blockIdx.x % bpf) * 256 + threadIdx.x;
  const uint4 rw = reinterpret_cast<const uint4*>(raw + (size_t)f * kNpix)[g];
  float4* o = reinterpret_cast<float4*>(out + (size_t)f * kNpix);
  o[2 * g] = make_float4((float)rw.x, (float)rw.y, 0.f, 0.f);
  o[2 * g + 1] = make_float4((float)rw.z, (float)rw.w, 0.f, 0.f);
}

// write-only / read-only halves
__global__ __launch_bounds__(256) void k_write_only(const uint16_t* raw, const float* ped, const float* gf, float* out,
                                                    int nframes) {
  const int bpf = kGroups / 256;
  const int f = blockIdx.x / bpf, g = (blockIdx.x % bpf) * 256 + threadIdx.x;
  float* o = out + (size_t)f * kNpix;
  stnt(reinterpret_cast<float4*>(o) + 2 * g, make_float4((float)g, 0.f, 0.f, 0.f));
  stnt(reinterpret_cast<float4*>(o) + 2 * g + 1, make_float4((float)f, 0.f, 0.f, 0.f));
}
__global__ __launch_bounds__(256) void k_read_only(const uint16_t* raw, const float* ped, const float* gf, float* out,
                                                   int nframes) {
  const int bpf = kGroups / 256;
  const int f = blockIdx.x / bpf, g = (blockIdx.x % bpf) * 256 + threadIdx.x;
  const float4* o = reinterpret_cast<const float4*>(out + (size_t)f * kNpix);
  const float4 a = o[2 * g], b = o[2 * g + 1];
  if (a.x + b.y == 12345.f) out[0] = a.z;   // never true for the zeroed buffer; keeps the loads
}

using K = void (*)(const uint16_t*, const float*, const float*, float*, int);

static double time_us(K k, dim3 grid, const uint16_t* raw, const float* ped, const float* gf, float* out, int nf) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(k, grid, dim3(256), 0, 0, raw, ped, gf, out, nf);
  CK(hipDeviceSynchronize());
  std::vector<float> t;
  for (int r = 0; r < 11; ++r) {
    CK(hipEventRecord(a));
    for (int i = 0; i < 10; ++i) hipLaunchKernelGGL(k, grid, dim3(256), 0, 0, raw, ped, gf, out, nf);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    t.push_back(ms);
  }
  std::sort(t.begin(), t.end());
  return 1e3 * t[t.size() / 2] / 10;
}

int main() {
  const int nf = 32;
  uint16_t* raw;
  float *ped, *gf, *out;
  CK(hipMalloc(&raw, (size_t)nf * kNpix * 2));
  CK(hipMalloc(&ped, (size_t)kNpix * 4));
  CK(hipMalloc(&gf, (size_t)kNpix * 4));
  CK(hipMalloc(&out, (size_t)nf * kNpix * 4));
  CK(hipMemset(raw, 1, (size_t)nf * kNpix * 2));
  CK(hipMemset(ped, 0, (size_t)kNpix * 4));
  CK(hipMemset(gf, 0, (size_t)kNpix * 4));
  CK(hipMemset(out, 0, (size_t)nf * kNpix * 4));
  const unsigned nblk = kGroups / 256;
  struct {
    const char* name;
    K k;
    dim3 grid;
  } runs[] = {{"frame_major", k_frame_major, dim3(nblk * nf)},
              {"table_major", k_table_major, dim3(nblk * nf)},
              {"frames_inner", k_frames_inner, dim3(nblk)},
              {"frame_major_ntload_plainstore", k_fm<true, false>, dim3(nblk * nf)},
              {"frame_major_plain", k_fm<false, false>, dim3(nblk * nf)},
              {"table_major_ntload_plainstore", k_tm<true, false>, dim3(nblk * nf)},
              {"table_major_plain", k_tm<false, false>, dim3(nblk * nf)},
              {"fm4_tables", k_fm4<true>, dim3(kNpix / 4 / 256 * nf)},
              {"fm4_no_tables", k_fm4<false>, dim3(kNpix / 4 / 256 * nf)},
              {"fm8_contig_stores", k_fm8c, dim3(nblk * nf)},
              {"no_tables", k_no_tables, dim3(nblk * nf)},
              {"no_tables_plain", k_no_tables_plain, dim3(nblk * nf)},
              {"write_only_f32", k_write_only, dim3(nblk * nf)},
              {"read_only_f32", k_read_only, dim3(nblk * nf)}};
  std::printf("{");
  for (size_t i = 0; i < sizeof(runs) / sizeof(runs[0]); ++i) {
    const double us = time_us(runs[i].k, runs[i].grid, raw, ped, gf, out, nf);
    const double dram_min = (double)nf * kNpix * 6;   // raw + out, tables once
    std::printf("%s\"%s_us_per_frame\": %.3f, \"%s_TBps_raw_out\": %.2f", i ? ", " : "", runs[i].name, us / nf,
                runs[i].name, dram_min / (us * 1e-6) / 1e12);
  }
  std::printf("}\n");
  return 0;
}
