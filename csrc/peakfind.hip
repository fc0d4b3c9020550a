// K-07 on-GPU peak finder for queue consumers (BASELINE config 5).
//
// Reference parity: psana-ray draws "Batches -> PyTorch Task" consumers
// (figures/psana-ray-architecture.png, README.md:3) and its setup.py:11 names PeakNet as the
// downstream, but ships no analysis code; this is the consumer-side analysis the framework
// provides.  Algorithm (peakfinder8-style, simplified, every knob a parameter):
//   candidate   v > thr_peak and v is the strict local maximum of its (2R+1)^2 window
//               (ties broken by linear index; pixels outside the panel are absent)
//   background  mean / population-std of the ring of Chebyshev radius R+1 .. R+2
//   snr         (v - bkg) / max(noise, 1e-6); kept if snr >= son_min
//   intensity   sum over the (2R+1)^2 window of (pixel - bkg)
// Per-frame summary: number of pixels above thr_peak and their sum (hit-finding statistics),
// reduced wave -> LDS -> one atomic per workgroup.
//
// MI355X design: output tiles staged with their halo once in LDS; candidates are rare so the
// divergent verification path is cheap; one atomic per accepted peak reserves its record slot
// (and bumps an optional 64-bit running total, so consumers never read counts back per batch).
// v1 (64x16 tile, 4 px per lane, scalar loads) is kept for A/B (PSANA_RAY_PF_V1=1).
#include "common.h"

namespace pr {

constexpr int kPfTX = 64, kPfTY = 16;

struct PfParams {
  float thr_peak;
  float son_min;
  int max_peaks;
  int n_panels, rows, cols;
};

template <int RAD>
__global__ __launch_bounds__(256) void peakfind_v1_kernel(const FramePtrs fp, const PfParams pp,
                                                       float* __restrict__ peaks,     // [F][max][8]
                                                       int* __restrict__ counts,      // [F]
                                                       float* __restrict__ summary,   // [F][2]
                                                       unsigned long long* __restrict__ total) {
  constexpr int H = RAD + 2;
  constexpr int LW = kPfTX + 2 * H, LH = kPfTY + 2 * H;
  __shared__ float t[LH][LW + 1];
  __shared__ float red_sum[4];
  __shared__ int red_cnt[4];

  const int f = blockIdx.y;
  const int tiles_x = (pp.cols + kPfTX - 1) / kPfTX;
  const int tiles_y = (pp.rows + kPfTY - 1) / kPfTY;
  const int panel = blockIdx.x / (tiles_x * tiles_y);
  const int trem = blockIdx.x % (tiles_x * tiles_y);
  const int ty0 = (trem / tiles_x) * kPfTY, tx0 = (trem % tiles_x) * kPfTX;
  const PR_GLOBAL float* img = gin<float>(fp.in[f]) + (int64_t)panel * pp.rows * pp.cols;
  const float NaN = __int_as_float(0x7fc00000);

  for (int i = threadIdx.x; i < LH * LW; i += 256) {
    const int ly = i / LW, lx = i % LW;
    const int gy = ty0 + ly - H, gx = tx0 + lx - H;
    t[ly][lx] = (gy >= 0 && gy < pp.rows && gx >= 0 && gx < pp.cols) ? img[(int64_t)gy * pp.cols + gx] : NaN;
  }
  __syncthreads();

  const int ly = threadIdx.x / (kPfTX / 4);
  const int lx0 = (threadIdx.x % (kPfTX / 4)) * 4;
  float above_sum = 0.0f;
  int above_cnt = 0;
  for (int k = 0; k < 4; ++k) {
    const int cy = ly + H, cx = lx0 + k + H;
    const float v = t[cy][cx];
    if (!(v > pp.thr_peak)) continue;  // also rejects NaN (outside the panel)
    above_sum += v;
    ++above_cnt;
    bool is_max = true;
#pragma unroll
    for (int dy = -RAD; dy <= RAD; ++dy)
#pragma unroll
      for (int dx = -RAD; dx <= RAD; ++dx) {
        if (dy == 0 && dx == 0) continue;
        const float n = t[cy + dy][cx + dx];
        if (n != n) continue;
        const bool before = (dy < 0) || (dy == 0 && dx < 0);
        if (before ? !(v > n) : !(v >= n)) is_max = false;
      }
    if (!is_max) continue;
    float s = 0.0f, s2 = 0.0f;
    int nr = 0;
#pragma unroll
    for (int dy = -H; dy <= H; ++dy)
#pragma unroll
      for (int dx = -H; dx <= H; ++dx) {
        const int d = max(abs(dy), abs(dx));
        if (d <= RAD) continue;
        const float n = t[cy + dy][cx + dx];
        if (n != n) continue;
        s += n;
        s2 += n * n;
        ++nr;
      }
    const float bkg = nr > 0 ? s / nr : 0.0f;
    const float var = nr > 0 ? fmaxf(s2 / nr - bkg * bkg, 0.0f) : 0.0f;
    const float noise = sqrtf(var);
    const float snr = (v - bkg) / fmaxf(noise, 1e-6f);
    if (snr < pp.son_min) continue;
    float inten = 0.0f;
#pragma unroll
    for (int dy = -RAD; dy <= RAD; ++dy)
#pragma unroll
      for (int dx = -RAD; dx <= RAD; ++dx) {
        const float n = t[cy + dy][cx + dx];
        if (n == n) inten += n - bkg;
      }
    const int slot = atomicAdd(counts + f, 1);
    if (slot < pp.max_peaks) {
      if (total != nullptr) atomicAdd(total, 1ull);
      float* rec = peaks + ((int64_t)f * pp.max_peaks + slot) * 8;
      rec[0] = (float)panel;
      rec[1] = (float)(ty0 + ly);
      rec[2] = (float)(tx0 + lx0 + k);
      rec[3] = v;
      rec[4] = inten;
      rec[5] = bkg;
      rec[6] = noise;
      rec[7] = snr;
    }
  }
  // block reduction of the hit statistics: wave shuffle -> LDS -> one atomic per block
  for (int o = 32; o > 0; o >>= 1) {
    above_sum += __shfl_down(above_sum, o);
    above_cnt += __shfl_down(above_cnt, o);
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) {
    red_sum[wave] = above_sum;
    red_cnt[wave] = above_cnt;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const float s = red_sum[0] + red_sum[1] + red_sum[2] + red_sum[3];
    const int c = red_cnt[0] + red_cnt[1] + red_cnt[2] + red_cnt[3];
    if (c > 0) {
      atomicAdd(summary + 2 * f, (float)c);
      atomicAdd(summary + 2 * f + 1, s);
    }
  }
}

// ---------------------------------------------------------------------------------------------
// v2 (default): 64x32 output tile per 256-thread workgroup.  The halo tile is loaded with 16-B
// aligned float4 loads (x halo rounded up to 4 columns; panels are a multiple of 4 wide, so a
// float4 is entirely inside or outside the panel) and stored with ds_write_b128; every lane owns
// ONE column x = lane and 8 rows, so a wave's neighbourhood reads t[y+dy][x+dx] hit 64
// consecutive words: bank-conflict free.  Half the workgroups of v1 for the same frame, 1.2x halo
// over-fetch instead of 1.5x.
// ---------------------------------------------------------------------------------------------
constexpr int kPf2TX = 64, kPf2TY = 32, kPf2HX = 4;

template <int RAD>
__device__ __forceinline__ void pf_candidate(const float (*t)[kPf2TX + 2 * kPf2HX], int cy, int cx, float v,
                                             const PfParams& pp, int f, int panel, int gy, int gx,
                                             float* __restrict__ peaks, int* __restrict__ counts,
                                             unsigned long long* __restrict__ total) {
  constexpr int H = RAD + 2;
#pragma unroll
  for (int dy = -RAD; dy <= RAD; ++dy)
#pragma unroll
    for (int dx = -RAD; dx <= RAD; ++dx) {
      if (dy == 0 && dx == 0) continue;
      const float n = t[cy + dy][cx + dx];
      if (n != n) continue;
      const bool before = (dy < 0) || (dy == 0 && dx < 0);
      if (before ? !(v > n) : !(v >= n)) return;   // not the strict local max (ties: lower index wins)
    }
  float s = 0.0f, s2 = 0.0f;
  int nr = 0;
#pragma unroll
  for (int dy = -H; dy <= H; ++dy)
#pragma unroll
    for (int dx = -H; dx <= H; ++dx) {
      const int d = max(abs(dy), abs(dx));
      if (d <= RAD) continue;
      const float n = t[cy + dy][cx + dx];
      if (n != n) continue;
      s += n;
      s2 += n * n;
      ++nr;
    }
  const float bkg = nr > 0 ? s / nr : 0.0f;
  const float var = nr > 0 ? fmaxf(s2 / nr - bkg * bkg, 0.0f) : 0.0f;
  const float noise = sqrtf(var);
  const float snr = (v - bkg) / fmaxf(noise, 1e-6f);
  if (snr < pp.son_min) return;
  float inten = 0.0f;
#pragma unroll
  for (int dy = -RAD; dy <= RAD; ++dy)
#pragma unroll
    for (int dx = -RAD; dx <= RAD; ++dx) {
      const float n = t[cy + dy][cx + dx];
      if (n == n) inten += n - bkg;
    }
  const int slot = atomicAdd(counts + f, 1);
  if (slot < pp.max_peaks) {
    if (total != nullptr) atomicAdd(total, 1ull);
    float* rec = peaks + ((int64_t)f * pp.max_peaks + slot) * 8;
    rec[0] = (float)panel;
    rec[1] = (float)gy;
    rec[2] = (float)gx;
    rec[3] = v;
    rec[4] = inten;
    rec[5] = bkg;
    rec[6] = noise;
    rec[7] = snr;
  }
}

template <int RAD>
__global__ __launch_bounds__(256) void peakfind_kernel(const FramePtrs fp, const PfParams pp,
                                                       float* __restrict__ peaks, int* __restrict__ counts,
                                                       float* __restrict__ summary,
                                                       unsigned long long* __restrict__ total) {
  constexpr int H = RAD + 2;
  static_assert(H <= kPf2HX, "x halo must cover the background ring");
  constexpr int LW = kPf2TX + 2 * kPf2HX;   // 72 floats = 18 float4 per row
  constexpr int LH = kPf2TY + 2 * H;
  constexpr int Q = LW / 4;
  __shared__ __attribute__((aligned(16))) float t[LH][LW];
  __shared__ float red_sum[4];
  __shared__ int red_cnt[4];

  const int f = blockIdx.y;
  const int tiles_x = (pp.cols + kPf2TX - 1) / kPf2TX;
  const int tiles_y = (pp.rows + kPf2TY - 1) / kPf2TY;
  const int panel = blockIdx.x / (tiles_x * tiles_y);
  const int trem = blockIdx.x % (tiles_x * tiles_y);
  const int ty0 = (trem / tiles_x) * kPf2TY, tx0 = (trem % tiles_x) * kPf2TX;
  const PR_GLOBAL float* img = gin<float>(fp.in[f]) + (int64_t)panel * pp.rows * pp.cols;
  const float NaN = __int_as_float(0x7fc00000);

  for (int i = threadIdx.x; i < LH * Q; i += 256) {
    const int ly = i / Q, q = i % Q;
    const int gy = ty0 + ly - H, gx = tx0 - kPf2HX + 4 * q;
    f32x4_t v = {NaN, NaN, NaN, NaN};
    if (gy >= 0 && gy < pp.rows && gx >= 0 && gx < pp.cols)
      v = *(const PR_GLOBAL f32x4_t*)(img + (int64_t)gy * pp.cols + gx);
    *reinterpret_cast<f32x4_t*>(&t[ly][4 * q]) = v;
  }
  __syncthreads();

  const int x = threadIdx.x & 63;
  const int y0 = threadIdx.x >> 6;
  const int gx = tx0 + x;
  float above_sum = 0.0f;
  int above_cnt = 0;
  if (gx < pp.cols) {
#pragma unroll
    for (int k = 0; k < kPf2TY / 4; ++k) {
      const int y = y0 + 4 * k;
      const float v = t[y + H][x + kPf2HX];   // NaN below the panel edge -> rejected
      if (!(v > pp.thr_peak)) continue;
      above_sum += v;
      ++above_cnt;
      pf_candidate<RAD>(t, y + H, x + kPf2HX, v, pp, f, panel, ty0 + y, gx, peaks, counts, total);
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    above_sum += __shfl_down(above_sum, o);
    above_cnt += __shfl_down(above_cnt, o);
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) {
    red_sum[wave] = above_sum;
    red_cnt[wave] = above_cnt;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const float s = red_sum[0] + red_sum[1] + red_sum[2] + red_sum[3];
    const int c = red_cnt[0] + red_cnt[1] + red_cnt[2] + red_cnt[3];
    if (c > 0) {
      atomicAdd(summary + 2 * f, (float)c);
      atomicAdd(summary + 2 * f + 1, s);
    }
  }
}

static bool pf_force_v1() {
  const char* e = getenv("PSANA_RAY_PF_V1");
  return e != nullptr && e[0] == '1';
}

void launch_peakfind(const FramePtrs& fp, int nframes, int n_panels, int rows, int cols, float thr_peak,
                     float son_min, int radius, int max_peaks, uint64_t peaks, uint64_t counts,
                     uint64_t summary, uint64_t total, uint64_t stream) {
  check(nframes >= 1 && nframes <= kMaxFrames, "peakfind: nframes out of range");
  check(radius == 1 || radius == 2, "peakfind: radius must be 1 or 2");
  check(max_peaks >= 1, "peakfind: max_peaks must be >= 1");
  check(cols % 4 == 0, "peakfind: panel width must be a multiple of 4");
  for (int f = 0; f < nframes; ++f) check(aligned16(fp.in[f]), "peakfind: frames must be 16-B aligned");
  PfParams pp{thr_peak, son_min, max_peaks, n_panels, rows, cols};
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  float* P = reinterpret_cast<float*>(peaks);
  int* C = reinterpret_cast<int*>(counts);
  float* S = reinterpret_cast<float*>(summary);
  unsigned long long* T = reinterpret_cast<unsigned long long*>(total);
  if (pf_force_v1()) {
    const int tiles = ((cols + kPfTX - 1) / kPfTX) * ((rows + kPfTY - 1) / kPfTY);
    const dim3 grid((unsigned)(tiles * n_panels), (unsigned)nframes);
    if (radius == 1)
      hipLaunchKernelGGL(peakfind_v1_kernel<1>, grid, dim3(256), 0, s, fp, pp, P, C, S, T);
    else
      hipLaunchKernelGGL(peakfind_v1_kernel<2>, grid, dim3(256), 0, s, fp, pp, P, C, S, T);
  } else {
    const int tiles = ((cols + kPf2TX - 1) / kPf2TX) * ((rows + kPf2TY - 1) / kPf2TY);
    const dim3 grid((unsigned)(tiles * n_panels), (unsigned)nframes);
    if (radius == 1)
      hipLaunchKernelGGL(peakfind_kernel<1>, grid, dim3(256), 0, s, fp, pp, P, C, S, T);
    else
      hipLaunchKernelGGL(peakfind_kernel<2>, grid, dim3(256), 0, s, fp, pp, P, C, S, T);
  }
  hip_check(hipGetLastError(), "peakfind launch");
}

}  // namespace pr
