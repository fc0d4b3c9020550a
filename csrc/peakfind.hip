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
// MI355X design: 64x16 output tile per 256-thread workgroup (4 consecutive pixels per lane),
// halo tile staged once in LDS, candidates are rare so the divergent verification path is
// cheap; one atomic per wave to reserve peak slots.
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
__global__ __launch_bounds__(256) void peakfind_kernel(const FramePtrs fp, const PfParams pp,
                                                       float* __restrict__ peaks,     // [F][max][8]
                                                       int* __restrict__ counts,      // [F]
                                                       float* __restrict__ summary) { // [F][2]
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

void launch_peakfind(const FramePtrs& fp, int nframes, int n_panels, int rows, int cols, float thr_peak,
                     float son_min, int radius, int max_peaks, uint64_t peaks, uint64_t counts,
                     uint64_t summary, uint64_t stream) {
  check(nframes >= 1 && nframes <= kMaxFrames, "peakfind: nframes out of range");
  check(radius == 1 || radius == 2, "peakfind: radius must be 1 or 2");
  check(max_peaks >= 1, "peakfind: max_peaks must be >= 1");
  PfParams pp{thr_peak, son_min, max_peaks, n_panels, rows, cols};
  const int tiles = ((cols + kPfTX - 1) / kPfTX) * ((rows + kPfTY - 1) / kPfTY);
  const dim3 grid((unsigned)(tiles * n_panels), (unsigned)nframes);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  float* P = reinterpret_cast<float*>(peaks);
  int* C = reinterpret_cast<int*>(counts);
  float* S = reinterpret_cast<float*>(summary);
  if (radius == 1)
    hipLaunchKernelGGL(peakfind_kernel<1>, grid, dim3(256), 0, s, fp, pp, P, C, S);
  else
    hipLaunchKernelGGL(peakfind_kernel<2>, grid, dim3(256), 0, s, fp, pp, P, C, S);
  hip_check(hipGetLastError(), "peakfind launch");
}

}  // namespace pr
