// K-03 common-mode correction, fused with K-01/K-02/K-04 in ONE pass over HBM.
//
// Reference parity: psana applies common mode inside det.calib (reached through
// psana_wrapper.iter_events, psana_ray/producer.py:88); psana-ray itself has no numerics.
// Semantics implemented here (psana "mode 7"-like, every knob a parameter):
//   v = ADU - ped[gain]                                   (pre-gain, ADU domain)
//   eligible = good-mask && gain in the CM gain set
//   rows:  for every ASIC row and every bank of `bank_cols` columns, median of the eligible
//          pixels with |v| < thr; if count >= npix_min and |median| <= maxcorr, subtract it
//          from every eligible pixel of that row-bank segment
//   cols:  then the same per ASIC column (all ASIC rows)
//   out = v * gain_factor   (mask folded into the gain factor -> masked pixels are 0)
// Median = numpy semantics (mean of the two middle elements for an even count).
//
// MI355X design: one 1024-thread workgroup (16 waves) owns one (frame, ASIC) tile.  The
// whole pre-gain tile lives in LDS (176 x 193 f32 incl. a 1-float row pad that makes column
// reads bank-conflict free, + 4 bits of per-pixel state = 152.8 KB of the 160 KB), so HBM is
// touched exactly once: raw u16 in, f32 out.  Medians are exact: every row-bank segment
// (<= 64 px) is one wave-register bitonic sort, every column (<= 256 px) a 4-register bitonic
// sort across the wave, with DPP / permlane-swap lane exchanges (VALU only, no LDS round trips).
#include "common.h"
#include "sortnet.h"

#include <cstdlib>

namespace pr {

// ---- lane exchange: y = x from lane (lane ^ J), VALU-only (no LDS-pipe round trip) ----
//  J = 1, 2 : one DPP quad_perm
//  J = 4, 8 : DPP row_shl:J / row_shr:J (16-lane rows) + lane select
//  J = 16   : gfx950 v_permlane16_swap (swaps odd rows of vdst with even rows of src)
//  J = 32   : gfx950 v_permlane32_swap (swaps the upper half of vdst with the lower of src)
template <int J>
__device__ __forceinline__ float xor_lane(float x, int lane) {
  const int xi = __float_as_int(x);
  int yi;
  if constexpr (J == 1) {
    yi = __builtin_amdgcn_update_dpp(0, xi, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
  } else if constexpr (J == 2) {
    yi = __builtin_amdgcn_update_dpp(0, xi, 0x4E, 0xF, 0xF, false);  // quad_perm [2,3,0,1]
  } else if constexpr (J == 4 || J == 8) {
    const int up = __builtin_amdgcn_update_dpp(0, xi, 0x100 + J, 0xF, 0xF, false);  // row_shl:J
    const int dn = __builtin_amdgcn_update_dpp(0, xi, 0x110 + J, 0xF, 0xF, false);  // row_shr:J
    yi = (lane & J) ? dn : up;
  } else if constexpr (J == 16) {
    const auto r = __builtin_amdgcn_permlane16_swap((unsigned)xi, (unsigned)xi, false, false);
    yi = (int)((lane & 16) ? r[0] : r[1]);
  } else {
    static_assert(J == 32, "xor_lane: J must be a power of two < 64");
    const auto r = __builtin_amdgcn_permlane32_swap((unsigned)xi, (unsigned)xi, false, false);
    yi = (int)((lane & 32) ? r[0] : r[1]);
  }
  return __int_as_float(yi);
}

// Self-test of the exchanges: out[j * 64 + lane] = source lane seen by `lane` for J = 1 << j.
__global__ void xor_lane_selftest_kernel(int* out) {
  const int lane = threadIdx.x & 63;
  const float x = (float)lane;
  out[0 * 64 + lane] = (int)xor_lane<1>(x, lane);
  out[1 * 64 + lane] = (int)xor_lane<2>(x, lane);
  out[2 * 64 + lane] = (int)xor_lane<4>(x, lane);
  out[3 * 64 + lane] = (int)xor_lane<8>(x, lane);
  out[4 * 64 + lane] = (int)xor_lane<16>(x, lane);
  out[5 * 64 + lane] = (int)xor_lane<32>(x, lane);
}

void launch_xor_selftest(uint64_t out, uint64_t stream) {
  hipLaunchKernelGGL(xor_lane_selftest_kernel, dim3(1), dim3(64), 0, reinterpret_cast<hipStream_t>(stream),
                     reinterpret_cast<int*>(out));
  hip_check(hipGetLastError(), "xor selftest launch");
}

// ---- bitonic sort of NR independent 64-element sequences (element index = lane) --------
template <int K, int J, int NR>
__device__ __forceinline__ void seg_step(float (&x)[NR], int lane) {
  const bool up = (lane & K) == 0;
  const bool lower = (lane & J) == 0;
  const bool take_min = (lower == up);
#pragma unroll
  for (int r = 0; r < NR; ++r) {
    const float y = xor_lane<J>(x[r], lane);
    x[r] = take_min ? fminf(x[r], y) : fmaxf(x[r], y);
  }
}
template <int K, int J, int NR>
__device__ __forceinline__ void seg_merge(float (&x)[NR], int lane) {
  seg_step<K, J, NR>(x, lane);
  if constexpr (J > 1) seg_merge<K, J / 2, NR>(x, lane);
}
template <int K, int NR>
__device__ __forceinline__ void seg_sort_from(float (&x)[NR], int lane) {
  seg_merge<K, K / 2, NR>(x, lane);
  if constexpr (K < 64) seg_sort_from<K * 2, NR>(x, lane);
}

// ---- bitonic sort of ONE 256-element sequence held as x[r] at element r*64 + lane -------
template <int K, int J>
__device__ __forceinline__ void col_step(float (&x)[4], int lane) {
  if constexpr (J >= 64) {
    constexpr int JR = J / 64;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if ((r & JR) == 0) {
        const int q = r | JR;
        const bool up = ((r * 64) & K) == 0;
        const float lo = fminf(x[r], x[q]);
        const float hi = fmaxf(x[r], x[q]);
        x[r] = up ? lo : hi;
        x[q] = up ? hi : lo;
      }
    }
  } else {
    const bool lower = (lane & J) == 0;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const bool up = ((r * 64 + lane) & K) == 0;
      const float y = xor_lane<J>(x[r], lane);
      x[r] = (lower == up) ? fminf(x[r], y) : fmaxf(x[r], y);
    }
  }
}
template <int K, int J>
__device__ __forceinline__ void col_merge(float (&x)[4], int lane) {
  col_step<K, J>(x, lane);
  if constexpr (J > 1) col_merge<K, J / 2>(x, lane);
}
template <int K>
__device__ __forceinline__ void col_sort_from(float (&x)[4], int lane) {
  col_merge<K, K / 2>(x, lane);
  if constexpr (K < 256) col_sort_from<K * 2>(x, lane);
}

__device__ __forceinline__ float lane_value(float x, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), l));
}

// numpy-median of the `cnt` smallest (sorted) values; element e lives in register e>>6, lane e&63.
__device__ __forceinline__ float median_sorted4(const float (&x)[4], int cnt) {
  const int i0 = __builtin_amdgcn_readfirstlane((cnt - 1) >> 1);
  const int i1 = __builtin_amdgcn_readfirstlane(cnt >> 1);
  const int r0 = i0 >> 6, r1 = i1 >> 6;
  const float s0 = r0 == 0 ? x[0] : (r0 == 1 ? x[1] : (r0 == 2 ? x[2] : x[3]));
  const float s1 = r1 == 0 ? x[0] : (r1 == 1 ? x[1] : (r1 == 2 ? x[2] : x[3]));
  const float a = lane_value(s0, i0 & 63);
  const float b = lane_value(s1, i1 & 63);
  return (a + b) * 0.5f;
}

struct CmParams {
  float thr;        // |v| < thr participates in the median estimate
  float maxcorr;    // a correction with |median| > maxcorr is not applied
  int npix_min;     // minimum participating pixels for a correction
  int flags;        // bit0: rows by bank, bit1: columns
  int bank_cols;    // columns per bank (<= 64, divides the ASIC width)
  int gather;       // 1: load only the candidate tables a pixel group uses (net kernels)
};

struct TileGeom {
  int panel_rows, panel_cols;  // H, W of one panel
  int asic_rows, asic_cols;    // R, C of one ASIC tile
  int asics_per_col, asics_per_row;  // H / R, W / C
  int64_t npix;                // pixels per frame
  int nframes;                 // frames of this launch (grid = n_asics * nframes, 1-D)
  int swizzle;                 // 1: XCD-aware remap (all frames of an ASIC on one XCD / L2); opt-in
};

// (asic, frame) of this workgroup.  Frame-minor logical order + the XCD remap put the blocks
// that read the SAME per-ASIC tables (574 KB for epix) on one XCD, so the tables come from its L2
// instead of HBM for every frame.
__device__ __forceinline__ void cm_block_coords(const TileGeom& tg, int& asic, int& f) {
  const int nwg = (int)gridDim.x;
  const int id = tg.swizzle ? xcd_swizzle((int)blockIdx.x, nwg) : (int)blockIdx.x;
  asic = id / tg.nframes;
  f = id % tg.nframes;
}

// Fused K-05 output (image mode with common mode).  Every panel is placed by an integer rotation
// + translation (geometry.py), so pixel (y, x) of panel p lands at image element
// desc[3p] + y * desc[3p+1] + x * desc[3p+2]; the corrected tile goes from LDS straight into the
// assembled image instead of a frame-shaped scratch buffer that a second kernel re-reads
// (saves a 2 x 8.65 MB HBM round trip per epix10k2M frame).  Gap pixels: launch_fill_runs.
struct ImgOut {
  const int32_t* desc;    // [n_panels][3] (base, step per panel row, step per panel column); nullptr: frame layout
  const uint8_t* omask;   // image-shaped output mask (truthy keeps) or nullptr
};

// Phase 3 of both common-mode kernels: gain factor (+ folded frame mask) applied to the corrected
// LDS tile; stored in frame layout (16-B stores) or, with io.desc, written into the image.  The
// image walk keeps consecutive lanes on consecutive image elements: tile rows when the panel's
// columns run along image rows (|sx| == 1), tile columns otherwise (column reads of the padded
// tile are LDS-conflict-free: odd pitch).
template <int NT>
__device__ __forceinline__ void cm_store(float* tile, const uint32_t* nib, const float* __restrict__ gf,
                                         const TileGeom& tg, const int R, const int C, int64_t base,
                                         PR_GLOBAL float* out, const ImgOut& io, int panel, int y0, int x0,
                                         bool gather) {
  const int LD = C + 1, C8 = C >> 3;
  const int tid = threadIdx.x;
  const bool img = io.desc != nullptr;
  for (int i = tid; i < R * C8; i += blockDim.x) {
    const int r = i / C8, c = (i % C8) * 8;
    const int64_t pix = base + (int64_t)r * tg.panel_cols + c;
    const uint32_t nb = nib[i];
    uint32_t need = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) need |= 1u << ((nb >> (4 * j)) & 3u);
    if (!gather) need = (1u << NT) - 1u;
    float ga[NT][8];
#pragma unroll
    for (int k = 0; k < NT; ++k) {
      float4 a = make_float4(0.f, 0.f, 0.f, 0.f), b = a;
      if ((need >> k) & 1u) {
        a = *reinterpret_cast<const float4*>(gf + k * tg.npix + pix);
        b = *reinterpret_cast<const float4*>(gf + k * tg.npix + pix + 4);
      }
      ga[k][0] = a.x; ga[k][1] = a.y; ga[k][2] = a.z; ga[k][3] = a.w;
      ga[k][4] = b.x; ga[k][5] = b.y; ga[k][6] = b.z; ga[k][7] = b.w;
    }
    float* trow = tile + r * LD + c;
    float o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint32_t q = (nb >> (4 * j)) & 0xFu;
      const int cand = q & 3;
      float gg;
      if constexpr (NT == 1) gg = ga[0][j];
      else if constexpr (NT == 2) gg = bsel(cand != 0, ga[1][j], ga[0][j]);
      else gg = bsel(cand == 0, ga[0][j], bsel(cand == 1, ga[1][j], ga[2][j]));
      o[j] = (q & 4u) ? trow[j] * gg : 0.0f;
    }
    if (img) {
#pragma unroll
      for (int j = 0; j < 8; ++j) trow[j] = o[j];
    } else {
      PR_GLOBAL float4* op = (PR_GLOBAL float4*)(out + pix);
      st_f4(op, make_float4(o[0], o[1], o[2], o[3]));
      st_f4(op + 1, make_float4(o[4], o[5], o[6], o[7]));
    }
  }
  if (!img) return;
  __syncthreads();
  const int32_t* d = io.desc + 3 * panel;
  const int sy = d[1], sx = d[2];
  const int64_t b0 = (int64_t)d[0] + (int64_t)y0 * sy + (int64_t)x0 * sx;
  const int n = R * C;
  const bool rows = sx == 1 || sx == -1;
  const int inner = rows ? C : R;
  const float inv = 1.0f / (float)inner;   // e < 2^24: floor((e + 0.5) / inner) is exact in f32
  for (int e = tid; e < n; e += blockDim.x) {
    const int a = (int)(((float)e + 0.5f) * inv);
    const int bb = e - a * inner;
    const int r = rows ? a : bb, c = rows ? bb : a;
    const int64_t q = b0 + (int64_t)r * sy + (int64_t)c * sx;
    float v = tile[r * LD + c];
    if (io.omask != nullptr && !io.omask[q]) v = 0.0f;
    out[q] = v;
  }
}

// per-pixel nibble in LDS: bits0-1 candidate, bit2 good, bit3 cm-eligible
template <int KIND>
__global__ __launch_bounds__(1024) void calib_cm_kernel(const FramePtrs fp, const float* __restrict__ ped,
                                                        const float* __restrict__ gf,
                                                        const uint8_t* __restrict__ pflags,
                                                        const TileGeom tg, const CmParams cp,
                                                        const ImgOut io) {
  constexpr int NT = KIND == kEpix10ka ? 2 : (KIND == kJungfrau ? 3 : 1);
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int R = tg.asic_rows, C = tg.asic_cols, LD = C + 1;
  float* tile = reinterpret_cast<float*>(smem);
  uint32_t* nib = reinterpret_cast<uint32_t*>(smem + (((size_t)R * LD * 4 + 15) & ~(size_t)15));
  const int C8 = C >> 3;

  int asic, f;
  cm_block_coords(tg, asic, f);
  const int per_panel = tg.asics_per_col * tg.asics_per_row;
  const int panel = asic / per_panel;
  const int ar = (asic % per_panel) / tg.asics_per_row;
  const int ac = (asic % per_panel) % tg.asics_per_row;
  const int64_t base = (int64_t)panel * tg.panel_rows * tg.panel_cols +
                       (int64_t)ar * R * tg.panel_cols + (int64_t)ac * C;
  const PR_GLOBAL uint16_t* raw = gin<uint16_t>(fp.in[f]);
  PR_GLOBAL float* out = gout<float>(fp.out[f]);
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int nwaves = blockDim.x >> 6;

  // ---- phase 1: decode + pedestal into LDS ---------------------------------------------
  for (int i = tid; i < R * C8; i += blockDim.x) {
    const int r = i / C8, c = (i % C8) * 8;
    const int64_t pix = base + (int64_t)r * tg.panel_cols + c;
    const uint4 rw = ld_nt_u4((const PR_GLOBAL uint4*)(raw + pix));
    const uint2 fl = *reinterpret_cast<const uint2*>(pflags + pix);
    const uint32_t w[4] = {rw.x, rw.y, rw.z, rw.w};
    const uint32_t fw[2] = {fl.x, fl.y};
    float pa[NT][8];
#pragma unroll
    for (int k = 0; k < NT; ++k) {
      const float4 a = *reinterpret_cast<const float4*>(ped + k * tg.npix + pix);
      const float4 b = *reinterpret_cast<const float4*>(ped + k * tg.npix + pix + 4);
      pa[k][0] = a.x; pa[k][1] = a.y; pa[k][2] = a.z; pa[k][3] = a.w;
      pa[k][4] = b.x; pa[k][5] = b.y; pa[k][6] = b.z; pa[k][7] = b.w;
    }
    uint32_t nb = 0;
    float* trow = tile + r * LD + c;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint32_t rv = (w[j >> 1] >> (16 * (j & 1))) & 0xFFFFu;
      const uint32_t pf = (fw[j >> 2] >> (8 * (j & 3))) & 0xFFu;
      bool valid;
      const int cand = decode_cand(rv, KIND, valid);
      float pp;
      if constexpr (NT == 1) pp = pa[0][j];
      else if constexpr (NT == 2) pp = bsel(cand != 0, pa[1][j], pa[0][j]);
      else pp = bsel(cand == 0, pa[0][j], bsel(cand == 1, pa[1][j], pa[2][j]));
      const bool good = valid && (pf & 1u);
      const bool elig = good && ((pf >> (1 + cand)) & 1u);
      trow[j] = decode_adu(rv, KIND) - pp;
      nb |= (uint32_t)(cand | (good ? 4 : 0) | (elig ? 8 : 0)) << (4 * j);
    }
    nib[r * C8 + (c >> 3)] = nb;
  }
  __syncthreads();

  const float INF = __int_as_float(0x7f800000);

  // ---- phase 2a: row common mode per bank segment ---------------------------------------
  if (cp.flags & 1) {
    const int L = cp.bank_cols;
    const int nbanks = C / L;
    for (int r = wave; r < R; r += nwaves) {
      float* trow = tile + r * LD;
      for (int b0 = 0; b0 < nbanks; b0 += 4) {
        float x[4];
        float v[4];
        bool el[4];
        int cnt[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int col = (b0 + j) * L + lane;
          const bool in = (b0 + j < nbanks) && (lane < L);
          v[j] = in ? trow[col] : 0.0f;
          el[j] = in && ((nib[r * C8 + (col >> 3)] >> (4 * (col & 7) + 3)) & 1u);
          const bool part = el[j] && (fabsf(v[j]) < cp.thr);
          x[j] = part ? v[j] : INF;
          cnt[j] = __popcll(__ballot(part));
        }
        seg_sort_from<2, 4>(x, lane);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if (cnt[j] >= cp.npix_min && cnt[j] > 0) {
            const int i0 = __builtin_amdgcn_readfirstlane((cnt[j] - 1) >> 1);
            const int i1 = __builtin_amdgcn_readfirstlane(cnt[j] >> 1);
            const float med = (lane_value(x[j], i0) + lane_value(x[j], i1)) * 0.5f;
            if (fabsf(med) <= cp.maxcorr && el[j]) trow[(b0 + j) * L + lane] = v[j] - med;
          }
        }
      }
    }
    __syncthreads();
  }

  // ---- phase 2b: column common mode -------------------------------------------------------
  if (cp.flags & 2) {
    for (int c = wave; c < C; c += nwaves) {
      float x[4], v[4];
      bool el[4];
      int cnt = 0;
      const uint32_t shift = 4 * (c & 7) + 3;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int r = k * 64 + lane;
        const bool in = r < R;
        v[k] = in ? tile[r * LD + c] : 0.0f;
        el[k] = in && ((nib[r * C8 + (c >> 3)] >> shift) & 1u);
        const bool part = el[k] && (fabsf(v[k]) < cp.thr);
        x[k] = part ? v[k] : INF;
        cnt += __popcll(__ballot(part));
      }
      col_sort_from<2>(x, lane);
      if (cnt >= cp.npix_min && cnt > 0) {
        const float med = median_sorted4(x, cnt);
        if (fabsf(med) <= cp.maxcorr) {
#pragma unroll
          for (int k = 0; k < 4; ++k)
            if (el[k]) tile[(k * 64 + lane) * LD + c] = v[k] - med;
        }
      }
    }
    __syncthreads();
  }

  // ---- phase 3: gain factor + mask, store -------------------------------------------------
  cm_store<NT>(tile, nib, gf, tg, R, C, base, out, io, panel, ar * R, ac * C, false);
}


// ==========================================================================================
// Fast path: per-lane in-register sorting networks (no cross-lane traffic in the sorts).
//
//  rows:    ONE lane owns one (row, bank) segment of L pixels; the lane sorts its L values with a
//           pruned Batcher network (L=48: 384 comparators = 768 VALU) -- 64 segments per wave
//           instruction instead of one.
//  columns: TWO lanes (an even/odd pair) own one column, M = ceil(R/2) rows each; each sorts its
//           half in registers (M=88: 957 comparators), then both evaluate the merge-path
//           identity  kth(A u B) = min_i max(A[i-1], B[k-i])  with the partner's registers
//           fetched by one DPP quad_perm each (all register indices compile-time).
//  Balanced +-inf padding: of the u non-participating elements, the first floor(u/2) become
//           -inf and the rest +inf.  The numpy median of the participating values then sits at
//           FIXED sorted positions (N/2-1, N/2 for even N), so no runtime register indexing.
// ==========================================================================================
__device__ __forceinline__ float dpp_xor1(float x) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0xB1, 0xF, 0xF, false));
}

template <int N>
__device__ __forceinline__ void fixed_median_pos(int cnt, int& lo, int& hi) {
  // positions of the lower/upper numpy-median elements after balanced +-inf padding of N slots
  const int u = N - cnt, a = u >> 1;
  lo = a + ((cnt - 1) >> 1);
  hi = a + (cnt >> 1);
}

// quad_perm DPP read of a lane of the same quad (CTRL = p0 | p1<<2 | p2<<4 | p3<<6)
template <int CTRL>
__device__ __forceinline__ float dpp_quad(float x) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), CTRL, 0xF, 0xF, false));
}
template <int CTRL>
__device__ __forceinline__ int dpp_quad_i(int x) {
  return __builtin_amdgcn_update_dpp(0, x, CTRL, 0xF, 0xF, false);
}

// Ascending sort of a V-shaped (non-increasing then non-decreasing) register sequence, virtually
// padded with +inf to the next power of two: the bitonic half-cleaner network restricted to the
// comparators between real positions (a comparator against a +inf pad is a no-op).
template <int N>
__device__ __forceinline__ void bitonic_merge_vpad(float (&z)[N]) {
  constexpr int P2 = N <= 1 ? 1 : (N <= 2 ? 2 : (N <= 4 ? 4 : (N <= 8 ? 8 : (N <= 16 ? 16 : (N <= 32 ? 32 : 64)))));
  static_assert(N <= 64, "bitonic_merge_vpad: at most 64 registers");
#pragma unroll
  for (int j = P2 / 2; j >= 1; j >>= 1) {
#pragma unroll
    for (int i = 0; i < N; ++i) {
      if ((i & j) == 0 && i + j < N) {
        const float a = z[i], b = z[i + j];
        z[i] = fminf(a, b);
        z[i + j] = fmaxf(a, b);
      }
    }
  }
}

// TR / TC: the tile (stripe) rows / columns as compile-time constants for the production shapes
// (0 = read from TileGeom).  With constants every LDS address in the unrolled median loops is a
// base VGPR + immediate offset; with runtime dims the compiler kept i*LD / i*C8 for all unrolled
// i as SGPRs, spilled them to VGPR lanes and re-read them with v_readlane + v_mul_lo per access.
template <int KIND, int L, int M, int BLOCK, int CQ, int TR = 0, int TC = 0>
__global__ __launch_bounds__(BLOCK, CQ == 4 ? (M <= 48 ? 4 : 2) : 512 / BLOCK) void calib_cm_net_kernel(const FramePtrs fp, const float* __restrict__ ped,
                                                            const float* __restrict__ gf,
                                                            const uint8_t* __restrict__ pflags,
                                                            const TileGeom tg, const CmParams cp,
                                                            const ImgOut io) {
  constexpr int NT = KIND == kEpix10ka ? 2 : (KIND == kJungfrau ? 3 : 1);
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int R = TR ? TR : tg.asic_rows, C = TC ? TC : tg.asic_cols, LD = C + 1;
  float* tile = reinterpret_cast<float*>(smem);
  uint32_t* nib = reinterpret_cast<uint32_t*>(smem + (((size_t)R * LD * 4 + 15) & ~(size_t)15));
  const int C8 = C >> 3;
  int asic, f;
  cm_block_coords(tg, asic, f);
  const int per_panel = tg.asics_per_col * tg.asics_per_row;
  const int panel = asic / per_panel;
  const int ar = (asic % per_panel) / tg.asics_per_row;
  const int ac = (asic % per_panel) % tg.asics_per_row;
  const int64_t base = (int64_t)panel * tg.panel_rows * tg.panel_cols + (int64_t)ar * R * tg.panel_cols +
                       (int64_t)ac * C;
  const PR_GLOBAL uint16_t* raw = gin<uint16_t>(fp.in[f]);
  PR_GLOBAL float* out = gout<float>(fp.out[f]);
  const int tid = threadIdx.x;
  const float INF = __int_as_float(0x7f800000);

  // ---- phase 1: decode + pedestal into LDS (same as the generic kernel) -------------------
  // select-then-load: a candidate table is read only by the 8-pixel groups that use it
  // (gain-switched pixels are rare, so the second/third table's lines are almost never fetched;
  // memory phases 5.6 -> see profiles/kernels_r1_cm_gather.jsonl)
  auto p1_need = [&](const uint4 rw) -> uint32_t {
    const uint32_t w[4] = {rw.x, rw.y, rw.z, rw.w};
    uint32_t need = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      bool vd;
      need |= 1u << decode_cand((w[j >> 1] >> (16 * (j & 1))) & 0xFFFFu, KIND, vd);
    }
    return cp.gather ? need : (1u << NT) - 1u;
  };
  auto p1_ped = [&](int64_t pix, uint32_t need, float (&pa)[NT][8], int k0 = 0) {
#pragma unroll
    for (int k = k0; k < NT; ++k) {
      float4 a = make_float4(0.f, 0.f, 0.f, 0.f), b = a;
      if ((need >> k) & 1u) {
        a = *reinterpret_cast<const float4*>(ped + k * tg.npix + pix);
        b = *reinterpret_cast<const float4*>(ped + k * tg.npix + pix + 4);
      }
      pa[k][0] = a.x; pa[k][1] = a.y; pa[k][2] = a.z; pa[k][3] = a.w;
      pa[k][4] = b.x; pa[k][5] = b.y; pa[k][6] = b.z; pa[k][7] = b.w;
    }
  };
  auto p1_store = [&](int i, const uint4 rw, const uint2 fl, const float (&pa)[NT][8]) {
    const int r = i / C8, c = (i % C8) * 8;
    const uint32_t w[4] = {rw.x, rw.y, rw.z, rw.w};
    const uint32_t fw[2] = {fl.x, fl.y};
    uint32_t nb = 0;
    float* trow = tile + r * LD + c;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint32_t rv = (w[j >> 1] >> (16 * (j & 1))) & 0xFFFFu;
      const uint32_t pf = (fw[j >> 2] >> (8 * (j & 3))) & 0xFFu;
      bool valid;
      const int cand = decode_cand(rv, KIND, valid);
      float pp;
      if constexpr (NT == 1) pp = pa[0][j];
      else if constexpr (NT == 2) pp = bsel(cand != 0, pa[1][j], pa[0][j]);
      else pp = bsel(cand == 0, pa[0][j], bsel(cand == 1, pa[1][j], pa[2][j]));
      const bool good = valid && (pf & 1u);
      const bool elig = good && ((pf >> (1 + cand)) & 1u);
      trow[j] = decode_adu(rv, KIND) - pp;
      nb |= (uint32_t)(cand | (good ? 4 : 0) | (elig ? 8 : 0)) << (4 * j);
    }
    nib[r * C8 + (c >> 3)] = nb;
  };
  auto p1_pix = [&](int i) -> int64_t {
    const int r = i / C8, c = (i % C8) * 8;
    return base + (int64_t)r * tg.panel_cols + c;
  };
  constexpr int NITEMS = (TR > 0 && TC > 0) ? TR * (TC / 8) : 0;
  constexpr int NI = NITEMS > 0 ? (NITEMS + BLOCK - 1) / BLOCK : 0;
  if constexpr (NI > 0 && NI <= 6) {
    // compile-time shape: all of this lane's raw / flag loads in flight at once, then all of its
    // pedestal loads (two dependent round trips per workgroup instead of two per item)
    // The first candidate table (the unswitched gain: nearly every pixel) is loaded together with
    // the raw words; only the rare switched candidates wait for the decoded raw (select-then-load).
    uint4 rw[NI];
    uint2 fl[NI];
    float pa[NI][NT][8];
#pragma unroll
    for (int u = 0; u < NI; ++u) {
      const int i = tid + u * BLOCK;
      if ((u + 1) * BLOCK <= NITEMS || i < NITEMS) {
        const int64_t pix = p1_pix(i);
        rw[u] = ld_nt_u4((const PR_GLOBAL uint4*)(raw + pix));
        fl[u] = *reinterpret_cast<const uint2*>(pflags + pix);
        p1_ped(pix, 1u, pa[u]);
      }
    }
#pragma unroll
    for (int u = 0; u < NI; ++u) {
      const int i = tid + u * BLOCK;
      if ((u + 1) * BLOCK <= NITEMS || i < NITEMS) p1_ped(p1_pix(i), p1_need(rw[u]), pa[u], 1);
    }
#pragma unroll
    for (int u = 0; u < NI; ++u) {
      const int i = tid + u * BLOCK;
      if ((u + 1) * BLOCK <= NITEMS || i < NITEMS) p1_store(i, rw[u], fl[u], pa[u]);
    }
  } else {
    for (int i = tid; i < R * C8; i += blockDim.x) {
      const int64_t pix = p1_pix(i);
      const uint4 rw = ld_nt_u4((const PR_GLOBAL uint4*)(raw + pix));
      const uint2 fl = *reinterpret_cast<const uint2*>(pflags + pix);
      float pa[NT][8];
      p1_ped(pix, p1_need(rw), pa);
      p1_store(i, rw, fl, pa);
    }
  }
  __syncthreads();

  // ---- phase 2a: rows by bank, one lane per segment ----------------------------------------
  // Non-participating elements are first marked NaN (a per-element select, no bit masks: 64-bit
  // mask extraction per element pushed the sorts into scratch), then turned into the balanced
  // -inf / +inf padding by a running counter.
  const float QNAN = __int_as_float(0x7fc00000);
  if (cp.flags & 1) {
    const int nbank = C / L;
    for (int sgi = tid; sgi < R * nbank; sgi += blockDim.x) {
      const int b = sgi / R, r = sgi % R;           // consecutive lanes -> consecutive rows: no bank conflicts
      float* seg = tile + r * LD + b * L;
      const uint32_t* nrow = nib + r * C8;
      // L % 8 == 0: the segment's eligibility bits are L/8 whole nibble words, read once and
      // indexed by compile-time j in both loops below
      constexpr int NW = (L % 8 == 0) ? L / 8 : 1;
      uint32_t nw[NW];
      if constexpr (L % 8 == 0) {
#pragma unroll
        for (int k = 0; k < NW; ++k) nw[k] = nrow[(b * L >> 3) + k];
      }
      auto elig = [&](int j) -> bool {
        if constexpr (L % 8 == 0) return (nw[j >> 3] >> (4 * (j & 7) + 3)) & 1u;
        const int col = b * L + j;
        return (nrow[col >> 3] >> (4 * (col & 7) + 3)) & 1u;
      };
      float x[L];
      int cnt = 0;
#pragma unroll
      for (int j = 0; j < L; ++j) {
        const float v = seg[j];
        const bool el = elig(j);
        const bool pt = el && (fabsf(v) < cp.thr);
        cnt += pt ? 1 : 0;
        x[j] = pt ? v : QNAN;
      }
      const int a = (L - cnt) >> 1;
      int ninv = 0;
#pragma unroll
      for (int j = 0; j < L; ++j) {
        const bool inv = x[j] != x[j];
        x[j] = inv ? (ninv < a ? -INF : INF) : x[j];
        ninv += inv ? 1 : 0;
      }
      asm volatile("" ::: "memory");   // keep the write-back's LDS reads below the sort (VGPR pressure)
      sort_regs<L>(x);
      asm volatile("" ::: "memory");
      // numpy median at fixed positions: lower = a + (cnt-1)/2, upper = a + cnt/2, which only
      // depend on the parity of cnt (L even: L/2-1 | L/2; L odd: (L-1)/2 | (L-3)/2,(L-1)/2)
      float s_lo, s_hi;
      if constexpr ((L & 1) == 0) {
        s_lo = x[L / 2 - 1];
        s_hi = (cnt & 1) ? x[L / 2 - 1] : x[L / 2];
      } else {
        s_lo = (cnt & 1) ? x[(L - 1) / 2] : x[(L - 3) / 2];
        s_hi = x[(L - 1) / 2];
      }
      const float med = (s_lo + s_hi) * 0.5f;
      if (cnt >= cp.npix_min && cnt > 0 && fabsf(med) <= cp.maxcorr) {
        // branch-free: every element is rewritten (v - 0 == v bitwise, -0 and NaN included), so
        // the 48 per-element exec-mask branches become selects
#pragma unroll
        for (int j = 0; j < L; ++j) {
          const float v = seg[j];
          seg[j] = v - (elig(j) ? med : 0.0f);
        }
      }
    }
    __syncthreads();
  }

  // ---- phase 2b (CQ = 4): columns, FOUR lanes (a quad) per column, M rows each ---------------
  //  each lane sorts its M values (sort_regs<M>); lanes (q, q^1) merge-split (lower lane keeps
  //  min(x[i], partner[M-1-i]), upper the max) and sort the resulting bitonic sequences (the
  //  lower lane negated so both are V-shaped: bitonic_merge_vpad); the two sorted halves of the
  //  pair (0,1) and of the pair (2,3) are then merged by merge-path for k = 2M-1 and 2M with ONE
  //  quad_perm(3,2,1,0) fetch per register.  Half the registers and half the serial comparator
  //  chain of the two-lane path; validated by a numpy emulation of the exact lane algorithm.
  if constexpr (CQ == 4) {
    if (cp.flags & 2) {
      const int nwork = 4 * C;
      for (int w = tid; w < ((nwork + 63) / 64) * 64; w += blockDim.x) {
        const bool act = w < nwork;
        const int c = act ? (w >> 2) : 0;
        const int q = w & 3;
        const bool lower = (q & 1) == 0;
        const uint32_t shift = 4 * (c & 7) + 3;
        // per-lane base addresses; the unrolled i then becomes an immediate LDS offset (i * LD,
        // i * C8 are constants for compile-time tile shapes)
        float* colp = tile + (q * M) * LD + c;
        const uint32_t* nibp = nib + (q * M) * C8 + (c >> 3);
        float x[M];
        int my_cnt = 0;
#pragma unroll
        for (int i = 0; i < M; ++i) {
          const bool in = act && q * M + i < R;
          const float v = in ? colp[i * LD] : 0.0f;
          const bool el = in && ((nibp[i * C8] >> shift) & 1u);
          const bool pt = el && (fabsf(v) < cp.thr);
          my_cnt += pt ? 1 : 0;
          x[i] = pt ? v : QNAN;
          if ((i & 15) == 15) asm volatile("" ::: "memory");
        }
        // quad totals + exclusive prefix of the non-participants: balanced +-inf padding
        const int my_inv = M - my_cnt;
        const int i0 = dpp_quad_i<0x00>(my_inv), i1 = dpp_quad_i<0x55>(my_inv);
        const int i2 = dpp_quad_i<0xAA>(my_inv), i3 = dpp_quad_i<0xFF>(my_inv);
        const int total_inv = i0 + i1 + i2 + i3;
        const int cnt = 4 * M - total_inv;
        const int a = total_inv >> 1;
        const int prefix = (q > 0 ? i0 : 0) + (q > 1 ? i1 : 0) + (q > 2 ? i2 : 0);
        const int neg_budget = min(my_inv, max(0, a - prefix));
        int ninv = 0;
#pragma unroll
        for (int i = 0; i < M; ++i) {
          const bool inv = x[i] != x[i];
          x[i] = inv ? (ninv < neg_budget ? -INF : INF) : x[i];
          ninv += inv ? 1 : 0;
        }
        asm volatile("" ::: "memory");
        sort_regs<M>(x);
        // level 1: merge-split with lane q^1 (partner read reversed)
        float z[M];
#pragma unroll
        for (int i = 0; i < M; ++i) {
          const float pv = dpp_quad<0xB1>(x[M - 1 - i]);
          const float y = lower ? fminf(x[i], pv) : fmaxf(x[i], pv);
          z[i] = lower ? -y : y;   // both lanes V-shaped
        }
        bitonic_merge_vpad<M>(z);
#pragma unroll
        for (int i = 0; i < M; ++i) x[i] = lower ? -z[M - 1 - i] : z[i];   // ascending half of the pair
        asm volatile("" ::: "memory");
        // level 2: merge-path of pair (0,1) with pair (2,3); lane 0 reads lane 3, lane 1 lane 2
        float k88 = INF, k87 = INF, plast = INF;
#pragma unroll
        for (int j = 0; j < M; ++j) {
          const float pj = dpp_quad<0x1B>(x[j]);
          k88 = fminf(k88, fmaxf(x[M - 1 - j], pj));
          if (j <= M - 2) k87 = fminf(k87, fmaxf(x[M - 2 - j], pj));
          if (j == M - 1) plast = pj;
        }
        const float e = dpp_quad<0xAA>(x[M - 1]);   // lane 2's last element
        const float extra = q == 0 ? fminf(plast, fmaxf(x[M - 1], e)) : x[M - 1];
        k87 = fminf(k87, extra);
        k87 = fminf(k87, dpp_quad<0xB1>(k87));
        k88 = fminf(k88, dpp_quad<0xB1>(k88));
        const float k_lo = dpp_quad<0x00>(k87), k_hi = dpp_quad<0x00>(k88);   // lane 0 has the answer
        const float med = (k_lo + ((cnt & 1) ? k_lo : k_hi)) * 0.5f;
        asm volatile("" ::: "memory");
        if (act) {   // branch-free per element (v - 0 == v bitwise), as in the row pass
          const float m = (cnt >= cp.npix_min && cnt > 0 && fabsf(med) <= cp.maxcorr) ? med : 0.0f;
#pragma unroll
          for (int i = 0; i < M; ++i) {
            if (q * M + i < R) {
              const float v = colp[i * LD];
              colp[i * LD] = v - (((nibp[i * C8] >> shift) & 1u) ? m : 0.0f);
            }
            if ((i & 15) == 15) asm volatile("" ::: "memory");
          }
        }
      }
      __syncthreads();
    }
  } else
  // ---- phase 2b (CQ = 2): columns, two lanes per column ------------------------------------
  if (cp.flags & 2) {
    const int nwork = 2 * C;
    for (int w = tid; w < ((nwork + 63) / 64) * 64; w += blockDim.x) {
      // whole waves iterate together (the DPP exchange needs both lanes of a pair)
      const bool act = w < nwork;
      const int c = act ? (w >> 1) : 0;
      const int h = w & 1;
      const uint32_t shift = 4 * (c & 7) + 3;
      float x[M];
      int my_cnt = 0;
#pragma unroll
      for (int i = 0; i < M; ++i) {
        const int r = h * M + i;
        const bool in = act && r < R;
        const float v = in ? tile[r * LD + c] : 0.0f;
        const bool el = in && ((nib[r * C8 + (c >> 3)] >> shift) & 1u);
        const bool pt = el && (fabsf(v) < cp.thr);
        my_cnt += pt ? 1 : 0;
        x[i] = pt ? v : QNAN;
        if ((i & 15) == 15) asm volatile("" ::: "memory");   // cap loads in flight (VGPR pressure)
      }
      const int other_cnt = __builtin_amdgcn_update_dpp(0, my_cnt, 0xB1, 0xF, 0xF, false);
      const int cnt = my_cnt + other_cnt;
      const int a = (2 * M - cnt) >> 1;
      const int my_inv = M - my_cnt, other_inv = M - other_cnt;
      // the even lane owns the first non-participating elements of the column
      const int neg_budget = h == 0 ? min(my_inv, a) : max(0, a - other_inv);
      int ninv = 0;
#pragma unroll
      for (int i = 0; i < M; ++i) {
        const bool inv = x[i] != x[i];
        x[i] = inv ? (ninv < neg_budget ? -INF : INF) : x[i];
        ninv += inv ? 1 : 0;
      }
      asm volatile("" ::: "memory");
      sort_regs<M>(x);
      asm volatile("" ::: "memory");
      // merge-path k-th of the union for k = M-1 and k = M (both lanes compute both)
      float k_lo = fminf(x[M - 1], dpp_xor1(x[M - 1]));   // i = M and i = 0 terms
      float k_hi = __int_as_float(0x7f800000);
#pragma unroll
      for (int i = 1; i < M; ++i) k_lo = fminf(k_lo, fmaxf(x[i - 1], dpp_xor1(x[M - 1 - i])));
#pragma unroll
      for (int i = 1; i <= M; ++i) k_hi = fminf(k_hi, fmaxf(x[i - 1], dpp_xor1(x[M - i])));
      // 2M slots: lower median at M-1; upper at M (even count) or M-1 (odd count)
      const float med = (k_lo + ((cnt & 1) ? k_lo : k_hi)) * 0.5f;
      asm volatile("" ::: "memory");
      if (act && cnt >= cp.npix_min && cnt > 0 && fabsf(med) <= cp.maxcorr) {
#pragma unroll
        for (int i = 0; i < M; ++i) {
          const int r = h * M + i;
          if (r < R && ((nib[r * C8 + (c >> 3)] >> shift) & 1u)) tile[r * LD + c] -= med;
          if ((i & 15) == 15) asm volatile("" ::: "memory");
        }
      }
    }
    __syncthreads();
  }

  // ---- phase 3: gain factor + mask, store ---------------------------------------------------
  cm_store<NT>(tile, nib, gf, tg, R, C, base, out, io, panel, ar * R, ac * C, cp.gather != 0);
}

// PSANA_RAY_CM_GENERIC=1 forces the generic wave-bitonic kernel (A/B benchmarking, read per launch)
static bool cm_force_generic() {
  const char* e = getenv("PSANA_RAY_CM_GENERIC");
  return e != nullptr && e[0] == '1';
}

size_t cm_lds_bytes(int asic_rows, int asic_cols) {
  const size_t tile = (((size_t)asic_rows * (asic_cols + 1) * 4) + 15) & ~(size_t)15;
  return tile + (size_t)asic_rows * (asic_cols / 8) * 4;
}

// Width of the LDS tile a workgroup owns.  Row medians are per bank segment and column medians
// need whole columns, so an ASIC may be cut into full-height stripes whose width is a multiple
// of the bank width without changing any median (Jungfrau: 256x256 ASIC = 289 KB > 160 KiB ->
// two 256x128 stripes of 145 KB).  0 = no stripe fits.
int cm_tile_cols(int asic_rows, int asic_cols, int bank_cols, int max_cols) {
  for (int w = std::min(asic_cols, max_cols > 0 ? max_cols : asic_cols); w >= bank_cols; --w) {
    if (asic_cols % w || w % bank_cols || w % 8) continue;
    if (cm_lds_bytes(asic_rows, w) <= 160 * 1024) return w;
  }
  return 0;
}

void launch_calib_cm(const FramePtrs& fp, int nframes, uint64_t ped, uint64_t gf, uint64_t pflags,
                     int kind, int n_panels, int panel_rows, int panel_cols, int asic_rows,
                     int asic_cols, float thr, float maxcorr, int npix_min, int flags,
                     int bank_cols, uint64_t stream, uint64_t img_desc, uint64_t img_omask) {
  check(nframes >= 1 && nframes <= kMaxFrames, "calib_cm: nframes out of range");
  check(asic_rows >= 1 && asic_rows <= 256, "calib_cm: ASIC rows must be in [1, 256]");
  check(asic_cols % 8 == 0 && asic_cols >= 8, "calib_cm: ASIC cols must be a multiple of 8");
  check(panel_rows % asic_rows == 0 && panel_cols % asic_cols == 0, "calib_cm: panel not tiled by ASICs");
  check(bank_cols >= 1 && bank_cols <= 64 && asic_cols % bank_cols == 0,
        "calib_cm: bank_cols must be <= 64 and divide the ASIC width");
  check(panel_cols % 8 == 0, "calib_cm: panel cols must be a multiple of 8");
  // stripe width: PSANA_RAY_CM_STRIPE caps it (A/B); a stripe of <= 128 columns runs 256-thread
  // workgroups, two of which fit one CU (LDS <= 80 KB each), so one block's HBM phases overlap
  // the other's sorts (one 512-thread block per CU cannot overlap anything)
  // Default: the widest stripe <= 128 columns whose tile fits half the LDS, when a sort-network
  // instantiation exists for it (epix10k2M: 176x96 stripes, 15.29 vs 15.82 us/frame full width,
  // 48 columns 22.8; profiles/kernels_r1_cm_stripes.jsonl).
  const int Mh = (asic_rows + 1) / 2;
  const bool net256 = !cm_force_generic() &&
      ((kind == kEpix10ka && bank_cols == 48 && Mh == 88) || (kind == kEpix10ka && bank_cols == 8 && Mh == 8) ||
       (kind == kPlain && bank_cols == 32 && Mh == 64) || (kind == kPlain && bank_cols == 8 && Mh == 4));
  int max_w = 0;
  if (net256) {
    for (int w = std::min(asic_cols, 128); w >= bank_cols; --w)
      if (asic_cols % w == 0 && w % bank_cols == 0 && w % 8 == 0 && cm_lds_bytes(asic_rows, w) <= 80 * 1024) {
        max_w = w;
        break;
      }
  }
  // PSANA_RAY_CM_CONSTDIMS=0 skips the compile-time-shape instantiations (A/B)
  const char* cd = getenv("PSANA_RAY_CM_CONSTDIMS");
  const bool const_dims = !(cd != nullptr && cd[0] == '0');
  // epix10k2M with the compile-time kernels: one-bank 176x48 stripes on 256-thread blocks, four
  // per CU (8.78 vs 9.16 us/frame for 176x96; profiles/kernels_r1_cm_stripes48.jsonl)
  if (const_dims && kind == kEpix10ka && bank_cols == 48 && asic_rows == 176 && asic_cols % 48 == 0) max_w = 48;
  if (const char* e = getenv("PSANA_RAY_CM_STRIPE"); e && *e) max_w = std::max(0, atoi(e));   // 0: full width
  const int full_cols = asic_cols;
  asic_cols = cm_tile_cols(asic_rows, full_cols, bank_cols, max_w);
  if (asic_cols == 0) asic_cols = cm_tile_cols(asic_rows, full_cols, bank_cols, 0);
  check(asic_cols > 0, "calib_cm: no full-height ASIC stripe fits in 160 KiB of LDS");
  const size_t lds = cm_lds_bytes(asic_rows, asic_cols);
  check(aligned16(ped) && aligned16(gf) && (pflags & 7) == 0, "calib_cm: misaligned constant tables");
  for (int f = 0; f < nframes; ++f)
    check(aligned16(fp.in[f]) && aligned16(fp.out[f]), "calib_cm: frame buffers must be 16-B aligned");
  const ImgOut io{reinterpret_cast<const int32_t*>(img_desc), reinterpret_cast<const uint8_t*>(img_omask)};
  check(img_omask == 0 || img_desc != 0, "calib_cm: an image mask needs the image output map");
  TileGeom tg;
  tg.panel_rows = panel_rows;
  tg.panel_cols = panel_cols;
  tg.asic_rows = asic_rows;
  tg.asic_cols = asic_cols;
  tg.asics_per_col = panel_rows / asic_rows;
  tg.asics_per_row = panel_cols / asic_cols;
  tg.npix = (int64_t)n_panels * panel_rows * panel_cols;
  CmParams cp{thr, maxcorr, npix_min, flags, bank_cols, 1};
  if (const char* e = getenv("PSANA_RAY_CM_GATHER"); e && *e) cp.gather = atoi(e) != 0;   // A/B
  tg.nframes = nframes;
  {
    // XCD-aware placement is OFF by default: measured slower (sort nets 17.4 vs 15.8 us/frame,
    // memory phases alone 6.5 vs 4.9; profiles/kernels_r1_cm_swizzle.jsonl) -- the per-ASIC tables
    // are already cache-served under round-robin placement.  PSANA_RAY_CM_SWZ=1 turns it on (A/B).
    const char* e = getenv("PSANA_RAY_CM_SWZ");
    tg.swizzle = (e != nullptr && e[0] == '1') ? 1 : 0;
  }
  const dim3 grid((unsigned)(n_panels * tg.asics_per_col * tg.asics_per_row * nframes));
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const float* P = reinterpret_cast<const float*>(ped);
  const float* G = reinterpret_cast<const float*>(gf);
  const uint8_t* F = reinterpret_cast<const uint8_t*>(pflags);
  const int M = (asic_rows + 1) / 2;
  bool done = false;
  const bool narrow = asic_cols <= 128;   // 2 lanes per column fit a 256-thread block
  // lanes per column: 4 (quad merge, <= 128 VGPRs, 4 waves/SIMD) unless PSANA_RAY_CM_COLQ=2 (A/B)
  int cq_req = 0;
  if (const char* e = getenv("PSANA_RAY_CM_COLQ"); e && *e) cq_req = atoi(e);
  const int M2 = (asic_rows + 1) / 2, M4 = (asic_rows + 3) / 4;
#define PR_CM_NET_T(KIND_, L_, M_, B_, CQ_, TR_, TC_)                                                   \
  if (!done && kind == KIND_ && bank_cols == L_ && (CQ_ == 4 ? M4 : M2) == M_ &&                        \
      (cq_req == 0 || cq_req == CQ_) && B_ == (narrow ? 256 : 512) * (CQ_ / 2) && !cm_force_generic() && \
      ((TR_ == 0 && TC_ == 0) || (const_dims && TR_ == asic_rows && TC_ == asic_cols))) {               \
    hip_check(hipFuncSetAttribute((const void*)calib_cm_net_kernel<KIND_, L_, M_, B_, CQ_, TR_, TC_>,   \
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds), "cm attr");   \
    hipLaunchKernelGGL((calib_cm_net_kernel<KIND_, L_, M_, B_, CQ_, TR_, TC_>), grid, dim3(B_), lds, s, fp, P, G, \
                       F, tg, cp, io);                                                                \
    done = true;                                                                                      \
  }
#define PR_CM_NET(KIND_, L_, M_, B_, CQ_) PR_CM_NET_T(KIND_, L_, M_, B_, CQ_, 0, 0)
  // epix10k2M 176x48 stripes (PSANA_RAY_CM_STRIPE=48): 256-thread blocks (176 row segments,
  // 192 column lanes), 38.7 KB LDS -> four workgroups per CU
  if (!done && const_dims && !cm_force_generic() && (cq_req == 0 || cq_req == 4) && kind == kEpix10ka &&
      bank_cols == 48 && asic_rows == 176 && asic_cols == 48) {
    // (192-thread blocks measured slower: 9.45 vs 8.82 us/frame; profiles/kernels_r1_cm_b48.jsonl)
    hip_check(hipFuncSetAttribute((const void*)calib_cm_net_kernel<kEpix10ka, 48, 44, 256, 4, 176, 48>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds), "cm attr");
    hipLaunchKernelGGL((calib_cm_net_kernel<kEpix10ka, 48, 44, 256, 4, 176, 48>), grid, dim3(256), lds, s, fp, P, G,
                       F, tg, cp, io);
    done = true;
  }
  PR_CM_NET_T(kEpix10ka, 48, 44, 512, 4, 176, 96)    // epix10k2M: 176x96 stripes
  PR_CM_NET_T(kJungfrau, 64, 64, 512, 4, 256, 128)   // Jungfrau: 256x128 stripes
  PR_CM_NET(kEpix10ka, 48, 44, 512, 4)
  PR_CM_NET(kEpix10ka, 48, 44, 1024, 4)
  PR_CM_NET(kEpix10ka, 48, 88, 512, 2)
  PR_CM_NET(kEpix10ka, 48, 88, 256, 2)
  PR_CM_NET(kEpix10ka, 8, 4, 512, 4)
  PR_CM_NET(kEpix10ka, 8, 8, 256, 2)
  PR_CM_NET(kJungfrau, 64, 64, 512, 4)
  PR_CM_NET(kPlain, 32, 32, 512, 4)
  PR_CM_NET(kPlain, 32, 64, 256, 2)
  PR_CM_NET(kPlain, 8, 4, 256, 2)
#undef PR_CM_NET
#undef PR_CM_NET_T
  if (!done) {
  switch (kind) {
    case kEpix10ka:
      hip_check(hipFuncSetAttribute((const void*)calib_cm_kernel<kEpix10ka>,
                                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds), "cm attr");
      hipLaunchKernelGGL(calib_cm_kernel<kEpix10ka>, grid, dim3(1024), lds, s, fp, P, G, F, tg, cp, io);
      break;
    case kJungfrau:
      hip_check(hipFuncSetAttribute((const void*)calib_cm_kernel<kJungfrau>,
                                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds), "cm attr");
      hipLaunchKernelGGL(calib_cm_kernel<kJungfrau>, grid, dim3(1024), lds, s, fp, P, G, F, tg, cp, io);
      break;
    case kPlain:
      hip_check(hipFuncSetAttribute((const void*)calib_cm_kernel<kPlain>,
                                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds), "cm attr");
      hipLaunchKernelGGL(calib_cm_kernel<kPlain>, grid, dim3(1024), lds, s, fp, P, G, F, tg, cp, io);
      break;
    default: check(false, "calib_cm: unknown gain kind");
  }
  }
  hip_check(hipGetLastError(), "calib_cm launch");
}

}  // namespace pr
