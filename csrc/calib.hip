// K-01 / K-02 / K-04: fused gain-decode + pedestal subtraction + gain factor + pixel mask.
// K-05 (fused variant): the same math evaluated directly at assembled-image positions.
//
// Reference parity: psana-ray never calibrates itself; it receives already calibrated frames
// from psana_wrapper.iter_events(mode) (psana_ray/producer.py:88, mode chosen at :156-159) and
// then applies `np.where(mask, data, 0)` (producer.py:92-95).  Here the whole chain is one
// memory-bound streaming pass on the GPU.
//
// Design (MI355X):
//  * one thread owns 4 consecutive pixels: one 8-B raw load + one 16-B f32 store per frame, so
//    consecutive lanes write consecutive 16 B (whole 128-B lines per store instruction).
//  * the per-pixel constants (pedestal and gain-factor for every candidate gain, the mask
//    folded into the gain factor) are loaded ONCE per thread and reused for every frame of the
//    batch (up to kMaxFrames per launch), so constant traffic is amortised over the batch and
//    the kernel streams raw-in + f32-out only: 6 B / pixel / frame.
//  * per-frame pointers travel in the kernel-argument block, so outputs can be scattered HBM
//    ring slots (no packing copy).
#include "common.h"

#include <algorithm>

namespace pr {

template <int KIND>
struct KindTraits;
template <>
struct KindTraits<kEpix10ka> { static constexpr int NT = 2; };
template <>
struct KindTraits<kJungfrau> { static constexpr int NT = 3; };
template <>
struct KindTraits<kPlain> { static constexpr int NT = 1; };

// 4-pixel-per-lane layout: 8-B raw loads and 16-B stores, consecutive lanes on consecutive
// 16-B output chunks, so every store instruction writes 1 KB contiguous (whole 128-B lines).
template <int NT>
__device__ __forceinline__ void load_tab4(const float* __restrict__ tab, int64_t npix, int64_t pix0,
                                          float (&t)[NT][4]) {
#pragma unroll
  for (int k = 0; k < NT; ++k) {
    const float4 a = *reinterpret_cast<const float4*>(tab + k * npix + pix0);
    t[k][0] = a.x; t[k][1] = a.y; t[k][2] = a.z; t[k][3] = a.w;
  }
}

template <int KIND, int NT>
__device__ __forceinline__ float4 calib4(const uint2 r, const float (&p)[NT][4], const float (&g)[NT][4]) {
  const uint32_t w[2] = {r.x, r.y};
  float o[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint32_t raw = (w[i >> 1] >> (16 * (i & 1))) & 0xFFFFu;
    bool valid;
    const int c = decode_cand(raw, KIND, valid);
    float pp, gg;
    if constexpr (NT == 1) {
      pp = p[0][i]; gg = g[0][i];
    } else if constexpr (NT == 2) {
      pp = bsel(c != 0, p[1][i], p[0][i]); gg = bsel(c != 0, g[1][i], g[0][i]);
    } else {
      pp = bsel(c == 0, p[0][i], bsel(c == 1, p[1][i], p[2][i]));
      gg = bsel(c == 0, g[0][i], bsel(c == 1, g[1][i], g[2][i]));
    }
    const float v = gmul(decode_adu(raw, KIND) - pp, gg);
    o[i] = valid ? v : 0.0f;
  }
  return make_float4(o[0], o[1], o[2], o[3]);
}

template <int KIND>
__global__ __launch_bounds__(256) void calib_basic4_kernel(const FramePtrs fp, const int nframes,
                                                           const float* __restrict__ ped,
                                                           const float* __restrict__ gf,
                                                           const int64_t npix, const int fpb) {
  constexpr int NT = KindTraits<KIND>::NT;
  const int64_t nq = npix >> 2;
  const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (q >= nq) return;
  const int f_begin = blockIdx.y * fpb;
  const int f_end = min(nframes, f_begin + fpb);
  const int64_t pix0 = q * 4;
  float p[NT][4], g[NT][4];
  load_tab4<NT>(ped, npix, pix0, p);
  load_tab4<NT>(gf, npix, pix0, g);
  int f = f_begin;
  for (; f + 8 <= f_end; f += 8) {
    uint2 r[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      r[k] = ld_nt_u2(gin<uint2>(fp.in[f + k]) + q);
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) st_f4(gout<float4>(fp.out[f + k]) + q, calib4<KIND, NT>(r[k], p, g));
  }
  for (; f < f_end; ++f) {
    st_f4(gout<float4>(fp.out[f]) + q, calib4<KIND, NT>(ld_nt_u2(gin<uint2>(fp.in[f]) + q), p, g));
  }
}

// Bandwidth reference for the same traffic mix (u16 in, f32 out, no calibration math).
__global__ __launch_bounds__(256) void convert_u16_f32_kernel(const FramePtrs fp, const int nframes,
                                                              const int64_t npix) {
  const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (q >= (npix >> 2)) return;
  for (int f = blockIdx.y * 8; f < min(nframes, (int)blockIdx.y * 8 + 8); ++f) {
    const uint2 x = ld_nt_u2(gin<uint2>(fp.in[f]) + q);
    st_f4(gout<float4>(fp.out[f]) + q,
          make_float4((float)(x.x & 0xFFFF), (float)(x.x >> 16), (float)(x.y & 0xFFFF), (float)(x.y >> 16)));
  }
}

void launch_convert_u16_f32(const FramePtrs& fp, int nframes, int64_t npix, uint64_t stream) {
  const dim3 grid((unsigned)((npix / 4 + 255) / 256), (unsigned)((nframes + 7) / 8));
  hipLaunchKernelGGL(convert_u16_f32_kernel, grid, dim3(256), 0, reinterpret_cast<hipStream_t>(stream), fp, nframes,
                     npix);
  hip_check(hipGetLastError(), "convert launch");
}

// Read-only bandwidth reference (what a frame-reading consumer kernel can reach): K float4 per
// lane, block reduction, one atomic per block.  NT = nontemporal loads.
template <int K, bool NT>
__global__ __launch_bounds__(256) void read_f32_kernel(const FramePtrs fp, const int64_t n4, float* __restrict__ sums) {
  __shared__ float red[4];
  const int f = blockIdx.y;
  const int64_t q0 = (int64_t)blockIdx.x * 256 * K + threadIdx.x;
  const PR_GLOBAL f32x4_t* in = gin<f32x4_t>(fp.in[f]);
  float acc = 0.0f;
  if ((int64_t)(blockIdx.x + 1) * 256 * K <= n4) {
    f32x4_t v[K];
#pragma unroll
    for (int k = 0; k < K; ++k) v[k] = NT ? ld_nt_f4(in + q0 + 256 * k) : in[q0 + 256 * k];
#pragma unroll
    for (int k = 0; k < K; ++k) acc += (v[k].x + v[k].y) + (v[k].z + v[k].w);
  } else {
    for (int k = 0; k < K; ++k)
      if (q0 + 256 * k < n4) {
        const f32x4_t v = in[q0 + 256 * k];
        acc += (v.x + v.y) + (v.z + v.w);
      }
  }
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_down(acc, o);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(sums + f, red[0] + red[1] + red[2] + red[3]);
}

void launch_read_f32(const FramePtrs& fp, int nframes, int64_t npix, int k, bool nt, uint64_t sums, uint64_t stream) {
  check(nframes >= 1 && nframes <= kMaxFrames && npix % 4 == 0, "read_f32: bad arguments");
  const int64_t n4 = npix / 4;
  const dim3 grid((unsigned)((n4 + 256 * k - 1) / (256 * k)), (unsigned)nframes);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  float* S = reinterpret_cast<float*>(sums);
#define PR_RD(K_, NT_) hipLaunchKernelGGL((read_f32_kernel<K_, NT_>), grid, dim3(256), 0, s, fp, n4, S)
  if (k == 4) { if (nt) PR_RD(4, true); else PR_RD(4, false); }
  else if (k == 8) { if (nt) PR_RD(8, true); else PR_RD(8, false); }
  else { check(k == 16, "read_f32: k must be 4, 8 or 16"); if (nt) PR_RD(16, true); else PR_RD(16, false); }
#undef PR_RD
  hip_check(hipGetLastError(), "read_f32 launch");
}

// Fused raw -> assembled image (image mode without common mode).  One thread owns 4
// consecutive output pixels; idx[o] is the flat source pixel of output o or -1 (gap).
// Constants are gathered once per thread and reused over the frame batch.
template <int KIND>
__global__ __launch_bounds__(256) void calib_image_kernel(const FramePtrs fp, const int nframes,
                                                          const float* __restrict__ ped,
                                                          const float* __restrict__ gf,
                                                          const int64_t npix,
                                                          const int32_t* __restrict__ idx,
                                                          const int64_t nout) {
  constexpr int NT = KindTraits<KIND>::NT;
  const int64_t o0 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
  if (o0 >= nout) return;
  int32_t src[4];
  float p[NT][4], g[NT][4];
  const bool full = (o0 + 4 <= nout);
  if (full) {
    const int4 s = *reinterpret_cast<const int4*>(idx + o0);
    src[0] = s.x; src[1] = s.y; src[2] = s.z; src[3] = s.w;
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i) src[i] = (o0 + i < nout) ? idx[o0 + i] : -1;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
#pragma unroll
    for (int k = 0; k < NT; ++k) {
      p[k][i] = src[i] >= 0 ? ped[k * npix + src[i]] : 0.0f;
      g[k][i] = src[i] >= 0 ? gf[k * npix + src[i]] : 0.0f;
    }
  }
  for (int f = 0; f < nframes; ++f) {
    const PR_GLOBAL uint16_t* raw = gin<uint16_t>(fp.in[f]);
    float o[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float val = 0.0f;
      if (src[i] >= 0) {
        const uint32_t r = raw[src[i]];
        bool valid;
        const int c = decode_cand(r, KIND, valid);
        float pp, gg;
        if constexpr (NT == 1) {
          pp = p[0][i]; gg = g[0][i];
        } else if constexpr (NT == 2) {
          pp = bsel(c != 0, p[1][i], p[0][i]); gg = bsel(c != 0, g[1][i], g[0][i]);
        } else {
          pp = bsel(c == 0, p[0][i], bsel(c == 1, p[1][i], p[2][i]));
          gg = bsel(c == 0, g[0][i], bsel(c == 1, g[1][i], g[2][i]));
        }
        val = valid ? gmul(decode_adu(r, KIND) - pp, gg) : 0.0f;
      }
      o[i] = val;
    }
    PR_GLOBAL float* out = gout<float>(fp.out[f]);
    if (full) {
      st_f4((PR_GLOBAL float4*)(out + o0), make_float4(o[0], o[1], o[2], o[3]));
    } else {
      for (int i = 0; i < 4 && o0 + i < nout; ++i) out[o0 + i] = o[i];
    }
  }
}

// ---------------------------------------------------------------------------------------
// host launchers
// ---------------------------------------------------------------------------------------
void launch_calib_basic(const FramePtrs& fp, int nframes, uint64_t ped, uint64_t gf, int64_t npix,
                        int kind, uint64_t stream) {
  check(nframes >= 1 && nframes <= kMaxFrames, "calib_basic: nframes out of range");
  check(npix % 8 == 0, "calib_basic: npix must be a multiple of 8");
  check(aligned16(ped) && aligned16(gf), "calib_basic: constant tables must be 16-B aligned");
  for (int f = 0; f < nframes; ++f)
    check(aligned16(fp.in[f]) && aligned16(fp.out[f]), "calib_basic: frame buffers must be 16-B aligned");
  // 4 pixels per lane (8-B raw loads, 16-B stores, every store instruction writes 1 KiB
  // contiguous) and the whole batch per block: the tables are loaded once per lane and reused for
  // every frame (round 1 A/B: 2.42 us/frame vs 2.72 for 8 px per lane in groups of 8 frames,
  // profiles/kernels_r1.jsonl)
  const int fpb = kMaxFrames;
  const dim3 g4((unsigned)((npix / 4 + 255) / 256), (unsigned)((nframes + fpb - 1) / fpb));
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const float* P = reinterpret_cast<const float*>(ped);
  const float* G = reinterpret_cast<const float*>(gf);
  switch (kind) {
    case kEpix10ka: hipLaunchKernelGGL(calib_basic4_kernel<kEpix10ka>, g4, dim3(256), 0, s, fp, nframes, P, G, npix, fpb); break;
    case kJungfrau: hipLaunchKernelGGL(calib_basic4_kernel<kJungfrau>, g4, dim3(256), 0, s, fp, nframes, P, G, npix, fpb); break;
    case kPlain: hipLaunchKernelGGL(calib_basic4_kernel<kPlain>, g4, dim3(256), 0, s, fp, nframes, P, G, npix, fpb); break;
    default: check(false, "calib_basic: unknown gain kind");
  }
  hip_check(hipGetLastError(), "calib_basic launch");
}

void launch_calib_image(const FramePtrs& fp, int nframes, uint64_t ped, uint64_t gf, int64_t npix,
                        int kind, uint64_t idx, int64_t nout, uint64_t stream) {
  check(nframes >= 1 && nframes <= kMaxFrames, "calib_image: nframes out of range");
  check(aligned16(idx), "calib_image: index map must be 16-B aligned");
  for (int f = 0; f < nframes; ++f) check(aligned16(fp.out[f]), "calib_image: outputs must be 16-B aligned");
  const int64_t nthr = (nout + 3) / 4;
  const dim3 grid((unsigned)((nthr + 255) / 256));
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const float* P = reinterpret_cast<const float*>(ped);
  const float* G = reinterpret_cast<const float*>(gf);
  const int32_t* I = reinterpret_cast<const int32_t*>(idx);
  switch (kind) {
    case kEpix10ka: hipLaunchKernelGGL(calib_image_kernel<kEpix10ka>, grid, dim3(256), 0, s, fp, nframes, P, G, npix, I, nout); break;
    case kJungfrau: hipLaunchKernelGGL(calib_image_kernel<kJungfrau>, grid, dim3(256), 0, s, fp, nframes, P, G, npix, I, nout); break;
    case kPlain: hipLaunchKernelGGL(calib_image_kernel<kPlain>, grid, dim3(256), 0, s, fp, nframes, P, G, npix, I, nout); break;
    default: check(false, "calib_image: unknown gain kind");
  }
  hip_check(hipGetLastError(), "calib_image launch");
}

}  // namespace pr
