// K-05 geometry assembly by LDS-staged tiles (image mode: the reference's DEFAULT retrieval mode,
// psana_ray/producer.py:22,156-159).
//
// A plain gather (assemble.hip: one source index per output pixel) reads the rotated panels of
// a pinwheel detector column-wise: consecutive output pixels are a whole panel row apart in the
// source, so every lane touches its own cache line (measured 16 us/frame for epix10k2M, 5x its
// streaming bound).  Here the host cuts the image into 32x64 output tiles and, for each, finds
// the dominant panel and the bounding box of the source pixels it needs (TileDesc; <= 2048 px:
// a 90-degree-rotated 32x64 tile is a 64x32 source box).  A 256-thread workgroup
//   1. stages the box into LDS with row-contiguous (coalesced) source reads -- calibrating raw
//      ADU on the way in for the fused path, the per-pixel pedestal/gain candidates held in
//      registers across the whole frame batch;
//   2. writes the output tile row-major (coalesced 256-B wave stores), each output pixel reading
//      the LDS word its precomputed code names.
// The box is stored with a (w+1)-word row pitch so the column walks of rotated tiles hit
// distinct banks.  Codes: >= 0 LDS offset, -1 gap / masked (0.0), <= -2 a source pixel outside
// the box (another panel at a tile border, or an irregular geometry), read directly.
// The image-space mask is folded into the codes on the host, so masked pixels cost nothing.
#include "common.h"

#include <type_traits>

namespace pr {

constexpr int kImgTH = 32, kImgTW = 64, kImgStage = 2048, kImgLds = 2176;

struct ImgGeom {
  int panel_rows, panel_cols;
  int img_h, img_w;
  int tiles_x;
  int64_t npix;
};

template <int KIND>
struct ImgTraits;
template <>
struct ImgTraits<kEpix10ka> { static constexpr int NT = 2; };
template <>
struct ImgTraits<kJungfrau> { static constexpr int NT = 3; };
template <>
struct ImgTraits<kPlain> { static constexpr int NT = 1; };

template <int NT>
__device__ __forceinline__ float img_pick(const float (&t)[NT], int c) {
  if constexpr (NT == 1) {
    return t[0];
  } else if constexpr (NT == 2) {
    return bsel(c != 0, t[1], t[0]);
  } else {
    return bsel(c == 0, t[0], bsel(c == 1, t[1], t[2]));
  }
}

// CALIB = true: in = raw u16 frames, calibrate (K-01/02/04) while staging.
// CALIB = false: in = calibrated f32 frames (after common mode), pure assembly.
template <int KIND, bool CALIB, int BLOCK>
__global__ __launch_bounds__(BLOCK) void image_tile_kernel(const FramePtrs fp, const int f0, const int f1,
                                                         const float* __restrict__ ped,
                                                         const float* __restrict__ gf,
                                                         const int32_t* __restrict__ tiles,   // [n][8]
                                                         const int32_t* __restrict__ codes,   // [img_h*img_w]
                                                         const ImgGeom g) {
  constexpr int NT = ImgTraits<KIND>::NT;
  constexpr int SJ = kImgStage / BLOCK;            // staged pixels per thread
  constexpr int OK = kImgTH * kImgTW / BLOCK;      // output pixels per thread
  __shared__ float stage[kImgLds];

  const int t = blockIdx.x;
  const int fa = f0 + (int)blockIdx.y * (f1 - f0 + (int)gridDim.y - 1) / (int)gridDim.y;
  const int fb = min(f1, f0 + ((int)blockIdx.y + 1) * (f1 - f0 + (int)gridDim.y - 1) / (int)gridDim.y);
  const int ty0 = (t / g.tiles_x) * kImgTH, tx0 = (t % g.tiles_x) * kImgTW;
  const int4 d = *reinterpret_cast<const int4*>(tiles + 8 * t);       // panel, r0, c0, h
  const int bw = tiles[8 * t + 4];                                     // w
  const int panel = d.x, r0 = d.y, c0 = d.z, bh = d.w;
  const int tid = threadIdx.x;

  // staged pixels of this thread: box index i -> (r, c) -> flat source pixel + LDS offset
  int32_t src[SJ], lds[SJ];
  float p[SJ][NT], q[SJ][NT];
#pragma unroll
  for (int j = 0; j < SJ; ++j) {
    const int i = tid + BLOCK * j;
    src[j] = -1;
    lds[j] = 0;
    if (panel >= 0 && i < bh * bw) {
      const int r = i / bw, c = i - (i / bw) * bw;
      src[j] = (int32_t)((int64_t)panel * g.panel_rows * g.panel_cols + (int64_t)(r0 + r) * g.panel_cols + c0 + c);
      lds[j] = r * (bw + 1) + c;
    }
    if constexpr (CALIB) {
#pragma unroll
      for (int k = 0; k < NT; ++k) {
        p[j][k] = src[j] >= 0 ? ped[k * g.npix + src[j]] : 0.0f;
        q[j][k] = src[j] >= 0 ? gf[k * g.npix + src[j]] : 0.0f;
      }
    }
  }
  // output pixels of this thread: (ty0 + tid/64 + 4k, tx0 + tid%64), k < 8 -- a wave covers 64
  // consecutive columns of one row, so stores are 256-B contiguous
  const int oy0 = ty0 + (tid >> 6), ox = tx0 + (tid & 63);
  const int64_t obase = (int64_t)oy0 * g.img_w + ox;
  const int64_t ostep = (int64_t)(BLOCK / kImgTW) * g.img_w;
  int32_t code[OK];
  unsigned valid_mask = 0;
#pragma unroll
  for (int k = 0; k < OK; ++k) {
    const bool in = ox < g.img_w && oy0 + (BLOCK / kImgTW) * k < g.img_h;
    valid_mask |= (unsigned)in << k;
    code[k] = in ? codes[obase + k * ostep] : -1;
  }

  // software pipeline: frame f+1's source words are loaded into registers while frame f is
  // written out (plain loads stay in flight across the LDS barriers)
  using InT = typename std::conditional<CALIB, uint16_t, float>::type;
  InT cur[SJ], nxt[SJ];
  auto load_frame = [&](int f, InT (&dst)[SJ]) {
    const PR_GLOBAL InT* in = gin<InT>(fp.in[f]);
#pragma unroll
    for (int j = 0; j < SJ; ++j) dst[j] = src[j] >= 0 ? in[src[j]] : InT(0);
  };
  if (fa < fb) load_frame(fa, nxt);
  for (int f = fa; f < fb; ++f) {
#pragma unroll
    for (int j = 0; j < SJ; ++j) cur[j] = nxt[j];
    if (f + 1 < fb) load_frame(f + 1, nxt);
#pragma unroll
    for (int j = 0; j < SJ; ++j) {
      if (src[j] < 0) continue;
      float v;
      if constexpr (CALIB) {
        const uint32_t r = cur[j];
        bool valid;
        const int c = decode_cand(r, KIND, valid);
        v = valid ? gmul(decode_adu(r, KIND) - img_pick<NT>(p[j], c), img_pick<NT>(q[j], c)) : 0.0f;
      } else {
        v = cur[j];
      }
      stage[lds[j]] = v;
    }
    __syncthreads();
    PR_GLOBAL float* out = gout<float>(fp.out[f]);
#pragma unroll
    for (int k = 0; k < OK; ++k) {
      if (!((valid_mask >> k) & 1u)) continue;
      const int cd = code[k];
      float v = 0.0f;
      if (cd >= 0) {
        v = stage[cd];
      } else if (cd <= -2) {   // outside the staged box: direct read (tile borders only)
        const int64_t s = (int64_t)(-(cd + 2));
        if constexpr (CALIB) {
          const uint32_t r = gin<uint16_t>(fp.in[f])[s];
          bool valid;
          const int c = decode_cand(r, KIND, valid);
          float pp[NT], qq[NT];
#pragma unroll
          for (int m = 0; m < NT; ++m) {
            pp[m] = ped[m * g.npix + s];
            qq[m] = gf[m * g.npix + s];
          }
          v = valid ? gmul(decode_adu(r, KIND) - img_pick<NT>(pp, c), img_pick<NT>(qq, c)) : 0.0f;
        } else {
          v = gin<float>(fp.in[f])[s];
        }
      }
      out[obase + k * ostep] = v;
    }
    __syncthreads();
  }
}

int image_tile_h() { return kImgTH; }
int image_tile_w() { return kImgTW; }
int image_tile_stage() { return kImgStage; }

// frames [0, nframes) of fp; calib: raw -> image, else f32 frames -> image
void launch_image_tiles(const FramePtrs& fp, int nframes, bool calib, int kind, uint64_t ped, uint64_t gf,
                        int64_t npix, int panel_rows, int panel_cols, uint64_t tiles, int n_tiles, int tiles_x,
                        uint64_t codes, int img_h, int img_w, uint64_t stream) {
  check(nframes >= 1 && nframes <= kMaxFrames, "image_tiles: nframes out of range");
  check(tiles != 0 && codes != 0 && aligned16(tiles), "image_tiles: tile map missing or misaligned");
  check(tiles_x == (img_w + kImgTW - 1) / kImgTW && n_tiles == tiles_x * ((img_h + kImgTH - 1) / kImgTH),
        "image_tiles: tile grid does not match the image");
  check(npix < (int64_t)1 << 31, "image_tiles: frames above 2^31 pixels");
  if (calib) check(ped != 0 && gf != 0, "image_tiles: calibration tables missing");
  ImgGeom g{panel_rows, panel_cols, img_h, img_w, tiles_x, npix};
  // frame groups: tables are loaded once per block and reused over its frames, but a block walks
  // its frames serially, so more groups = more blocks in flight (epix10k2M, 1250 tiles, 32 frames:
  // 1 group 7.98, 2: 6.45, 4: 5.94, 8: 6.42 us/frame; profiles/kernels_r1_image.jsonl)
  const int groups = std::min(n_tiles >= 8192 ? 1 : (n_tiles >= 4096 ? 2 : 4), nframes);
  const dim3 grid((unsigned)n_tiles, (unsigned)groups);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const float* P = reinterpret_cast<const float*>(ped);
  const float* G = reinterpret_cast<const float*>(gf);
  const int32_t* T = reinterpret_cast<const int32_t*>(tiles);
  const int32_t* Cd = reinterpret_cast<const int32_t*>(codes);
  // 512-thread blocks: half the per-thread staged pixels / codes of 256 (fewer VGPRs, more waves
  // in flight; round-1 A/B)
#define PR_IMG(K, CAL) \
  hipLaunchKernelGGL((image_tile_kernel<K, CAL, 512>), grid, dim3(512), 0, s, fp, 0, nframes, P, G, T, Cd, g)
  if (calib) {
    switch (kind) {
      case kEpix10ka: PR_IMG(kEpix10ka, true); break;
      case kJungfrau: PR_IMG(kJungfrau, true); break;
      case kPlain: PR_IMG(kPlain, true); break;
      default: check(false, "image_tiles: unknown gain kind");
    }
  } else {
    PR_IMG(kPlain, false);
  }
#undef PR_IMG
  hip_check(hipGetLastError(), "image_tiles launch");
}

}  // namespace pr
