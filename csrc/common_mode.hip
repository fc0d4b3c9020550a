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
// MI355X design.  Round 2 started VALU-bound (4.0M VALU wave-instructions per epix10k2M frame,
// ~6.6 us at the chip's ~614 G wave-instr/s); this version is at 3.3M and the memory phases now
// dominate (medians off: ~4.7-5.0 us/frame, vs a measured 3.0 us/frame floor for the same bytes,
// tools/bw_ceiling.hip; profiles/r2/cm_kernel.md):
//  * one workgroup owns one (frame, full-height ASIC stripe) tile in LDS: HBM is touched once;
//  * the tile holds v for CM-eligible pixels and NaN for every other pixel.  The median phases then
//    need no eligibility lookups at all: |NaN| < thr is false (never participates) and
//    NaN - median stays NaN (never corrected);
//  * the raw v of an 8-pixel group that has non-eligible but kept pixels (status-bad or
//    gain-switched, a few %) is parked in an LDS side slot (per-wave ranges claimed with a ballot,
//    no atomics) so the store phase never goes back to HBM for it; a full range falls back to a
//    recompute from raw + pedestal;
//  * eligibility arrives as per-8-pixel bit-planes (one byte per candidate gain table), selected by
//    the pixels' candidate bits with one v_bfi per 8 pixels (SWAR) instead of per-pixel shifts;
//  * row segments: one lane per (row, bank), values in registers, a median-cone-pruned Batcher
//    network (select_regs: 580 VALU for 48 values instead of a 768-VALU sort), toggle +-inf padding
//    so the median sits at fixed register positions;
//  * columns: four lanes (a quad) per column, per-lane sorts + DPP merge-split + merge-path;
//  * tile rows are 16-B aligned with an odd number of 16-B slots per row (pitch 52 floats for
//    48-column stripes) so the row phase moves whole segments with conflict-free ds_read_b128; the
//    candidate bits and side-slot numbers for the store phase live in the row pad;
//  * compile-time production shapes issue every load of a phase before the first use (phase 1:
//    raw + planes + first pedestal table, then the rare switched-gain tables; phase 3: first gain
//    table) -- 125 VGPRs, no scratch, four 256-thread workgroups per CU.
#include "common.h"
#include "sortnet.h"

#include <algorithm>

// Workgroups of the epix10k2M kernel per CU (LDS sizing).  4: the kernel alone fills the CU; 3: a
// quarter of every CU's LDS and VGPRs stays free, so the consumer's peak finder can run BESIDE the
// producer's common mode on the same CUs (device-resident pipeline).
// Frames per workgroup of the epix10k2M kernel.  2 = frame k+1's raw words prefetched during frame
// k's medians (3 workgroups per CU, 168 VGPRs): measured equal to 1 on the same MI355X (6.59-6.60
// vs 6.59-6.61 us/frame, device-resident pipeline 118.9k vs 118.4k fr/s on that box,
// tools/gpu_cm_ab.sh), so the simpler single-frame form ships.
#ifndef PR_CM_FPW
#define PR_CM_FPW 1
#endif
#ifndef PR_CM_GPRE
#define PR_CM_GPRE 0
#endif
// Raw-word loads of the compile-time (production) kernels: 1 = non-temporal (stream cache policy),
// 0 = plain.  (The read-ceiling probe at four workgroups per CU read 5.00 TB/s non-temporal vs 6.03
// plain, profiles/r2/pf/read_ceiling.md.)
#ifndef PR_CM_RAW_NT
#define PR_CM_RAW_NT 1
#endif
// Output stores of the production kernels: 0 = plain; 1 = non-temporal (streaming) for calib-mode
// frames; 2 = non-temporal for the image placement too; 3 = calib-mode frames non-temporal for the
// 128-B lines a tile row owns, plain for the lines it shares with its neighbour tile (cm_flush).  Same-box A/B, device-resident pipeline
// (common mode + peak finder), two boxes (profiles/r4/cm_pass1, cm_pass2): level 1 calib 144.6k /
// 145.0k / 144.9k / 143.6k vs plain 140.6k / 141.3k / 141.2k / 139.8k fr/s (+2.7 %), image mode
// unchanged; level 2 costs image mode 13 % (100.9k vs 115.8k: partial-line image runs).  Kernel
// alone: memory phases 4.14 vs 4.26 us/frame, full kernel within 0.5 %.
#ifndef PR_CM_NT_STORE
#define PR_CM_NT_STORE 1
#endif
// Threads per workgroup of the epix10k2M production kernel (4 or 6 waves; the tile and four
// workgroups per CU are unchanged: 6 waves leave each wave 80 VGPRs)
#ifndef PR_CM_EPIX_BLOCK
#define PR_CM_EPIX_BLOCK 256
#endif
#ifndef PR_CM_EPIX_WG_PER_CU
#define PR_CM_EPIX_WG_PER_CU ((PR_CM_FPW > 1 || PR_CM_GPRE) ? 3 : 4)
#endif

namespace pr {

// ---- phase stamps (diagnostic build only: -DPR_CM_STAMPS=1, tools/cm_stamps.py) ----------------
// Every wave of the epix10k2M production kernel records the shader clock at its phase boundaries
// (before and after each barrier) and the 100-MHz real-time clock at entry and exit; lane 0 writes
// them with ONE vector store per value at the end.  Record per wave (16 x u64):
//   [0] realtime entry  [1] realtime exit  [2] HW_ID  [3] XCC_ID  [4..15] shader-clock stamps
constexpr int kCmStampWords = 16;
#ifndef PR_CM_STAMPS
#define PR_CM_STAMPS 0
#endif
#if PR_CM_STAMPS
__device__ uint64_t* g_cm_stamps = nullptr;
#define PR_STAMP(k) st_[(k)] = __builtin_amdgcn_s_memtime()
#else
#define PR_STAMP(k) ((void)0)
#endif
void cm_set_stamp_buffer(uint64_t p) {
#if PR_CM_STAMPS
  uint64_t* q = reinterpret_cast<uint64_t*>(p);
  hip_check(hipMemcpyToSymbol(HIP_SYMBOL(g_cm_stamps), &q, sizeof(q)), "cm stamps");
#else
  (void)p;
  check(false, "cm_set_stamp_buffer: this build has no phase stamps (-DPR_CM_STAMPS=1)");
#endif
}

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
};

struct TileGeom {
  int panel_rows, panel_cols;        // H, W of one panel
  int asic_rows, asic_cols;          // R, C of one tile (a full-height ASIC stripe)
  int asics_per_col, asics_per_row;  // H / R, W / C
  int64_t npix;                      // pixels per frame
  int nframes;                       // frames of this launch
  int fpw;                           // frames per workgroup (grid = n_tiles * ceil(nframes / fpw), 1-D)
  int side_slots;                    // LDS side slots after the tile (SideCtx)
  int pitch;                         // LDS floats per tile row (values + candidate bits + pad)
  int xcd_map;                       // XCD-grouped tile order (cm_coords): few frames per launch
  uint64_t plain_mask;               // bit f: frame f's calib-layout stores are plain, not streaming
                                     // (frames written into ANOTHER process's ring: QueueFabric direct
                                     // grants -- streaming stores through an IPC mapping were seen stale
                                     // by the ring's owner, profiles/r6/README.md)
};

// Fused K-05 output (image mode with common mode).  Every panel is placed by an integer rotation
// + translation (geometry.py), so pixel (y, x) of panel p lands at image element
// desc[3p] + y * desc[3p+1] + x * desc[3p+2]; the corrected tile goes from LDS straight into the
// assembled image instead of a frame-shaped scratch buffer that a second kernel re-reads
// (saves a 2 x 8.65 MB HBM round trip per epix10k2M frame).  The gap pixels between panels are
// zeroed by the same kernel from a gap table of image elements no panel covers: aligned 16-B chunks
// (entry = first element, >= 0, a multiple of 4) first, then single elements (entry = -1 - element);
// workgroup (tile t, frame f) takes its 1/n_tiles share.
struct ImgOut {
  const int32_t* desc;    // [n_panels][3] (base, step per panel row, step per panel column); nullptr: frame layout
  const int32_t* gaps;    // [n_gaps] gap table (geometry.py gap_fill_table)
  int n_gaps;
};

// ---- tile layout ------------------------------------------------------------------------
// Candidate bits per pixel kept for the store phase (which gain-factor table): 1 for 2-table
// kinds, 2 for Jungfrau's 3 tables.  Eligibility bit-planes per 8-pixel group in global memory:
// PB bytes, byte k = pixels eligible when they decode to candidate k.
template <int NT>
struct CmLayout {
  static constexpr int kCandBits = NT == 3 ? 2 : 1;
  static constexpr int kPlaneBytes = NT == 3 ? 4 : NT;   // stride of the eligibility planes
};

// Tile row: C values, then the row pad = candidate bits (C * cand_bits / 8 bytes) + one side-slot
// byte per 8-pixel group (C / 8 bytes); rows are 16-B aligned with an odd number of 16-B slots.
__host__ __device__ constexpr int cm_pitch(int cols, int cand_bits) {
  int p = cols + (cols * (cand_bits + 1) + 31) / 32;
  while (p % 8 != 4) ++p;
  return p;
}

// Side slots: the raw values v of the (few) 8-pixel groups holding non-eligible pixels, so the
// store phase never goes back to HBM for them.  Every wave owns a fixed slot range (no atomics);
// a group that finds its wave's range full is marked kSideOverflow and recomputed from global
// memory instead (correct, just slower).
constexpr uint32_t kNoSide = 0xFF, kSideOverflow = 0xFE, kMaxSideSlots = 254;

struct SideCtx {
  float* side;    // slot s = 8 floats at side + 8 s
  int base, end;  // this wave's slots [base, end)
  int used;       // wave-uniform running count
};

__device__ __forceinline__ SideCtx side_ctx(float* side, int nslots, int wave, int nw) {
  const int per = nslots / nw;
  return SideCtx{side, wave * per, wave * per + per, 0};
}
__device__ __forceinline__ SideCtx side_ctx(float* side, int nslots) {
  return side_ctx(side, nslots, (int)threadIdx.x >> 6, (int)(blockDim.x >> 6));
}

// Claims a slot for every lane with `needs` (call convergently: all lanes of the wave) and writes
// v[8] into it.  Returns the group's slot byte.
__device__ __forceinline__ uint32_t side_put(SideCtx& sc, bool needs, const float (&v)[8]) {
  const uint64_t bal = __ballot(needs);
  const int before =
      (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
  const int slot = sc.base + sc.used + before;
  sc.used += __popcll(bal);
  if (!needs) return kNoSide;
  if (slot >= sc.end) return kSideOverflow;
  float* d = sc.side + 8 * slot;
  *reinterpret_cast<float4*>(d) = make_float4(v[0], v[1], v[2], v[3]);
  *reinterpret_cast<float4*>(d + 4) = make_float4(v[4], v[5], v[6], v[7]);
  return (uint32_t)slot;
}

// (m & a) | (~m & b) as ONE v_bfi_b32 (the compiler emits and / xor / and / or for the
// constant-operand and sign-extended-mask forms below: 4-5 VALU per pixel)
__device__ __forceinline__ uint32_t bfi(uint32_t m, uint32_t a, uint32_t b) {
  uint32_t r;
  asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "v"(m), "v"(a), "v"(b));
  return r;
}

// Decode one 8-pixel group: v = ADU - pedestal (0 for Jungfrau's invalid gain code), el = CM
// eligibility bits, cbits = candidate bits for the store phase.
//   rw: raw words (2 pixels each), pa: candidate pedestals, ep: eligibility bit-planes
// SG (signed pedestal tables, CalibConstants.cm_signed_pedestals): the pedestal of a pixel that is
// not CM-eligible for that candidate is stored negated -- the tables carry the eligibility in their
// sign bits (every pedestal is >= +0), so v = ADU - |p| and no bit-plane is loaded (ep unused).
template <int KIND, int NT, bool SG = false>
__device__ __forceinline__ void cm_decode8(const uint4 rw, const uint32_t ep, const float (&pa)[NT][8], float (&v)[8],
                                           uint32_t& el, uint32_t& cbits) {
  const uint32_t w[4] = {rw.x, rw.y, rw.z, rw.w};
  uint32_t c0 = 0, c1 = 0;   // candidate bit planes (bit j of pixel j): gain bit 14 / 15
  uint32_t es = 0;           // SG: eligibility from the selected pedestal's sign
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const uint32_t wj = w[j >> 1];
    const int sh = 16 * (j & 1);
    if constexpr (KIND == kPlain) {
      const float p = pa[0][j];
      v[j] = (float)__builtin_amdgcn_ubfe(wj, sh, 16) - (SG ? fabsf(p) : p);
      if constexpr (SG) es |= ((~__float_as_uint(p)) >> 31) << j;
    } else {
      const float adu = (float)__builtin_amdgcn_ubfe(wj, sh, 14);
      const uint32_t g0 = (uint32_t)__builtin_amdgcn_sbfe((int)wj, sh + 14, 1);   // all ones: gain bit 14
      if constexpr (KIND == kEpix10ka) {
        const float p = __uint_as_float(bfi(g0, __float_as_uint(pa[1][j]), __float_as_uint(pa[0][j])));
        v[j] = adu - (SG ? fabsf(p) : p);
        if constexpr (SG) es |= ((~__float_as_uint(p)) >> 31) << j;
        c0 |= g0 & (1u << j);
      } else {   // Jungfrau: gain bits 0 -> G0, 1 -> G1, 3 -> G2, 2 -> invalid (never eligible, output 0)
        const uint32_t g1 = (uint32_t)__builtin_amdgcn_sbfe((int)wj, sh + 15, 1);
        const uint32_t p01 = (g0 & __float_as_uint(pa[1][j])) | (~g0 & __float_as_uint(pa[0][j]));
        const uint32_t sel2 = g0 & g1;
        const float p = __uint_as_float((sel2 & __float_as_uint(pa[2][j])) | (~sel2 & p01));
        const float vj = adu - (SG ? fabsf(p) : p);
        v[j] = __uint_as_float(__float_as_uint(vj) & ~(~g0 & g1));
        if constexpr (SG) es |= (((~__float_as_uint(p)) >> 31) & ~((~g0 & g1) >> 31)) << j;   // invalid: never
        c0 |= g0 & (1u << j);
        c1 |= g1 & (1u << j);
      }
    }
  }
  if constexpr (SG) {
    el = es;
    if constexpr (NT == 1) {
      cbits = 0;
    } else if constexpr (NT == 2) {
      cbits = c0;
    } else {
      uint32_t cb = 0;
#pragma unroll
      for (int j = 0; j < 8; ++j) cb |= ((((c0 >> j) & 1u) + (((c0 & c1) >> j) & 1u)) << (2 * j));
      cbits = cb;
    }
  } else if constexpr (NT == 1) {
    el = ep & 0xFFu;
    cbits = 0;
  } else if constexpr (NT == 2) {
    el = ((c0 & (ep >> 8)) | (~c0 & ep)) & 0xFFu;   // v_bfi: plane 1 where the pixel switched
    cbits = c0;
  } else {
    // cand 0: !b14 !b15, cand 1: b14 !b15, cand 2: b14 b15, invalid: !b14 b15
    el = ((~c0 & ~c1 & ep) | (c0 & ~c1 & (ep >> 8)) | (c0 & c1 & (ep >> 16))) & 0xFFu;
    uint32_t cb = 0;   // 2-bit candidate field per pixel: 0, 1, 2
#pragma unroll
    for (int j = 0; j < 8; ++j) cb |= ((((c0 >> j) & 1u) + (((c0 & c1) >> j) & 1u)) << (2 * j));
    cbits = cb;
  }
}

// PR_CM_BASE_FAST = 1: wave-uniform fast paths for items in which no pixel of the whole wave left the
// first candidate table (no gain switch: epix10ka bit 14 / Jungfrau bits 14-15 clear everywhere) --
// in the decode (v = ADU - table-0 pedestal, no per-pixel mask / select, no candidate bits) and in
// the store phase (table-0 gain factor, no per-pixel select).  Gain switching marks bright pixels
// only (synthetic epix10k2M: 2e-5 of the 8-pixel groups), so nearly every item takes them; a wave
// that meets one switched pixel runs the general path for that item.
#ifndef PR_CM_BASE_FAST
#define PR_CM_BASE_FAST 1
#endif
template <int KIND>
__device__ __forceinline__ bool cm_base_only(const uint4 rw) {
  const uint32_t b = rw.x | rw.y | rw.z | rw.w;
  if constexpr (KIND == kEpix10ka) return (b & 0x40004000u) == 0u;
  else if constexpr (KIND == kJungfrau) return (b & 0xC000C000u) == 0u;
  else return true;
}
// cm_decode8 for a group whose pixels all decode to candidate 0 (cm_base_only)
template <int KIND>
__device__ __forceinline__ void cm_decode8_base(const uint4 rw, const uint32_t ep, const float (&pa0)[8], float (&v)[8],
                                                uint32_t& el) {
  const uint32_t w[4] = {rw.x, rw.y, rw.z, rw.w};
#pragma unroll
  for (int j = 0; j < 8; ++j)
    v[j] = (float)__builtin_amdgcn_ubfe(w[j >> 1], 16 * (j & 1), KIND == kPlain ? 16 : 14) - pa0[j];
  el = ep & 0xFFu;
}

// cm_decode8_base for signed pedestal tables: the tile values straight from the sign bits (v where
// the pedestal is >= +0, NaN where it is negated); returns true when some pixel is not eligible
template <int KIND>
__device__ __forceinline__ bool cm_decode8_base_sg(const uint4 rw, const float (&pa0)[8], float (&v)[8], float (&x)[8]) {
  const uint32_t w[4] = {rw.x, rw.y, rw.z, rw.w};
  const uint32_t qnan = 0x7fc00000u;
  uint32_t acc = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float p = pa0[j];
    v[j] = (float)__builtin_amdgcn_ubfe(w[j >> 1], 16 * (j & 1), KIND == kPlain ? 16 : 14) - fabsf(p);
    const uint32_t m = (uint32_t)((int)__float_as_uint(p) >> 31);
    x[j] = __uint_as_float(bfi(m, qnan, __float_as_uint(v[j])));
    acc |= m;
  }
  return acc != 0u;
}

// tile value: v where eligible, NaN elsewhere
__device__ __forceinline__ void cm_tile_values(const float (&v)[8], uint32_t el, float (&x)[8]) {
  const uint32_t qnan = 0x7fc00000u;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const uint32_t m = (uint32_t)__builtin_amdgcn_sbfe((int)el, j, 1);
    x[j] = __uint_as_float(bfi(m, __float_as_uint(v[j]), qnan));
  }
}

// row pad accessors (group k of the row)
template <int NT>
__device__ __forceinline__ void cm_put_meta(uint8_t* pad, int C, int k, uint32_t cbits, uint32_t slot) {
  if constexpr (CmLayout<NT>::kCandBits == 1) pad[k] = (uint8_t)cbits;
  else reinterpret_cast<uint16_t*>(pad)[k] = (uint16_t)cbits;
  pad[(C * CmLayout<NT>::kCandBits) / 8 + k] = (uint8_t)slot;
}
template <int NT>
__device__ __forceinline__ void cm_get_meta(const uint8_t* pad, int C, int k, uint32_t& cbits, uint32_t& slot) {
  if constexpr (CmLayout<NT>::kCandBits == 1) cbits = pad[k];
  else cbits = reinterpret_cast<const uint16_t*>(pad)[k];
  slot = pad[(C * CmLayout<NT>::kCandBits) / 8 + k];
}

template <int NT>
__device__ __forceinline__ uint32_t cm_need(uint32_t cbits) {
  // which candidate tables an 8-pixel group touches (bit k = table k)
  if constexpr (NT == 1) return 1u;
  else if constexpr (NT == 2) return 1u | (cbits ? 2u : 0u);
  else return 1u | ((cbits & 0x5555u) ? 2u : 0u) | ((cbits & 0xAAAAu) ? 4u : 0u);
}

#ifndef PR_CM_UNDEF_TABLES
#define PR_CM_UNDEF_TABLES 1
#endif
// A table the group does not need (no pixel selects that candidate) is left UNDEFINED, not zeroed:
// every consumer selects it only for pixels of that candidate (v_bfi on the candidate bits), and a
// zero fill costs 8 v_mov per group (phase 1 and phase 3: 80 VALU per lane of the production kernel).
template <int NT>
__device__ __forceinline__ void load8(const float* __restrict__ t, int64_t npix, int64_t pix, uint32_t need,
                                      float (&a)[NT][8], int k0 = 0) {
#pragma unroll
  for (int k = k0; k < NT; ++k) {
    f32x4_t u, w;
    if ((need >> k) & 1u) {
      u = *reinterpret_cast<const f32x4_t*>(t + k * npix + pix);
      w = *reinterpret_cast<const f32x4_t*>(t + k * npix + pix + 4);
    } else {   // an empty asm "defines" the registers: no instruction (freeze(undef) would be a v_mov 0)
#if PR_CM_UNDEF_TABLES
      asm("" : "=v"(u));
      asm("" : "=v"(w));
#else
      u = f32x4_t{0.f, 0.f, 0.f, 0.f};
      w = u;
#endif
    }
    a[k][0] = u.x; a[k][1] = u.y; a[k][2] = u.z; a[k][3] = u.w;
    a[k][4] = w.x; a[k][5] = w.y; a[k][6] = w.z; a[k][7] = w.w;
  }
}

// PR_CM_OFF32: the production kernel's per-item loads address a per-frame uniform global base (SGPR)
// plus a 32-bit element offset within the tile, instead of a 64-bit per-item pointer (64-bit VALU
// adds per load; generic-pointer flat loads for the tables).  Same-box A/B (profiles/r4/off32/):
// kernel 5.39-5.43 vs 5.48-5.50 us/frame (flags 0: 4.05-4.07 vs 4.15-4.17), 120 -> 109 VGPRs,
// device-resident pipeline 151.0-153.8k vs 149.2-151.7k.
#ifndef PR_CM_OFF32
#define PR_CM_OFF32 1
#endif
// tables[k] = base of candidate table k at the tile origin (uniform); o = element offset in the tile
template <int NT>
__device__ __forceinline__ void load8o(const PR_GLOBAL float* const (&tb)[NT], uint32_t o, uint32_t need,
                                       float (&a)[NT][8], int k0 = 0) {
#pragma unroll
  for (int k = k0; k < NT; ++k) {
    f32x4_t u, w;
    if ((need >> k) & 1u) {
      u = *reinterpret_cast<const PR_GLOBAL f32x4_t*>(tb[k] + o);
      w = *reinterpret_cast<const PR_GLOBAL f32x4_t*>(tb[k] + o + 4);
    } else {
      asm("" : "=v"(u));
      asm("" : "=v"(w));
    }
    a[k][0] = u.x; a[k][1] = u.y; a[k][2] = u.z; a[k][3] = u.w;
    a[k][4] = w.x; a[k][5] = w.y; a[k][6] = w.z; a[k][7] = w.w;
  }
}
template <int NT>
__device__ __forceinline__ uint32_t load_planes_o(const PR_GLOBAL uint8_t* planes_tile, uint32_t o) {
  const uint32_t g = o >> 3;   // o is a multiple of 8 (8-pixel groups, 8-aligned tiles and rows)
  if constexpr (NT == 1) return planes_tile[g];
  else if constexpr (NT == 2) return *reinterpret_cast<const PR_GLOBAL uint16_t*>(planes_tile + 2 * g);
  else return *reinterpret_cast<const PR_GLOBAL uint32_t*>(planes_tile + 4 * g);
}

template <int NT>
__device__ __forceinline__ uint32_t load_planes(const uint8_t* __restrict__ planes, int64_t pix) {
  const int64_t g = pix >> 3;
  if constexpr (NT == 1) return planes[g];
  else if constexpr (NT == 2) return *reinterpret_cast<const uint16_t*>(planes + 2 * g);
  else return *reinterpret_cast<const uint32_t*>(planes + 4 * g);
}

template <int NT>
__device__ __forceinline__ uint32_t need_from_raw(const uint4 rw) {
  // candidate tables the group's raw gain bits select (select-then-load of the rare tables)
  const uint32_t b = (rw.x | rw.y | rw.z | rw.w);
  if constexpr (NT == 1) return 1u;
  else if constexpr (NT == 2) return 1u | ((b & 0x40004000u) ? 2u : 0u);
  else return 1u | ((b & 0x40004000u) ? 6u : 0u);
}

// gain factor of pixel j from the group's candidate bits
template <int NT>
__device__ __forceinline__ float cm_gain(const float (&ga)[NT][8], uint32_t cb, int j) {
  if constexpr (NT == 1) {
    return ga[0][j];
  } else if constexpr (NT == 2) {
    const uint32_t m = (uint32_t)__builtin_amdgcn_sbfe((int)cb, j, 1);
    return __uint_as_float(bfi(m, __float_as_uint(ga[1][j]), __float_as_uint(ga[0][j])));
  } else {
    const uint32_t cj = (cb >> (2 * j)) & 3u;
    return bsel(cj == 0, ga[0][j], bsel(cj == 1, ga[1][j], ga[2][j]));
  }
}

// NaN-fill: x if x is a number, else s -- ONE v_med3_f32 instead of v_cmp_u + v_cndmask.  With no
// NaN operand med3(x, s, x) = x; with a NaN operand v_med3_f32 returns v_min3_f32 of its operands,
// whose minNum semantics drop the NaNs: med3(NaN, s, NaN) = s (s is never NaN: a raw value or a
// recomputed ADU - pedestal).  The third operand is x itself (no opaque copy: an asm barrier would
// cost a v_mov per pixel in a VALU-bound kernel).  That relies on LLVM keeping
// amdgcn.fmed3(x, s, x) as a med3 and not folding it to x, which
// tests/test_med3_fill_isa.py checks on the compiled gfx950 code (v_med3_f32 vA, vX, vS, vX
// present) and the bitwise GPU tests check numerically; PR_CM_MED3_FILL=0 builds the compare +
// select reference.
#ifndef PR_CM_MED3_FILL
#define PR_CM_MED3_FILL 1
#endif
__device__ __forceinline__ float nan_fill(float x, float s) {
#if PR_CM_MED3_FILL
  return __builtin_amdgcn_fmed3f(x, s, x);
#else
  return x != x ? s : x;
#endif
}

// Store-phase output of one 8-pixel group.  NaN tile entries are pixels that were not CM-eligible:
// their raw value comes from the group's side slot (or, on slot overflow, is recomputed from raw
// + pedestal in global memory); masked pixels have a zero gain factor, Jungfrau's invalid gain
// code a zero value, so both come out 0.
// PR_CM_LDS_PROBE = 1 (diagnostic, WRONG results): the store phase's tile reads and the flush's reads
// use bank-conflict-free addresses instead of the tile layout's -- the timing bound of removing the
// memory phases' LDS read conflicts (tools/lds_bank_model.py attributes all 660 conflict cycles per
// tile to those phases: phase-1 / phase-3 b128 writes 176 + 176, phase-3 b128 reads 176, flush 132).
#ifndef PR_CM_LDS_PROBE
#define PR_CM_LDS_PROBE 0
#endif
template <int KIND, int NT, bool BASE = false, bool SG = false>
__device__ __forceinline__ void cm_out8(const float* tile_row, const float* side, uint32_t cb, uint32_t slot,
                                        const float (&ga)[NT][8], const PR_GLOBAL uint16_t* raw,
                                        const float* __restrict__ ped, int64_t npix, int64_t pix, float (&o)[8]) {
#if PR_CM_LDS_PROBE
  tile_row = side - 8 * 1024 + 4 * (int)threadIdx.x;   // the tile base is side - R * P; 4 dwords per lane
  const float4 t0 = *reinterpret_cast<const float4*>(tile_row);
  const float4 t1 = *reinterpret_cast<const float4*>(tile_row + 1024);
#else
  const float4 t0 = *reinterpret_cast<const float4*>(tile_row);
  const float4 t1 = *reinterpret_cast<const float4*>(tile_row + 4);
#endif
  float xv[8] = {t0.x, t0.y, t0.z, t0.w, t1.x, t1.y, t1.z, t1.w};
  if (slot < kSideOverflow) {
    const float4 s0 = *reinterpret_cast<const float4*>(side + 8 * slot);
    const float4 s1 = *reinterpret_cast<const float4*>(side + 8 * slot + 4);
    const float sv[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
#pragma unroll
    for (int j = 0; j < 8; ++j) xv[j] = nan_fill(xv[j], sv[j]);
  } else if (slot == kSideOverflow) {
    const uint4 rw = ld_nt_u4((const PR_GLOBAL uint4*)(raw + pix));
    float pa[NT][8];
    load8<NT>(ped, npix, pix, need_from_raw<NT>(rw), pa);
    float v[8];
    uint32_t el, cb2;
    cm_decode8<KIND, NT, SG>(rw, 0u, pa, v, el, cb2);
#pragma unroll
    for (int j = 0; j < 8; ++j) xv[j] = nan_fill(xv[j], v[j]);
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = gmul(xv[j], BASE ? ga[0][j] : cm_gain<NT>(ga, cb, j));
}

// Store phase, part 2.  Part 1 leaves the finished output tile in LDS; part 2 only reads LDS
// and writes global memory.  On CDNA the vector-memory counter counts stores as well as loads,
// so a load between two stores would make the wave wait for the earlier stores to retire; with
// no loads in this loop every store is fire-and-forget (the round-1 form that interleaved the
// gain-factor loads with the stores serialised one store round trip per 8-pixel group).
// Frame layout: 16 B per lane, consecutive lanes along tile rows.
template <int LEVEL>
__device__ __forceinline__ void st_out4(PR_GLOBAL float4* p, const float4 v) {
  if constexpr (LEVEL == 1 ? PR_CM_NT_STORE >= 1 : PR_CM_NT_STORE == 2) {
    f32x4_t x;
    x.x = v.x; x.y = v.y; x.z = v.z; x.w = v.w;
    __builtin_nontemporal_store(x, (PR_GLOBAL f32x4_t*)p);
  } else {
    st_f4(p, v);
  }
}

// Flush of the float4 chunks [j0, j0 + nj) of every tile row; NT: streaming (non-temporal) stores.
template <bool NT>
__device__ __forceinline__ void cm_flush_cols(const float* tile, int P, int R, PR_GLOBAL float* ob, int panel_cols,
                                              int j0, int nj) {
  if (nj <= 0) return;
  // (row, chunk) advance incrementally by blockDim.x chunks per iteration (one division per thread)
  const int dr = (int)blockDim.x / nj, dj = (int)blockDim.x - dr * nj;
  int r = (int)threadIdx.x / nj, j = (int)threadIdx.x - r * nj;
  for (int e = threadIdx.x; e < R * nj; e += blockDim.x) {
    const float4 v = *reinterpret_cast<const float4*>(tile + r * P + 4 * (j0 + j));
    PR_GLOBAL float4* d = (PR_GLOBAL float4*)(ob + (uint32_t)(r * panel_cols + 4 * (j0 + j)));
    if constexpr (NT) st_out4<1>(d, v);
    else st_f4(d, v);
    r += dr;
    j += dj;
    if (j >= nj) {
      j -= nj;
      ++r;
    }
  }
}

// PR_CM_NT_STORE = 3 (calib mode): non-temporal stores for the 128-B lines a tile row owns whole, plain
// stores for the lines it shares with its neighbour tile (a 48-float stripe row is 192 B: every other
// line is half this tile's, half the next one's).  A streaming store evicts its partial line before the
// neighbour's half arrives, so the L2 writes it back twice: +9 % WRITE_SIZE per frame with every store
// non-temporal (profiles/r5/README.md); the neighbour tile of the same frame runs on the same XCD
// (table-major order, 64 frames per launch), so a plain store's half line waits in L2 for its partner.
__device__ __forceinline__ void cm_flush(const float* tile, int P, int R, int C, PR_GLOBAL float* out, int64_t base,
                                         int panel_cols, bool nt = true) {
  const int C4 = C >> 2;
  if (!nt) {   // plain stores (a frame for another process's ring), workgroup-uniform
    cm_flush_cols<false>(tile, P, R, out + base, panel_cols, 0, C4);
    return;
  }
#if PR_CM_NT_STORE == 3 && !PR_CM_LDS_PROBE
  if ((panel_cols & 31) == 0) {   // every tile row starts at the same offset within its 128-B line
    PR_GLOBAL float* const ob = out + base;
    const int s = (int)(reinterpret_cast<uintptr_t>(ob) & 127);        // byte offset of the rows in their lines
    const int jlo = min(C4, ((128 - s) & 127) >> 4);                    // first chunk of a whole line
    const int jhi = max(jlo, (((s + 16 * C4) & ~127) - s) >> 4);        // end of the last whole line
    cm_flush_cols<true>(tile, P, R, ob, panel_cols, jlo, jhi - jlo);
    cm_flush_cols<false>(tile, P, R, ob, panel_cols, 0, jlo);
    cm_flush_cols<false>(tile, P, R, ob, panel_cols, jhi, C4 - jhi);
    return;
  }
#endif
#ifndef PR_CM_FLUSH32
#define PR_CM_FLUSH32 PR_CM_OFF32
#endif
#if PR_CM_FLUSH32
  PR_GLOBAL float* const ob = out + base;   // uniform tile origin; 32-bit offsets per store
  // (row, float4 column) of element e advance incrementally by blockDim.x elements per iteration:
  // one integer division per thread instead of one per element
  const int dr = (int)blockDim.x / C4, dj = (int)blockDim.x - dr * C4;
  int r = (int)threadIdx.x / C4, j = (int)threadIdx.x - r * C4;
  for (int e = threadIdx.x; e < R * C4; e += blockDim.x) {
#if PR_CM_LDS_PROBE
    const float4 v = *reinterpret_cast<const float4*>(tile + 4 * e);
#else
    const float4 v = *reinterpret_cast<const float4*>(tile + r * P + 4 * j);
#endif
#if PR_CM_MEMPROBE & 8
    if (__float_as_uint(v.x) == 0x7fc01234u)   // never: the flush's LDS reads and loop stay, the stores go
#endif
    st_out4<1>((PR_GLOBAL float4*)(ob + (uint32_t)(r * panel_cols + 4 * j)), v);
    r += dr;
    j += dj;
    if (j >= C4) {
      j -= C4;
      ++r;
    }
  }
#else
  for (int e = threadIdx.x; e < R * C4; e += blockDim.x) {
    const int r = e / C4, j = e - r * C4;
    const float4 v = *reinterpret_cast<const float4*>(tile + r * P + 4 * j);
    st_out4<1>((PR_GLOBAL float4*)(out + base + (int64_t)r * panel_cols + 4 * j), v);
  }
#endif
}

// Image layout (fused K-05): every panel sits in the image by an integer rotation + translation,
// so either tile rows or tile columns are contiguous image runs (step +-1).  Each run is cut into
// 16-B aligned image chunks.  Stores are issue-bound here (a 4-B-per-lane store costs the issue slot
// of a 16-B one), so the FULL chunks go out first, one 16-B store per lane and no partial-chunk
// branch in the loop, and the (at most 3 + 3) ragged elements of every run after them, one 4-B
// store per element over all lanes.  (The round-2 form handled partial chunks inside the chunk loop:
// every wave iteration that met one issued 1 + 4 store instructions.)  The image mask is folded
// into the gain factors of this plan (Calibrator), so no mask loads sit between the stores.

// Gap table share of this workgroup, preloaded into registers BEFORE the store phase's barrier (the
// loads' latency hides behind the barrier and the placement; a load between stores would wait for
// them).  kGapPre entries per thread cover the share; a larger share loops.
constexpr int kGapPre = 4;
struct GapPre {
  int v[kGapPre];
  int r0, r1;
};
__device__ __forceinline__ GapPre cm_gap_preload(const ImgOut& io, int tile, int ntiles) {
  GapPre g;
  g.r0 = io.n_gaps > 0 ? (int)((int64_t)io.n_gaps * tile / ntiles) : 0;
  g.r1 = io.n_gaps > 0 ? (int)((int64_t)io.n_gaps * (tile + 1) / ntiles) : 0;
#pragma unroll
  for (int k = 0; k < kGapPre; ++k) {
    const int e = g.r0 + (int)threadIdx.x + k * (int)blockDim.x;
    g.v[k] = e < g.r1 ? io.gaps[e] : INT32_MIN;
  }
  return g;
}
__device__ __forceinline__ void cm_gap_store(PR_GLOBAL float* out, int v) {
  if (v >= 0) st_f4((PR_GLOBAL float4*)(out + v), make_float4(0.f, 0.f, 0.f, 0.f));
  else if (v != INT32_MIN) out[-1 - (int64_t)v] = 0.0f;
}
__device__ __forceinline__ void cm_fill_gaps(const ImgOut& io, const GapPre& g, PR_GLOBAL float* out) {
#pragma unroll
  for (int k = 0; k < kGapPre; ++k) cm_gap_store(out, g.v[k]);
  for (int e = g.r0 + (int)threadIdx.x + kGapPre * (int)blockDim.x; e < g.r1; e += (int)blockDim.x)
    cm_gap_store(out, io.gaps[e]);   // shares beyond kGapPre entries per thread (not the production shapes)
}

// PR_CM_PLACEPROBE (diagnostic, WRONG results): bit 1 drops the ragged 4-B stores, bit 2 the
// full-chunk stores of row-run panels, bit 4 those of column-run panels (the LDS reads stay).
#ifndef PR_CM_PLACEPROBE
#define PR_CM_PLACEPROBE 0
#endif
#ifndef PR_CM_PLACE_CQ
#define PR_CM_PLACE_CQ 4
#endif
#define PR_PLACE_KEEP(bit, v) (!(PR_CM_PLACEPROBE & (bit)) || __float_as_uint((v)) == 0x7fc01234u)
// PR_CM_IMG_NT (bit 1 = row-run panels, bit 2 = column-run panels; shipped 3 with PR_CM_PLACE_LA):
// image placement stores streaming (non-temporal) for the 128-B
// lines that lie wholly inside one image run, plain for the lines a run shares with a gap or a
// neighbour tile (the image form of PR_CM_NT_STORE 3; all-streaming placement stores cost 13 %).
// With the round-5 column walk (a wave: 4 chunks x 16 runs) it LOST: kernel (--mode image --no-gaps,
// flags 3) 5.78-5.80 vs 5.37-5.39 us/frame, image pipeline 125.2-126.5k vs 136.2-137.7k fr/s
// (profiles/r6/image/); split by panel kind (profiles/r6/image_ntrc/) row-run panels only 5.34-5.37
// (neutral), column-run panels only 5.88-5.97: every line arrived as two half-line streaming writes
// from two instructions.  With the line-aligned column walk (PR_CM_PLACE_LA: each store instruction
// writes 8 whole lines) it WINS: flags 0 4.60-4.64 vs 5.05-5.08, flags 3 5.32 vs 5.38-5.40, image
// pipeline 142.8-146.8k vs 136.0-137.8k (profiles/r6/image_la/; line-aligned alone: neutral).
#ifndef PR_CM_IMG_NT
#define PR_CM_IMG_NT 3
#endif
// PR_CM_IMG_T = 1 (A/B, not kept): column-run panels read each image chunk's four tile elements as
// one ds_read_b128 of a tile ROW per lane and transpose 4x4 blocks in the quad with DPP (VERDICT r5
// next #3: one LDS read per 16-B store instead of four ds_read_b32).  Bitwise (45 CM / image tests);
// same box, 3 rounds: kernel (--mode image --no-gaps, flags 3) 5.44 / 5.44 / 5.46 vs 5.38 / 5.40 /
// 5.40 us/frame, image pipeline 135.5k / 136.9k / 136.6k vs 139.9k / 137.8k / 136.4k fr/s
// (profiles/r6/image_t/): the LDS reads are not what the placement waits on (cf. r5 sections 14, 19).
#ifndef PR_CM_IMG_T
#define PR_CM_IMG_T 0
#endif
// Column-run panels, line-aligned walk (see cm_place); 0 = the round-5 walk (PR_CM_PLACE_CQ chunks
// x 64 / CQ runs per wave, lines split between instructions)
#ifndef PR_CM_PLACE_LA
#define PR_CM_PLACE_LA 1
#endif
// quad_perm exchange with bound_ctrl (no `old` operand to materialise)
template <int CTRL>
__device__ __forceinline__ float quad_x(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, true));
}
template <int NTMASK = 3>
__device__ __forceinline__ void st_img4(PR_GLOBAL float* out, int32_t e, int32_t run_lo, int len, const float4 v,
                                        bool nt) {
#if PR_CM_IMG_NT
  if ((PR_CM_IMG_NT & NTMASK) && nt && (e & ~31) >= run_lo && (e | 31) < run_lo + len) {
    f32x4_t x;
    x.x = v.x; x.y = v.y; x.z = v.z; x.w = v.w;
    __builtin_nontemporal_store(x, (PR_GLOBAL f32x4_t*)(out + e));
    return;
  }
#endif
  st_out4<2>((PR_GLOBAL float4*)(out + e), v);
}
// nt = false: plain stores only (a frame for another process's ring, as cm_flush)
__device__ __forceinline__ void cm_place(const float* tile, int P, int R, int C, const ImgOut& io, int panel, int y0,
                                         int x0, PR_GLOBAL float* out, bool nt) {
  const int32_t* d = io.desc + 3 * panel;
  const int sy = d[1], sx = d[2];
  const int64_t b0 = (int64_t)d[0] + (int64_t)y0 * sy + (int64_t)x0 * sx;
  const bool rows = sx == 1 || sx == -1;           // image runs along tile rows (else along columns)
  const int len = rows ? C : R;                     // run length
  const int nruns = rows ? R : C;
  const int step = rows ? sx : sy;                  // +-1 along the run
  const int64_t outer = rows ? sy : sx;             // image step between runs
  const int nb = (int)blockDim.x;
  if ((outer & 3) != 0) {                           // runs not equally aligned: 4-B stores
    for (int e = threadIdx.x; e < R * C; e += nb) {
      const int a = e / len, t = e - a * len;
      const int r = rows ? a : t, c = rows ? t : a;
      out[b0 + (int64_t)r * sy + (int64_t)c * sx] = tile[r * P + c];
    }
    return;
  }
  const int64_t lo = step > 0 ? b0 : b0 - (len - 1);   // lowest image address of run 0
  const int head = (int)(lo & 3);                       // the same for every run
  // full chunks ch in [ch_lo, ch_lo + nfull): chunk ch covers positions t = 4 ch - head .. + 3 in
  // lowest-address order; positions [0, t_lo) and [t_hi, len) are ragged
  const int ch_lo = (head + 3) >> 2;
  const int nfull = max(0, ((len + head) >> 2) - ch_lo);
  const int t_lo = nfull > 0 ? 4 * ch_lo - head : len;
  const int t_hi = nfull > 0 ? t_lo + 4 * nfull : len;
  const int rb_step = rows ? P : 1;                     // tile address of run `run`, element i:
  const int ie = rows ? 1 : P;                          //   run * rb_step + i * ie
  const int di = step > 0 ? ie : -ie;
  auto tile_at = [&](int run, int t) { return tile + run * rb_step + (step > 0 ? t : len - 1 - t) * ie; };
  // lanes -> (run, full chunk): rows-case runs are tile rows (contiguous in LDS too), so consecutive
  // lanes take consecutive chunks of one run; column-case runs are tile columns, so a wave takes 4
  // chunks (64 B of image) of 16 neighbouring columns -- LDS reads 2-way instead of 32-way
  // bank-conflicted, global stores 16 segments of 64 B.  The (run, chunk) walk is incremental (one
  // integer division per thread, not per chunk).
  // One loop per layout (no per-item selects on the uniform `rows`), tile and image addresses
  // linear in (run, chunk) with the direction folded into a signed stride, 32-bit image offsets
  // (the image is < 2^31 elements; Geometry.panel_placement): 6.85-6.91 vs 7.04-7.07 us/frame for
  // the round-2 loop with per-item selects (profiles/r3/image/place2_ab/).
  if (nfull > 0) {
    const float* tb = tile + (step > 0 ? t_lo : len - 1 - t_lo) * ie;   // element t_lo of run 0
    const int32_t ob = (int32_t)((lo & ~(int64_t)3) + 4 * ch_lo);      // chunk 0 of run 0
    const int32_t oo = (int32_t)outer;
    if (rows) {
      // items e = tid + nb * i over (run, chunk) run-major: consecutive lanes, consecutive chunks
      int run = (int)threadIdx.x / nfull, k = (int)threadIdx.x - run * nfull;
      const int drun = nb / nfull, dk = nb - drun * nfull;
      for (; run < nruns;) {
        const float* tp = tb + run * P + 4 * k * di;
        const float4 v4 = make_float4(tp[0], tp[di], tp[2 * di], tp[3 * di]);
        if (PR_PLACE_KEEP(2, v4.x)) st_img4<1>(out, ob + run * oo + 4 * k, (int32_t)lo + run * oo, len, v4, nt);
        run += drun;
        k += dk;
        if (k >= nfull) {
          k -= nfull;
          ++run;
        }
      }
    } else if (PR_CM_PLACE_LA) {
      // line-aligned: a wave takes 8 runs x one 128-B image line each (lane = run offset x chunk of
      // the line), so a store instruction writes 8 whole lines instead of 16 half lines (the runs'
      // line phases differ: each lane locates its chunk from its run's own phase)
      const int lane = (int)threadIdx.x & 63, ro = lane >> 3, j = lane & 7;
      const int nrg = (nruns + 7) >> 3, ng = (nfull + 14) >> 3, nw = nb >> 6;
      for (int u = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6); u < nrg * ng; u += nw) {
        const int rg = u / ng, g = u - rg * ng;
        const int run = 8 * rg + ro;
        const int32_t a0 = ob + run * oo;             // chunk 0 of this run (16-B aligned)
        const int k = 8 * g - ((a0 >> 2) & 7) + j;    // this lane's chunk: line g of the run
        if (run < nruns && k >= 0 && k < nfull) {
          const float* tp = tb + run + 4 * k * di;
          const float4 v4 = make_float4(tp[0], tp[di], tp[2 * di], tp[3 * di]);
          st_img4<2>(out, a0 + 4 * k, (int32_t)lo + run * oo, len, v4, nt);
        }
      }
    } else if (PR_CM_IMG_T && (nruns & 3) == 0) {
      // quad transpose: lane q of a quad reads tile row (position t_lo + 4k + q) of 4 neighbouring
      // columns as ONE ds_read_b128, the quad transposes the 4x4 block with DPP exchanges, and lane q
      // stores chunk k of column c0 + q.  A wave takes 4 chunks x 16 columns (the shipped CQ 4 shape).
      const int q = (int)threadIdx.x & 3, quad = ((int)threadIdx.x & 63) >> 2;
      const int nq = (nfull + 3) >> 2, ncg = (nruns + 15) >> 4, nw = nb >> 6;
      for (int u = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6); u < ncg * nq; u += nw) {
        const int g = u / nq, a = u - g * nq;
        const int c0 = 16 * g + 4 * (quad & 3), k = 4 * a + (quad >> 2);
        const bool ok = c0 < nruns && k < nfull;          // uniform over the quad
        const int tq = t_lo + 4 * (ok ? k : 0) + q;
        const int r = step > 0 ? tq : len - 1 - tq;
        const float4 m = *reinterpret_cast<const float4*>(tile + r * P + (ok ? c0 : 0));
        // (every exchange runs on all four lanes: the opaque asm keeps the compiler from sinking a
        // DPP read into the lane-divergent select, where it would read a disabled partner)
        const bool odd = q & 1, hi = q & 2;
        float p0 = quad_x<0xB1>(m.x), p1 = quad_x<0xB1>(m.y), p2 = quad_x<0xB1>(m.z), p3 = quad_x<0xB1>(m.w);
        asm volatile("" : "+v"(p0), "+v"(p1), "+v"(p2), "+v"(p3));
        const float y0 = odd ? p1 : m.x, y1 = odd ? m.y : p0, y2 = odd ? p3 : m.z, y3 = odd ? m.w : p2;
        float s0 = quad_x<0x4E>(y0), s1 = quad_x<0x4E>(y1), s2 = quad_x<0x4E>(y2), s3 = quad_x<0x4E>(y3);
        asm volatile("" : "+v"(s0), "+v"(s1), "+v"(s2), "+v"(s3));
        const float z0 = hi ? s2 : y0, z1 = hi ? s3 : y1, z2 = hi ? y2 : s0, z3 = hi ? y3 : s1;
        if (ok) st_img4(out, ob + (c0 + q) * oo + 4 * k, (int32_t)lo + (c0 + q) * oo, len, make_float4(z0, z1, z2, z3), nt);
      }
    } else {
      // a wave takes PR_CM_PLACE_CQ chunks (16 B each) of 64 / PR_CM_PLACE_CQ neighbouring columns
      // (see the general form)
      constexpr int CQ = PR_CM_PLACE_CQ;
      const int per = CQ * nruns, nq = (nfull + CQ - 1) / CQ;
      int a = (int)threadIdx.x / per, w = (int)threadIdx.x - a * per;
      const int da = nb / per, dw = nb - da * per;
      for (; a < nq;) {
        const int run = w / CQ, k = CQ * a + (w % CQ);
        if (k < nfull) {
          const float* tp = tb + run + 4 * k * di;
          const float4 v4 = make_float4(tp[0], tp[di], tp[2 * di], tp[3 * di]);
          if (PR_PLACE_KEEP(4, v4.x)) st_img4<2>(out, ob + run * oo + 4 * k, (int32_t)lo + run * oo, len, v4, nt);
        }
        a += da;
        w += dw;
        if (w >= per) {
          w -= per;
          ++a;
        }
      }
    }
  }
  // ragged elements: n_rag per run, the same for every run
  const int n_head = t_lo, n_rag = t_lo + (len - t_hi);
  if (n_rag > 0) {
    for (int e = threadIdx.x; e < nruns * n_rag; e += nb) {
      const int run = e / n_rag, j = e - run * n_rag;
      const int t = j < n_head ? j : t_hi + (j - n_head);
      const float v1 = *tile_at(run, t);
      if (PR_PLACE_KEEP(1, v1)) out[lo + (int64_t)run * outer + t] = v1;
    }
  }
}

__device__ __forceinline__ void cm_put8(float* trow, const float (&o)[8]) {
  *reinterpret_cast<float4*>(trow) = make_float4(o[0], o[1], o[2], o[3]);
  *reinterpret_cast<float4*>(trow + 4) = make_float4(o[4], o[5], o[6], o[7]);
}

struct NoMark {
  __device__ void operator()(int) const {}
};
// mark(k): phase-stamp hook of the diagnostic build (k = 9 after the barrier, 10 after placement)
template <typename Mark = NoMark>
__device__ __forceinline__ void cm_write_out(const float* tile, int P, int R, int C, const TileGeom& tg,
                                             const ImgOut& io, int tile_id, int panel, int y0, int x0, int64_t base,
                                             PR_GLOBAL float* out, bool nt, const Mark& mark = Mark()) {
  GapPre gp;
  if (io.desc != nullptr) gp = cm_gap_preload(io, tile_id, (int)gridDim.x / ((tg.nframes + tg.fpw - 1) / tg.fpw));
  __syncthreads();
  mark(9);
  if (io.desc != nullptr) {
    cm_place(tile, P, R, C, io, panel, y0, x0, out, nt);
    mark(10);
    cm_fill_gaps(io, gp, out);
  } else {
    cm_flush(tile, P, R, C, out, base, tg.panel_cols, nt);
  }
}

// Phase 3 (runtime-shape loop form).
template <int KIND, int NT>
__device__ __forceinline__ void cm_store(float* tile, const float* side, const int P, const int R, const int C,
                                         const TileGeom& tg, const PR_GLOBAL uint16_t* raw,
                                         const float* __restrict__ ped, const float* __restrict__ gf, int64_t base,
                                         PR_GLOBAL float* out, const ImgOut& io, int tile_id, int panel, int y0,
                                         int x0, bool nt) {
  const int C8 = C >> 3;
  for (int i = threadIdx.x; i < R * C8; i += blockDim.x) {
    const int r = i / C8, k = i - r * C8, c = k * 8;
    const int64_t pix = base + (int64_t)r * tg.panel_cols + c;
    uint32_t cb, slot;
    cm_get_meta<NT>(reinterpret_cast<const uint8_t*>(tile + r * P + C), C, k, cb, slot);
    float ga[NT][8];
    load8<NT>(gf, tg.npix, pix, cm_need<NT>(cb), ga);
    float o[8];
    cm_out8<KIND, NT>(tile + r * P + c, side, cb, slot, ga, raw, ped, tg.npix, pix, o);
    cm_put8(tile + r * P + c, o);
  }
  cm_write_out(tile, P, R, C, tg, io, tile_id, panel, y0, x0, base, out, nt);
}

// (tile, frame) of this workgroup and the tile's first pixel
struct TileCoord {
  int f, tile, panel, ar, ac;
  int64_t base;
};
// Table-major order: consecutive workgroups take the same tile of consecutive frames, so the
// constant tables of a tile are fetched from HBM about once per XCD and then hit in L2.  (A/B on
// MI355X, 32 epix10k2M frames: frame-major order 5.7 us/frame vs 5.0 table-major with the medians
// off; an XCD-grouping remap of the table-major order changed nothing, 4.75 vs 4.65, and an
// XCD-local frame-major order lost, 5.29 vs 4.90.)
// With tg.fpw > 1 a workgroup takes fpw consecutive frames of its tile (t.f = the first).
// Image layout (desc != null, PR_CM_IMG_ORDER): in a panel whose tile COLUMNS are image rows (90 / 270
// degree placements) the tile that continues an image row is the next ASIC row, so those panels
// number their tiles ASIC-row fastest: the two tiles sharing the 128-B lines at a run's ends then run
// 64 workgroups apart on the same XCD (as row-run panels' neighbours do) instead of 64 x ASICs per
// row, and the L2 merges the halves before a partial line is written back.
#ifndef PR_CM_IMG_ORDER
#define PR_CM_IMG_ORDER 0
#endif
// XCD-grouped order for launches of at most PR_CM_XCD_MAX_FRAMES frames (TileGeom.xcd_map): with few
// frames per launch a tile's constant tables are re-read per frame group on every XCD and dominate
// the traffic (Jungfrau-16M, 8-frame chunks: 43.4 -> 37.7 us/frame; epix10k2M at 8 frames 6.35 ->
// 5.76), while at 32-64 frames the plain table-major order spreads the raw / output streams better
// (epix10k2M 64 frames: 4.59 vs 4.72), profiles/r5/README.md section 20
#ifndef PR_CM_XCD_MAX_FRAMES
#define PR_CM_XCD_MAX_FRAMES 12
#endif
__device__ __forceinline__ TileCoord cm_coords(const TileGeom& tg, int R, int C, const int id = (int)blockIdx.x,
                                               const int32_t* desc = nullptr) {
  TileCoord t;
  const int ng = (tg.nframes + tg.fpw - 1) / tg.fpw;
  const int per_panel = tg.asics_per_col * tg.asics_per_row;
  int tile = id / ng;
  t.f = (id - tile * ng) * tg.fpw;
  if (tg.xcd_map) {
    // XCD-grouped table-major order: workgroups go to the 8 XCDs round-robin, so ids 8j + x of a
    // block of 8 tiles x ng frame groups run tile (block, x) on XCD x -- every frame of a tile on
    // ONE XCD, whose L2 then fetches the tile's tables once per launch instead of once per XCD
    // (the launcher sets xcd_map only when the tiles per frame are a multiple of 8)
    const int blk = id / (8 * ng), rem = id - blk * 8 * ng;
    tile = blk * 8 + (rem & 7);
    t.f = (rem >> 3) * tg.fpw;
  }
  t.tile = tile;
  t.panel = tile / per_panel;
  t.ar = (tile % per_panel) / tg.asics_per_row;
  t.ac = (tile % per_panel) % tg.asics_per_row;
  if (PR_CM_IMG_ORDER && desc != nullptr) {
    const int sx = desc[3 * t.panel + 2];
    if (sx != 1 && sx != -1) {   // column runs: ASIC rows fastest
      t.ar = (tile % per_panel) % tg.asics_per_col;
      t.ac = (tile % per_panel) / tg.asics_per_col;
    }
  }
  t.base = (int64_t)t.panel * tg.panel_rows * tg.panel_cols + (int64_t)t.ar * R * tg.panel_cols + (int64_t)t.ac * C;
  return t;
}

// Phase 1 (runtime-shape loop form): decode + pedestal into the tile, side slots for groups with
// non-eligible pixels.  Whole waves iterate together (side_put is a wave-wide ballot).
template <int KIND, int NT>
__device__ __forceinline__ void cm_phase1(float* tile, SideCtx& sc, const int P, const int R, const int C,
                                          const TileGeom& tg, const PR_GLOBAL uint16_t* raw,
                                          const float* __restrict__ ped, const uint8_t* __restrict__ planes,
                                          int64_t base) {
  const int C8 = C >> 3;
  const int n = R * C8;
  for (int i0 = threadIdx.x & ~63; i0 < n; i0 += blockDim.x) {
    const int i = i0 + (threadIdx.x & 63);
    const bool act = i < n;
    const int r = act ? i / C8 : 0, k = act ? i - r * C8 : 0, c = k * 8;
    const int64_t pix = base + (int64_t)r * tg.panel_cols + c;
    float v[8];
    uint32_t el = 0xFFu, cb = 0;
    if (act) {
      const uint4 rw = ld_nt_u4((const PR_GLOBAL uint4*)(raw + pix));
      const uint32_t ep = load_planes<NT>(planes, pix);
      float pa[NT][8];
      load8<NT>(ped, tg.npix, pix, need_from_raw<NT>(rw), pa);
      cm_decode8<KIND, NT>(rw, ep, pa, v, el, cb);
      float x[8];
      cm_tile_values(v, el, x);
      float* trow = tile + r * P + c;
      *reinterpret_cast<float4*>(trow) = make_float4(x[0], x[1], x[2], x[3]);
      *reinterpret_cast<float4*>(trow + 4) = make_float4(x[4], x[5], x[6], x[7]);
    }
    const uint32_t slot = side_put(sc, act && el != 0xFFu, v);
    if (act) cm_put_meta<NT>(reinterpret_cast<uint8_t*>(tile + r * P + C), C, k, cb, slot);
  }
}

// ==========================================================================================
// Generic kernel (any ASIC shape): 1024 threads, one wave per row segment / column with
// cross-lane bitonic sorts.  Fallback for shapes without a compile-time instantiation below.
// ==========================================================================================
template <int KIND>
__global__ __launch_bounds__(1024) void calib_cm_kernel(const FramePtrs fp, const float* __restrict__ ped,
                                                        const float* __restrict__ gf,
                                                        const uint8_t* __restrict__ planes, const TileGeom tg,
                                                        const CmParams cp, const ImgOut io) {
  constexpr int NT = KIND == kEpix10ka ? 2 : (KIND == kJungfrau ? 3 : 1);
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int R = tg.asic_rows, C = tg.asic_cols, P = tg.pitch;
  float* tile = reinterpret_cast<float*>(smem);
  float* side = tile + R * P;
  SideCtx sc = side_ctx(side, tg.side_slots);
  const TileCoord t = cm_coords(tg, R, C);
  const PR_GLOBAL uint16_t* raw = gin<uint16_t>(fp.in[t.f]);
  PR_GLOBAL float* out = gout<float>(fp.out[t.f]);
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int nwaves = blockDim.x >> 6;

  cm_phase1<KIND, NT>(tile, sc, P, R, C, tg, raw, ped, planes, t.base);
  __syncthreads();
  const float INF = __int_as_float(0x7f800000);

  // ---- rows per bank segment: a wave sorts up to 4 segments (one element per lane) --------
  if (cp.flags & 1) {
    const int L = cp.bank_cols;
    const int nbanks = C / L;
    for (int r = wave; r < R; r += nwaves) {
      float* trow = tile + r * P;
      for (int b0 = 0; b0 < nbanks; b0 += 4) {
        float x[4], v[4];
        int cnt[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const bool in = (b0 + j < nbanks) && (lane < L);
          v[j] = in ? trow[(b0 + j) * L + lane] : __int_as_float(0x7fc00000);
          const bool part = fabsf(v[j]) < cp.thr;   // NaN (not eligible / outside) never participates
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
            if (fabsf(med) <= cp.maxcorr && (b0 + j < nbanks) && lane < L) trow[(b0 + j) * L + lane] = v[j] - med;
          }
        }
      }
    }
    __syncthreads();
  }

  // ---- columns: one wave per column (<= 256 rows, 4 per lane) --------------------------------
  if (cp.flags & 2) {
    for (int c = wave; c < C; c += nwaves) {
      float x[4], v[4];
      int cnt = 0;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int r = k * 64 + lane;
        v[k] = r < R ? tile[r * P + c] : __int_as_float(0x7fc00000);
        const bool part = fabsf(v[k]) < cp.thr;
        x[k] = part ? v[k] : INF;
        cnt += __popcll(__ballot(part));
      }
      col_sort_from<2>(x, lane);
      if (cnt >= cp.npix_min && cnt > 0) {
        const float med = median_sorted4(x, cnt);
        if (fabsf(med) <= cp.maxcorr) {
#pragma unroll
          for (int k = 0; k < 4; ++k)
            if (k * 64 + lane < R) tile[(k * 64 + lane) * P + c] = v[k] - med;   // NaN stays NaN
        }
      }
    }
    __syncthreads();
  }

  cm_store<KIND, NT>(tile, side, P, R, C, tg, raw, ped, gf, t.base, out, io, t.tile, t.panel, t.ar * R, t.ac * C,
                     !((tg.plain_mask >> t.f) & 1));
}

// ==========================================================================================
// Production kernel: per-lane in-register selection / sorting networks.
//
//  rows:    ONE lane owns one (row, bank) segment of L pixels (12 x ds_read_b128 for L = 48),
//           pads non-participants with alternating -inf/+inf (the first gets -inf), so the numpy
//           median of the participants is x[L/2] (odd count) or (x[L/2-1] + x[L/2]) / 2 (even)
//           after the median-cone network select_regs<L, L/2-1, L/2>.
//  columns: FOUR lanes (a quad) per column, M = ceil(R/4) rows each: per-lane sorts, a DPP
//           merge-split between lanes (q, q^1), then merge-path between the two pairs for the two
//           fixed middle positions of the balanced-padded 4M elements.
// ==========================================================================================
template <int CTRL>
__device__ __forceinline__ float dpp_quad(float x) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), CTRL, 0xF, 0xF, false));
}
template <int CTRL>
__device__ __forceinline__ int dpp_quad_i(int x) {
  return __builtin_amdgcn_mov_dpp(x, CTRL, 0xF, 0xF, false);
}

// max(+-quad_perm(a), +-b) as ONE v_max_f32 with a DPP source (the builtin mov_dpp + v_maximum3 is
// two VALU: v_maximum3 is VOP3, which takes no DPP operand on gfx950).  v_max_f32 is IEEE maxNum: it
// differs from maximum only for NaN operands and the order of -0 / +0, and the median networks
// carry neither a NaN nor a sign of zero that matters (a -0 median subtracts like +0).  The s_nop
// covers the VALU-write -> DPP-read hazard (2 wait states), which the compiler does not insert for
// inline asm.  PERM: 0xB1 = quad_perm [1,0,3,2] (lane q^1), 0x1B = [3,2,1,0] (lane q^3).
#ifndef PR_CM_DPP_MAX
#define PR_CM_DPP_MAX 1
#endif
#define PR_DPP_MAX_ASM(PERMSTR, SA, SB) \
  asm("s_nop 1\n\tv_max_f32_dpp %0, " SA "%1, " SB "%2 quad_perm:" PERMSTR " row_mask:0xf bank_mask:0xf" \
      : "=v"(r) : "v"(a), "v"(b))
template <int PERM, bool NEG_A, bool NEG_B>
__device__ __forceinline__ float max_dpp(float a, float b) {
#if PR_CM_DPP_MAX
  static_assert(PERM == 0xB1 || PERM == 0x1B, "max_dpp: quad permutation");
  float r;
  if constexpr (PERM == 0xB1) {
    if constexpr (NEG_A && NEG_B) PR_DPP_MAX_ASM("[1,0,3,2]", "-", "-");
    else if constexpr (NEG_A) PR_DPP_MAX_ASM("[1,0,3,2]", "-", "");
    else if constexpr (NEG_B) PR_DPP_MAX_ASM("[1,0,3,2]", "", "-");
    else PR_DPP_MAX_ASM("[1,0,3,2]", "", "");
  } else {
    if constexpr (NEG_A && NEG_B) PR_DPP_MAX_ASM("[3,2,1,0]", "-", "-");
    else if constexpr (NEG_A) PR_DPP_MAX_ASM("[3,2,1,0]", "-", "");
    else if constexpr (NEG_B) PR_DPP_MAX_ASM("[3,2,1,0]", "", "-");
    else PR_DPP_MAX_ASM("[3,2,1,0]", "", "");
  }
  return r;
#else
  const float p = dpp_quad<PERM>(a);
  return vmax(NEG_A ? -p : p, NEG_B ? -b : b);
#endif
}
#undef PR_DPP_MAX_ASM

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
        z[i] = vmin(a, b);
        z[i + j] = vmax(a, b);
      }
    }
  }
}

__device__ __forceinline__ uint4 ld_raw_u4(const PR_GLOBAL uint4* p) {
#if PR_CM_RAW_NT
  return ld_nt_u4(p);
#else
  const u32x4_t v = *(const PR_GLOBAL u32x4_t*)p;
  return make_uint4(v.x, v.y, v.z, v.w);
#endif
}

// PR_CM_MEMPROBE (diagnostic, WRONG results; flags-0 timing of the memory phases): bit 1 = no pedestal
// loads in phase 1, 2 = no gain-factor loads in phase 3, 4 = no raw loads, 8 = no flush stores,
// 16 = no eligibility-plane loads.  A removed load is replaced by an opaque per-lane value (base
// gain, every pixel eligible), so the rest of the kernel runs the same instruction stream.
#ifndef PR_CM_MEMPROBE
#define PR_CM_MEMPROBE 0
#endif
#if PR_CM_MEMPROBE
template <int NT, bool RAW_IN>
__device__ __forceinline__ void cm_probe_loads(const PR_GLOBAL uint16_t* raw_t, const PR_GLOBAL uint8_t* pl_t,
                                               const PR_GLOBAL float* const (&ped_t)[NT], uint32_t o, int tid,
                                               uint4& rw, uint32_t& ep, float (&pa0)[1][8]) {
  if constexpr (!RAW_IN) {
    if constexpr (PR_CM_MEMPROBE & 4) {
      uint32_t z = 0x01000100u + ((uint32_t)tid & 0xffu) * 0x00010001u;
      asm volatile("" : "+v"(z));
      rw = make_uint4(z, z ^ 0x00010001u, z ^ 0x00020002u, z ^ 0x00030003u);
    } else {
      rw = ld_raw_u4((const PR_GLOBAL uint4*)(raw_t + o));
    }
  }
  if constexpr (PR_CM_MEMPROBE & 16) {
    uint32_t z = 0xFFFFFFFFu;
    asm volatile("" : "+v"(z));
    ep = z;
  } else {
    ep = load_planes_o<NT>(pl_t, o);
  }
  if constexpr (PR_CM_MEMPROBE & 1) {
    for (int j = 0; j < 8; ++j) {
      uint32_t z = 0x42c80000u + (uint32_t)j;   // ~100.0
      asm volatile("" : "+v"(z));
      pa0[0][j] = __uint_as_float(z);
    }
  } else {
    load8o<1>(reinterpret_cast<const PR_GLOBAL float* const(&)[1]>(ped_t), o, 1u, pa0);
  }
}
#endif

// TR / TC: the tile rows / columns as compile-time constants for the production shapes (0 = from
// TileGeom): every LDS address in the unrolled loops is then a base VGPR + immediate offset.
// Phase 1, compile-time tile shape: decode + pedestal of the tile into LDS by BLOCK threads
// (thread index tid in [0, BLOCK)).
template <int KIND, int NT, int BLOCK, int TR, int TC, bool RAW_IN, bool SG>
__device__ __forceinline__ void cm_load_net(float* tile, SideCtx& sc, const int P, const TileGeom& tg,
                                            const PR_GLOBAL uint16_t* raw, const float* __restrict__ ped,
                                            const uint8_t* __restrict__ planes, const int64_t base, const int tid,
                                            uint4 (&rw)[(TR * (TC / 8) + BLOCK - 1) / BLOCK],
                                            const PR_GLOBAL uint16_t* raw_next) {
  constexpr int C = TC;
  constexpr int NITEMS = TR * (TC / 8);
  constexpr int NI = (NITEMS + BLOCK - 1) / BLOCK;
  // all of this lane's raw / plane / first-table loads in flight at once; the rare switched-gain
  // tables are loaded per group while decoding (select-then-load, the wave waits only when one of
  // its lanes needs them), which keeps the live registers at raw + planes + one table.  RAW_IN: the
  // raw words were prefetched by the previous frame's phase 1 (they arrived during its medians).
  constexpr int C8 = TC / 8;
  uint32_t ep[NI];
  float pa0[NI][1][8];
#if PR_CM_OFF32
  // uniform (SGPR) bases at the tile origin; per item one 32-bit offset
  const PR_GLOBAL uint16_t* raw_t = raw + base;
  const PR_GLOBAL uint8_t* pl_t = (const PR_GLOBAL uint8_t*)planes + CmLayout<NT>::kPlaneBytes * (base >> 3);
  const PR_GLOBAL float* ped_t[NT];
#pragma unroll
  for (int k = 0; k < NT; ++k) ped_t[k] = (const PR_GLOBAL float*)ped + k * tg.npix + base;
#endif
#pragma unroll
  for (int u = 0; u < NI; ++u) {
    const int i = tid + u * BLOCK;
    if ((u + 1) * BLOCK <= NITEMS || i < NITEMS) {
      const int r = i / C8, c = (i % C8) * 8;
#if PR_CM_OFF32
      const uint32_t o = (uint32_t)(r * tg.panel_cols + c);
#if PR_CM_MEMPROBE
      cm_probe_loads<NT, RAW_IN>(raw_t, pl_t, ped_t, o, tid, rw[u], ep[u], pa0[u]);
#else
      if constexpr (!RAW_IN) rw[u] = ld_raw_u4((const PR_GLOBAL uint4*)(raw_t + o));
      if constexpr (SG) ep[u] = 0u;   // eligibility rides in the pedestals' sign bits
      else ep[u] = load_planes_o<NT>(pl_t, o);
      load8o<1>(reinterpret_cast<const PR_GLOBAL float* const(&)[1]>(ped_t), o, 1u, pa0[u]);
#endif
#else
      const int64_t pix = base + (int64_t)r * tg.panel_cols + c;
      if constexpr (!RAW_IN) rw[u] = ld_raw_u4((const PR_GLOBAL uint4*)(raw + pix));
      ep[u] = load_planes<NT>(planes, pix);
      load8<1>(ped, tg.npix, pix, 1u, pa0[u]);
#endif
    }
  }
#pragma unroll
  for (int u = 0; u < NI; ++u) {
    const int i = tid + u * BLOCK;
    const bool act = (u + 1) * BLOCK <= NITEMS || i < NITEMS;
    const int r = act ? i / C8 : 0, k = act ? i % C8 : 0, c = k * 8;
    float v[8];
    float x[8];
    uint32_t el = 0xFFu, cb = 0;
    if (act) {
      if (PR_CM_BASE_FAST && NT > 1 && __builtin_amdgcn_ballot_w64(!cm_base_only<KIND>(rw[u])) == 0) {
        // wave-uniform: no switched pixel
        if constexpr (SG) {
          el = cm_decode8_base_sg<KIND>(rw[u], pa0[u][0], v, x) ? 0u : 0xFFu;   // only el != 0xFF is read
        } else {
          cm_decode8_base<KIND>(rw[u], ep[u], pa0[u][0], v, el);
          cm_tile_values(v, el, x);
        }
      } else {
        float pa[NT][8];
#pragma unroll
        for (int j = 0; j < 8; ++j) pa[0][j] = pa0[u][0][j];
        if constexpr (NT > 1) {
#if PR_CM_OFF32
          load8o<NT>(ped_t, (uint32_t)(r * tg.panel_cols + c), need_from_raw<NT>(rw[u]), pa, 1);
#else
          load8<NT>(ped, tg.npix, base + (int64_t)r * tg.panel_cols + c, need_from_raw<NT>(rw[u]), pa, 1);
#endif
        }
        cm_decode8<KIND, NT, SG>(rw[u], ep[u], pa, v, el, cb);
        cm_tile_values(v, el, x);
      }
      float* trow = tile + r * P + c;
      *reinterpret_cast<float4*>(trow) = make_float4(x[0], x[1], x[2], x[3]);
      *reinterpret_cast<float4*>(trow + 4) = make_float4(x[4], x[5], x[6], x[7]);
    }
    const uint32_t slot = side_put(sc, act && el != 0xFFu, v);   // convergent: whole wave
    if (act) cm_put_meta<NT>(reinterpret_cast<uint8_t*>(tile + r * P + C), C, k, cb, slot);
  }
  // the next frame's raw words: in flight during this frame's medians and store (no barrier waits
  // on vector memory; the registers are free again)
  if (raw_next != nullptr) {
#pragma unroll
    for (int u = 0; u < NI; ++u) {
      const int i = tid + u * BLOCK;
      if ((u + 1) * BLOCK <= NITEMS || i < NITEMS) {
        const int r = i / C8, c = (i % C8) * 8;
        rw[u] = ld_raw_u4((const PR_GLOBAL uint4*)(raw_next + base + (int64_t)r * tg.panel_cols + c));
      }
    }
  }
}

// Row-segment medians (one lane per (row, bank) segment), threads t0, t0 + nt, ... of the workgroup.
template <int L>
__device__ __forceinline__ void cm_rows(float* tile, const int P, const int R, const int C, const CmParams& cp,
                                        const int t0, const int nt) {
  const float INF = __int_as_float(0x7f800000);
  const int nbank = C / L;
  for (int sgi = t0; sgi < R * nbank; sgi += nt) {
    const int b = sgi / R, r = sgi % R;           // consecutive lanes -> consecutive rows
    float* seg = tile + r * P + b * L;
    float x[L];
    int cnt = 0;
    float pad = -INF;
    if constexpr (L % 4 == 0) {
#pragma unroll
      for (int j = 0; j < L; j += 4) {
        const float4 q = *reinterpret_cast<const float4*>(seg + j);
        const float e[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const bool pt = fabsf(e[u]) < cp.thr;
          cnt += pt ? 1 : 0;
          x[j + u] = pt ? e[u] : pad;
          pad = pt ? pad : -pad;
        }
      }
    } else {
#pragma unroll
      for (int j = 0; j < L; ++j) {
        const float e = seg[j];
        const bool pt = fabsf(e) < cp.thr;
        cnt += pt ? 1 : 0;
        x[j] = pt ? e : pad;
        pad = pt ? pad : -pad;
      }
    }
    asm volatile("" ::: "memory");   // keep the write-back's LDS reads below the network
    constexpr int PA = (L & 1) ? (L - 1) / 2 : L / 2 - 1;
    constexpr int PB = PA + 1;
    select_regs<L, PA, PB>(x);
    asm volatile("" ::: "memory");
    // toggle padding: L even -> odd count: x[L/2], even: mean of x[L/2-1], x[L/2];
    //                 L odd  -> odd count: x[(L-1)/2], even: mean of x[(L-1)/2], x[(L+1)/2]
    float med;
    if constexpr ((L & 1) == 0) med = (cnt & 1) ? x[PB] : (x[PA] + x[PB]) * 0.5f;
    else med = (cnt & 1) ? x[PA] : (x[PA] + x[PB]) * 0.5f;
    if (cnt >= cp.npix_min && cnt > 0 && fabsf(med) <= cp.maxcorr) {
      // every element minus the median: NaN (non-eligible) stays NaN
      if constexpr (L % 4 == 0) {
#pragma unroll
        for (int j = 0; j < L; j += 4) {
          float4 q = *reinterpret_cast<const float4*>(seg + j);
          q.x -= med; q.y -= med; q.z -= med; q.w -= med;
          *reinterpret_cast<float4*>(seg + j) = q;
        }
      } else {
#pragma unroll
        for (int j = 0; j < L; ++j) seg[j] -= med;
      }
    }
  }
}

// PR_CM_COL_ONELOAD = 1: the column phase reads its values from LDS once (pass 2 from registers)
#ifndef PR_CM_COL_ONELOAD
#define PR_CM_COL_ONELOAD 1
#endif
// PR_CM_PK_COLSUB = 0: the column correction one v_sub_f32 per row (A/B of the packed form)
#ifndef PR_CM_PK_COLSUB
#define PR_CM_PK_COLSUB 1
#endif
// Column medians, FOUR lanes (a quad) per column, M rows each (t0 a multiple of 4).
//  Sign domain: the odd lane of each pair (q = 1, 3) holds its values NEGATED, so both lanes of a
//  pair run identical instructions where the classic merge-split needs lane-dependent min / max:
//   1. pass 1 counts the participants (|v| < thr); the quad's totals fix how many non-participants
//      become -inf (the rest +inf: balanced padding puts the median at fixed ranks 2M-1, 2M);
//      pass 2 reloads the column and writes sign-domain values and pads (no NaN survives);
//   2. every lane sorts its M values ascending (sort_regs<M>);
//   3. level 1, lanes (q, q^1): z[i] = max(partner[i], -x[i]) is the V-shaped merge-split half for
//      BOTH lanes (even lane: -min(l[i], u[M-1-i]); odd lane: max(l[i], u[M-1-i])), one DPP fetch
//      and ONE v_maximum3 (neg modifier) per register; bitonic_merge_vpad sorts it.  Afterwards
//      the even lane holds -A[M-1-i], the odd lane A[M+i] (A = the pair's 2M sorted values);
//   4. level 2, lanes (q, q^3) -- merge path of pair (0,1) with pair (2,3): lanes 1 and 3 each
//      see half of the split terms max(A[a], B[k-1-a]) as max(z[t], -partner[t]) (k = 2M) and
//      max(z[t], -partner[t+1]) (k = 2M-1), plus the end terms z[M-1] and max(A[M-1], B[M-1]);
//      the k-th value is the min over both lanes.
template <int M>
__device__ __forceinline__ void cm_cols(float* tile, const int P, const int R, const int C, const CmParams& cp,
                                        const int t0, const int nt) {
  static_assert(M % 2 == 0, "cm_cols: M must be even (interleaved rows)");
  const float INF = __int_as_float(0x7f800000);
  const float QNAN = __int_as_float(0x7fc00000);
  const int nwork = 4 * C;
  for (int w = t0; w < ((nwork + 63) / 64) * 64; w += nt) {
    const bool act = w < nwork;
    const int c = act ? (w >> 2) : 0;
    const int q = w & 3;
    // Rows of the column per lane: lane q takes rows 8j + 2q + b (b = 0, 1), so for a fixed
    // element the quad's four addresses differ by 2P rows -- 8 banks apart for the pitches in use
    // (P = 52: 2P = 104 = 8 mod 32; P = 140: 280 = 24 mod 32) -- and the 8 columns of a half wave
    // fill all 32 banks.  The median does not depend on which lane holds which row.
    float* colp = tile + 2 * q * P + c;
    auto row_of = [&](int i) { return 8 * (i >> 1) + 2 * q + (i & 1); };
    auto off_of = [&](int i) { return (8 * (i >> 1) + (i & 1)) * P; };
    auto load = [&](int i) { return (act && row_of(i) < R) ? colp[off_of(i)] : QNAN; };
    float x[M];
#if PR_CM_COL_ONELOAD
    // ONE pass over LDS: the column into registers, participants counted on the way (inactive lanes
    // -- whole quads past the tile's columns -- read column 0 and never write: no per-element select)
    int my_cnt = 0;
#pragma unroll
    for (int i = 0; i < M; ++i) {
      x[i] = row_of(i) < R ? colp[off_of(i)] : QNAN;
      my_cnt += fabsf(x[i]) < cp.thr ? 1 : 0;
      if ((i & 15) == 15) asm volatile("" ::: "memory");
    }
#else
    // pass 1: participants of this lane
    int my_cnt = 0;
#pragma unroll
    for (int i = 0; i < M; ++i) {
      my_cnt += fabsf(load(i)) < cp.thr ? 1 : 0;
      if ((i & 15) == 15) asm volatile("" ::: "memory");
    }
#endif
    // quad totals + exclusive prefix of the non-participants: balanced +-inf padding
    const int my_inv = M - my_cnt;
    const int i0 = dpp_quad_i<0x00>(my_inv), i1 = dpp_quad_i<0x55>(my_inv);
    const int i2 = dpp_quad_i<0xAA>(my_inv), i3 = dpp_quad_i<0xFF>(my_inv);
    const int total_inv = i0 + i1 + i2 + i3;
    const int cnt = 4 * M - total_inv;
    const int a = total_inv >> 1;
    const int prefix = (q > 0 ? i0 : 0) + (q > 1 ? i1 : 0) + (q > 2 ? i2 : 0);
    // pass 2: sign-domain values; pads are -inf while s >= 0 (the first neg_budget of them)
    int s = min(my_inv, max(0, a - prefix)) - 1;
    const uint32_t flip = (q & 1) ? 0x80000000u : 0u;
    uint32_t pad_base = 0xff800000u ^ flip;
    asm volatile("" : "+v"(pad_base));   // one v_bitop3 per pad below, not bitop3 + xor
#pragma unroll
    for (int i = 0; i < M; ++i) {
      const float v = PR_CM_COL_ONELOAD ? x[i] : load(i);
      const bool pt = fabsf(v) < cp.thr;
      const uint32_t padb = ((uint32_t)s & 0x80000000u) ^ pad_base;
      x[i] = __uint_as_float(pt ? (__float_as_uint(v) ^ flip) : padb);
      s -= pt ? 0 : 1;
      if ((i & 15) == 15) asm volatile("" ::: "memory");
    }
    asm volatile("" ::: "memory");
    sort_regs3<M>(x);
    // level 1: merge-split with lane q^1, both lanes V-shaped
    float z[M];
#pragma unroll
    for (int i = 0; i < M; ++i) z[i] = max_dpp<0xB1, false, true>(x[i], x[i]);
    if constexpr (have_vmerge3<M>()) vmerge_regs3<M>(z);
    else bitonic_merge_vpad<M>(z);
    asm volatile("" ::: "memory");
    // level 2: merge path with lane q^3 (lanes 1 and 3 hold the terms)
    float kh = INF, kl = INF;
    const float p0 = dpp_quad<0x1B>(z[0]);
#pragma unroll
    for (int t = 0; t < M; ++t) {
      kh = vmin(kh, max_dpp<0x1B, true, false>(z[t], z[t]));            // max(z[t], -partner z[t])
      if (t + 1 < M) kl = vmin(kl, max_dpp<0x1B, true, false>(z[t + 1], z[t]));   // max(z[t], -partner z[t+1])
    }
    const float e = -vmin(p0, dpp_quad<0xB1>(z[0]));   // max(A[M-1], B[M-1]) on lanes 1 and 3
    kl = vmin(kl, vmin(z[M - 1], e));
    const float k_lo = vmin(dpp_quad<0x55>(kl), dpp_quad<0xFF>(kl));
    const float k_hi = vmin(dpp_quad<0x55>(kh), dpp_quad<0xFF>(kh));
    const float med = (k_lo + ((cnt & 1) ? k_lo : k_hi)) * 0.5f;
    asm volatile("" ::: "memory");
    if (act && cnt >= cp.npix_min && cnt > 0 && fabsf(med) <= cp.maxcorr) {
      // every element minus the median (NaN -- non-eligible -- stays NaN), two rows per v_pk_add_f32:
      // rows 2j and 2j + 1 of a lane are one ds_read2_b32 / ds_write2_b32 pair
      const f32x2_t m2 = {med, med};
#pragma unroll
      for (int i = 0; i < M; i += 2) {
        if (PR_CM_PK_COLSUB && row_of(i + 1) < R) {
          f32x2_t v = {colp[off_of(i)], colp[off_of(i + 1)]};
          v -= m2;
          colp[off_of(i)] = v.x;
          colp[off_of(i + 1)] = v.y;
        } else {
          if (row_of(i) < R) colp[off_of(i)] -= med;
          if (!PR_CM_PK_COLSUB && row_of(i + 1) < R) colp[off_of(i + 1)] -= med;
        }
        if ((i & 14) == 14) asm volatile("" ::: "memory");
      }
    }
  }
}

// PR_CM_MAX_VGPR > 0: cap the net kernel's VGPRs (diagnostic builds: leave room on each SIMD for
// a co-resident consumer kernel's wave)
#ifndef PR_CM_MAX_VGPR
#define PR_CM_MAX_VGPR 0
#endif
#if PR_CM_MAX_VGPR > 0
#define PR_CM_VGPR_ATTR __attribute__((amdgpu_num_vgpr(PR_CM_MAX_VGPR / 2)))   // gfx950: the request counts twice (VGPR + AGPR file)
#else
#define PR_CM_VGPR_ATTR
#endif
#ifndef PR_CM_NET_MAXNI
#define PR_CM_NET_MAXNI 8
#endif
// signed pedestal tables for the production shapes (0: always the bit-planes, the A/B build)
#ifndef PR_CM_SG
#define PR_CM_SG 1
#endif
// Jungfrau stripe width: 128 (one 256x128 tile per CU, 512 threads) or 64 (two 256x64 tiles per CU,
// 256 threads each -- one workgroup's median phases overlap the other's memory phases)
#ifndef PR_CM_JF_W
#define PR_CM_JF_W 64
#endif
template <int KIND, int L, int M, int BLOCK, int TR = 0, int TC = 0, bool SG = false>
__global__ __launch_bounds__(BLOCK, M <= 48 ? (BLOCK / 64) * PR_CM_EPIX_WG_PER_CU / 4 : 2) PR_CM_VGPR_ATTR void calib_cm_net_kernel(
    const FramePtrs fp, const float* __restrict__ ped, const float* __restrict__ gf,
    const uint8_t* __restrict__ planes, const TileGeom tg, const CmParams cp, const ImgOut io) {
  constexpr int NT = KIND == kEpix10ka ? 2 : (KIND == kJungfrau ? 3 : 1);
  constexpr int PC = (TC > 0) ? cm_pitch(TC, CmLayout<NT>::kCandBits) : 0;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int R = TR ? TR : tg.asic_rows, C = TC ? TC : tg.asic_cols;
  const int P = PC ? PC : tg.pitch;
  float* tile = reinterpret_cast<float*>(smem);
  float* side = tile + R * P;
  SideCtx sc = side_ctx(side, tg.side_slots);
  const TileCoord t = cm_coords(tg, R, C, (int)blockIdx.x, io.desc);
  const int tid = threadIdx.x;
  constexpr int NITEMS = (TR > 0 && TC > 0) ? TR * (TC / 8) : 0;
  constexpr int NI = NITEMS > 0 ? (NITEMS + BLOCK - 1) / BLOCK : 0;
  // compile-time phase-1 / store form when every lane's items fit in registers: up to 6 items at the
  // epix10k2M kernel's 128-VGPR budget (four workgroups per CU), up to PR_CM_NET_MAXNI (8) for the
  // Jungfrau 256x128 stripe, whose 135-KB tile allows one workgroup per CU (256 VGPRs)
  constexpr bool kNet = NI > 0 && NI <= (M <= 48 ? 6 : PR_CM_NET_MAXNI);
  // signed pedestals (no bit-planes, `planes` may be null) only in the compile-time phase-1 / store form
  static_assert(!SG || kNet, "calib_cm_net_kernel: signed pedestal tables need the compile-time tile form");
  // frames of this workgroup (tg.fpw consecutive frames of one tile; the compile-time production
  // shapes prefetch frame k+1's raw words during frame k's medians)
  const int nf = min(tg.fpw, tg.nframes - t.f);
  uint4 rw[kNet ? NI : 1];
  // Median-phase work -> lanes: thread t takes row segment / column lane t (spreading the work
  // evenly over the four waves measured neutral: the same instruction stream per wave either way)
  const int rows_t0 = tid, rows_nt = (int)blockDim.x, cols_t0 = tid, cols_nt = (int)blockDim.x;
#if PR_CM_STAMPS
  uint64_t st_[12] = {};
  const uint64_t rt0 = __builtin_amdgcn_s_memrealtime();
  PR_STAMP(0);
#endif
  auto frame = [&](const int fi) {
    const int f = t.f + fi;
    const PR_GLOBAL uint16_t* raw = gin<uint16_t>(fp.in[f]);
    PR_GLOBAL float* out = gout<float>(fp.out[f]);
    if (fi > 0) {
      __syncthreads();   // the previous frame's store phase read the tile
      sc.used = 0;
    }
    // opaque per-frame copies of the tile base and the table pointers: the compiler must not keep
    // every per-item address of the frame body live across the loop (loop-invariant hoisting of
    // ~40 VGPRs of 64-bit addresses spills the kernel)
    int64_t tb = t.base;
    const float* pedp = ped;
    const float* gfp = gf;
    const uint8_t* plp = planes;
    asm volatile("" : "+s"(tb), "+s"(pedp), "+s"(gfp), "+s"(plp));

    // ---- phase 1: decode + pedestal into LDS ----------------------------------------------
    if constexpr (kNet) {
      const PR_GLOBAL uint16_t* raw_next = fi + 1 < nf ? gin<uint16_t>(fp.in[f + 1]) : nullptr;
      if (fi == 0)
        cm_load_net<KIND, NT, BLOCK, TR, TC, false, SG>(tile, sc, P, tg, raw, pedp, plp, tb, tid, rw, raw_next);
      else
        cm_load_net<KIND, NT, BLOCK, TR, TC, true, SG>(tile, sc, P, tg, raw, pedp, plp, tb, tid, rw, raw_next);
    } else {
      cm_phase1<KIND, NT>(tile, sc, P, R, C, tg, raw, pedp, plp, tb);
    }
    PR_STAMP(1);
    // PR_CM_GPRE: the first gain table of every item is loaded now and arrives during the medians,
    // so the store phase has no memory round trip before its first output (+40 VGPRs)
    float g0[kNet ? NI : 1][1][8];
    if constexpr (kNet && PR_CM_GPRE) {
      constexpr int C8 = TC / 8;
#pragma unroll
      for (int u = 0; u < NI; ++u) {
        const int i = tid + u * BLOCK;
        if ((u + 1) * BLOCK <= NITEMS || i < NITEMS)
          load8<1>(gfp, tg.npix, tb + (int64_t)(i / C8) * tg.panel_cols + (i % C8) * 8, 1u, g0[u]);
      }
    }
    __syncthreads();
    PR_STAMP(2);

    // ---- phase 2a: rows by bank, one lane per segment ------------------------------------
    if (cp.flags & 1) {
      cm_rows<L>(tile, P, R, C, cp, rows_t0, rows_nt);
      PR_STAMP(3);
      __syncthreads();
      PR_STAMP(4);
    }

    // ---- phase 2b: columns -----------------------------------------------------------------
    if (cp.flags & 2) {
      cm_cols<M>(tile, P, R, C, cp, cols_t0, cols_nt);
      PR_STAMP(5);
      __syncthreads();
      PR_STAMP(6);
    }

    // ---- phase 3: gain factor + mask, store ----------------------------------------------
    if constexpr (kNet) {
      // compile-time shape: every gain-factor load of this lane in flight before the first use
      constexpr int C8 = TC / 8;
      // (the first gain table of every item up front; the switched-gain tables are rare and are
      // loaded per item, which keeps the production kernel within 128 VGPRs)
      uint32_t cbs[NI], slots[NI];
#if PR_CM_OFF32
      const PR_GLOBAL float* gf_t[NT];
#pragma unroll
      for (int k = 0; k < NT; ++k) gf_t[k] = (const PR_GLOBAL float*)gfp + k * tg.npix + tb;
#endif
#pragma unroll
      for (int u = 0; u < NI; ++u) {
        const int i = tid + u * BLOCK;
        if ((u + 1) * BLOCK <= NITEMS || i < NITEMS) {
          const int r = i / C8, k = i % C8, c = k * 8;
          cm_get_meta<NT>(reinterpret_cast<const uint8_t*>(tile + r * P + C), C, k, cbs[u], slots[u]);
#if PR_CM_OFF32
#if PR_CM_MEMPROBE & 2
          for (int j = 0; j < 8; ++j) {
            uint32_t z = 0x3f800000u + (uint32_t)j;
            asm volatile("" : "+v"(z));
            g0[u][0][j] = __uint_as_float(z);
          }
#else
          if constexpr (!PR_CM_GPRE)
            load8o<1>(reinterpret_cast<const PR_GLOBAL float* const(&)[1]>(gf_t), (uint32_t)(r * tg.panel_cols + c), 1u,
                      g0[u]);
#endif
#else
          if constexpr (!PR_CM_GPRE) load8<1>(gfp, tg.npix, tb + (int64_t)r * tg.panel_cols + c, 1u, g0[u]);
#endif
        }
      }
#pragma unroll
      for (int u = 0; u < NI; ++u) {
        const int i = tid + u * BLOCK;
        if ((u + 1) * BLOCK <= NITEMS || i < NITEMS) {
          const int r = i / C8, c = (i % C8) * 8;
          const int64_t pix = tb + (int64_t)r * tg.panel_cols + c;
          float ga[NT][8];
#pragma unroll
          for (int j = 0; j < 8; ++j) ga[0][j] = g0[u][0][j];
          float o[8];
          if (PR_CM_BASE_FAST && NT > 1 && __builtin_amdgcn_ballot_w64(cbs[u] != 0u) == 0) {
            // wave-uniform: every pixel of the item takes the table-0 gain factor
            cm_out8<KIND, NT, true, SG>(tile + r * P + c, side, cbs[u], slots[u], ga, raw, pedp, tg.npix, pix, o);
          } else {
#if PR_CM_OFF32
            if constexpr (NT > 1) load8o<NT>(gf_t, (uint32_t)(r * tg.panel_cols + c), cm_need<NT>(cbs[u]), ga, 1);
#else
            if constexpr (NT > 1) load8<NT>(gfp, tg.npix, pix, cm_need<NT>(cbs[u]), ga, 1);
#endif
            cm_out8<KIND, NT, false, SG>(tile + r * P + c, side, cbs[u], slots[u], ga, raw, pedp, tg.npix, pix, o);
          }
          cm_put8(tile + r * P + c, o);
        }
      }
      PR_STAMP(7);
#if PR_CM_STAMPS
      cm_write_out(tile, P, R, C, tg, io, t.tile, t.panel, t.ar * R, t.ac * C, tb, out, !((tg.plain_mask >> f) & 1),
                   [&](int k) { st_[k] = __builtin_amdgcn_s_memtime(); });
#else
      cm_write_out(tile, P, R, C, tg, io, t.tile, t.panel, t.ar * R, t.ac * C, tb, out, !((tg.plain_mask >> f) & 1));
#endif
      PR_STAMP(8);
    } else {
      cm_store<KIND, NT>(tile, side, P, R, C, tg, raw, pedp, gfp, tb, out, io, t.tile, t.panel, t.ar * R,
                         t.ac * C, !((tg.plain_mask >> f) & 1));
    }
  };
  if constexpr (kNet) {
#pragma unroll
    for (int fi = 0; fi < PR_CM_FPW; ++fi)   // straight-line frames (a loop hoists every address)
      if (fi < nf) frame(fi);
  } else {
    for (int fi = 0; fi < nf; ++fi) frame(fi);
  }
#if PR_CM_STAMPS
  if (kNet && g_cm_stamps != nullptr && (threadIdx.x & 63) == 0) {
    // stores of wave-uniform values: plain global stores from VGPRs
    uint64_t* rec = g_cm_stamps + ((uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * kCmStampWords;
    rec[0] = rt0;
    rec[1] = __builtin_amdgcn_s_memrealtime();
    rec[2] = (uint64_t)__builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));    // HW_REG_HW_ID
    rec[3] = (uint64_t)__builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (31 << 11));   // HW_REG_XCC_ID
#pragma unroll
    for (int k = 0; k < 12; ++k) rec[4 + k] = st_[k];
  }
#endif
}


// The production shapes whose compile-time kernels read the signed pedestal tables (launch_calib_cm
// picks them with the same predicate); Calibrator builds the tables only for these.
bool cm_signed_shape(int kind, int asic_rows, int asic_cols, int bank_cols) {
  if (!PR_CM_SG) return false;
  if (kind == kEpix10ka) return bank_cols == 48 && asic_rows == 176 && asic_cols % 48 == 0;
  if (kind == kJungfrau) return PR_CM_NET_MAXNI >= 8 && bank_cols == 64 && asic_rows == 256 && asic_cols % 128 == 0;
  return false;
}

size_t cm_lds_bytes(int asic_rows, int asic_cols, int kind) {
  const int cand_bits = kind == kJungfrau ? 2 : 1;
  return (size_t)asic_rows * cm_pitch(asic_cols, cand_bits) * 4;
}

// Width of the LDS tile a workgroup owns.  Row medians are per bank segment and column medians
// need whole columns, so an ASIC may be cut into full-height stripes whose width is a multiple
// of the bank width without changing any median (Jungfrau: 256x256 ASIC -> two 256x128 stripes).
// 0 = no stripe fits.
int cm_tile_cols(int asic_rows, int asic_cols, int bank_cols, int max_cols, int kind) {
  for (int w = std::min(asic_cols, max_cols > 0 ? max_cols : asic_cols); w >= bank_cols; --w) {
    if (asic_cols % w || w % bank_cols || w % 8) continue;
    if (cm_lds_bytes(asic_rows, w, kind) <= 160 * 1024) return w;
  }
  return 0;
}

template <typename K>
static void cm_launch(K kernel, dim3 grid, int block, size_t lds, hipStream_t s, const FramePtrs& fp,
                      const float* P, const float* G, const uint8_t* F, const TileGeom& tg, const CmParams& cp,
                      const ImgOut& io) {
  hip_check(hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds),
            "cm attr");
  hipLaunchKernelGGL(kernel, grid, dim3(block), lds, s, fp, P, G, F, tg, cp, io);
}

void launch_calib_cm(const FramePtrs& fp, int nframes, uint64_t ped, uint64_t gf, uint64_t planes, int kind,
                     int n_panels, int panel_rows, int panel_cols, int asic_rows, int asic_cols, float thr,
                     float maxcorr, int npix_min, int flags, int bank_cols, uint64_t stream, uint64_t img_desc,
                     uint64_t gap_runs, int n_gap_runs, uint64_t ped_sg, uint64_t plain_mask) {
  check(nframes >= 1 && nframes <= kMaxFrames, "calib_cm: nframes out of range");
  check(asic_rows >= 1 && asic_rows <= 256, "calib_cm: ASIC rows must be in [1, 256]");
  check(asic_cols % 8 == 0 && asic_cols >= 8, "calib_cm: ASIC cols must be a multiple of 8");
  check(panel_rows % asic_rows == 0 && panel_cols % asic_cols == 0, "calib_cm: panel not tiled by ASICs");
  check(bank_cols >= 1 && bank_cols <= 64 && asic_cols % bank_cols == 0,
        "calib_cm: bank_cols must be <= 64 and divide the ASIC width");
  check(panel_cols % 8 == 0, "calib_cm: panel cols must be a multiple of 8");
  check(kind == kEpix10ka || kind == kJungfrau || kind == kPlain, "calib_cm: unknown gain kind");
  check(flags >= 0 && flags <= 3, "calib_cm: flags must be in [0, 3] (bit0 rows, bit1 columns)");
  // Tile shape (one decision per shape, no run-time knobs):
  //  * epix10k2M (176-row ASICs, 48-column banks): one-bank 176x48 stripes on 256-thread blocks,
  //    four workgroups per CU (round 1: 8.8 us/frame vs 9.2 for 176x96, 15.8 full width);
  //  * Jungfrau (256x256 ASICs, 64-column banks): 256x64 stripes (one bank), 256-thread blocks, two
  //    workgroups per CU (PR_CM_JF_W; 256x128 on 512 threads, one per CU: 52.8 vs 37.3 us/frame);
  //  * otherwise: the widest stripe <= 128 columns whose tile fits half the LDS (two blocks per CU)
  //    when a compile-time network exists for the shape, else the widest that fits at all.
  const int M4 = (asic_rows + 3) / 4;
  const bool epix_prod = kind == kEpix10ka && bank_cols == 48 && asic_rows == 176 && asic_cols % 48 == 0;
  const bool jf_prod = kind == kJungfrau && bank_cols == 64 && asic_rows == 256 && asic_cols % 128 == 0;
  const bool net = epix_prod || jf_prod || (kind == kEpix10ka && bank_cols == 48 && M4 == 44) ||
                   (kind == kEpix10ka && bank_cols == 8 && M4 == 4);
  int max_w = 0;
  if (epix_prod) {
    max_w = 48;
  } else if (jf_prod) {
    max_w = PR_CM_JF_W;
  } else if (net) {
    for (int w = std::min(asic_cols, 128); w >= bank_cols; --w)
      if (asic_cols % w == 0 && w % bank_cols == 0 && w % 8 == 0 && cm_lds_bytes(asic_rows, w, kind) <= 80 * 1024) {
        max_w = w;
        break;
      }
  }
  const int full_cols = asic_cols;
  asic_cols = cm_tile_cols(asic_rows, full_cols, bank_cols, max_w, kind);
  if (asic_cols == 0) asic_cols = cm_tile_cols(asic_rows, full_cols, bank_cols, 0, kind);
  check(asic_cols > 0, "calib_cm: no full-height ASIC stripe fits in 160 KiB of LDS");
  const size_t lds = cm_lds_bytes(asic_rows, asic_cols, kind);
  check(aligned16(ped) && aligned16(gf) && aligned16(ped_sg) && (planes & 3) == 0,
        "calib_cm: misaligned constant tables");
  for (int f = 0; f < nframes; ++f)
    check(aligned16(fp.in[f]) && aligned16(fp.out[f]), "calib_cm: frame buffers must be 16-B aligned");
  check(n_gap_runs == 0 || (img_desc != 0 && gap_runs != 0 && gap_runs % 4 == 0), "calib_cm: bad gap table");
  const ImgOut io{reinterpret_cast<const int32_t*>(img_desc), reinterpret_cast<const int32_t*>(gap_runs),
                  img_desc != 0 ? n_gap_runs : 0};
  // signed pedestal tables (eligibility in the sign bits, no bit-plane loads): the production kernels,
  // whose phase 1 is the compile-time form (cm_load_net); the loop form (cm_phase1 / cm_store) of the
  // other shapes reads the bit-planes
  // (-DPR_CM_SG=0: always the bit-planes, the A/B build)
  if (!PR_CM_SG) ped_sg = 0;
  const float* PS = reinterpret_cast<const float*>(ped_sg);
  const bool sg_kernel = ((epix_prod && asic_cols == 48) ||
                          (jf_prod && asic_cols == PR_CM_JF_W && PR_CM_NET_MAXNI >= 8)) && ped_sg != 0;
  check(sg_kernel || planes != 0, "calib_cm: this shape needs the eligibility bit-planes");
  // LDS budget of one workgroup: the epix10k2M 176x48 stripe runs PR_CM_EPIX_WG_PER_CU workgroups
  // per CU, the two 256x64 Jungfrau stripes two, the narrow compile-time kernels two,
  // everything else one; what the tiles leave is side slots
  const size_t lds_tiles = lds;
  const size_t budget = (epix_prod && asic_cols == 48) ? (160 * 1024) / PR_CM_EPIX_WG_PER_CU
                        : (jf_prod && asic_cols == 64) ? 80 * 1024     // two 256x64 Jungfrau stripes per CU
                        : (net && !jf_prod && asic_cols <= 128) ? 80 * 1024
                                                                : 160 * 1024;
  const int side_slots = (int)std::min<size_t>(kMaxSideSlots, lds_tiles < budget ? (budget - lds_tiles) / 32 : 0);
  TileGeom tg;
  tg.panel_rows = panel_rows;
  tg.panel_cols = panel_cols;
  tg.asic_rows = asic_rows;
  tg.asic_cols = asic_cols;
  tg.asics_per_col = panel_rows / asic_rows;
  tg.asics_per_row = panel_cols / asic_cols;
  tg.plain_mask = plain_mask;
  tg.npix = (int64_t)n_panels * panel_rows * panel_cols;
  tg.nframes = nframes;
  // frames per workgroup: the epix10k2M production kernel takes PR_CM_FPW consecutive frames of
  // its tile (next frame's raw words prefetched during the medians); everything else one
  tg.fpw = (epix_prod && asic_cols == 48) ? PR_CM_FPW : 1;
  tg.side_slots = side_slots;
  tg.pitch = cm_pitch(asic_cols, kind == kJungfrau ? 2 : 1);
  tg.xcd_map = (nframes <= PR_CM_XCD_MAX_FRAMES &&
                ((int64_t)n_panels * tg.asics_per_col * tg.asics_per_row) % 8 == 0) ? 1 : 0;
  const CmParams cp{thr, maxcorr, npix_min, flags, bank_cols};
  const dim3 grid((unsigned)(n_panels * tg.asics_per_col * tg.asics_per_row * ((nframes + tg.fpw - 1) / tg.fpw)));
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const float* P = reinterpret_cast<const float*>(ped);
  const float* G = reinterpret_cast<const float*>(gf);
  const uint8_t* F = reinterpret_cast<const uint8_t*>(planes);
  const bool narrow = asic_cols <= 128;
  const size_t lds_all = lds_tiles + 32 * (size_t)side_slots;
  if (sg_kernel && epix_prod) {
    cm_launch(calib_cm_net_kernel<kEpix10ka, 48, 44, PR_CM_EPIX_BLOCK, 176, 48, true>, grid, PR_CM_EPIX_BLOCK, lds_all, s,
              fp, PS, G, nullptr, tg, cp, io);
  } else if (sg_kernel) {
#if PR_CM_NET_MAXNI >= 8
    cm_launch(calib_cm_net_kernel<kJungfrau, 64, 64, 4 * PR_CM_JF_W, 256, PR_CM_JF_W, true>, grid, 4 * PR_CM_JF_W,
              lds_all, s, fp, PS, G, nullptr, tg, cp, io);
#endif
  } else if (epix_prod && asic_cols == 48) {
    cm_launch(calib_cm_net_kernel<kEpix10ka, 48, 44, PR_CM_EPIX_BLOCK, 176, 48>, grid, PR_CM_EPIX_BLOCK, lds_all, s, fp, P,
              G, F, tg, cp, io);
  } else if (jf_prod && asic_cols == PR_CM_JF_W) {
    cm_launch(calib_cm_net_kernel<kJungfrau, 64, 64, 4 * PR_CM_JF_W, 256, PR_CM_JF_W>, grid, 4 * PR_CM_JF_W, lds_all, s,
              fp, P, G, F, tg, cp, io);
  } else if (kind == kEpix10ka && bank_cols == 48 && M4 == 44 && narrow) {
    cm_launch(calib_cm_net_kernel<kEpix10ka, 48, 44, 512>, grid, 512, lds_all, s, fp, P, G, F, tg, cp, io);
  } else if (kind == kEpix10ka && bank_cols == 8 && M4 == 4 && narrow) {
    cm_launch(calib_cm_net_kernel<kEpix10ka, 8, 4, 512>, grid, 512, lds_all, s, fp, P, G, F, tg, cp, io);
  } else if (kind == kEpix10ka) {
    cm_launch(calib_cm_kernel<kEpix10ka>, grid, 1024, lds_all, s, fp, P, G, F, tg, cp, io);
  } else if (kind == kJungfrau) {
    cm_launch(calib_cm_kernel<kJungfrau>, grid, 1024, lds_all, s, fp, P, G, F, tg, cp, io);
  } else {
    cm_launch(calib_cm_kernel<kPlain>, grid, 1024, lds_all, s, fp, P, G, F, tg, cp, io);
  }
  hip_check(hipGetLastError(), "calib_cm launch");
}

}  // namespace pr
