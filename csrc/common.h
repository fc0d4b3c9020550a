// Shared definitions for the psana_ray_amd HIP kernels (gfx950 / CDNA4 only).
//
// Everything here is written for 64-lane wavefronts and launched on caller-provided
// hipStream_t handles (the Python layer passes torch's current stream as an integer),
// so the extension has no dependency on the torch C++ ABI.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdexcept>
#include <string>

namespace pr {

constexpr int kWave = 64;
// Max frames per launch: per-frame input/output pointers travel in the kernel argument
// block (2 * 32 * 8 B = 512 B), so ring slots need not be contiguous.
constexpr int kMaxFrames = 64;

struct FramePtrs {
  uint64_t in[kMaxFrames];
  uint64_t out[kMaxFrames];
};

// Runs of whole frames copied by one launch of copy_runs_kernel (queue fabric): run i moves n16[i]
// 16-B words from src[i] to dst[i]; cstart is filled by the launcher (first chunk of each run).
constexpr int kMaxCopyRuns = 64;
struct CopyRuns {
  uint64_t src[kMaxCopyRuns];
  uint64_t dst[kMaxCopyRuns];
  int64_t n16[kMaxCopyRuns];
  int32_t cstart[kMaxCopyRuns + 1];
  int32_t n;
};

// Gain decoding families (parameters, not verified psana facts).
//  kEpix10ka: ADU = raw & 0x3FFF; bit 14 selects candidate table b (auto-ranging switched)
//             vs a.  Candidates per pixel are pre-resolved from the pixel gain config on
//             the host (FH/FM/FL/AHL/AML -> (a, b) gain indices), so the kernel sees 2 tables.
//  kJungfrau: ADU = raw & 0x3FFF; gain bits = raw >> 14: 0 -> G0, 1 -> G1, 3 -> G2,
//             2 -> invalid (pixel output 0).  3 tables.
//  kPlain:    ADU = raw (no gain bits), 1 table.
enum GainKind : int { kEpix10ka = 0, kJungfrau = 1, kPlain = 2 };

__device__ __forceinline__ int decode_cand(uint32_t raw, int kind, bool& valid) {
  valid = true;
  if (kind == kEpix10ka) return (raw >> 14) & 1;
  if (kind == kJungfrau) {
    uint32_t g = raw >> 14;
    valid = (g != 2u);
    return g == 3u ? 2 : (int)(g & 1u);
  }
  return 0;
}

__device__ __forceinline__ float decode_adu(uint32_t raw, int kind) {
  return (float)(kind == kPlain ? raw : (raw & 0x3FFFu));
}

// value x gain factor with a +0 addend: a pixel the mask folded to gain factor 0 comes out +0 for
// a negative value too (a plain product gives -0), bit-identical to the reference's
// np.where(mask, data, 0) (psana_ray/producer.py:92-95).  Same instruction count: the multiply
// becomes v_fma_f32 / v_pk_fma_f32; every non-zero product is unchanged.
__device__ __forceinline__ float gmul(float v, float g) { return __builtin_fmaf(v, g, 0.0f); }

inline void check(bool ok, const std::string& msg) {
  if (!ok) throw std::runtime_error("psana_ray_amd: " + msg);
}

inline void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess)
    throw std::runtime_error(std::string("psana_ray_amd HIP error in ") + what + ": " +
                             hipGetErrorString(e));
}

inline bool aligned16(uint64_t p) { return (p & 15u) == 0; }

// Switches the calling thread to `device` and restores the previous device on scope exit.  Every
// native entry a Python thread can reach goes through this: a bare hipSetDevice would silently move
// the caller's current device, and torch's next 'cuda' tensor would land on the wrong GPU in a
// process that drives several.  device < 0: no-op.
class DeviceGuard {
 public:
  explicit DeviceGuard(int device) {
    if (device < 0) return;
    int cur = -1;
    if (hipGetDevice(&cur) != hipSuccess) cur = -1;
    if (cur == device) return;
    hip_check(hipSetDevice(device), "hipSetDevice");
    prev_ = cur;
  }
  ~DeviceGuard() {
    if (prev_ >= 0) (void)hipSetDevice(prev_);
  }
  DeviceGuard(const DeviceGuard&) = delete;
  DeviceGuard& operator=(const DeviceGuard&) = delete;

 private:
  int prev_ = -1;
};

// Bijective XCD-aware block remap (guide T1): the hardware deals workgroups round-robin over the
// 8 XCDs (block b and b+8 share an L2), so hand each XCD a CONTIGUOUS range of logical ids.
// Speed only -- every logical id is still produced exactly once.
__device__ __forceinline__ int xcd_swizzle(int orig, int nwg) {
  constexpr int kXcd = 8;
  const int q = nwg / kXcd, r = nwg % kXcd, xcd = orig % kXcd;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / kXcd;
}

// Register-only select.  A plain `c ? t[1][i] : t[0][i]` lets LLVM fold the select into an
// indexed access t[c][i], which forces the whole register table into scratch/LDS; the integer
// blend keeps both operands in VGPRs.
__device__ __forceinline__ float bsel(bool c, float a, float b) {
  const int m = -(int)c;
  return __int_as_float((__float_as_int(a) & m) | (__float_as_int(b) & ~m));
}

typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));

// Frame buffers arrive as integer addresses (kernarg FramePtrs).  A pointer made from an integer
// is GENERIC to the compiler, which then emits FLAT loads/stores (tracked by both vmcnt and
// lgkmcnt).  Every frame access goes through these address_space(1) (global) views so the ISA
// uses global_load/store with scalar bases and LDS waits stay independent of HBM waits in the
// LDS-heavy kernels.  (No speed-up of the streaming calib kernel is claimed: the only FLAT-vs-
// global comparison was taken with host-bound timing and could not separate them.)
#define PR_GLOBAL __attribute__((address_space(1)))
template <typename T>
__device__ __forceinline__ const PR_GLOBAL T* gin(uint64_t p) {
  return (const PR_GLOBAL T*)p;
}
template <typename T>
__device__ __forceinline__ PR_GLOBAL T* gout(uint64_t p) {
  return (PR_GLOBAL T*)p;
}

// 16-B / 8-B streaming (non-temporal) global loads: data read exactly once (raw frames).
__device__ __forceinline__ uint4 ld_nt_u4(const PR_GLOBAL uint4* p) {
  const u32x4_t v = __builtin_nontemporal_load((const PR_GLOBAL u32x4_t*)p);
  return make_uint4(v.x, v.y, v.z, v.w);
}
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));
// 16-B global store (HIP_vector_type has no address-space-qualified operator=)
__device__ __forceinline__ void st_f4(PR_GLOBAL float4* p, const float4 v) {
  f32x4_t x;
  x.x = v.x; x.y = v.y; x.z = v.z; x.w = v.w;
  *(PR_GLOBAL f32x4_t*)p = x;
}
__device__ __forceinline__ f32x4_t ld_nt_f4(const PR_GLOBAL f32x4_t* p) { return __builtin_nontemporal_load(p); }
__device__ __forceinline__ uint2 ld_nt_u2(const PR_GLOBAL uint2* p) {
  const u32x2_t v = __builtin_nontemporal_load((const PR_GLOBAL u32x2_t*)p);
  return make_uint2(v.x, v.y);
}

}  // namespace pr
