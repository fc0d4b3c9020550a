// Batch gather for training consumers: leased ring slots (scattered HBM frames) -> one contiguous
// [n, *frame] batch tensor, optionally converted to bf16, in ONE launch.
//
// Reference parity: the reference's consumer receives one numpy frame per actor RPC
// (psana_ray/data_reader.py:35) and the architecture figure feeds a "PyTorch Task" (PeakNet,
// setup.py:11); a training step wants a contiguous batch.  Per-frame hipMemcpyAsync D2D would be
// n blit launches; here one grid covers (chunks of the frame) x (frames), each lane moving 2 x 16 B
// (nontemporal reads: the slot is released right after), and the bf16 variant halves the batch
// bytes (round-to-nearest-even, NaN kept quiet) so the model's first layer reads half as much.
#include "common.h"

#include <algorithm>
#include <cstdlib>

namespace pr {

__device__ __forceinline__ uint32_t f32_to_bf16_bits(float f) {
  const uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (u >> 16) | 0x40u;   // NaN: keep it quiet
  return (u + 0x7fffu + ((u >> 16) & 1u)) >> 16;
}

template <bool BF16>
__global__ __launch_bounds__(256) void gather_frames_kernel(const FramePtrs fp, const int64_t n4) {
  const int f = blockIdx.y;
  const PR_GLOBAL f32x4_t* in = gin<f32x4_t>(fp.in[f]);
  const int64_t q0 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 2;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int64_t q = q0 + k;
    if (q >= n4) return;
    const f32x4_t v = ld_nt_f4(in + q);
    if constexpr (BF16) {
      u32x2_t o;
      o.x = f32_to_bf16_bits(v.x) | (f32_to_bf16_bits(v.y) << 16);
      o.y = f32_to_bf16_bits(v.z) | (f32_to_bf16_bits(v.w) << 16);
      gout<u32x2_t>(fp.out[f])[q] = o;
    } else {
      gout<f32x4_t>(fp.out[f])[q] = v;
    }
  }
}

void launch_gather_frames(const FramePtrs& fp, int nframes, int64_t nelem, bool bf16, uint64_t stream) {
  check(nframes >= 1 && nframes <= kMaxFrames, "gather_frames: 1..kMaxFrames frames per launch");
  check(nelem > 0 && nelem % 4 == 0, "gather_frames: frame size must be a multiple of 4 elements");
  for (int i = 0; i < nframes; ++i)
    check(aligned16(fp.in[i]) && (fp.out[i] % (bf16 ? 8 : 16)) == 0, "gather_frames: misaligned frame");
  const int64_t n4 = nelem / 4;
  const dim3 grid((unsigned)((n4 + 511) / 512), (unsigned)nframes);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (bf16)
    hipLaunchKernelGGL(gather_frames_kernel<true>, grid, dim3(256), 0, s, fp, n4);
  else
    hipLaunchKernelGGL(gather_frames_kernel<false>, grid, dim3(256), 0, s, fp, n4);
  hip_check(hipGetLastError(), "gather_frames launch");
}

// Output mask of psana-calibrated frames (psana_wrapper fallback path, R-05: np.where(mask, data, 0),
// psana_ray/producer.py:92-95) over a whole uploaded chunk in ONE launch, in place: frame f's pixel
// i becomes 0 where zero[i] != 0.  Each lane owns 4 pixels (one 32-bit load of mask bytes, one
// 16-B frame load) and stores only when one of them is masked; a frame size that is not a multiple
// of 4 pixels leaves a scalar tail to lane 0 of the last workgroup.
__global__ __launch_bounds__(256) void mask_frames_kernel(const FramePtrs fp, const uint8_t* __restrict__ zero,
                                                          const int64_t npix) {
  const int f = blockIdx.y;
  PR_GLOBAL float* out = gout<float>(fp.out[f]);
  const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t n4 = npix >> 2;
  if (q < n4) {
    const uint32_t m = reinterpret_cast<const uint32_t*>(zero)[q];
    if (m != 0u) {
      f32x4_t v = reinterpret_cast<PR_GLOBAL f32x4_t*>(out)[q];
      if (m & 0x000000FFu) v.x = 0.0f;
      if (m & 0x0000FF00u) v.y = 0.0f;
      if (m & 0x00FF0000u) v.z = 0.0f;
      if (m & 0xFF000000u) v.w = 0.0f;
      reinterpret_cast<PR_GLOBAL f32x4_t*>(out)[q] = v;
    }
  }
  if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0)
    for (int64_t i = n4 * 4; i < npix; ++i)
      if (zero[i]) out[i] = 0.0f;
}

void launch_mask_frames(const FramePtrs& fp, int nframes, uint64_t zero, int64_t npix, uint64_t stream) {
  check(nframes >= 1 && nframes <= kMaxFrames, "mask_frames: 1..kMaxFrames frames per launch");
  check(npix > 0 && zero != 0 && zero % 4 == 0, "mask_frames: needs a 4-B aligned byte mask of npix entries");
  for (int i = 0; i < nframes; ++i) check(aligned16(fp.out[i]), "mask_frames: frames must be 16-B aligned");
  const int64_t n4 = npix / 4;
  const dim3 grid((unsigned)std::max<int64_t>(1, (n4 + 255) / 256), (unsigned)nframes);
  hipLaunchKernelGGL(mask_frames_kernel, grid, dim3(256), 0, reinterpret_cast<hipStream_t>(stream), fp,
                     reinterpret_cast<const uint8_t*>(zero), npix);
  hip_check(hipGetLastError(), "mask_frames launch");
}

// Zero fill of fixed element runs in every output frame (the gaps between panels of an image
// written by the fused common-mode kernel).  One wave per run (host splits runs to <= 1024
// elements so the waves are balanced), consecutive lanes on consecutive elements.
__global__ __launch_bounds__(256) void fill_runs_kernel(const FramePtrs fp, const int2* __restrict__ runs,
                                                        const int n_runs) {
  const int w = (int)blockIdx.x * 4 + ((int)threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (w >= n_runs) return;
  const int2 rr = runs[w];
  PR_GLOBAL float* out = gout<float>(fp.out[blockIdx.y]);
  for (int k = lane; k < rr.y; k += 64) out[(int64_t)rr.x + k] = 0.0f;
}

void launch_fill_runs(const FramePtrs& fp, int nframes, uint64_t runs, int n_runs, uint64_t stream) {
  check(nframes >= 1 && nframes <= kMaxFrames, "fill_runs: 1..kMaxFrames frames per launch");
  if (n_runs <= 0) return;
  check(runs % 8 == 0, "fill_runs: misaligned run table");
  const dim3 grid((unsigned)((n_runs + 3) / 4), (unsigned)nframes);
  hipLaunchKernelGGL(fill_runs_kernel, grid, dim3(256), 0, reinterpret_cast<hipStream_t>(stream), fp,
                     reinterpret_cast<const int2*>(runs), n_runs);
  hip_check(hipGetLastError(), "fill_runs launch");
}

// ---------------------------------------------------------------------------------------------
// Host -> HBM staging copy as OUR kernel: the pinned pool
// (or registered run file) is read straight over PCIe by a FEW persistent workgroups, each lane
// keeping 4 x 16 B nontemporal loads in flight (64 workgroups x 256 lanes x 64 B = 1 MiB in flight,
// ~8x the PCIe Gen5 bandwidth-delay product), instead of the runtime's blit kernel, whose
// workgroups occupy CUs across the chip while stalled on PCIe latency and stretch the concurrent
// calibration / peak-finder kernels (profiles/rocprof_bench_n1_host_r1d.md).
// ---------------------------------------------------------------------------------------------
template <int U>
__global__ __launch_bounds__(256) void copy_h2d_kernel(const f32x4_t* __restrict__ src, f32x4_t* __restrict__ dst,
                                                       const int64_t n16) {
  const int64_t stride = (int64_t)gridDim.x * 256 * U;
  for (int64_t base = (int64_t)blockIdx.x * 256 * U + threadIdx.x; base < n16; base += stride) {
    f32x4_t v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t q = base + 256 * u;
      if (q < n16) v[u] = __builtin_nontemporal_load(src + q);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t q = base + 256 * u;
      if (q < n16) dst[q] = v[u];
    }
  }
}

bool launch_copy_h2d(uint64_t dst, uint64_t host_src, int64_t bytes, int workgroups, uint64_t stream) {
  if (workgroups <= 0 || bytes <= 0 || (dst | host_src | (uint64_t)bytes) % 16 != 0) return false;
  void* dsrc = nullptr;
  if (hipHostGetDevicePointer(&dsrc, reinterpret_cast<void*>(host_src), 0) != hipSuccess || dsrc == nullptr) {
    (void)hipGetLastError();   // not pinned / not mapped: the caller falls back to hipMemcpyAsync
    return false;
  }
  constexpr int U = 4;   // 16-B loads in flight per lane (round-1 A/B: 8 no faster)
  const int64_t n16 = bytes / 16;
  const int64_t need = (n16 + 256 * U - 1) / (256 * U);
  const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>(workgroups, need));
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const f32x4_t* sp = reinterpret_cast<const f32x4_t*>(dsrc);
  f32x4_t* dp = reinterpret_cast<f32x4_t*>(dst);
  hipLaunchKernelGGL(copy_h2d_kernel<U>, dim3(grid), dim3(256), 0, s, sp, dp, n16);
  hip_check(hipGetLastError(), "copy_h2d launch");
  return true;
}

// ---------------------------------------------------------------------------------------------
// Queue-fabric frame copies (csrc/fabric.cpp): every frame a producer routes to OTHER processes in
// one fabric pass -- to any number of consumer rings, each an IPC mapping of a peer's HBM (another
// GPU over xGMI, or this GPU) -- moves in ONE launch on the fabric's own hardware queue.  The
// runtime path was one blit launch per contiguous run per link, each on an ordinary stream
// multiplexed with the staging and calibration streams.  Work unit: a 16-KB
// chunk (256 lanes x U x 16 B in flight); the grid strides over the chunks of all runs, so the
// writes to different consumers (different xGMI links) are in flight at the same time.  Loads are
// nontemporal (the producer slot is freed right after); stores are plain (a same-GPU consumer reads
// the slot next).  Visibility: the consumer is told only after this kernel's completion event; when
// a dispatch writes another GPU's ring, the fabric follows it with ONE system-scope release on every
// XCD (launch_release_fence, verify.hip: buffer_wbl2 sc0 sc1 writes back L2 lines of peer memory
// before the completion signal) instead of relying on the dispatch packet's release scope, and the
// consumer issues the matching acquire (verify.h).  PR_COPY_RELEASE=1 builds the round-6 variant with
// a release at the end of every wave instead: 2 ranks on one GPU, route=remote_only window 83.0k /
// 84.0k vs 108.2k / 109.7k fr/s without it (profiles/r6/README.md section 3).
// ---------------------------------------------------------------------------------------------
#ifndef PR_COPY_RELEASE
#define PR_COPY_RELEASE 0
#endif
template <int U>
__global__ __launch_bounds__(256) void copy_runs_kernel(const CopyRuns cr, const int total_chunks) {
  constexpr int kChunk16 = 256 * U;
  int e = 0;   // run of the current chunk: chunks ascend per workgroup, so the scan only moves forward
  for (int c = blockIdx.x; c < total_chunks; c += gridDim.x) {
    while (e + 1 < cr.n && cr.cstart[e + 1] <= c) ++e;
    const PR_GLOBAL f32x4_t* src = gin<f32x4_t>(cr.src[e]);
    PR_GLOBAL f32x4_t* dst = gout<f32x4_t>(cr.dst[e]);
    const int64_t n16 = cr.n16[e];
    const int64_t base = (int64_t)(c - cr.cstart[e]) * kChunk16 + threadIdx.x;
    f32x4_t v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t q = base + 256 * u;
      if (q < n16) v[u] = ld_nt_f4(src + q);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t q = base + 256 * u;
      if (q < n16) dst[q] = v[u];
    }
  }
#if PR_COPY_RELEASE
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
#endif
}

int launch_copy_runs(CopyRuns& cr, int workgroups, uint64_t stream) {
  constexpr int U = 4;
  constexpr int64_t kChunk16 = 256 * U;
  check(cr.n >= 1 && cr.n <= kMaxCopyRuns, "copy_runs: 1..kMaxCopyRuns runs per launch");
  int64_t total = 0;
  for (int i = 0; i < cr.n; ++i) {
    check(aligned16(cr.src[i]) && aligned16(cr.dst[i]) && cr.n16[i] > 0, "copy_runs: misaligned or empty run");
    cr.cstart[i] = (int32_t)total;
    total += (cr.n16[i] + kChunk16 - 1) / kChunk16;
    check(total < (int64_t(1) << 30), "copy_runs: too many chunks in one launch");
  }
  cr.cstart[cr.n] = (int32_t)total;
  const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(workgroups > 0 ? workgroups : 256, total));
  hipLaunchKernelGGL(copy_runs_kernel<U>, dim3(grid), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), cr,
                     (int)total);
  hip_check(hipGetLastError(), "copy_runs launch");
  return grid;
}

}  // namespace pr
