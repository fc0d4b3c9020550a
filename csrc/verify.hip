// Device side of the fabric's end-to-end frame checks (csrc/verify.h): the 64-bit content
// checksum of up to kMaxFrames frames per launch, and the system-scope acquire a consumer issues
// before reading frames another process wrote into its ring.
#include "verify.h"

#include <algorithm>

namespace pr {

// Two launches: (blocks per frame, frames) blocks each sum the mixes of a strided set of 16-B words
// (DPP-lowered shuffles, then LDS across the block's 4 waves) and store ONE partial per block; then
// one block per frame adds its partials in a fixed order and stores the tagged sum into pinned host
// memory, where the host reads it after the launch's event (producer: into the notice; consumer:
// compared with the producer's -- no device-side counters, so no cross-XCD atomics at all).  The kernel boundary
// orders the partials' stores before their reads on every XCD: a single-launch "last block adds
// the others' atomics" form gave sums that differed from the host's on gfx950 (the blocks of a
// frame run on all 8 XCDs, whose L2s are not coherent for device-scope atomics on plain memory).
constexpr int kCkBlocks = kCkPartials;   // max blocks per frame (partials per frame)

__global__ __launch_bounds__(256) void frame_partials_kernel(const CkFrames a, const int64_t n16,
                                                             uint64_t* __restrict__ part) {
  const int f = blockIdx.y;
  const PR_GLOBAL u32x4_t* p = gin<u32x4_t>(a.ptr[f]);
  uint64_t s = 0;
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x; q < n16; q += stride) {
    const u32x4_t v = p[q];
    s += ck_word((uint64_t)v.x | ((uint64_t)v.y << 32), (uint64_t)v.z | ((uint64_t)v.w << 32), (uint64_t)q);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor((unsigned long long)s, o);
  __shared__ uint64_t w[4];
  if ((threadIdx.x & 63) == 0) w[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) part[(int64_t)f * kCkBlocks + blockIdx.x] = w[0] + w[1] + w[2] + w[3];
}

__global__ __launch_bounds__(64) void frame_finish_kernel(const int nblk, const uint64_t* __restrict__ part,
                                                          int64_t* out) {
  const int f = blockIdx.x;
  uint64_t s = 0;
  for (int b = threadIdx.x; b < nblk; b += 64) s += part[(int64_t)f * kCkBlocks + b];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor((unsigned long long)s, o);
  if (threadIdx.x != 0) return;
  out[f] = ck_tag(s);   // pinned host memory: read on the host once the launch's event completed
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
}

void launch_frame_checksums(const CkFrames& a, int nframes, int64_t n16, uint64_t part, uint64_t out,
                            uint64_t stream) {
  check(nframes >= 1 && nframes <= kMaxFrames, "frame_checksums: 1..kMaxFrames frames per launch");
  check(n16 > 0 && part != 0 && out != 0, "frame_checksums: empty frame, no scratch or no result buffer");
  for (int i = 0; i < nframes; ++i) check(aligned16(a.ptr[i]), "frame_checksums: frames must be 16-B aligned");
  const int64_t per = (n16 + 256 * 8 - 1) / (256 * 8);   // ~8 words per lane, at most kCkBlocks blocks a frame
  const int nblk = (int)std::max<int64_t>(1, std::min<int64_t>(kCkBlocks, per));
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  auto* pp = reinterpret_cast<uint64_t*>(part);
  hipLaunchKernelGGL(frame_partials_kernel, dim3((unsigned)nblk, (unsigned)nframes), dim3(256), 0, s, a, n16, pp);
  hipLaunchKernelGGL(frame_finish_kernel, dim3((unsigned)nframes), dim3(64), 0, s, nblk, pp,
                     reinterpret_cast<int64_t*>(out));
  hip_check(hipGetLastError(), "frame_checksums launch");
}

// buffer_inv sc0 sc1: drops this CU's L1 and its XCD's L2 lines that a peer's writes may have made
// stale.  Workgroups are dealt round-robin over the 8 XCDs, so 64 of them reach every XCD's L2.
__global__ __launch_bounds__(64) void acquire_fence_kernel() { __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, ""); }

// buffer_wbl2 sc0 sc1: writes back the dirty L2 lines of this XCD (peer memory included), so frames
// that kernels of this GPU wrote into another GPU's ring reach it before the completion signal that
// the notice is posted after.  64 workgroups reach every XCD's L2.
__global__ __launch_bounds__(64) void release_fence_kernel() { __builtin_amdgcn_fence(__ATOMIC_RELEASE, ""); }

void launch_release_fence(uint64_t stream) {
  hipLaunchKernelGGL(release_fence_kernel, dim3(64), dim3(64), 0, reinterpret_cast<hipStream_t>(stream));
  hip_check(hipGetLastError(), "release_fence launch");
}

void launch_acquire_fence(uint64_t stream) {
  hipLaunchKernelGGL(acquire_fence_kernel, dim3(64), dim3(64), 0, reinterpret_cast<hipStream_t>(stream));
  hip_check(hipGetLastError(), "acquire_fence launch");
}

}  // namespace pr
