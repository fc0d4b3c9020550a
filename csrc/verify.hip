// Device side of the fabric's end-to-end frame checks (csrc/verify.h): the 64-bit content
// checksum of up to kMaxFrames frames per launch, and the system-scope acquire a consumer issues
// before reading frames another process wrote into its ring.
#include "verify.h"

#include <algorithm>

namespace pr {

// Grid (blocks per frame, frames).  Each lane sums the mixes of a strided set of 16-B words, the
// block reduces them (DPP-lowered shuffles, then LDS across its 4 waves), and one lane adds the
// block's sum to the frame's scratch accumulator.  The LAST block of a frame (ticket) reads the
// total, leaves the scratch zero for the next launch on this row, and publishes: the tagged sum
// (producer, into pinned host memory) or the comparison (consumer, device counters).
template <bool kCompare>
__global__ __launch_bounds__(256) void frame_checksum_kernel(const CkFrames a, const int64_t n16,
                                                             unsigned long long* __restrict__ acc,
                                                             unsigned int* __restrict__ cnt, int64_t* out,
                                                             unsigned long long* counters) {
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
  __shared__ uint64_t part[4];
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x != 0) return;
  s = part[0] + part[1] + part[2] + part[3];
  atomicAdd(&acc[f], (unsigned long long)s);
  __threadfence();
  const unsigned t = atomicAdd(&cnt[f], 1u);
  if (t != gridDim.x - 1) return;
  __threadfence();
  const uint64_t tot = atomicExch(&acc[f], 0ull);
  atomicExch(&cnt[f], 0u);
  const int64_t tg = ck_tag(tot);
  if constexpr (!kCompare) {
    out[f] = tg;   // pinned host memory: read by the fabric thread once the copy's event completed
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  } else if (tg == a.expect[f]) {
    atomicAdd(&counters[0], 1ull);
  } else {
    atomicAdd(&counters[1], 1ull);
    atomicExch(&counters[2], (unsigned long long)a.gevt[f]);
  }
}

void launch_frame_checksums(const CkFrames& a, int nframes, int64_t n16, uint64_t acc, uint64_t cnt, bool compare,
                            uint64_t out, uint64_t counters, uint64_t stream) {
  check(nframes >= 1 && nframes <= kMaxFrames, "frame_checksums: 1..kMaxFrames frames per launch");
  check(n16 > 0 && acc != 0 && cnt != 0, "frame_checksums: empty frame or no scratch");
  check(compare ? counters != 0 : out != 0, "frame_checksums: no result buffer");
  for (int i = 0; i < nframes; ++i) check(aligned16(a.ptr[i]), "frame_checksums: frames must be 16-B aligned");
  const int64_t per = (n16 + 256 * 8 - 1) / (256 * 8);   // ~8 words per lane, at most 128 blocks a frame
  const dim3 grid((unsigned)std::max<int64_t>(1, std::min<int64_t>(128, per)), (unsigned)nframes);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  auto* pa = reinterpret_cast<unsigned long long*>(acc);
  auto* pc = reinterpret_cast<unsigned int*>(cnt);
  if (compare)
    hipLaunchKernelGGL(frame_checksum_kernel<true>, grid, dim3(256), 0, s, a, n16, pa, pc, nullptr,
                       reinterpret_cast<unsigned long long*>(counters));
  else
    hipLaunchKernelGGL(frame_checksum_kernel<false>, grid, dim3(256), 0, s, a, n16, pa, pc,
                       reinterpret_cast<int64_t*>(out), nullptr);
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
