// K-05 geometry assembly (image mode) as a deterministic GATHER.
//
// Reference parity: image mode is psana-ray's DEFAULT (`--calib` absent,
// psana_ray/producer.py:22,156-159); psana scatters calibrated panel pixels into a 2-D image.
// Here every output pixel carries a precomputed source index (or -1 for gaps), so writes are
// coalesced 16-B stores, there are no atomics and the result is deterministic.  The index map
// is loaded once per thread and reused over the whole frame batch.
#include "common.h"

namespace pr {

__global__ __launch_bounds__(256) void assemble_kernel(const FramePtrs fp, const int nframes,
                                                       const int32_t* __restrict__ idx,
                                                       const int64_t nout,
                                                       const uint8_t* __restrict__ omask) {
  const int64_t o0 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
  if (o0 >= nout) return;
  const bool full = (o0 + 4 <= nout);
  int32_t src[4];
  if (full) {
    const int4 s = *reinterpret_cast<const int4*>(idx + o0);
    src[0] = s.x; src[1] = s.y; src[2] = s.z; src[3] = s.w;
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i) src[i] = (o0 + i < nout) ? idx[o0 + i] : -1;
  }
  if (omask != nullptr) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (o0 + i < nout && omask[o0 + i] == 0) src[i] = -1;
  }
  for (int f = 0; f < nframes; ++f) {
    const PR_GLOBAL float* in = gin<float>(fp.in[f]);
    float o[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) o[i] = src[i] >= 0 ? in[src[i]] : 0.0f;
    PR_GLOBAL float* out = gout<float>(fp.out[f]);
    if (full) {
      st_f4((PR_GLOBAL float4*)(out + o0), make_float4(o[0], o[1], o[2], o[3]));
    } else {
      for (int i = 0; i < 4 && o0 + i < nout; ++i) out[o0 + i] = o[i];
    }
  }
}

void launch_assemble(const FramePtrs& fp, int nframes, uint64_t idx, int64_t nout, uint64_t omask,
                     uint64_t stream) {
  check(nframes >= 1 && nframes <= kMaxFrames, "assemble: nframes out of range");
  check(aligned16(idx), "assemble: index map must be 16-B aligned");
  for (int f = 0; f < nframes; ++f) check(aligned16(fp.out[f]), "assemble: outputs must be 16-B aligned");
  const int64_t nthr = (nout + 3) / 4;
  const dim3 grid((unsigned)((nthr + 255) / 256));
  hipLaunchKernelGGL(assemble_kernel, grid, dim3(256), 0, reinterpret_cast<hipStream_t>(stream), fp,
                     nframes, reinterpret_cast<const int32_t*>(idx), nout,
                     reinterpret_cast<const uint8_t*>(omask));
  hip_check(hipGetLastError(), "assemble launch");
}

}  // namespace pr
