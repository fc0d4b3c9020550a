// Column-median probe ("build the non-sorting median select"): the epix10k2M
// common-mode COLUMN phase -- the exact numpy median of the participating (|v| < thr) values of each
// of the 48 columns of a 176 x 48 LDS tile, subtracted from the column -- in three forms, on the
// same tiles, same lane mapping (a quad of lanes per column, 44 rows per lane), same LDS footprint:
//
//   net   the shipped routine (csrc/common_mode.hip cm_cols<44>): per-lane sorting network, DPP
//         merge-split, merge path -- included verbatim from the production source;
//   hist  a two-level LDS-histogram radix select (non-sorting): 32 value bins per column
//         (ds_add_u32 per participant), quad prefix scan to the bin holding rank k, 32 sub-bins
//         of that bin, then exact extraction of the k-th value among the few candidates left
//         (iterative quad-min), and of rank k+1 for even counts;
//   bisect a count-bisection on the values: per step every lane counts its values below the pivot,
//         a quad DPP sum, and the interval halves until it holds rank k's value alone.
//
// Each kernel loads T tiles from HBM into LDS (pitch 52), runs the column phase REPS times (the
// timing of interest: (t(reps = 1 + n) - t(reps = 1)) / n), and writes the tile back; with reps = 1
// every output is compared BITWISE with a host reference (numpy-semantics median).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I csrc tools/median_probe.hip -o tools/median_probe_bin
//   tools/median_probe_bin [tiles=16384]
#include "../csrc/common_mode.hip"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

namespace pr {

constexpr int kR = 176, kC = 48, kP = 52, kM = 44, kBins = 32;
// unroll factor of the passes over a lane's values: full for register-resident values (an indexed
// register array must be fully unrolled), partial when they are re-read from the LDS tile
#ifndef LDSX
#define LDSX 0   // 1: hist / bisect re-read the values from the LDS tile in every pass (few VGPRs)
#endif
#ifndef UNR
#define UNR 44
#endif

__device__ __forceinline__ int quad_sum_i(int v) {
  return dpp_quad_i<0x00>(v) + dpp_quad_i<0x55>(v) + dpp_quad_i<0xAA>(v) + dpp_quad_i<0xFF>(v);
}
__device__ __forceinline__ float quad_min_f(float v) {
  return fminf(fminf(dpp_quad<0x00>(v), dpp_quad<0x55>(v)), fminf(dpp_quad<0xAA>(v), dpp_quad<0xFF>(v)));
}

// rank-r value (0-based) among the quad's values with cand set: iterative minimum extraction over
// distinct values (duplicates counted); r < number of candidates
template <int M, typename XF>
__device__ __forceinline__ float extract_rank(const XF& X, const uint64_t cand, int r) {
  const float INF = __int_as_float(0x7f800000);
  float prev = -INF;
  float ans = 0.f;
  for (int guard = 0; guard < 4 * M; ++guard) {   // every iteration retires >= 1 candidate value
    float m = INF;
#pragma unroll UNR
    for (int i = 0; i < M; ++i) {
      const float xi = X(i);
      m = ((cand >> i) & 1ull) && xi > prev ? fminf(m, xi) : m;
    }
    const float cur = quad_min_f(m);
    int eq = 0;
#pragma unroll UNR
    for (int i = 0; i < M; ++i) eq += ((cand >> i) & 1ull) && X(i) == cur ? 1 : 0;
    eq = quad_sum_i(eq);
    if (r < eq) {
      ans = cur;
      break;
    }
    r -= eq;
    prev = cur;
  }
  return ans;
}

// The exact median of the quad's participants given rank k1's value: rank k2 = k1 + (cnt even).
template <int M, typename XF>
__device__ __forceinline__ float finish_median(const XF& X, const uint64_t part, int cnt, float v1) {
  if (cnt & 1) return (v1 + v1) * 0.5f;
  const float INF = __int_as_float(0x7f800000);
  int le = 0;
  float nxt = INF;
#pragma unroll UNR
  for (int i = 0; i < M; ++i) {
    const bool p = (part >> i) & 1ull;
    const float xi = X(i);
    le += p && xi <= v1 ? 1 : 0;
    nxt = p && xi > v1 ? fminf(nxt, xi) : nxt;
  }
  le = quad_sum_i(le);
  const int k2 = cnt / 2;
  const float v2 = le > k2 ? v1 : quad_min_f(nxt);
  return (v1 + v2) * 0.5f;
}

// ---- two-level LDS-histogram radix select ---------------------------------------------------
template <int M>
__device__ void cols_hist(float* tile, int P, int R, int C, const CmParams& cp, int t0, int nt, uint32_t* hist) {
  const float QNAN = __int_as_float(0x7fc00000);
  const int nwork = 4 * C;
  const float S = (float)kBins / (2.0f * cp.thr);
  for (int w = t0; w < ((nwork + 63) / 64) * 64; w += nt) {
    const bool act = w < nwork;
    const int c = act ? (w >> 2) : 0;
    const int q = w & 3;
    float* colp = tile + 2 * q * P + c;
    auto row_of = [&](int i) { return 8 * (i >> 1) + 2 * q + (i & 1); };
    auto off_of = [&](int i) { return (8 * (i >> 1) + (i & 1)) * P; };
#if LDSX
    auto X = [&](int i) -> float { return (act && row_of(i) < R) ? colp[off_of(i)] : QNAN; };
#else
    float x[M];
#pragma unroll
    for (int i = 0; i < M; ++i) x[i] = (act && row_of(i) < R) ? colp[off_of(i)] : QNAN;
    auto X = [&](int i) -> float { return x[i]; };
#endif
    uint64_t part = 0;
    int my = 0;
#pragma unroll UNR
    for (int i = 0; i < M; ++i) {
      const bool p = fabsf(X(i)) < cp.thr;
      part |= (uint64_t)p << i;
      my += p ? 1 : 0;
    }
    const int cnt = quad_sum_i(my);
    uint32_t* h = hist + c * kBins;
    float med = 0.f;
    if (cnt > 0) {
      const int k1 = (cnt - 1) / 2;
      // level 1: bins of width 2 thr / 32 over (-thr, thr)
      *reinterpret_cast<uint4*>(h + 8 * q) = make_uint4(0, 0, 0, 0);
      *reinterpret_cast<uint4*>(h + 8 * q + 4) = make_uint4(0, 0, 0, 0);
#pragma unroll UNR
      for (int i = 0; i < M; ++i)
        if ((part >> i) & 1ull) atomicAdd(h + min(kBins - 1, (int)((X(i) + cp.thr) * S)), 1u);
      auto locate = [&](int k, int& bin, int& below) {
        const uint4 a = *reinterpret_cast<const uint4*>(h + 8 * q);
        const uint4 b = *reinterpret_cast<const uint4*>(h + 8 * q + 4);
        const int hv[8] = {(int)a.x, (int)a.y, (int)a.z, (int)a.w, (int)b.x, (int)b.y, (int)b.z, (int)b.w};
        int s = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) s += hv[j];
        const int s0 = dpp_quad_i<0x00>(s), s1 = dpp_quad_i<0x55>(s), s2 = dpp_quad_i<0xAA>(s);
        int pre = (q > 0 ? s0 : 0) + (q > 1 ? s1 : 0) + (q > 2 ? s2 : 0);
        int mb = -1, mbelow = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          if (mb < 0 && k >= pre && k < pre + hv[j]) {   // only the lane whose bins hold rank k
            mb = 8 * q + j;
            mbelow = pre;
          }
          pre += hv[j];
        }
        // exactly one lane of the quad found it: broadcast with a quad max
        const int code = mb >= 0 ? (mb << 16) | mbelow : -1;
        const int cm = max(max(dpp_quad_i<0x00>(code), dpp_quad_i<0x55>(code)),
                           max(dpp_quad_i<0xAA>(code), dpp_quad_i<0xFF>(code)));
        bin = cm >> 16;
        below = cm & 0xFFFF;
      };
      int b1, l1;
      locate(k1, b1, l1);
      // level 2: 32 sub-bins of bin b1 (from the same scaled value, so membership and order agree)
      *reinterpret_cast<uint4*>(h + 8 * q) = make_uint4(0, 0, 0, 0);
      *reinterpret_cast<uint4*>(h + 8 * q + 4) = make_uint4(0, 0, 0, 0);
      uint64_t inb = 0;
#pragma unroll UNR
      for (int i = 0; i < M; ++i) {
        // non-participants (NaN, |v| >= thr) never reach the float -> int conversion: converting a
        // NaN is poison in LLVM, and `p && poison` may fold to poison
        const bool p = (part >> i) & 1ull;
        const float t = p ? (X(i) + cp.thr) * S : 0.f;
        const bool in = p && min(kBins - 1, (int)t) == b1;
        inb |= (uint64_t)in << i;
        if (in) atomicAdd(h + min(kBins - 1, (int)((t - (float)b1) * (float)kBins)), 1u);
      }
      int b2, l2;
      locate(k1 - l1, b2, l2);
      uint64_t cand = 0;
#pragma unroll UNR
      for (int i = 0; i < M; ++i) {
        const bool p = (inb >> i) & 1ull;
        const float t = p ? (X(i) + cp.thr) * S : (float)b1;
        const bool in = p && min(kBins - 1, (int)((t - (float)b1) * (float)kBins)) == b2;
        cand |= (uint64_t)in << i;
      }
      const float v1 = extract_rank<M>(X, cand, k1 - l1 - l2);
      med = finish_median<M>(X, part, cnt, v1);
    }
    if (act && cnt >= cp.npix_min && cnt > 0 && fabsf(med) <= cp.maxcorr) {
#pragma unroll
      for (int i = 0; i < M; ++i)
        if (row_of(i) < R) colp[off_of(i)] -= med;
    }
  }
}

// ---- count-bisection on the values ------------------------------------------------------------
template <int M>
__device__ void cols_bisect(float* tile, int P, int R, int C, const CmParams& cp, int t0, int nt) {
  const float QNAN = __int_as_float(0x7fc00000);
  const int nwork = 4 * C;
  for (int w = t0; w < ((nwork + 63) / 64) * 64; w += nt) {
    const bool act = w < nwork;
    const int c = act ? (w >> 2) : 0;
    const int q = w & 3;
    float* colp = tile + 2 * q * P + c;
    auto row_of = [&](int i) { return 8 * (i >> 1) + 2 * q + (i & 1); };
    auto off_of = [&](int i) { return (8 * (i >> 1) + (i & 1)) * P; };
#if LDSX
    auto X = [&](int i) -> float { return (act && row_of(i) < R) ? colp[off_of(i)] : QNAN; };
#else
    float x[M];
#pragma unroll
    for (int i = 0; i < M; ++i) x[i] = (act && row_of(i) < R) ? colp[off_of(i)] : QNAN;
    auto X = [&](int i) -> float { return x[i]; };
#endif
    uint64_t part = 0;
    int my = 0;
#pragma unroll UNR
    for (int i = 0; i < M; ++i) {
      const bool p = fabsf(X(i)) < cp.thr;
      part |= (uint64_t)p << i;
      my += p ? 1 : 0;
    }
    const int cnt = quad_sum_i(my);
    float med = 0.f;
    if (cnt > 0) {
      const int k1 = (cnt - 1) / 2;
      // invariant: #(v < lo) <= k1 < #(v < hi); stop when [lo, hi) holds few participants
      float lo = -cp.thr, hi = cp.thr;
      int below = 0, inside = cnt;
      for (int step = 0; step < 40 && inside > 2; ++step) {
        const float mid = 0.5f * (lo + hi);
        if (!(mid > lo && mid < hi)) break;   // interval exhausted at float resolution
        int n = 0;
#pragma unroll UNR
        for (int i = 0; i < M; ++i) n += ((part >> i) & 1ull) && X(i) < mid ? 1 : 0;
        n = quad_sum_i(n);
        if (k1 < n) {
          hi = mid;
          inside = n - below;
        } else {
          lo = mid;
          inside -= n - below;
          below = n;
        }
      }
      uint64_t cand = 0;
#pragma unroll UNR
      for (int i = 0; i < M; ++i) {
        const float xi = X(i);
        cand |= (uint64_t)(((part >> i) & 1ull) && xi >= lo && xi < hi) << i;
      }
      const float v1 = extract_rank<M>(X, cand, k1 - below);
      med = finish_median<M>(X, part, cnt, v1);
    }
    if (act && cnt >= cp.npix_min && cnt > 0 && fabsf(med) <= cp.maxcorr) {
#pragma unroll
      for (int i = 0; i < M; ++i)
        if (row_of(i) < R) colp[off_of(i)] -= med;
    }
  }
}

template <int MODE>
__global__ __launch_bounds__(256) void probe_cols_kernel(const float* __restrict__ in, float* __restrict__ out,
                                                          int ntiles, CmParams cp, int reps) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* tile = reinterpret_cast<float*>(smem);
  uint32_t* hist = reinterpret_cast<uint32_t*>(tile + kR * kP);
  for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const float* src = in + (int64_t)t * kR * kC;
    for (int e = threadIdx.x; e < kR * kC / 4; e += blockDim.x) {
      const int r = e / (kC / 4), j = e % (kC / 4);
      *reinterpret_cast<float4*>(tile + r * kP + 4 * j) = *reinterpret_cast<const float4*>(src + r * kC + 4 * j);
    }
    __syncthreads();
    for (int k = 0; k < reps; ++k) {
      if constexpr (MODE == 0) cm_cols<kM>(tile, kP, kR, kC, cp, threadIdx.x, blockDim.x);
      else if constexpr (MODE == 1) cols_hist<kM>(tile, kP, kR, kC, cp, threadIdx.x, blockDim.x, hist);
      else cols_bisect<kM>(tile, kP, kR, kC, cp, threadIdx.x, blockDim.x);
      __syncthreads();
    }
    float* dst = out + (int64_t)t * kR * kC;
    for (int e = threadIdx.x; e < kR * kC / 4; e += blockDim.x) {
      const int r = e / (kC / 4), j = e % (kC / 4);
      *reinterpret_cast<float4*>(dst + r * kC + 4 * j) = *reinterpret_cast<const float4*>(tile + r * kP + 4 * j);
    }
    __syncthreads();
  }
}

}  // namespace pr

using namespace pr;

static float host_median(std::vector<float>& v) {
  std::sort(v.begin(), v.end());
  const size_t n = v.size();
  return (v[(n - 1) / 2] + v[n / 2]) * 0.5f;
}

int main(int argc, char** argv) {
  const int ntiles = argc > 1 ? atoi(argv[1]) : 16384;
  const size_t n = (size_t)ntiles * kR * kC;
  std::vector<float> h(n);
  std::mt19937 rng(7);
  std::normal_distribution<float> nd(0.f, 5.f);
  std::uniform_real_distribution<float> u(0.f, 1.f);
  for (size_t i = 0; i < n; ++i) {
    float v = nd(rng) + 0.37f * (float)((i / kC) % 7);
    const float r = u(rng);
    if (r < 0.03f) v = __builtin_nanf("");          // non-eligible pixels are NaN in the tile
    else if (r < 0.06f) v = 200.f + 100.f * u(rng);  // photon hits: above thr, never participate
    else if (r < 0.07f) v = std::round(v);           // exact duplicates inside the median's range
    h[i] = v;
  }
  // a few degenerate columns: all equal, one participant, none
  for (int r = 0; r < kR; ++r) {
    h[(size_t)r * kC + 0] = 1.25f;
    h[(size_t)r * kC + 1] = r == 7 ? -3.5f : 500.f;
    h[(size_t)r * kC + 2] = 999.f;
  }
  const CmParams cp{30.f, 1e30f, 1, 2, 48};
  float *din, *dout;
  hipMalloc(&din, n * 4);
  hipMalloc(&dout, n * 4);
  hipMemcpy(din, h.data(), n * 4, hipMemcpyHostToDevice);
  // expected outputs (reps = 1)
  std::vector<float> exp(h);
  for (int t = 0; t < ntiles; ++t)
    for (int c = 0; c < kC; ++c) {
      std::vector<float> p;
      for (int r = 0; r < kR; ++r) {
        const float v = h[((size_t)t * kR + r) * kC + c];
        if (std::fabs(v) < cp.thr) p.push_back(v);
      }
      if (p.empty()) continue;
      const float med = host_median(p);
      if (!(std::fabs(med) <= cp.maxcorr)) continue;
      for (int r = 0; r < kR; ++r) exp[((size_t)t * kR + r) * kC + c] -= med;
    }
  const size_t lds = (size_t)kR * kP * 4 + (size_t)kC * kBins * 4;   // same footprint for every form
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  int dev = 0, cus = 0;
  hipGetDevice(&dev);
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const char* names[3] = {"net", LDSX ? "hist_lds" : "hist_reg", LDSX ? "bisect_lds" : "bisect_reg"};
  void (*kerns[3])(const float*, float*, int, CmParams, int) = {probe_cols_kernel<0>, probe_cols_kernel<1>,
                                                                probe_cols_kernel<2>};
  int rc = 0;
  printf("{\"tiles\": %d, \"lds_bytes\": %zu, \"results\": [", ntiles, lds);
  for (int k = 0; k < 3; ++k) {
    hipFuncSetAttribute((const void*)kerns[k], hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    int per = 0;
    hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, (const void*)kerns[k], 256, lds);
    const int grid = cus * per;
    // correctness, reps = 1
    hipLaunchKernelGGL(kerns[k], dim3(grid), dim3(256), lds, 0, din, dout, ntiles, cp, 1);
    std::vector<float> got(n);
    hipMemcpy(got.data(), dout, n * 4, hipMemcpyDeviceToHost);
    // bitwise mismatches, and value mismatches (+0 / -0 equal: a median of a +0 and a -0 has either
    // sign depending on which the sort put first, in the reference as well)
    size_t bad = 0, badv = 0;
    for (size_t i = 0; i < n; ++i) {
      uint32_t a, b;
      std::memcpy(&a, &got[i], 4);
      std::memcpy(&b, &exp[i], 4);
      const bool nan2 = std::isnan(got[i]) && std::isnan(exp[i]);
      if (a != b && !nan2) ++bad;
      if (!(got[i] == exp[i]) && !nan2) ++badv;
    }
    if (badv) rc = 1;
    auto timed = [&](int reps) {
      float best = 1e30f;
      for (int it = 0; it < 5; ++it) {
        hipEventRecord(e0, 0);
        hipLaunchKernelGGL(kerns[k], dim3(grid), dim3(256), lds, 0, din, dout, ntiles, cp, reps);
        hipEventRecord(e1, 0);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        best = std::min(best, ms);
      }
      return best;
    };
    const float t1 = timed(1), t9 = timed(9);
    const double us_per_tile_phase = 1e3 * (t9 - t1) / 8.0 / ntiles;
    // epix10k2M: 256 tiles per frame
    printf("%s{\"form\": \"%s\", \"wg_per_cu\": %d, \"bitwise_mismatches\": %zu, \"value_mismatches\": %zu, "
           "\"ms_reps1\": %.4f, \"ms_reps9\": %.4f, \"column_phase_us_per_frame\": %.4f}",
           k ? ", " : "", names[k], per, bad, badv, t1, t9, us_per_tile_phase * 256.0);
    fflush(stdout);
  }
  printf("]}\n");
  hipFree(din);
  hipFree(dout);
  return rc;
}
