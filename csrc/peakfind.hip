// K-07 on-GPU peak finder for queue consumers (BASELINE config 5).
//
// Reference parity: psana-ray draws "Batches -> PyTorch Task" consumers
// (figures/psana-ray-architecture.png, README.md:3) and its setup.py:11 names PeakNet as the
// downstream, but ships no analysis code; this is the consumer-side analysis the framework
// provides.  Algorithm (peakfinder8-style, simplified, every knob a parameter):
//   candidate   v > thr_peak and v is the strict local maximum of its (2R+1)^2 window
//               (ties broken by linear index; pixels outside the panel are absent)
//   background  mean / population-std of the ring of Chebyshev radius R+1 .. R+2
//   snr         (v - bkg) / max(noise, 1e-6); kept if snr >= son_min
//   intensity   sum over the (2R+1)^2 window of (pixel - bkg)
// Per-frame summary: number of pixels above thr_peak and their sum (hit-finding statistics),
// reduced wave -> LDS -> one atomic per workgroup.
//
// MI355X design: candidates are rare in detector frames, so the kernel reads every
// pixel once with coalesced 16-B loads, thresholds in registers, and sends only the rare
// candidates through the neighbourhood test (direct, cache-hit reads); one atomic per accepted
// peak reserves its record slot (and bumps an optional 64-bit running total, so consumers never
// read counts back per batch).  Round-1 A/B, epix10k2M: this stream form 2.21 us/frame, 64x32 LDS
// halo tiles 2.76-2.86, 64x16 tiles with scalar loads 5.88 (profiles/kernels_r1_peakfind_ab.jsonl;
// the losing variants are retired).
#include "common.h"
#include "kernels.h"

#include <map>
#include <mutex>

#include <algorithm>

namespace pr {


struct PfParams {
  float thr_peak;
  float son_min;
  int max_peaks;
  int n_panels, rows, cols;
};

// The test of one candidate.  at(dy, dx): neighbour value, NaN outside the panel.  Returns whether
// it is a peak and, if so, its record fields.
template <int RAD, typename At>
__device__ __forceinline__ bool pf_eval(const At& at, float v, const PfParams& pp, float& bkg, float& noise,
                                        float& snr, float& inten) {
  constexpr int H = RAD + 2;
  constexpr int D = 2 * H + 1;
  // the whole (2H+1)^2 neighbourhood is loaded up front: ONE round of independent loads instead of
  // one per test below (the tests run after the stream, so their latency is the kernel's tail;
  // measured 1.824-1.828 vs 1.836-1.842 us/frame, 32 epix10k2M frames)
  float w[D][D];
#pragma unroll
  for (int dy = -H; dy <= H; ++dy)
#pragma unroll
    for (int dx = -H; dx <= H; ++dx) w[dy + H][dx + H] = (dy == 0 && dx == 0) ? v : at(dy, dx);
  bkg = 0.0f, noise = 0.0f, snr = 0.0f, inten = 0.0f;
#pragma unroll
  for (int dy = -RAD; dy <= RAD; ++dy)
#pragma unroll
    for (int dx = -RAD; dx <= RAD; ++dx) {
      if (dy == 0 && dx == 0) continue;
      const float n = w[dy + H][dx + H];
      if (n != n) continue;
      const bool before = (dy < 0) || (dy == 0 && dx < 0);
      if (before ? !(v > n) : !(v >= n)) return false;   // not the strict local max (ties: lower index wins)
    }
  float s = 0.0f, s2 = 0.0f;
  int nr = 0;
#pragma unroll
  for (int dy = -H; dy <= H; ++dy)
#pragma unroll
    for (int dx = -H; dx <= H; ++dx) {
      const int d = max(abs(dy), abs(dx));
      if (d <= RAD) continue;
      const float n = w[dy + H][dx + H];
      if (n != n) continue;
      s += n;
      s2 += n * n;
      ++nr;
    }
  bkg = nr > 0 ? s / nr : 0.0f;
  const float var = nr > 0 ? fmaxf(s2 / nr - bkg * bkg, 0.0f) : 0.0f;
  noise = sqrtf(var);
  snr = (v - bkg) / fmaxf(noise, 1e-6f);
  if (snr < pp.son_min) return false;
#pragma unroll
  for (int dy = -RAD; dy <= RAD; ++dy)
#pragma unroll
    for (int dx = -RAD; dx <= RAD; ++dx) {
      const float n = w[dy + H][dx + H];
      if (n == n) inten += n - bkg;
    }
  return true;
}

// one record = two 16-B stores (records are 32-B aligned)
__device__ __forceinline__ void pf_store(float* __restrict__ peaks, const PfParams& pp, int f, int slot,
                                         const f32x4_t& a, const f32x4_t& b) {
  f32x4_t* rec = reinterpret_cast<f32x4_t*>(peaks + ((int64_t)f * pp.max_peaks + slot) * 8);
  rec[0] = a;
  rec[1] = b;
}

// Slot index among the lanes here with `pending` set, per frame: ONE atomic on ctr[f] per (wave,
// frame) -- same-address atomics serialise, so never one per lane.  ctr is an LDS counter array
// (the workgroup's per-frame tallies) or the global per-frame counts (in-stream path).
__device__ __forceinline__ int pf_claim(bool pending, int f, int* ctr) {
  const int lane = (int)(threadIdx.x & 63);
  int loc = 0;
  for (;;) {
    const uint64_t m = __ballot(pending);
    if (m == 0) break;
    const int leader = __ffsll((unsigned long long)m) - 1;
    const int f0 = __shfl(f, leader);
    const uint64_t mf = __ballot(pending && f == f0);
    int base = 0;
    if (lane == leader) base = atomicAdd(ctr + f0, __popcll(mf));
    base = __shfl(base, leader);
    if (pending && f == f0) {
      loc = base + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(mf >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mf, 0u));
      pending = false;
    }
  }
  return loc;
}

// records written by the active lanes with `wrote` set, added to the running total (one atomic
// per wave)
__device__ __forceinline__ void pf_add_total(unsigned long long* total, bool wrote) {
  if (total == nullptr) return;
  const uint64_t wr = __ballot(wrote);
  const int leader = __ffsll((unsigned long long)__ballot(1)) - 1;
  if ((int)(threadIdx.x & 63) == leader && wr != 0) atomicAdd(total, (unsigned long long)__popcll(wr));
}

// ---------------------------------------------------------------------------------------------
// Streaming form: candidates are rare in detector frames (synthetic epix10k2M: 0.02 % of pixels
// above thr_peak, 0.5 % of 64-pixel wave rows contain one), so an LDS halo tile is overhead: every
// pixel is read ONCE with coalesced 16-B loads (4 float4 per lane in flight), thresholded in
// registers, and only the rare candidates -- parked in LDS until the stream ends, then tested one
// per lane -- read their neighbourhood directly from global memory (just-touched lines, L1/L2
// hits).  No halo over-fetch; LDS only for the parked candidates and the statistics reduction.
// ---------------------------------------------------------------------------------------------
// The per-frame hit statistics are device-scope atomics to ONE address pair per frame, and
// same-address atomics serialise (~3 ns each, measured: read_f32 with one atomic per 8-KB block
// 3.09 us/frame vs 1.81 with one per 16 KB), so a workgroup owns many 16-KB chunks and issues its
// two atomics once per frame it touches.  The next chunk's loads are issued before the current
// chunk's rare candidates are parked, so the memory pipe stays busy.
//
// Self-resetting outputs (`scratch` != nullptr): the slot counters and hit statistics accumulate in
// a persistent scratch block instead of in `counts` / `summary`; the LAST workgroup to finish
// (device-scope done counter) moves them to the outputs and zeroes the scratch for the next
// launch on the stream -- so a consumer needs no per-batch fill kernel before the peak finder.
// ONE scratch block per stream: two launches in flight on different streams sharing a block would
// mix their counters and race on the done ticket (PeakFinderConsumer owns one per consumer stream;
// kernels.peakfind documents the rule).
struct PfScratch {
  int tickets[kMaxFrames];
  float acc[2 * kMaxFrames];
  unsigned int done;
};

// Frame loads of the stream: 1 = non-temporal (each pixel is read once; the frames do not push the
// producer's common-mode tables out of L2 when both run on the GPU), 0 = plain.
#ifndef PR_PF_NT_LOAD
#define PR_PF_NT_LOAD 0
#endif
constexpr int kPfCandCap = 512;   // candidates parked per workgroup (2 KiB of LDS)
static_assert(sizeof(PfScratch) <= kPfScratchHeader, "PfScratch outgrew its header");
// spill entry: pixel | frame << 26 (frames of < 2^26 pixels; larger frames test overflow inline)
constexpr int kPfSpillShift = 26;

// Balanced grid: ONE resident wave of workgroups (CUs x occupancy) over the batch's (frame, chunk)
// sequence, each taking a contiguous range of T / G chunks, so every workgroup ends within one
// chunk of the others.  (The round-2 2-D grid -- 64 workgroups per frame striding over the frame's
// 528 chunks -- gave 16 of every 64 a ninth chunk: 1.92-1.99 vs 1.88-1.89 us/frame for this form,
// 32 epix10k2M frames, tools/pf_probe.py; K = 8 / 16 float4 per lane: 2.19 / 2.25, lower occupancy.)
// A range crosses at most a couple of frame boundaries; the hit statistics are flushed at each.
// PR_PF_WAVES_PER_EU > 0: VGPR budget 512 / N (diagnostic builds: co-residency with the
// common-mode kernel's waves, which leave 64 VGPRs per SIMD lane free)
#ifndef PR_PF_WAVES_PER_EU
#define PR_PF_WAVES_PER_EU 0
#endif
#if PR_PF_WAVES_PER_EU > 0
#define PR_PF_WAVES_ATTR __attribute__((amdgpu_waves_per_eu(PR_PF_WAVES_PER_EU, PR_PF_WAVES_PER_EU)))
#else
#define PR_PF_WAVES_ATTR
#endif
template <int RAD, int K>
__global__ __launch_bounds__(256) PR_PF_WAVES_ATTR void peakfind_range_kernel(const FramePtrs fp, const PfParams pp,
                                                             float* __restrict__ peaks, int* __restrict__ counts_out,
                                                             float* __restrict__ summary_out,
                                                             unsigned long long* __restrict__ total,
                                                             PfScratch* __restrict__ scratch, const int nframes,
                                                             const bool spill_ok) {
  __shared__ float red_sum[4];
  __shared__ int red_cnt[4];
  __shared__ int is_last;
  __shared__ int cand_n;
  __shared__ int cand_p[kPfCandCap];
  __shared__ unsigned char cand_f[kPfCandCap];
  __shared__ int wg_cnt[kMaxFrames], wg_n0[kMaxFrames], wg_base[kMaxFrames];   // per-frame tallies
  int* counts = scratch != nullptr ? scratch->tickets : counts_out;
  float* summary = scratch != nullptr ? scratch->acc : summary_out;
  // the running total: with a scratch block the last workgroup adds the launch's record count in
  // ONE atomic (per-peak atomics on one address serialise, ~3 ns each: 1,800 per 32-frame launch
  // kept the kernel's completion ~5 us behind its last wave); without one, one atomic per record
  unsigned long long* const total_per_peak = scratch != nullptr ? nullptr : total;
  const int64_t hw = (int64_t)pp.rows * pp.cols;
  const int64_t n4 = (int64_t)pp.n_panels * hw / 4;
  const int ncpf = (int)((n4 + 256 * K - 1) / (256 * K));
  const int64_t T = (int64_t)ncpf * nframes;
  const int64_t g0 = T * blockIdx.x / gridDim.x, g1 = T * (blockIdx.x + 1) / gridDim.x;
  const float NaN = __int_as_float(0x7fc00000);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  // this workgroup's spill list (hit-rich frames; none without a scratch block or past kPfSpillWgs)
  uint32_t* const spill = (scratch != nullptr && spill_ok && (int)blockIdx.x < kPfSpillWgs)
                              ? reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(scratch) + kPfScratchHeader) +
                                    (int64_t)blockIdx.x * kPfSpillCap
                              : nullptr;
  const int cap = kPfCandCap + (spill != nullptr ? kPfSpillCap : 0);
  f32x4_t v[K];
#ifndef PR_PF_DEPTH
#define PR_PF_DEPTH 1
#endif
  f32x4_t v2[PR_PF_DEPTH > 1 ? K : 1];   // PR_PF_DEPTH 2: a second chunk in flight
  #ifndef PR_PF_FASTLOAD
#define PR_PF_FASTLOAD 1
#endif
// chunk g's float4s: a uniform base (SGPR) + a 32-bit lane offset; interior chunks (all but a
  // frame's last) load without per-load bounds checks (each cost a 64-bit compare, an exec-mask
  // branch and four NaN moves: ~1/3 of the stream loop's VALU)
  auto load_to = [&](f32x4_t(&v)[K], int64_t g) {
    const int f = (int)(g / ncpf);
    const int64_t c0 = (g - (int64_t)f * ncpf) * 256 * K;   // first float4 of the chunk (uniform)
    const PR_GLOBAL f32x4_t* cp = reinterpret_cast<const PR_GLOBAL f32x4_t*>(gin<float>(fp.in[f])) + c0;
    const uint32_t t = threadIdx.x;
    if (PR_PF_FASTLOAD && c0 + 256 * K <= n4) {
#pragma unroll
      for (int k = 0; k < K; ++k) {
#if PR_PF_NT_LOAD
        v[k] = ld_nt_f4(cp + t + 256 * k);
#else
        v[k] = cp[t + 256 * k];
#endif
      }
    } else {
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const bool in = c0 + t + 256 * k < n4;
#if PR_PF_NT_LOAD
        v[k] = in ? ld_nt_f4(cp + t + 256 * k) : f32x4_t{NaN, NaN, NaN, NaN};
#else
        v[k] = in ? cp[t + 256 * k] : f32x4_t{NaN, NaN, NaN, NaN};
#endif
      }
    }
  };
  auto load = [&](int64_t g) { load_to(v, g); };
  // A candidate's (2H+1)^2 neighbourhood, H = RAD + 2, as THREE aligned 16-B loads per row (the
  // 4-float groups holding columns x-H .. x+H; panels are a multiple of 4 wide, so a group is wholly
  // inside or outside its row) instead of (2H+1) 4-B loads: 21 vector loads for RAD 1 where 49 scalar
  // ones kept the texture units busy on hit-rich frames (tens of thousands of candidates per frame).
  // Returns whether the candidate is a peak; its record in (ra, rb).
  auto test = [&](int f, int64_t p, f32x4_t& ra, f32x4_t& rb) -> bool {
    constexpr int H = RAD + 2, D = 2 * H + 1;
    static_assert(D <= 9, "three 4-float groups per row cover at most 9 columns at any alignment");
    const PR_GLOBAL float* img = gin<float>(fp.in[f]);
    const int panel = (int)(p / hw);
    const int64_t rem = p - (int64_t)panel * hw;
    const int y = (int)(rem / pp.cols), x = (int)(rem - (int64_t)(rem / pp.cols) * pp.cols);
    const PR_GLOBAL float* pim = img + (int64_t)panel * hw;
    const int base = (x - H) & ~3;          // first group (may start left of the panel)
    const int off = (x - H) - base;         // 0..3: column x-H inside it
    float wv[D][D];
#pragma unroll
    for (int dy = -H; dy <= H; ++dy) {
      const int yy = y + dy;
      const bool row_ok = yy >= 0 && yy < pp.rows;
      float e[12];
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const int c0 = base + 4 * k;
        const f32x4_t q = (row_ok && c0 >= 0 && c0 < pp.cols)
                              ? *(const PR_GLOBAL f32x4_t*)(pim + (int64_t)yy * pp.cols + c0)
                              : f32x4_t{NaN, NaN, NaN, NaN};
        e[4 * k] = q.x; e[4 * k + 1] = q.y; e[4 * k + 2] = q.z; e[4 * k + 3] = q.w;
      }
#pragma unroll
      for (int dx = 0; dx < D; ++dx)   // register select on the run-time alignment (no indexed access)
        wv[dy + H][dx] = off == 0 ? e[dx] : off == 1 ? e[dx + 1] : off == 2 ? e[dx + 2] : e[dx + 3];
    }
    const float val = wv[H][H];
    float bkg, noise, snr, inten;
    const bool ok = pf_eval<RAD>([&](int dy, int dx) { return wv[dy + H][dx + H]; }, val, pp, bkg, noise, snr, inten);
    ra = f32x4_t{(float)panel, (float)y, (float)x, val};
    rb = f32x4_t{inten, bkg, noise, snr};
    return ok;
  };
  // in-stream path (a workgroup past its LDS and spill capacity): slots straight from the global
  // per-frame counts, one atomic per (wave, frame)
  auto test_now = [&](int f, int64_t p) {
    f32x4_t ra, rb;
    const bool ok = test(f, p, ra, rb);
    const int slot = pf_claim(ok, f, counts);
    const bool wrote = ok && slot < pp.max_peaks;
    if (wrote) pf_store(peaks, pp, f, slot, ra, rb);
    pf_add_total(total_per_peak, wrote);
  };
  // block-reduce this frame's statistics and add them (one atomic pair per workgroup and frame)
  auto flush = [&](int f, float s, int c) {
    for (int o = 32; o > 0; o >>= 1) {
      s += __shfl_down(s, o);
      c += __shfl_down(c, o);
    }
    __syncthreads();
    if (lane == 0) {
      red_sum[wave] = s;
      red_cnt[wave] = c;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      const float sm = red_sum[0] + red_sum[1] + red_sum[2] + red_sum[3];
      const int cn = red_cnt[0] + red_cnt[1] + red_cnt[2] + red_cnt[3];
      if (cn > 0) {
        const float o0 = atomicAdd(summary + 2 * f, (float)cn);
        const float o1 = atomicAdd(summary + 2 * f + 1, sm);
        if (scratch != nullptr) asm volatile("" ::"v"(o0), "v"(o1));
      }
    }
  };
  if (threadIdx.x == 0) cand_n = 0;
  if (threadIdx.x < kMaxFrames) wg_cnt[threadIdx.x] = 0;
  __syncthreads();
  float above_sum = 0.0f;
  int above_cnt = 0;
  int fcur = (int)(g0 / ncpf);
  // one chunk: candidate bits and hit statistics from its registers, the next load issued (`refill`),
  // then the candidates parked
  auto chunk = [&](f32x4_t(&cv)[K], int64_t g, auto refill) {
    const int f = (int)(g / ncpf);   // wave-uniform
    if (f != fcur) {
      flush(fcur, above_sum, above_cnt);
      above_sum = 0.0f;
      above_cnt = 0;
      fcur = f;
    }
    uint64_t cand = 0;
#pragma unroll
    for (int k = 0; k < K; ++k) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float val = cv[k][e];
        const bool hit = val > pp.thr_peak;
        above_sum += hit ? val : 0.0f;
        above_cnt += hit ? 1 : 0;
        cand |= (uint64_t)hit << (4 * k + e);
      }
    }
    const int64_t q0 = (g - (int64_t)f * ncpf) * 256 * K + threadIdx.x;
    refill();
#ifdef PR_PF_DIAG_STREAM_ONLY
    cand = 0;   // diagnostic builds only: the stream without any candidate handling
#endif
    if (cand) {
      int slot = atomicAdd(&cand_n, __popcll(cand));
      while (cand) {
        const int b = __builtin_ctzll(cand);
        cand &= cand - 1;
        const int64_t p = 4 * (q0 + 256 * (b >> 2)) + (b & 3);
        if (slot < kPfCandCap) {
          cand_p[slot] = (int)p;
          cand_f[slot] = (unsigned char)f;
        } else if (slot < cap) {
          spill[slot - kPfCandCap] = (uint32_t)p | ((uint32_t)f << kPfSpillShift);
        } else {
          test_now(f, p);   // past LDS and spill: tested in the stream (correct, slow)
        }
        ++slot;
      }
    }
  };
#if PR_PF_DEPTH > 1
  if (g0 < g1) load_to(v, g0);
  if (g0 + 1 < g1) load_to(v2, g0 + 1);
  for (int64_t g = g0; g < g1; g += 2) {
    chunk(v, g, [&] { if (g + 2 < g1) load_to(v, g + 2); });
    if (g + 1 < g1) chunk(v2, g + 1, [&] { if (g + 3 < g1) load_to(v2, g + 3); });
  }
#else
  if (g0 < g1) load(g0);
  for (int64_t g = g0; g < g1; ++g) chunk(v, g, [&] { if (g + 1 < g1) load(g + 1); });
#endif
  if (g0 < g1) flush(fcur, above_sum, above_cnt);
  __syncthreads();
  // Parked, then spilled candidates, one per thread and round (the spill stores above are visible:
  // the barrier orders them for the whole workgroup).  Record slots are reserved ONCE per
  // (workgroup, frame) from the global counts, not per (wave, round): tallies go to LDS counters
  // first.  (Per-wave global atomics on the few per-frame count words cost 2.6 us/frame on a
  // hit-rich batch -- 44k candidates / 32k peaks per epix10k2M frame; one returning atomic on one
  // word saturates near 88 per us, MI355X_MICROARCH.md dequeue row.)
  //   round 0 (threads 0..255)  test, keep the record in registers, claim a local index
  //   rounds >= 1               test, count only
  //   reserve                   one global atomic per frame this workgroup accepted peaks in
  //   write                     round 0 from registers; rounds >= 1 re-tested, only for frames
  //                             whose reserved range still reaches below max_peaks (a hit-rich
  //                             frame past its record capacity needs counts, not records)
#ifdef PR_PF_DIAG_STREAM_ONLY
  const int nc = 0;
#else
  const int nc = min(cand_n, cap);
#endif
  auto cand_at = [&](int i, int& f, int64_t& p) {
    if (i < kPfCandCap) {
      f = cand_f[i];
      p = cand_p[i];
    } else {
      const uint32_t e = spill[i - kPfCandCap];
      f = (int)(e >> kPfSpillShift);
      p = (int64_t)(e & ((1u << kPfSpillShift) - 1u));
    }
  };
  const int tid = (int)threadIdx.x;
  int f0 = 0, loc0 = 0;
  f32x4_t ra0{}, rb0{};
  bool ok0 = false;
  if (tid < nc) {
    int64_t p;
    cand_at(tid, f0, p);
    ok0 = test(f0, p, ra0, rb0);
  }
  loc0 = pf_claim(ok0, f0, wg_cnt);
  __syncthreads();
  if (tid < nframes) wg_n0[tid] = wg_cnt[tid];
  for (int i = tid + 256; i < nc; i += 256) {
    int f;
    int64_t p;
    cand_at(i, f, p);
    f32x4_t ra, rb;
    const bool ok = test(f, p, ra, rb);
    pf_claim(ok, f, wg_cnt);
  }
  __syncthreads();
  if (tid < nframes) {
    const int c = wg_cnt[tid];
    wg_base[tid] = c > 0 ? atomicAdd(counts + tid, c) : 0;
    wg_cnt[tid] = wg_n0[tid];   // running local index of rounds >= 1
  }
  __syncthreads();
  {
    const bool wrote = ok0 && wg_base[f0] + loc0 < pp.max_peaks;
    if (wrote) pf_store(peaks, pp, f0, wg_base[f0] + loc0, ra0, rb0);
    pf_add_total(total_per_peak, wrote);
  }
  for (int i = tid + 256; i < nc; i += 256) {
    int f;
    int64_t p;
    cand_at(i, f, p);
    f32x4_t ra, rb;
    const bool ok = wg_base[f] + wg_n0[f] < pp.max_peaks && test(f, p, ra, rb);
    const int slot = wg_base[f] + pf_claim(ok, f, wg_cnt);
    const bool wrote = ok && slot < pp.max_peaks;
    if (wrote) pf_store(peaks, pp, f, slot, ra, rb);
    pf_add_total(total_per_peak, wrote);
  }
  if (scratch == nullptr) return;
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned prev = atomicAdd(&scratch->done, 1u);
    is_last = prev == gridDim.x - 1;
  }
  __syncthreads();
  if (!is_last) return;
  int written = 0;   // records written by this launch (slots below max_peaks)
  for (int i = threadIdx.x; i < nframes; i += blockDim.x) {
    const int c = atomicExch(&scratch->tickets[i], 0);
    counts_out[i] = c;
    written += min(c, pp.max_peaks);
    summary_out[2 * i] = atomicExch(&scratch->acc[2 * i], 0.0f);
    summary_out[2 * i + 1] = atomicExch(&scratch->acc[2 * i + 1], 0.0f);
  }
  if (total != nullptr) {
    for (int o = 32; o > 0; o >>= 1) written += __shfl_down(written, o);
    if (lane == 0) red_cnt[wave] = written;
    __syncthreads();
    if (threadIdx.x == 0) {
      const int n = red_cnt[0] + red_cnt[1] + red_cnt[2] + red_cnt[3];
      if (n > 0) atomicAdd(total, (unsigned long long)n);
    }
  }
  if (threadIdx.x == 0) atomicExch(&scratch->done, 0u);
}

// resident workgroups of a 256-thread kernel on the CURRENT device, queried once per (device,
// kernel) under a lock: a process that drives several GPUs, or launches from several threads, sizes
// every grid from its own device's answer (speed only: the last-workgroup protocol needs no
// co-residency)
template <typename Kern>
static int pf_resident_blocks(int which, Kern k) {
  static std::mutex mu;
  static std::map<std::pair<int, int>, int> cache;
  int dev = 0;
  hip_check(hipGetDevice(&dev), "pf device");
  std::lock_guard<std::mutex> lk(mu);
  int& n = cache[{dev, which}];
  if (n == 0) {
    int cus = 0, per = 0;
    hip_check(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev), "pf cu count");
    hip_check(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, (const void*)k, 256, 0), "pf occupancy");
    n = std::max(1, cus * std::max(1, per));
  }
  return n;
}

void launch_peakfind(const FramePtrs& fp, int nframes, int n_panels, int rows, int cols, float thr_peak,
                     float son_min, int radius, int max_peaks, uint64_t peaks, uint64_t counts,
                     uint64_t summary, uint64_t total, uint64_t stream, uint64_t scratch) {
  check(nframes >= 1 && nframes <= kMaxFrames, "peakfind: nframes out of range");
  check(radius == 1 || radius == 2, "peakfind: radius must be 1 or 2");
  check(max_peaks >= 1, "peakfind: max_peaks must be >= 1");
  check(cols % 4 == 0, "peakfind: panel width must be a multiple of 4");
  check((int64_t)n_panels * rows * cols < (int64_t)1 << 31, "peakfind: frame too large for 32-bit pixel ids");
  for (int f = 0; f < nframes; ++f) check(aligned16(fp.in[f]), "peakfind: frames must be 16-B aligned");
  PfParams pp{thr_peak, son_min, max_peaks, n_panels, rows, cols};
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  float* P = reinterpret_cast<float*>(peaks);
  int* C = reinterpret_cast<int*>(counts);
  float* S = reinterpret_cast<float*>(summary);
  unsigned long long* T = reinterpret_cast<unsigned long long*>(total);
  PfScratch* X = reinterpret_cast<PfScratch*>(scratch);
  check(scratch % 8 == 0, "peakfind: misaligned scratch");
  constexpr int K = 4;   // float4 per lane per chunk (16 KB per 256-thread chunk)
  const int64_t n4 = (int64_t)n_panels * rows * cols / 4;
  const int64_t chunks = (n4 + 256 * K - 1) / (256 * K) * nframes;
  auto kern = radius == 1 ? peakfind_range_kernel<1, K> : peakfind_range_kernel<2, K>;
  const int g = (int)std::min<int64_t>(chunks, pf_resident_blocks(radius == 1 ? 0 : 1, kern));
  const bool spill_ok = (int64_t)n_panels * rows * cols < ((int64_t)1 << kPfSpillShift) && nframes <= 64;
  hipLaunchKernelGGL(kern, dim3(g), dim3(256), 0, s, fp, pp, P, C, S, T, X, nframes, spill_ok);
  hip_check(hipGetLastError(), "peakfind launch");
}

}  // namespace pr
