// Native producer engine + calibration-plan dispatcher.
//
// Reference parity: psana_ray/producer.py:78-117 (produce_data) is a Python loop that, per
// event, calls psana (CPU calibration), applies masks, and performs a blocking Ray RPC.  Here
// the per-chunk loop is a C++ thread (no interpreter, no GIL): pinned host frames ->
// hipMemcpyAsync on a side stream -> calibration kernels on a compute stream writing straight
// into HBM ring slots -> commit into the SlotPool (event-ordered, no host sync).  Backpressure
// is a condition-variable wait inside SlotPool::acquire_produce (replaces the sleep-based
// exponential backoff of producer.py:105-111).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "runtime.h"

namespace pr {

class QueueFabric;   // fabric.h

enum PlanMode : int {
  kPlanRawCopy = 0,     // mode=raw: copy raw frames into the slot
  kPlanCalib = 1,       // K-01/02/04
  kPlanCalibCm = 2,     // K-01..K-04 with K-03 common mode
  kPlanImageFused = 3,  // K-01/02/04 evaluated at image positions (no scratch)
  kPlanImageScratch = 4, // calib (+cm if use_cm) into scratch, then K-05 assemble (+image mask)
  kPlanImageCm = 5       // common-mode kernel writing the assembled image directly + gap fill
};

struct CalibPlan {
  int mode = kPlanCalib;
  int kind = 0;
  int64_t npix = 0;
  uint64_t ped = 0, gf = 0, elig = 0;
  uint64_t ped_sg = 0;  // common mode: pedestals with the eligibility in their sign bits (0 = bit-planes)
  int n_panels = 0, panel_rows = 0, panel_cols = 0, asic_rows = 0, asic_cols = 0;
  float thr = 0, maxcorr = 0;
  int npix_min = 0, cm_flags = 0, bank_cols = 0;
  int use_cm = 0;
  uint64_t idx = 0;
  int64_t nout = 0;
  uint64_t omask = 0;
  uint64_t scratch = 0;  // >= kMaxFrames * npix f32 (kPlanImageScratch)
  // LDS-tiled assembly (csrc/image.hip); use_tiles = 0 falls back to the plain gather kernels
  int use_tiles = 0;
  uint64_t tiles = 0, codes = 0;
  int n_tiles = 0, tiles_x = 0, img_h = 0, img_w = 0;
  // kPlanImageCm: per-panel (base, row step, col step) image placement + gap runs (int2 start, len)
  uint64_t img_desc = 0, gap_runs = 0;
  int n_gap_runs = 0;
  int64_t raw_frame_bytes = 0;
  int64_t out_frame_bytes = 0;
};

// Launch the plan for n frames (any n; split into kMaxFrames launches) on `stream`.
// plain: per frame, 1 = plain (not streaming) output stores (frames for another process's ring)
void run_calib_plan(const CalibPlan& plan, const std::vector<uint64_t>& in, const std::vector<uint64_t>& out,
                    uint64_t stream, const std::vector<uint8_t>* plain = nullptr);

class ProducerEngine {
 public:
  // copy_workgroups: host->HBM staging copies by copy_h2d_kernel with this many workgroups
  // (0 = hipMemcpyAsync, the runtime's blit / SDMA path); gpu_timing: event-time every chunk's
  // H2D copy and calibration (diagnostics)
  ProducerEngine(SlotPool* pool, int64_t slot_bytes, int device, const CalibPlan& plan,
                 int chunk, int n_raw_bufs, int64_t rank, int64_t size, int copy_workgroups = 32,
                 bool gpu_timing = false);
  ~ProducerEngine();
  ProducerEngine(const ProducerEngine&) = delete;
  ProducerEngine& operator=(const ProducerEngine&) = delete;

  // cycled source: frame k of this rank reads host_frames[k % n] (pinned host or device memory)
  void set_cycled_source(const std::vector<uint64_t>& frames, const std::vector<double>& photon_energy);
  // raw-run file source: rank-local event k is file record rank + k*size, read by the native
  // thread pool into pinned staging (one region per raw buffer) while the previous chunk's
  // H2D copy runs; (gevt, photon energy) come from the records.  The reader must outlive the run.
  void set_file_source(RawRunReader* reader);
  bool device_resident() const { return device_resident_; }
  // the `rank` field written into frame headers (default: the event-sharding rank).  Panel-sharded
  // producers (SURVEY P-04) shard EVENTS over rank groups but tag frames with their own rank, so a
  // consumer can tell the panel shard (rank % shards) apart from the event (gevt).
  void set_header_rank(int64_t r) { hdr_rank_ = r; }
  // Calibrate straight into consumer slots the queue fabric offers (QueueFabric::take_direct; null =
  // off).  Before start(); the fabric must outlive the run (ProducerPipeline clears it after join).
  void set_fabric(QueueFabric* f) { fabric_ = f; }
  int64_t direct_frames() const { return direct_frames_.load(); }
  // Direct headroom (0 = off): `slots` of the producer budget are kept for direct frames; frames
  // calibrated into LOCAL slots (the copy path's backlog) stay within budget - slots.  While the
  // fabric offers grants, a chunk whose local share would pass that waits for grants to cover it
  // (or for the backlog to drain) instead of queueing more frames for a second pass; wait_s > 0
  // bounds that wait (then local frames may use headroom slots).  Before start().
  void set_direct_headroom(int slots, double wait_s) {
    headroom_ = slots;
    headroom_wait_s_ = wait_s;
  }
  int direct_headroom() const { return headroom_; }
  // seconds the engine waited for grants (direct headroom)
  double direct_wait_s() const { return direct_wait_s_.load(); }
  // rank-local events [k0, n_local_events) (n_local_events < 0: endless), at most max_steps of them
  void start(int64_t n_local_events, int64_t max_steps, int64_t k0 = 0);
  void request_stop() { stop_.store(true); }
  bool join(double timeout_s);   // true when the thread has exited
  void halt();                   // stop the producing thread and join it (process exit)
  bool running() const { return running_.load(); }
  // frames whose calibration was ENQUEUED (committed to the pool; the kernels may still run)
  int64_t frames() const { return frames_.load(); }
  // Completion log (sustained-rate accounting): every chunk records a timing event
  // after its calibration; once it has completed on the device the chunk is logged as
  // (frames completed so far, device ms since the engine's origin event).  completions(i) returns
  // the entries with index >= i (older entries are trimmed past 64k chunks) and polls first.
  int64_t completed() const;
  std::vector<std::pair<int64_t, double>> completions(int64_t since, int64_t* first_index) const;
  // Device ms since the origin of the event recorded now on `stream` (host waits for it): puts a
  // point of another stream (a consumer's) on the completion log's clock.
  double mark(uint64_t stream) const;
  int64_t full_waits() const { return full_waits_.load(); }
  std::string error() const;
  // host-side time (seconds) spent per loop part: [stage copies, acquire slots, launch kernels, commit, total]
  std::vector<double> timing() const;
  // GPU-side per-stage time from timing events (gpu_timing=true at construction):
  // [h2d ms total, h2d chunks measured, calib ms total, calib chunks measured]; zeros when off
  std::vector<double> gpu_timing() const;
  // (copies that moved a multi-frame span, copies of a single frame) in cycled-host mode
  // {span copies, single-frame copies, copies done by copy_h2d_kernel (the rest went through hipMemcpyAsync)}
  std::vector<int64_t> copy_stats() const { return {span_copies_.load(), frame_copies_.load(), kernel_copies_.load()}; }
  bool gpu_timing_enabled() const { return gpu_timing_; }
  // Chunks alternate over n compute streams (before start; 1..4): chunk c+1's calibration starts
  // filling the CUs while chunk c's last workgroups drain, instead of after them.  Plans with one
  // shared scratch buffer (kPlanImageScratch) stay on one stream.
  // kind: StreamKind (streams.h) -- kStreamDedicated gives every compute stream its own hardware
  // queue.
  void set_compute_streams(int n, int kind = 0);
  int compute_streams() const { return (int)cstreams_.size(); }

 private:
  void loop(int64_t n_local_events, int64_t max_steps, int64_t k0);

  SlotPool* pool_;
  int64_t slot_bytes_;
  int device_;
  CalibPlan plan_;
  int chunk_;
  int n_raw_bufs_;
  int64_t rank_, size_, hdr_rank_;
  QueueFabric* fabric_ = nullptr;
  std::atomic<int64_t> direct_frames_{0};
  int headroom_ = 0;
  double headroom_wait_s_ = 0.002;
  std::atomic<double> direct_wait_s_{0.0};
  std::vector<uint64_t> src_frames_;
  std::vector<double> src_pe_;
  bool device_resident_ = false;   // source frames live in this GPU's HBM: no staging copies
  RawRunReader* file_ = nullptr;   // file source (instead of the cycled pool)
  void* file_staging_ = nullptr;   // pinned, n_raw_bufs x chunk frames
  std::vector<std::vector<std::pair<int64_t, double>>> buf_meta_;   // per raw buffer: (gevt, pe)
  hipStream_t h2d_ = nullptr, compute_ = nullptr;   // compute_ == cstreams_[0]
  std::vector<hipStream_t> cstreams_;
  int stream_kind_ = 0;   // placement of cstreams_ and h2d_ (streams.h): the constructor's are ordinary
  std::vector<hipEvent_t> buf_free_, h2d_done_;
  // optional GPU timing: start events per raw buffer, harvested (non-blocking) when the buffer is
  // reused or at the end of the run
  bool gpu_timing_ = false;
  int copy_workgroups_ = 32;
  std::vector<hipEvent_t> h2d_start_, calib_start_;
  std::vector<char> h2d_pending_, calib_pending_;
  double gpu_h2d_ms_ = 0, gpu_calib_ms_ = 0;
  int64_t gpu_h2d_n_ = 0, gpu_calib_n_ = 0;
  void harvest(int b, bool block);
  void* raw_bufs_ = nullptr;
  // raw chunk region b: chunk x (frame + kCopySlack) bytes.  Host frames spaced by a constant
  // stride <= frame + kCopySlack (records of a mapped run file: payload + record / datagram
  // headers) are staged with ONE copy of the whole span; dev_in_[b][q] is frame q's position.
  static constexpr int64_t kCopySlack = 4096;
  int64_t region_bytes_ = 0;
  std::vector<std::vector<uint64_t>> dev_in_;
  std::atomic<int64_t> span_copies_{0}, frame_copies_{0}, kernel_copies_{0};
  // completion log (see completed()); done_mu_ guards everything below it
  void note_chunk_done_locked() const;
  void record_chunk_done(int n, hipStream_t s);
  mutable std::mutex done_mu_;
  hipEvent_t origin_ = nullptr;
  bool origin_recorded_ = false;
  mutable std::vector<hipEvent_t> done_free_;
  std::vector<hipEvent_t> done_all_;
  mutable std::deque<std::pair<hipEvent_t, int64_t>> done_pending_;   // (event, cumulative frames)
  mutable std::vector<std::pair<int64_t, double>> done_log_;
  mutable int64_t done_base_ = 0, done_frames_ = 0;
  mutable double done_ms_ = 0;   // the log's times are prefix-completion times (monotone)
  int64_t enq_frames_ = 0;
  std::thread thread_;
  std::atomic<bool> stop_{false}, running_{false};
  std::mutex halt_mu_;   // halt() from the destructor and from halt_native_threads()
  std::atomic<int64_t> frames_{0}, full_waits_{0};
  double t_stage_ = 0, t_acquire_ = 0, t_launch_ = 0, t_commit_ = 0, t_total_ = 0;
  mutable std::mutex err_mu_;
  std::string error_;
};

}  // namespace pr
