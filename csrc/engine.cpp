#include "engine.h"
#include "fabric.h"
#include "trace.h"

#include <chrono>
#include <thread>
#include <stdexcept>

#include "common.h"
#include "kernels.h"
#include "lifecycle.h"
#include "streams.h"

namespace pr {

static FramePtrs ptrs_of(const std::vector<uint64_t>& in, const std::vector<uint64_t>& out, size_t a, size_t b) {
  FramePtrs fp{};
  for (size_t i = a; i < b; ++i) {
    fp.in[i - a] = in[i];
    fp.out[i - a] = out[i];
  }
  return fp;
}

void run_calib_plan(const CalibPlan& p, const std::vector<uint64_t>& in, const std::vector<uint64_t>& out,
                    uint64_t stream, const std::vector<uint8_t>* plain) {
  check(in.size() == out.size(), "run_calib_plan: in/out size mismatch");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  for (size_t a = 0; a < in.size(); a += kMaxFrames) {
    const size_t b = std::min(in.size(), a + (size_t)kMaxFrames);
    const int n = (int)(b - a);
    uint64_t plain_mask = 0;   // frames written into another process's ring: plain stores (fabric.h direct)
    if (plain != nullptr)
      for (size_t i = a; i < b && i < plain->size(); ++i)
        if ((*plain)[i]) plain_mask |= 1ull << (i - a);
    switch (p.mode) {
      case kPlanRawCopy:
        for (size_t i = a; i < b; ++i)
          hip_check(hipMemcpyAsync(reinterpret_cast<void*>(out[i]), reinterpret_cast<const void*>(in[i]),
                                   (size_t)p.raw_frame_bytes, hipMemcpyDeviceToDevice, s),
                    "raw copy");
        break;
      case kPlanCalib:
        launch_calib_basic(ptrs_of(in, out, a, b), n, p.ped, p.gf, p.npix, p.kind, stream);
        break;
      case kPlanCalibCm:
        launch_calib_cm(ptrs_of(in, out, a, b), n, p.ped, p.gf, p.elig, p.kind, p.n_panels, p.panel_rows,
                        p.panel_cols, p.asic_rows, p.asic_cols, p.thr, p.maxcorr, p.npix_min, p.cm_flags,
                        p.bank_cols, stream, 0, 0, 0, p.ped_sg, plain_mask);
        break;
      case kPlanImageFused:
        if (p.use_tiles)
          launch_image_tiles(ptrs_of(in, out, a, b), n, true, p.kind, p.ped, p.gf, p.npix, p.panel_rows,
                             p.panel_cols, p.tiles, p.n_tiles, p.tiles_x, p.codes, p.img_h, p.img_w, stream);
        else
          launch_calib_image(ptrs_of(in, out, a, b), n, p.ped, p.gf, p.npix, p.kind, p.idx, p.nout, stream);
        break;
      case kPlanImageCm: {
        check(p.use_cm && p.img_desc != 0, "run_calib_plan: fused image plan without common mode / placement");
        const FramePtrs fp = ptrs_of(in, out, a, b);
        launch_calib_cm(fp, n, p.ped, p.gf, p.elig, p.kind, p.n_panels, p.panel_rows, p.panel_cols, p.asic_rows,
                        p.asic_cols, p.thr, p.maxcorr, p.npix_min, p.cm_flags, p.bank_cols, stream, p.img_desc, p.gap_runs,
                        p.n_gap_runs, p.ped_sg);
        break;
      }
      case kPlanImageScratch: {
        check(p.scratch != 0, "run_calib_plan: image plan without scratch");
        std::vector<uint64_t> tmp(n);
        for (int i = 0; i < n; ++i) tmp[i] = p.scratch + (uint64_t)i * (uint64_t)p.npix * 4u;
        std::vector<uint64_t> ina(in.begin() + a, in.begin() + b), outa(out.begin() + a, out.begin() + b);
        if (p.use_cm)
          launch_calib_cm(ptrs_of(ina, tmp, 0, n), n, p.ped, p.gf, p.elig, p.kind, p.n_panels, p.panel_rows,
                          p.panel_cols, p.asic_rows, p.asic_cols, p.thr, p.maxcorr, p.npix_min, p.cm_flags,
                          p.bank_cols, stream, 0, 0, 0, p.ped_sg);
        else
          launch_calib_basic(ptrs_of(ina, tmp, 0, n), n, p.ped, p.gf, p.npix, p.kind, stream);
        if (p.use_tiles)
          launch_image_tiles(ptrs_of(tmp, outa, 0, n), n, false, p.kind, 0, 0, p.npix, p.panel_rows,
                             p.panel_cols, p.tiles, p.n_tiles, p.tiles_x, p.codes, p.img_h, p.img_w, stream);
        else
          launch_assemble(ptrs_of(tmp, outa, 0, n), n, p.idx, p.nout, p.omask, stream);
        break;
      }
      default:
        check(false, "run_calib_plan: unknown plan mode");
    }
  }
}

// ---------------------------------------------------------------------------------------
ProducerEngine::ProducerEngine(SlotPool* pool, int64_t slot_bytes, int device,
                               const CalibPlan& plan, int chunk, int n_raw_bufs, int64_t rank, int64_t size,
                               int copy_workgroups, bool gpu_timing)
    : pool_(pool), slot_bytes_(slot_bytes), device_(device), plan_(plan),
      chunk_(std::max(1, std::min(chunk, kMaxFrames))), n_raw_bufs_(std::max(2, n_raw_bufs)), rank_(rank),
      size_(size), hdr_rank_(rank), gpu_timing_(gpu_timing), copy_workgroups_(std::max(0, copy_workgroups)) {
  check(pool != nullptr && device >= 0, "ProducerEngine needs a device SlotPool");
  check(plan.raw_frame_bytes > 0 && plan.raw_frame_bytes % 16 == 0, "ProducerEngine: bad raw frame size");
  DeviceGuard dg(device_);
  hip_check(hipStreamCreateWithFlags(&h2d_, hipStreamNonBlocking), "hipStreamCreate");
  hip_check(hipStreamCreateWithFlags(&compute_, hipStreamNonBlocking), "hipStreamCreate");
  cstreams_.push_back(compute_);
  const unsigned ev_flags = gpu_timing_ ? hipEventDefault : hipEventDisableTiming;
  buf_free_.resize(n_raw_bufs_);
  h2d_done_.resize(n_raw_bufs_);
  for (int i = 0; i < n_raw_bufs_; ++i) {
    hip_check(hipEventCreateWithFlags(&buf_free_[i], ev_flags), "hipEventCreate");
    hip_check(hipEventCreateWithFlags(&h2d_done_[i], ev_flags), "hipEventCreate");
  }
  if (gpu_timing_) {
    h2d_start_.resize(n_raw_bufs_);
    calib_start_.resize(n_raw_bufs_);
    for (int i = 0; i < n_raw_bufs_; ++i) {
      hip_check(hipEventCreate(&h2d_start_[i]), "hipEventCreate");
      hip_check(hipEventCreate(&calib_start_[i]), "hipEventCreate");
    }
    h2d_pending_.assign(n_raw_bufs_, 0);
    calib_pending_.assign(n_raw_bufs_, 0);
  }
  hip_check(hipEventCreate(&origin_), "hipEventCreate (origin)");
  region_bytes_ = (int64_t)chunk_ * (plan.raw_frame_bytes + kCopySlack);
  hip_check(hipMalloc(&raw_bufs_, (size_t)n_raw_bufs_ * region_bytes_), "hipMalloc raw chunks");
  dev_in_.assign(n_raw_bufs_, std::vector<uint64_t>(chunk_, 0));
  register_native_thread_owner(this, [this] { halt(); });
}

void ProducerEngine::halt() {
  std::lock_guard<std::mutex> lk(halt_mu_);
  stop_.store(true);
  pool_->wake_producers();
  if (thread_.joinable()) thread_.join();
}

ProducerEngine::~ProducerEngine() {
  unregister_native_thread_owner(this);
  halt();
  DeviceGuard dg(device_);
  if (h2d_) (void)hipStreamSynchronize(h2d_);
  for (auto cs : cstreams_) (void)hipStreamSynchronize(cs);
  for (auto e : buf_free_) (void)hipEventDestroy(e);
  for (auto e : h2d_done_) (void)hipEventDestroy(e);
  for (auto e : h2d_start_) (void)hipEventDestroy(e);
  for (auto e : calib_start_) (void)hipEventDestroy(e);
  for (auto e : done_all_) (void)hipEventDestroy(e);
  if (origin_) (void)hipEventDestroy(origin_);
  if (raw_bufs_) (void)hipFree(raw_bufs_);
  if (file_staging_) (void)hipHostFree(file_staging_);
  release_stream(device_, stream_kind_, h2d_);
  for (auto cs : cstreams_) release_stream(device_, stream_kind_, cs);
}

void ProducerEngine::set_compute_streams(int n, int kind) {
  check(!running_.load() && !thread_.joinable(), "ProducerEngine: set_compute_streams before start");
  check(n >= 1 && n <= 8, "ProducerEngine: compute streams must be 1..8");
  {
    std::lock_guard<std::mutex> lk(done_mu_);
    check(!origin_recorded_, "ProducerEngine: set_compute_streams after the first start");
  }
  if (plan_.mode == kPlanImageScratch) n = 1;   // one scratch buffer: never two launches in flight
  DeviceGuard dg(device_);
  for (auto cs : cstreams_) release_stream(device_, stream_kind_, cs);
  cstreams_.clear();
  const int old_kind = stream_kind_;
  stream_kind_ = kind;
  for (int i = 0; i < n; ++i) cstreams_.push_back(acquire_stream(device_, kind));
  compute_ = cstreams_[0];
  // the staging copies get the same placement: a copy stream multiplexed onto a queue that runs
  // calibration or peak-finder kernels would wait behind them and idle the PCIe link
  release_stream(device_, old_kind, h2d_);
  h2d_ = acquire_stream(device_, kind);
}

void ProducerEngine::set_cycled_source(const std::vector<uint64_t>& frames, const std::vector<double>& pe) {
  check(!running_.load(), "ProducerEngine: cannot change the source while running");
  check(!frames.empty() && frames.size() == pe.size(), "ProducerEngine: bad cycled source");
  src_frames_ = frames;
  src_pe_ = pe;
  // frames already resident in this GPU's memory are calibrated in place: no staging copy
  DeviceGuard dg(device_);
  bool all_dev = true;
  for (uint64_t f : frames) {
    hipPointerAttribute_t a{};
    if (hipPointerGetAttributes(&a, reinterpret_cast<const void*>(f)) != hipSuccess ||
        a.type != hipMemoryTypeDevice || a.device != device_) {
      (void)hipGetLastError();   // pageable host memory reports an error: clear it
      all_dev = false;
      break;
    }
  }
  device_resident_ = all_dev;
}

void ProducerEngine::set_file_source(RawRunReader* reader) {
  check(!running_.load(), "ProducerEngine: cannot change the source while running");
  check(reader != nullptr, "ProducerEngine: null reader");
  check(reader->frame_bytes() == plan_.raw_frame_bytes, "ProducerEngine: file frame size != detector raw frame");
  DeviceGuard dg(device_);
  if (file_staging_ == nullptr)
    hip_check(hipHostMalloc(&file_staging_, (size_t)n_raw_bufs_ * chunk_ * plan_.raw_frame_bytes, hipHostMallocDefault),
              "hipHostMalloc file staging");
  file_ = reader;
  device_resident_ = false;
  src_frames_.assign(1, 0);     // non-empty marker; the cycled pool is not used
  src_pe_.assign(1, 0.0);
  buf_meta_.assign(n_raw_bufs_, {});
}

void ProducerEngine::start(int64_t n_local_events, int64_t max_steps, int64_t k0) {
  check(!src_frames_.empty() || file_ != nullptr, "ProducerEngine: no source");
  if (file_ != nullptr) check(n_local_events >= 0, "ProducerEngine: a file source needs its event count");
  check(k0 >= 0, "ProducerEngine: negative start event");
  check(!running_.load() && !thread_.joinable(), "ProducerEngine: already started");
  stop_.store(false);
  {
    std::lock_guard<std::mutex> lk(done_mu_);
    if (!origin_recorded_) {   // the completion log's clock starts here
      DeviceGuard dg(device_);
      hip_check(hipEventRecord(origin_, compute_), "record origin");
      origin_recorded_ = true;
    }
  }
  running_.store(true);
  thread_ = std::thread([this, n_local_events, max_steps, k0] { loop(n_local_events, max_steps, k0); });
}

bool ProducerEngine::join(double timeout_s) {
  if (!thread_.joinable()) return true;
  const auto t_end = std::chrono::steady_clock::now() + std::chrono::duration<double>(timeout_s);
  while (running_.load()) {
    if (timeout_s >= 0 && std::chrono::steady_clock::now() >= t_end) return false;
    std::this_thread::sleep_for(std::chrono::microseconds(200));
  }
  std::lock_guard<std::mutex> lk(halt_mu_);   // never two joins of one thread (halt() at exit)
  if (thread_.joinable()) thread_.join();
  return true;
}

std::vector<double> ProducerEngine::timing() const {
  std::lock_guard<std::mutex> lk(err_mu_);
  return {t_stage_, t_acquire_, t_launch_, t_commit_, t_total_};
}

// Fold the finished measurements of raw buffer b into the totals (block: wait for them).
void ProducerEngine::harvest(int b, bool block) {
  if (!gpu_timing_) return;
  auto take = [&](char& pending, hipEvent_t a, hipEvent_t z, double& tot, int64_t& n) {
    if (!pending) return;
    if (block) (void)hipEventSynchronize(z);
    else if (hipEventQuery(z) != hipSuccess) return;   // keep pending; try again next time
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, a, z) == hipSuccess) {
      std::lock_guard<std::mutex> lk(err_mu_);   // gpu_timing() reads these from another thread
      tot += ms;
      ++n;
    }
    (void)hipGetLastError();
    pending = 0;
  };
  take(h2d_pending_[b], h2d_start_[b], h2d_done_[b], gpu_h2d_ms_, gpu_h2d_n_);
  take(calib_pending_[b], calib_start_[b], buf_free_[b], gpu_calib_ms_, gpu_calib_n_);
}

std::vector<double> ProducerEngine::gpu_timing() const {
  std::lock_guard<std::mutex> lk(err_mu_);
  return {gpu_h2d_ms_, (double)gpu_h2d_n_, gpu_calib_ms_, (double)gpu_calib_n_};
}

// Move completed chunks from the pending queue into the log (done_mu_ held).  Polling stops at the
// first chunk still running; with several compute streams a later chunk can finish first, so an
// entry's time is when ALL frames up to it had completed (the max over the prefix).
void ProducerEngine::note_chunk_done_locked() const {
  while (!done_pending_.empty()) {
    hipEvent_t e = done_pending_.front().first;
    const hipError_t q = hipEventQuery(e);
    if (q == hipErrorNotReady) return;
    hip_check(q, "hipEventQuery (chunk done)");
    float ms = 0.f;
    hip_check(hipEventElapsedTime(&ms, origin_, e), "hipEventElapsedTime (chunk done)");
    done_frames_ = done_pending_.front().second;
    done_ms_ = std::max(done_ms_, (double)ms);
    done_log_.emplace_back(done_frames_, done_ms_);
    done_pending_.pop_front();
    done_free_.push_back(e);
  }
  if (done_log_.size() > (size_t(1) << 17)) {   // bounded: keep the newest 64k chunks
    const size_t drop = done_log_.size() - (size_t(1) << 16);
    done_log_.erase(done_log_.begin(), done_log_.begin() + (ptrdiff_t)drop);
    done_base_ += (int64_t)drop;
  }
}

void ProducerEngine::record_chunk_done(int n, hipStream_t s) {
  std::lock_guard<std::mutex> lk(done_mu_);
  note_chunk_done_locked();
  hipEvent_t e;
  if (!done_free_.empty()) {
    e = done_free_.back();
    done_free_.pop_back();
  } else {
    hip_check(hipEventCreate(&e), "hipEventCreate (chunk done)");
    done_all_.push_back(e);
  }
  hip_check(hipEventRecord(e, s), "record chunk done");
  enq_frames_ += n;
  done_pending_.emplace_back(e, enq_frames_);
}

int64_t ProducerEngine::completed() const {
  std::lock_guard<std::mutex> lk(done_mu_);
  DeviceGuard dg(device_);
  note_chunk_done_locked();
  return done_frames_;
}

std::vector<std::pair<int64_t, double>> ProducerEngine::completions(int64_t since, int64_t* first_index) const {
  std::lock_guard<std::mutex> lk(done_mu_);
  DeviceGuard dg(device_);
  note_chunk_done_locked();
  const int64_t a = std::max(since, done_base_);
  if (first_index != nullptr) *first_index = a;
  std::vector<std::pair<int64_t, double>> out;
  for (int64_t i = a; i < done_base_ + (int64_t)done_log_.size(); ++i) out.push_back(done_log_[(size_t)(i - done_base_)]);
  return out;
}

double ProducerEngine::mark(uint64_t stream) const {
  hipEvent_t e;
  {
    std::lock_guard<std::mutex> lk(done_mu_);
    check(origin_recorded_, "ProducerEngine.mark: the engine has not started");
  }
  DeviceGuard dg(device_);
  hip_check(hipEventCreate(&e), "hipEventCreate (mark)");
  float ms = 0.f;
  hipError_t err = hipEventRecord(e, reinterpret_cast<hipStream_t>(stream));
  if (err == hipSuccess) err = hipEventSynchronize(e);
  if (err == hipSuccess) err = hipEventElapsedTime(&ms, origin_, e);
  (void)hipEventDestroy(e);
  hip_check(err, "ProducerEngine.mark");
  return (double)ms;
}

std::string ProducerEngine::error() const {
  std::lock_guard<std::mutex> lk(err_mu_);
  return error_;
}

void ProducerEngine::loop(int64_t n_local_events, int64_t max_steps, int64_t k0) {
  using clk = std::chrono::steady_clock;
  auto secs = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double>(b - a).count(); };
  const auto t_begin = clk::now();
  try {
    hip_check(hipSetDevice(device_), "hipSetDevice");
    // absolute rank-local event bound: [k0, limit)
    int64_t limit = n_local_events;
    if (max_steps >= 0 && (limit < 0 || k0 + max_steps < limit)) limit = k0 + max_steps;
    const int n_cs = (int)cstreams_.size();
    std::vector<char> used(n_raw_bufs_, 0);
    std::vector<uint64_t> in, out;
    std::vector<int> slots;
    std::vector<SlotHeader> hdrs;
    const size_t nsrc = src_frames_.size();
    // host-side software pipeline: the copy of chunk c+1 is queued on the side stream BEFORE
    // chunk c waits for slots / launches, so the copy engine never runs dry behind host work
    const int64_t fb = plan_.raw_frame_bytes;
    // host->HBM staging copies by our own kernel with copy_workgroups_ workgroups (default 32;
    // 0 = hipMemcpyAsync, i.e. the runtime's blit / SDMA copies).  Measured in the pipeline:
    // 12.98-12.99k fr/s with 32 workgroups vs 12.53-12.77k with blit copies on the same box
    // (profiles/bench_r1/copy_kernel/)
    const int copy_kernel_wgs = copy_workgroups_;
    auto stage = [&](int64_t k0, int n, int b) {
      char* buf = static_cast<char*>(raw_bufs_) + (size_t)b * region_bytes_;
      std::vector<uint64_t>& dev = dev_in_[b];
      if (file_ != nullptr) {
        // staging region b is rewritten only after its previous H2D copy finished (host wait; with
        // n_raw_bufs regions it is n_raw_bufs chunks old by now)
        char* stg = static_cast<char*>(file_staging_) + (size_t)b * chunk_ * plan_.raw_frame_bytes;
        if (used[b]) hip_check(hipEventSynchronize(h2d_done_[b]), "wait staging free");
        std::vector<int64_t> ev(n);
        std::vector<uint64_t> dst(n);
        for (int i = 0; i < n; ++i) {
          ev[i] = rank_ + (k0 + i) * size_;
          dst[i] = reinterpret_cast<uint64_t>(stg) + (uint64_t)i * plan_.raw_frame_bytes;
        }
        {
          trace::Range r("producer.file_read");
          buf_meta_[b] = file_->read(ev, dst);   // native pread thread pool
        }
        if (used[b]) hip_check(hipStreamWaitEvent(h2d_, buf_free_[b], 0), "wait buf free");
        used[b] = 1;
        if (gpu_timing_) {
          harvest(b, false);
          hip_check(hipEventRecord(h2d_start_[b], h2d_), "record h2d start");
          h2d_pending_[b] = 1;
        }
        if (copy_kernel_wgs > 0 && launch_copy_h2d(reinterpret_cast<uint64_t>(buf), reinterpret_cast<uint64_t>(stg),
                                                   (int64_t)n * plan_.raw_frame_bytes, copy_kernel_wgs,
                                                   reinterpret_cast<uint64_t>(h2d_)))
          kernel_copies_.fetch_add(1, std::memory_order_relaxed);
        else
          hip_check(hipMemcpyAsync(buf, stg, (size_t)n * plan_.raw_frame_bytes, hipMemcpyHostToDevice, h2d_),
                    "stage copy");
        hip_check(hipEventRecord(h2d_done_[b], h2d_), "record h2d");
        for (int q = 0; q < n; ++q) dev[q] = reinterpret_cast<uint64_t>(buf) + (uint64_t)q * fb;
        return;
      }
      if (used[b]) hip_check(hipStreamWaitEvent(h2d_, buf_free_[b], 0), "wait buf free");
      used[b] = 1;
      if (gpu_timing_) {
        harvest(b, false);
        hip_check(hipEventRecord(h2d_start_[b], h2d_), "record h2d start");
        h2d_pending_[b] = 1;
      }
      // coalesce runs of frames spaced by one constant stride d (fb <= d <= fb + slack, d a
      // multiple of 16 so every frame lands 16-B aligned) into ONE copy of the whole span: a
      // pinned pool (d == fb) or the records of a registered run file (d = record size)
      int i = 0;
      int64_t pos = 0;
      while (i < n) {
        const uint64_t s0 = src_frames_[(k0 + i) % nsrc];
        int j = i + 1;
        int64_t d = 0;
        if (j < n) {
          d = (int64_t)(src_frames_[(k0 + j) % nsrc] - s0);
          if (d < fb || d > fb + kCopySlack || d % 16 != 0) d = 0;
        }
        if (d > 0)
          while (j < n && src_frames_[(k0 + j) % nsrc] == s0 + (uint64_t)((j - i) * d)) ++j;
        else
          j = i + 1;
        const int64_t span = (int64_t)(j - i - 1) * d + fb;
        pos = (pos + 255) & ~int64_t(255);
        check(pos + span <= region_bytes_, "ProducerEngine: staging region overflow");
        if (copy_kernel_wgs > 0 && !device_resident_ &&
            launch_copy_h2d(reinterpret_cast<uint64_t>(buf + pos), s0, span, copy_kernel_wgs,
                            reinterpret_cast<uint64_t>(h2d_)))
          kernel_copies_.fetch_add(1, std::memory_order_relaxed);
        else
          hip_check(hipMemcpyAsync(buf + pos, reinterpret_cast<const void*>(s0), (size_t)span, hipMemcpyDefault, h2d_),
                    "stage copy");
        for (int q = i; q < j; ++q) dev[q] = reinterpret_cast<uint64_t>(buf) + (uint64_t)(pos + (q - i) * d);
        (j - i > 1 ? span_copies_ : frame_copies_).fetch_add(1, std::memory_order_relaxed);
        pos += span;
        i = j;
      }
      hip_check(hipEventRecord(h2d_done_[b], h2d_), "record h2d");
    };
    auto chunk_len = [&](int64_t k0) -> int {
      int n = chunk_;
      if (limit >= 0) n = (int)std::max<int64_t>(0, std::min<int64_t>(n, limit - k0));
      return n;
    };
    // Prefetch depth: H2D copies of this many chunks stay queued on the copy stream ahead of the
    // chunk being calibrated, so a host hiccup (slot wait, descheduling) of up to depth x 2.5 ms
    // does not idle the PCIe link.  depth < n_raw_bufs: a buffer is re-staged only after the
    // calibration that read it was launched (its buf_free event recorded; the copy stream waits on
    // it device-side), and its pointers / file metadata were consumed.
    const int depth = std::min(3, n_raw_bufs_ - 1);
    int64_t st_k = k0;   // first event not staged yet
    int64_t st_no = 0;   // chunks staged so far
    auto stage_upto = [&](int64_t last_no) {   // stage chunks st_no .. last_no
      while (st_no <= last_no) {
        const int ns = chunk_len(st_k);
        if (ns <= 0) break;
        stage(st_k, ns, (int)(st_no % n_raw_bufs_));
        st_k += ns;
        ++st_no;
      }
    };
    int64_t k = k0;      // first event of the current chunk
    int64_t chunk_no = 0;
    int n = chunk_len(k0);
    if (n > 0 && !device_resident_) {
      const auto t0 = clk::now();
      stage_upto(0);
      t_stage_ += secs(t0, clk::now());
    }
    while (n > 0 && !stop_.load()) {
      const int b = (int)(chunk_no % n_raw_bufs_);
      hipStream_t cs = cstreams_[(size_t)(chunk_no % n_cs)];
      const uint64_t stream_c = reinterpret_cast<uint64_t>(cs);
      const int64_t k_next = k + n;
      const int n_next = chunk_len(k_next);
      trace::Range chunk_range("producer.chunk");
      auto t0 = clk::now();
      if (n_next > 0 && !device_resident_) {
        trace::Range r("producer.stage_h2d");
        stage_upto(chunk_no + depth);
      }
      auto t1 = clk::now();
      t_stage_ += secs(t0, t1);
      // direct headroom: frames in LOCAL slots stay within budget - headroom, the producer budget the
      // queue_size accounting gives (the headroom slots only carry direct frames' headers: their data
      // sits in the consumer's ring).  While the fabric offers grants the engine takes them first,
      // and a chunk whose local share would pass the cap waits for grants to cover it or for the
      // local backlog to drain, whichever comes first (headroom_wait_s_ > 0: at most that long, then
      // the chunk may use headroom slots for local frames).
      std::vector<QueueFabric::DirectGrant> dg;
      if (fabric_ != nullptr && headroom_ > 0) {
        trace::Range r("producer.direct_wait");
        const auto tw = clk::now();
        const int64_t cap = (int64_t)pool_->producer_budget() - headroom_;
        for (;;) {
          const bool offering = fabric_->direct_offering();
          if (offering) {
            const auto more = fabric_->take_direct(n - (int)dg.size());
            dg.insert(dg.end(), more.begin(), more.end());
          }
          const int64_t local =
              (int64_t)(pool_->producer_budget() - pool_->producer_room()) - fabric_->direct_inflight();
          if ((int)dg.size() >= n || local + (n - (int64_t)dg.size()) <= cap) break;
          if (stop_.load() || pool_->closed()) break;
          if (headroom_wait_s_ > 0 && offering && secs(tw, clk::now()) > headroom_wait_s_) break;
          std::this_thread::sleep_for(std::chrono::microseconds(20));
        }
        direct_wait_s_.store(direct_wait_s_.load() + secs(tw, clk::now()));
      }
      slots.clear();
      trace::push("producer.acquire");
      while (slots.empty() && !stop_.load()) {   // all n slots at once, one event wait per batch
        slots = pool_->acquire_batch(n, 0.05, stream_c);
        if (slots.empty()) {
          if (pool_->closed()) break;
          full_waits_.fetch_add(1);
        }
      }
      trace::pop();
      auto t2 = clk::now();
      t_acquire_ += secs(t1, t2);
      if ((int)slots.size() < n) {   // stopped while waiting
        if (!dg.empty()) {
          std::vector<int64_t> tk;
          for (const auto& g : dg) tk.push_back(g.token);
          fabric_->cancel_direct(tk);
        }
        break;
      }
      in.resize(n);
      out.resize(n);
      if (device_resident_) {   // calibrate straight from the resident source frames
        for (int q = 0; q < n; ++q) in[q] = src_frames_[(size_t)((k + q) % (int64_t)nsrc)];
      } else {
        hip_check(hipStreamWaitEvent(cs, h2d_done_[b], 0), "wait h2d");
        for (int q = 0; q < n; ++q) in[q] = dev_in_[b][q];
      }
      for (int q = 0; q < n; ++q) out[q] = pool_->slot_ptr(slots[q]);
      // frames with a direct grant are calibrated straight into that consumer's slot (the local slot
      // only carries the header and the queue_size accounting; QueueFabric::take_direct)
      if (fabric_ != nullptr && headroom_ == 0) dg = fabric_->take_direct(n);   // opportunistic: never waits
      for (size_t q = 0; q < dg.size(); ++q) out[q] = dg[q].ptr;
      if (gpu_timing_) {
        if (device_resident_) harvest(b, false);
        hip_check(hipEventRecord(calib_start_[b], cs), "record calib start");
        calib_pending_[b] = 1;
      }
      {
        trace::Range r("producer.launch_calib");
        if (dg.empty()) {
          run_calib_plan(plan_, in, out, stream_c);
        } else {
          std::vector<uint8_t> plain(n, 0);
          for (size_t q = 0; q < dg.size(); ++q) plain[q] = 1;
          run_calib_plan(plan_, in, out, stream_c, &plain);
        }
      }
      if (!device_resident_ || gpu_timing_) hip_check(hipEventRecord(buf_free_[b], cs), "record buf free");
      auto t3 = clk::now();
      t_launch_ += secs(t2, t3);
      hdrs.resize(n);
      for (int q = 0; q < n; ++q) {
        hdrs[q].rank = hdr_rank_;
        hdrs[q].idx = k + q;
        if (file_ != nullptr) {
          hdrs[q].gevt = buf_meta_[b][q].first;
          hdrs[q].photon_energy = buf_meta_[b][q].second;
        } else {
          hdrs[q].gevt = rank_ + (k + q) * size_;
          hdrs[q].photon_energy = src_pe_[(k + q) % src_pe_.size()];
        }
      }
      if (!dg.empty()) {   // bound BEFORE the commit: the fabric must never route these as copies
        std::vector<int> ds(slots.begin(), slots.begin() + (int64_t)dg.size());
        std::vector<int64_t> tk(dg.size());
        for (size_t q = 0; q < dg.size(); ++q) tk[q] = dg[q].token;
        fabric_->bind_direct(ds, tk);
        direct_frames_.fetch_add((int64_t)dg.size());
      }
      pool_->commit_batch(slots, hdrs, stream_c);   // one ready event for the whole chunk
      record_chunk_done(n, cs);
      t_commit_ += secs(t3, clk::now());
      frames_.fetch_add(n);
      k = k_next;
      n = n_next;
      ++chunk_no;
    }
    for (auto c : cstreams_) hip_check(hipStreamSynchronize(c), "final sync");
    hip_check(hipStreamSynchronize(h2d_), "final sync");
    {
      std::lock_guard<std::mutex> lk(done_mu_);
      note_chunk_done_locked();
    }
    for (int b = 0; b < n_raw_bufs_; ++b) harvest(b, true);
  } catch (const std::exception& e) {
    std::lock_guard<std::mutex> lk(err_mu_);
    error_ = e.what();
  }
  {
    std::lock_guard<std::mutex> lk(err_mu_);
    t_total_ = secs(t_begin, clk::now());
  }
  running_.store(false);
}

}  // namespace pr
