// pybind11 bindings of psana_ray_amd._C.  Device buffers and streams cross the boundary as
// integers (tensor.data_ptr(), torch.cuda.current_stream().cuda_stream), so this module does
// not depend on the torch C++ ABI; the Python layer validates shapes/dtypes/devices first.
#include <execinfo.h>
#include <signal.h>
#include <stdlib.h>
#include <unistd.h>

#include <algorithm>
#include <memory>

#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "common.h"
#include "runtime.h"

namespace py = pybind11;

#include "engine.h"
#include "fabric.h"
#include "lifecycle.h"
#include "kernels.h"
#include "streams.h"
#include "trace.h"
#include "verify.h"
#include "xtc2.h"


using pr::FramePtrs;

// Minimal DLPack (v0.8 ABI, unversioned "dltensor" capsule) so HBM ring segments we allocate with
// hipMalloc become torch tensors (torch.from_dlpack) without any torch C++ dependency.
namespace dl {
struct Device {
  int32_t device_type;  // kDLROCM = 10, kDLCPU = 1
  int32_t device_id;
};
struct DataType {
  uint8_t code;  // kDLUInt = 1
  uint8_t bits;
  uint16_t lanes;
};
struct Tensor {
  void* data;
  Device device;
  int32_t ndim;
  DataType dtype;
  int64_t* shape;
  int64_t* strides;
  uint64_t byte_offset;
};
struct Managed {
  Tensor dl_tensor;
  void* manager_ctx;
  void (*deleter)(Managed* self);
};
struct Ctx {
  std::shared_ptr<pr::DeviceBuffer> buf;
  int64_t shape[1];
};
}  // namespace dl

static py::capsule device_buffer_dlpack(std::shared_ptr<pr::DeviceBuffer> buf) {
  auto* ctx = new dl::Ctx{buf, {buf->bytes()}};
  auto* m = new dl::Managed{};
  m->dl_tensor.data = reinterpret_cast<void*>(buf->ptr());
  m->dl_tensor.device = dl::Device{10, buf->device()};
  m->dl_tensor.ndim = 1;
  m->dl_tensor.dtype = dl::DataType{1, 8, 1};
  m->dl_tensor.shape = ctx->shape;
  m->dl_tensor.strides = nullptr;
  m->dl_tensor.byte_offset = 0;
  m->manager_ctx = ctx;
  m->deleter = [](dl::Managed* self) {
    delete static_cast<dl::Ctx*>(self->manager_ctx);
    delete self;
  };
  // a capsule never consumed (renamed "used_dltensor") frees the tensor itself
  return py::capsule(m, "dltensor", [](PyObject* cap) {
    if (PyCapsule_IsValid(cap, "dltensor")) {
      auto* mm = static_cast<dl::Managed*>(PyCapsule_GetPointer(cap, "dltensor"));
      if (mm != nullptr && mm->deleter != nullptr) mm->deleter(mm);
    }
  });
}

static FramePtrs make_ptrs(const std::vector<uint64_t>& in, const std::vector<uint64_t>& out) {
  pr::check(in.size() == out.size(), "input/output pointer lists differ in length");
  pr::check(!in.empty() && (int)in.size() <= pr::kMaxFrames, "1..32 frames per launch");
  FramePtrs fp{};
  for (size_t i = 0; i < in.size(); ++i) {
    pr::check(in[i] != 0 && out[i] != 0, "null frame pointer");
    fp.in[i] = in[i];
    fp.out[i] = out[i];
  }
  return fp;
}

// Diagnostic (PSANA_RAY_AMD_SEGV_TRACE=1): a SIGSEGV prints the native stack first, then the
// handler that was installed before (Python's faulthandler, or the default) runs on the re-fault.
static struct sigaction g_prev_segv;
static void segv_trace_handler(int sig, siginfo_t* info, void* uctx) {
  (void)info;
  (void)uctx;
  void* frames[64];
  const int n = backtrace(frames, 64);
  const char hdr[] = "\n[psana_ray_amd] native stack at SIGSEGV:\n";
  (void)!write(2, hdr, sizeof(hdr) - 1);
  backtrace_symbols_fd(frames, n, 2);
  sigaction(sig, &g_prev_segv, nullptr);   // the faulting instruction re-runs into the old handler
}
static void maybe_install_segv_trace() {
  const char* e = getenv("PSANA_RAY_AMD_SEGV_TRACE");
  if (e == nullptr || e[0] != '1') return;
  // already ours (installed at import, called again at shutdown): keep the FIRST saved handler --
  // saving our own as "previous" would make a SIGSEGV re-enter this handler forever
  struct sigaction cur {};
  if (sigaction(SIGSEGV, nullptr, &cur) == 0 && (cur.sa_flags & SA_SIGINFO) && cur.sa_sigaction == segv_trace_handler)
    return;
  struct sigaction sa {};
  sa.sa_sigaction = segv_trace_handler;
  sa.sa_flags = SA_SIGINFO;
  sigemptyset(&sa.sa_mask);
  sigaction(SIGSEGV, &sa, &g_prev_segv);
}

// Peer-access / link topology of every GPU this process sees (bench topology record):
// {"n", "can_access"[i][j], "link_type"[i][j], "hops"[i][j]} (diagonal: -1)
static py::dict device_topology() {
  int n = 0;
  py::dict d;
  if (hipGetDeviceCount(&n) != hipSuccess) {
    (void)hipGetLastError();
    n = 0;
  }
  py::list acc, typ, hop;
  for (int i = 0; i < n; ++i) {
    py::list ra, rt, rh;
    for (int j = 0; j < n; ++j) {
      int can = -1;
      uint32_t lt = 0, hc = 0;
      int t = -1, h = -1;
      if (i != j) {
        if (hipDeviceCanAccessPeer(&can, i, j) != hipSuccess) {
          (void)hipGetLastError();
          can = -1;
        }
        if (hipExtGetLinkTypeAndHopCount(i, j, &lt, &hc) == hipSuccess) {
          t = (int)lt;
          h = (int)hc;
        } else {
          (void)hipGetLastError();
        }
      }
      ra.append(can);
      rt.append(t);
      rh.append(h);
    }
    acc.append(ra);
    typ.append(rt);
    hop.append(rh);
  }
  d["n"] = n;
  d["can_access"] = acc;
  d["link_type"] = typ;
  d["hops"] = hop;
  return d;
}

PYBIND11_MODULE(_C, m) {
  maybe_install_segv_trace();
  m.def("device_topology", &device_topology,
        "peer access (hipDeviceCanAccessPeer) and link type / hop count (hipExtGetLinkTypeAndHopCount) "
        "between every pair of visible GPUs");
  m.def("install_segv_trace", &maybe_install_segv_trace);
  m.def("frame_checksum_host", [](uint64_t ptr, int64_t bytes) {
        return pr::frame_checksum_host(reinterpret_cast<const void*>(ptr), bytes);
      }, py::arg("ptr"), py::arg("bytes"), "content checksum of a host buffer (csrc/verify.h)");
  m.def("checksum_tag", [](uint64_t sum) { return pr::ck_tag(sum); }, py::arg("sum"));
  py::class_<pr::FrameVerifier, std::shared_ptr<pr::FrameVerifier>>(m, "FrameVerifier")
      .def(py::init<int, int64_t>(), py::arg("device"), py::arg("frame_bytes"))
      .def("checksum_async", &pr::FrameVerifier::checksum_async, py::arg("ptrs"), py::arg("stream"))
      .def("result", &pr::FrameVerifier::result, py::arg("index"))
      .def("verify", &pr::FrameVerifier::verify, py::arg("ptrs"), py::arg("expect"), py::arg("gevt"),
           py::arg("stream"))
      .def("acquire", &pr::FrameVerifier::acquire, py::arg("stream"))
      .def("counts", &pr::FrameVerifier::counts);
  m.doc() = "psana_ray_amd native extension: gfx950 HIP kernels + host runtime";
  m.attr("MAX_FRAMES_PER_LAUNCH") = pr::kMaxFrames;
  m.attr("KIND_EPIX10KA") = (int)pr::kEpix10ka;
  m.attr("KIND_JUNGFRAU") = (int)pr::kJungfrau;
  m.attr("KIND_PLAIN") = (int)pr::kPlain;

  m.def("calib_basic",
        [](const std::vector<uint64_t>& in, const std::vector<uint64_t>& out, uint64_t ped, uint64_t gf,
           int64_t npix, int kind, uint64_t stream) {
          pr::launch_calib_basic(make_ptrs(in, out), (int)in.size(), ped, gf, npix, kind, stream);
        },
        py::arg("raw_ptrs"), py::arg("out_ptrs"), py::arg("ped"), py::arg("gf"), py::arg("npix"),
        py::arg("kind"), py::arg("stream"));
  m.def("calib_image",
        [](const std::vector<uint64_t>& in, const std::vector<uint64_t>& out, uint64_t ped, uint64_t gf,
           int64_t npix, int kind, uint64_t idx, int64_t nout, uint64_t stream) {
          pr::launch_calib_image(make_ptrs(in, out), (int)in.size(), ped, gf, npix, kind, idx, nout, stream);
        },
        py::arg("raw_ptrs"), py::arg("out_ptrs"), py::arg("ped"), py::arg("gf"), py::arg("npix"),
        py::arg("kind"), py::arg("idx"), py::arg("nout"), py::arg("stream"));
  m.def("calib_cm",
        [](const std::vector<uint64_t>& in, const std::vector<uint64_t>& out, uint64_t ped, uint64_t gf,
           uint64_t elig, int kind, int n_panels, int panel_rows, int panel_cols, int asic_rows,
           int asic_cols, float thr, float maxcorr, int npix_min, int flags, int bank_cols, uint64_t stream,
           uint64_t ped_sg) {
          pr::launch_calib_cm(make_ptrs(in, out), (int)in.size(), ped, gf, elig, kind, n_panels, panel_rows,
                              panel_cols, asic_rows, asic_cols, thr, maxcorr, npix_min, flags, bank_cols, stream, 0, 0,
                              0, ped_sg);
        },
        py::arg("raw_ptrs"), py::arg("out_ptrs"), py::arg("ped"), py::arg("gf"), py::arg("elig"),
        py::arg("kind"), py::arg("n_panels"), py::arg("panel_rows"), py::arg("panel_cols"),
        py::arg("asic_rows"), py::arg("asic_cols"), py::arg("thr"), py::arg("maxcorr"), py::arg("npix_min"),
        py::arg("flags"), py::arg("bank_cols"), py::arg("stream"), py::arg("ped_sg") = 0);
  m.def("cm_lds_bytes", &pr::cm_lds_bytes, py::arg("asic_rows"), py::arg("asic_cols"), py::arg("kind"));
  m.def("cm_signed_shape", &pr::cm_signed_shape, py::arg("kind"), py::arg("asic_rows"), py::arg("asic_cols"),
        py::arg("bank_cols"));
  m.def("cm_tile_cols", &pr::cm_tile_cols, py::arg("asic_rows"), py::arg("asic_cols"), py::arg("bank_cols"),
        py::arg("max_cols") = 0, py::arg("kind") = 0);
  m.def("image_tile_shape", [] { return py::make_tuple(pr::image_tile_h(), pr::image_tile_w(), pr::image_tile_stage()); });
  m.def("image_tiles",
        [](const std::vector<uint64_t>& in, const std::vector<uint64_t>& out, bool calib, int kind, uint64_t ped,
           uint64_t gf, int64_t npix, int panel_rows, int panel_cols, uint64_t tiles, int n_tiles, int tiles_x,
           uint64_t codes, int img_h, int img_w, uint64_t stream) {
          pr::launch_image_tiles(make_ptrs(in, out), (int)in.size(), calib, kind, ped, gf, npix, panel_rows,
                                 panel_cols, tiles, n_tiles, tiles_x, codes, img_h, img_w, stream);
        },
        py::arg("in_ptrs"), py::arg("out_ptrs"), py::arg("calib"), py::arg("kind"), py::arg("ped"), py::arg("gf"),
        py::arg("npix"), py::arg("panel_rows"), py::arg("panel_cols"), py::arg("tiles"), py::arg("n_tiles"),
        py::arg("tiles_x"), py::arg("codes"), py::arg("img_h"), py::arg("img_w"), py::arg("stream"));
  m.def("roctx_enabled", &pr::trace::enabled);
  m.def("roctx_push", [](const std::string& n) { pr::trace::push(n.c_str()); });
  m.def("roctx_pop", &pr::trace::pop);
  m.def("roctx_mark", [](const std::string& n) { pr::trace::mark(n.c_str()); });
  m.def("gather_frames",
        [](const std::vector<uint64_t>& in, const std::vector<uint64_t>& out, int64_t nelem, bool bf16,
           uint64_t stream) { pr::launch_gather_frames(make_ptrs(in, out), (int)in.size(), nelem, bf16, stream); },
        py::arg("in_ptrs"), py::arg("out_ptrs"), py::arg("nelem"), py::arg("bf16"), py::arg("stream"));
  m.def("mask_frames",
        [](const std::vector<uint64_t>& frames, uint64_t zero, int64_t npix, uint64_t stream) {
          pr::launch_mask_frames(make_ptrs(frames, frames), (int)frames.size(), zero, npix, stream);
        },
        py::arg("frame_ptrs"), py::arg("zero_mask"), py::arg("npix"), py::arg("stream"),
        "in place: pixel i of every frame -> 0 where zero_mask[i] != 0 (u8), one launch for <= 64 frames");
  m.def("copy_runs",
        [](const std::vector<uint64_t>& src, const std::vector<uint64_t>& dst, const std::vector<int64_t>& bytes,
           int workgroups, uint64_t stream) {
          pr::check(src.size() == dst.size() && src.size() == bytes.size(), "copy_runs: list lengths differ");
          pr::check(!src.empty() && (int)src.size() <= pr::kMaxCopyRuns, "copy_runs: 1..64 runs per launch");
          pr::CopyRuns cr{};
          cr.n = (int32_t)src.size();
          for (size_t i = 0; i < src.size(); ++i) {
            pr::check(src[i] != 0 && dst[i] != 0 && bytes[i] > 0 && bytes[i] % 16 == 0,
                      "copy_runs: null pointer or a size that is not a positive multiple of 16 B");
            cr.src[i] = src[i];
            cr.dst[i] = dst[i];
            cr.n16[i] = bytes[i] / 16;
          }
          return pr::launch_copy_runs(cr, workgroups, stream);
        },
        py::arg("src_ptrs"), py::arg("dst_ptrs"), py::arg("bytes"), py::arg("workgroups"), py::arg("stream"),
        "the queue fabric's batched D2D copy kernel (copy_runs_kernel); returns the grid size");
  m.def("convert_u16_f32",
        [](const std::vector<uint64_t>& in, const std::vector<uint64_t>& out, int64_t npix, uint64_t stream) {
          pr::launch_convert_u16_f32(make_ptrs(in, out), (int)in.size(), npix, stream);
        },
        "bandwidth reference: u16 -> f32 streaming copy (same traffic as calib_basic)");
  m.def("read_f32",
        [](const std::vector<uint64_t>& in, int64_t npix, int k, bool nt, uint64_t sums, uint64_t stream) {
          pr::launch_read_f32(make_ptrs(in, in), (int)in.size(), npix, k, nt, sums, stream);
        },
        "bandwidth reference: read-only f32 frame sweep (what the peak finder's input read can reach)");
  m.def("xor_lane_selftest", &pr::launch_xor_selftest, py::arg("out"), py::arg("stream"));
  m.def("cm_set_stamp_buffer", &pr::cm_set_stamp_buffer, py::arg("ptr"));
  m.def("assemble",
        [](const std::vector<uint64_t>& in, const std::vector<uint64_t>& out, uint64_t idx, int64_t nout,
           uint64_t omask, uint64_t stream) {
          pr::launch_assemble(make_ptrs(in, out), (int)in.size(), idx, nout, omask, stream);
        },
        py::arg("in_ptrs"), py::arg("out_ptrs"), py::arg("idx"), py::arg("nout"), py::arg("omask"),
        py::arg("stream"));
  m.def("peakfind",
        [](const std::vector<uint64_t>& in, int n_panels, int rows, int cols, float thr_peak, float son_min,
           int radius, int max_peaks, uint64_t peaks, uint64_t counts, uint64_t summary, uint64_t stream,
           uint64_t total, uint64_t scratch) {
          pr::launch_peakfind(make_ptrs(in, in), (int)in.size(), n_panels, rows, cols, thr_peak, son_min,
                              radius, max_peaks, peaks, counts, summary, total, stream, scratch);
        },
        py::arg("in_ptrs"), py::arg("n_panels"), py::arg("rows"), py::arg("cols"), py::arg("thr_peak"),
        py::arg("son_min"), py::arg("radius"), py::arg("max_peaks"), py::arg("peaks"), py::arg("counts"),
        py::arg("summary"), py::arg("stream"), py::arg("total") = 0, py::arg("scratch") = 0);
  m.attr("PF_SCRATCH_BYTES") = pr::kPfScratchBytes;
  // consumer hot path: ring slots -> peak finder with self-resetting outputs, one native call
  m.def("peakfind_slots",
        [](const pr::SlotPool& pool, int64_t slot_bytes, const std::vector<int>& slots, int n_panels, int rows,
           int cols, float thr_peak, float son_min, int radius, int max_peaks, uint64_t peaks, uint64_t counts,
           uint64_t summary, uint64_t total, uint64_t stream, uint64_t scratch) {
          const int n = (int)slots.size();
          pr::check(n >= 1, "peakfind_slots: no slots");
          pr::check(slot_bytes >= (int64_t)n_panels * rows * cols * 4, "peakfind_slots: frame larger than a slot");
          pr::check(scratch != 0, "peakfind_slots: needs a zero-initialised scratch block (PF_SCRATCH_BYTES)");
          for (int a = 0; a < n; a += pr::kMaxFrames) {
            const int m = std::min(pr::kMaxFrames, n - a);
            std::vector<uint64_t> in(m);
            for (int i = 0; i < m; ++i) in[i] = pool.slot_ptr(slots[a + i]);
            pr::launch_peakfind(make_ptrs(in, in), m, n_panels, rows, cols, thr_peak, son_min, radius, max_peaks,
                                peaks + (uint64_t)a * max_peaks * 32, counts + (uint64_t)a * 4,
                                summary + (uint64_t)a * 8, total, stream, scratch);
          }
        },
        py::arg("pool"), py::arg("slot_bytes"), py::arg("slots"), py::arg("n_panels"), py::arg("rows"),
        py::arg("cols"), py::arg("thr_peak"), py::arg("son_min"), py::arg("radius"), py::arg("max_peaks"),
        py::arg("peaks"), py::arg("counts"), py::arg("summary"), py::arg("total"), py::arg("stream"),
        py::arg("scratch"), py::call_guard<py::gil_scoped_release>());

  m.def("copy_h2d_kernel",
        [](uint64_t dst, uint64_t src, int64_t bytes, int workgroups, uint64_t stream) {
          return pr::launch_copy_h2d(dst, src, bytes, workgroups, stream);
        },
        py::arg("dst"), py::arg("src"), py::arg("bytes"), py::arg("workgroups"), py::arg("stream") = 0,
        "host (pinned) -> HBM copy by copy_h2d_kernel; False = not applicable (unaligned / unmapped)");
  m.def("memcpy_h2d_async", &pr::memcpy_h2d_async, py::arg("dst"), py::arg("src"), py::arg("bytes"),
        py::arg("stream"));
  m.def("memcpy_h2d_batch", &pr::memcpy_h2d_batch, py::arg("dst"), py::arg("src"), py::arg("bytes"),
        py::arg("stream"));

  py::class_<pr::DeviceBuffer, std::shared_ptr<pr::DeviceBuffer>>(m, "DeviceBuffer")
      .def(py::init<int64_t, int>(), py::arg("bytes"), py::arg("device"))
      .def_property_readonly("ptr", &pr::DeviceBuffer::ptr)
      .def_property_readonly("nbytes", &pr::DeviceBuffer::bytes)
      .def_property_readonly("device", &pr::DeviceBuffer::device)
      .def("__dlpack__", [](std::shared_ptr<pr::DeviceBuffer> b, py::kwargs) { return device_buffer_dlpack(b); })
      .def("__dlpack_device__", [](const pr::DeviceBuffer& b) { return py::make_tuple(10, b.device()); });

  // ---- elastic queue fabric (fabric.h)
  m.def("pid_alive", &pr::pid_alive, py::arg("pid"));
  // stop and join every fabric / engine thread still running (registered with atexit by the loader)
  m.def("halt_native_threads", &pr::halt_native_threads, py::call_guard<py::gil_scoped_release>());
  // streams with a chosen hardware-queue placement (streams.h); torch wraps them as ExternalStream
  m.def("stream_create", [](int device, int kind) { return reinterpret_cast<uint64_t>(pr::acquire_stream(device, kind)); },
        py::arg("device"), py::arg("kind"));
  m.def("stream_release", [](int device, int kind, uint64_t s) {
        pr::release_stream(device, kind, reinterpret_cast<hipStream_t>(s)); },
        py::arg("device"), py::arg("kind"), py::arg("stream"), py::call_guard<py::gil_scoped_release>());
  m.def("close_stream_pool", &pr::close_stream_pool, py::call_guard<py::gil_scoped_release>());
  m.def("shm_remove", &pr::shm_remove, py::arg("name"));
  py::class_<pr::ShmRegion>(m, "ShmRegion", py::buffer_protocol())
      .def(py::init<const std::string&, int64_t, bool, double>(), py::arg("name"), py::arg("bytes"),
           py::arg("create"), py::arg("timeout_s") = 10.0, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("ptr", &pr::ShmRegion::ptr)
      .def_property_readonly("nbytes", &pr::ShmRegion::bytes)
      .def_property_readonly("name", &pr::ShmRegion::name)
      .def("unlink", &pr::ShmRegion::unlink)
      .def_buffer([](pr::ShmRegion& r) -> py::buffer_info {
        return py::buffer_info(reinterpret_cast<void*>(r.ptr()), 1, py::format_descriptor<uint8_t>::format(), 1,
                               {(py::ssize_t)r.bytes()}, {(py::ssize_t)1});
      });
  py::class_<pr::FabricStats>(m, "FabricStats")
      .def_readonly("iterations", &pr::FabricStats::iterations)
      .def_readonly("idle_iterations", &pr::FabricStats::idle_iterations)
      .def_readonly("frames_local", &pr::FabricStats::frames_local)
      .def_readonly("frames_sent", &pr::FabricStats::frames_sent)
      .def_readonly("frames_recv", &pr::FabricStats::frames_recv)
      .def_readonly("frames_requeued", &pr::FabricStats::frames_requeued)
      .def_readonly("grants_given", &pr::FabricStats::grants_given)
      .def_readonly("grants_returned", &pr::FabricStats::grants_returned)
      .def_readonly("grants_reclaimed", &pr::FabricStats::grants_reclaimed)
      .def_readonly("bytes_sent", &pr::FabricStats::bytes_sent)
      .def_readonly("bytes_recv", &pr::FabricStats::bytes_recv)
      .def_readonly("batches", &pr::FabricStats::batches)
      .def_readonly("links_opened", &pr::FabricStats::links_opened)
      .def_readonly("peers_dead", &pr::FabricStats::peers_dead)
      .def_readonly("links_failed", &pr::FabricStats::links_failed)
      .def_readonly("frames_returned", &pr::FabricStats::frames_returned)
      .def_readonly("frames_reclaimed", &pr::FabricStats::frames_reclaimed)
      .def_readonly("frames_dropped", &pr::FabricStats::frames_dropped)
      .def_readonly("returns_rejected", &pr::FabricStats::returns_rejected)
      .def_readonly("readahead", &pr::FabricStats::readahead)
      .def_readonly("copy_s", &pr::FabricStats::copy_s)
      .def_readonly("copy_launches", &pr::FabricStats::copy_launches)
      .def_readonly("copy_dev_ms", &pr::FabricStats::copy_dev_ms)
      .def_readonly("copy_dev_bytes", &pr::FabricStats::copy_dev_bytes)
      .def_readonly("taken_local", &pr::FabricStats::taken_local)
      .def_readonly("taken_remote", &pr::FabricStats::taken_remote)
      .def_readonly("frames_checksummed", &pr::FabricStats::frames_checksummed)
      .def_readonly("frames_direct", &pr::FabricStats::frames_direct)
      .def_readonly("frames_lost_direct", &pr::FabricStats::frames_lost_direct)
      .def_readonly("frames_corrupted", &pr::FabricStats::frames_corrupted);
  py::class_<pr::CopySample>(m, "CopySample")
      .def_readonly("dev_ms", &pr::CopySample::dev_ms)
      .def_readonly("issue_to_done_ms", &pr::CopySample::issue_to_done_ms)
      .def_readonly("bytes", &pr::CopySample::bytes)
      .def_readonly("frames", &pr::CopySample::frames)
      .def_readonly("links", &pr::CopySample::links);
  py::class_<pr::LinkStatus>(m, "LinkStatus")
      .def_readonly("peer", &pr::LinkStatus::peer)
      .def_readonly("outgoing", &pr::LinkStatus::outgoing)
      .def_readonly("attached", &pr::LinkStatus::attached)
      .def_readonly("eos", &pr::LinkStatus::eos)
      .def_readonly("detached", &pr::LinkStatus::detached)
      .def_readonly("dead", &pr::LinkStatus::dead)
      .def_readonly("closed", &pr::LinkStatus::closed)
      .def_readonly("keeper", &pr::LinkStatus::keeper)
      .def_readonly("taken", &pr::LinkStatus::taken)
      .def_readonly("outstanding", &pr::LinkStatus::outstanding)
      .def_readonly("frames", &pr::LinkStatus::frames)
      .def_readonly("consumer_device", &pr::LinkStatus::consumer_device)
      .def_readonly("kernel_copy", &pr::LinkStatus::kernel_copy)
      .def_readonly("peer_access", &pr::LinkStatus::peer_access)
      .def_readonly("link_type", &pr::LinkStatus::link_type)
      .def_readonly("hops", &pr::LinkStatus::hops);
  py::class_<pr::QueueFabric>(m, "QueueFabric")
      .def(py::init<pr::SlotPool*, int64_t, int, bool, bool, int, int64_t>(), py::arg("pool"),
           py::arg("slot_bytes"), py::arg("device"), py::arg("is_producer"), py::arg("is_consumer"),
           py::arg("policy"), py::arg("self_mid"), py::keep_alive<1, 2>())
      .def("export_host_ring", &pr::QueueFabric::export_host_ring, py::arg("shm_name"))
      .def("export_ipc_ring", &pr::QueueFabric::export_ipc_ring)
      .def_property_readonly("export_segments", &pr::QueueFabric::export_segments)
      .def("add_in_link", &pr::QueueFabric::add_in_link, py::arg("producer_mid"), py::arg("name"))
      .def("add_out_link", &pr::QueueFabric::add_out_link, py::arg("consumer_mid"), py::arg("name"))
      .def("drop_peer", &pr::QueueFabric::drop_peer, py::arg("mid"))
      .def("set_policy", &pr::QueueFabric::set_policy, py::arg("policy"))
      .def("set_producer_finished", &pr::QueueFabric::set_producer_finished)
      .def("set_consumer_closed", &pr::QueueFabric::set_consumer_closed)
      .def("start", &pr::QueueFabric::start)
      .def("request_stop", &pr::QueueFabric::request_stop)
      .def("join", &pr::QueueFabric::join, py::arg("timeout_s"), py::call_guard<py::gil_scoped_release>())
      .def("step", &pr::QueueFabric::step, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("running", &pr::QueueFabric::running)
      .def_property_readonly("producer_drained", &pr::QueueFabric::producer_drained)
      .def_property_readonly("consumer_quiesced", &pr::QueueFabric::consumer_quiesced)
      .def_property_readonly("policy", &pr::QueueFabric::policy)
      .def("error", &pr::QueueFabric::error)
      .def("last_link_error", &pr::QueueFabric::last_link_error)
      .def("set_grant_filter", &pr::QueueFabric::set_grant_filter, py::arg("on"))
      .def("set_prefetch", &pr::QueueFabric::set_prefetch, py::arg("n"))
      .def_property_readonly("prefetch", &pr::QueueFabric::prefetch)
      .def("set_keeper", &pr::QueueFabric::set_keeper, py::arg("on"))
      .def("set_peer_grantable", &pr::QueueFabric::set_peer_grantable, py::arg("mid"), py::arg("on"))
      .def("stats", &pr::QueueFabric::stats)
      .def("set_copy_engine", &pr::QueueFabric::set_copy_engine, py::arg("engine"), py::arg("workgroups") = 0,
           py::arg("stream_kind") = 1)
      .def_property_readonly("copy_engine", &pr::QueueFabric::copy_engine)
      .def_property_readonly("copy_workgroups", &pr::QueueFabric::copy_workgroups)
      .def("copy_samples", &pr::QueueFabric::copy_samples)
      .def("set_verify_every", &pr::QueueFabric::set_verify_every, py::arg("every"))
      .def("set_direct", &pr::QueueFabric::set_direct, py::arg("on"))
      .def("direct", &pr::QueueFabric::direct)
      .def("verify_every", &pr::QueueFabric::verify_every)
      .def("verify_counts", &pr::QueueFabric::verify_counts)
      .def_static("copy_grid_for", &pr::QueueFabric::copy_grid_for, py::arg("consumer_devices"), py::arg("device"),
                  py::arg("per_peer"))
      .def("links", &pr::QueueFabric::links);

  py::class_<pr::PinnedBuffer>(m, "PinnedBuffer", py::buffer_protocol())
      .def(py::init<size_t>(), py::arg("bytes"))
      .def_property_readonly("ptr", &pr::PinnedBuffer::ptr)
      .def_property_readonly("nbytes", &pr::PinnedBuffer::bytes)
      .def_buffer([](pr::PinnedBuffer& b) -> py::buffer_info {
        return py::buffer_info(b.raw(), 1, py::format_descriptor<uint8_t>::format(), 1, {(py::ssize_t)b.bytes()},
                               {(py::ssize_t)1});
      });

  py::class_<pr::SlotHeader>(m, "SlotHeader")
      .def(py::init<>())
      .def(py::init([](int64_t rank, int64_t idx, int64_t gevt, double pe, int64_t aux) {
             pr::SlotHeader h;
             h.rank = rank;
             h.idx = idx;
             h.gevt = gevt;
             h.photon_energy = pe;
             h.aux = aux;
             return h;
           }),
           py::arg("rank"), py::arg("idx"), py::arg("gevt"), py::arg("photon_energy"), py::arg("aux") = 0)
      .def_readwrite("rank", &pr::SlotHeader::rank)
      .def_readwrite("idx", &pr::SlotHeader::idx)
      .def_readwrite("gevt", &pr::SlotHeader::gevt)
      .def_readwrite("photon_energy", &pr::SlotHeader::photon_energy)
      .def_readwrite("aux", &pr::SlotHeader::aux);

  py::class_<pr::PoolStats>(m, "PoolStats")
      .def_readonly("produced", &pr::PoolStats::produced)
      .def_readonly("routed_local", &pr::PoolStats::routed_local)
      .def_readonly("sent", &pr::PoolStats::sent)
      .def_readonly("received", &pr::PoolStats::received)
      .def_readonly("got", &pr::PoolStats::got)
      .def_readonly("released", &pr::PoolStats::released)
      .def_readonly("produce_full", &pr::PoolStats::produce_full);

  using SP = pr::SlotPool;
  py::class_<SP>(m, "SlotPool")
      .def(py::init<int, int, int>(), py::arg("producer_budget"), py::arg("consumer_budget"), py::arg("device"))
      .def_property_readonly("n_slots", &SP::n_slots)
      .def("set_slot_ptrs", &SP::set_slot_ptrs, py::arg("ptrs"))
      .def("slot_ptr", &SP::slot_ptr, py::arg("slot"))
      .def_property_readonly("producer_budget", &SP::producer_budget)
      .def_property_readonly("consumer_budget", &SP::consumer_budget)
      .def("try_acquire_produce", &SP::try_acquire_produce)
      .def("acquire_produce", &SP::acquire_produce, py::arg("timeout_s"), py::call_guard<py::gil_scoped_release>())
      .def("commit_produce", &SP::commit_produce, py::arg("slot"), py::arg("header"), py::arg("stream"))
      .def("abort_produce", &SP::abort_produce)
      .def("produced", &SP::produced, py::arg("max_n"))
      .def("n_produced", &SP::n_produced)
      .def("producer_held", &SP::producer_held)
      .def("route_local", &SP::route_local)
      .def("begin_send", &SP::begin_send)
      .def("end_send", &SP::end_send, py::arg("slot"), py::arg("stream"))
      .def("credits", &SP::credits)
      .def("begin_recv", &SP::begin_recv)
      .def("end_recv", &SP::end_recv, py::arg("slot"), py::arg("header"), py::arg("stream"))
      .def("try_get", &SP::try_get)
      .def("get", &SP::get, py::arg("timeout_s"), py::call_guard<py::gil_scoped_release>())
      .def("release", &SP::release, py::arg("slot"), py::arg("stream"))
      .def("n_ready", &SP::n_ready)
      .def("consumer_held", &SP::consumer_held)
      .def("wait_ready_on", &SP::wait_ready_on, py::arg("slot"), py::arg("stream"))
      .def("check_frames", &SP::check_frames, py::arg("slots"), py::arg("stream"),
           py::call_guard<py::gil_scoped_release>())
      .def("wait_free_on", &SP::wait_free_on, py::arg("slot"), py::arg("stream"))
      .def("sync_ready", &SP::sync_ready, py::call_guard<py::gil_scoped_release>())
      .def("header", &SP::header)
      .def("state", &SP::state)
      .def("stats", &SP::stats)
      .def("wake_all", &SP::wake_all)
      .def("wake_producers", &SP::wake_producers)
      .def("closed", &SP::closed)
      .def("set_auto_route", &SP::set_auto_route)
      .def("get_batch", &SP::get_batch, py::arg("max_n"), py::arg("timeout_s"), py::arg("stream"),
           py::call_guard<py::gil_scoped_release>())
      .def("release_batch", &SP::release_batch, py::arg("slots"), py::arg("stream"))
      .def("headers", &SP::headers)
      .def("acquire_batch", &SP::acquire_batch, py::arg("n"), py::arg("timeout_s"), py::arg("stream"),
           py::call_guard<py::gil_scoped_release>())
      .def("commit_batch", &SP::commit_batch, py::arg("slots"), py::arg("headers"), py::arg("stream"))
      .def("begin_send_batch", &SP::begin_send_batch, py::arg("slots"), py::arg("stream"))
      .def("begin_recv_batch", &SP::begin_recv_batch, py::arg("n"), py::arg("stream"))
      .def("end_send_batch", &SP::end_send_batch, py::arg("slots"), py::arg("stream"))
      .def("end_recv_batch", &SP::end_recv_batch, py::arg("slots"), py::arg("headers"), py::arg("stream"))
      .def("grant_batch", &SP::grant_batch, py::arg("max_n"))
      .def("complete_recv_batch", &SP::complete_recv_batch, py::arg("slots"), py::arg("headers"))
      .def("cancel_recv_batch", &SP::cancel_recv_batch, py::arg("slots"))
      .def("reoffer_batch", &SP::reoffer_batch, py::arg("slots"), py::arg("stream"))
      .def("relay_ready", &SP::relay_ready, py::arg("max_n"))
      .def("set_external_held", &SP::set_external_held, py::arg("n"))
      .def("producer_room", &SP::producer_room)
      .def("set_track_origins", &SP::set_track_origins, py::arg("on"))
      .def("take_got_origins", &SP::take_got_origins)
      .def("origin", &SP::origin, py::arg("slot"))
      .def("pop_ready_for_return", &SP::pop_ready_for_return, py::arg("max_n"))
      .def("unsend_batch", &SP::unsend_batch, py::arg("slots"))
      .def_property_readonly("event_records", &SP::event_records);

  py::class_<pr::CalibPlan>(m, "CalibPlan")
      .def(py::init<>())
      .def_readwrite("mode", &pr::CalibPlan::mode)
      .def_readwrite("kind", &pr::CalibPlan::kind)
      .def_readwrite("npix", &pr::CalibPlan::npix)
      .def_readwrite("ped", &pr::CalibPlan::ped)
      .def_readwrite("gf", &pr::CalibPlan::gf)
      .def_readwrite("elig", &pr::CalibPlan::elig)
      .def_readwrite("ped_sg", &pr::CalibPlan::ped_sg)
      .def_readwrite("n_panels", &pr::CalibPlan::n_panels)
      .def_readwrite("panel_rows", &pr::CalibPlan::panel_rows)
      .def_readwrite("panel_cols", &pr::CalibPlan::panel_cols)
      .def_readwrite("asic_rows", &pr::CalibPlan::asic_rows)
      .def_readwrite("asic_cols", &pr::CalibPlan::asic_cols)
      .def_readwrite("thr", &pr::CalibPlan::thr)
      .def_readwrite("maxcorr", &pr::CalibPlan::maxcorr)
      .def_readwrite("npix_min", &pr::CalibPlan::npix_min)
      .def_readwrite("cm_flags", &pr::CalibPlan::cm_flags)
      .def_readwrite("bank_cols", &pr::CalibPlan::bank_cols)
      .def_readwrite("use_cm", &pr::CalibPlan::use_cm)
      .def_readwrite("idx", &pr::CalibPlan::idx)
      .def_readwrite("nout", &pr::CalibPlan::nout)
      .def_readwrite("omask", &pr::CalibPlan::omask)
      .def_readwrite("scratch", &pr::CalibPlan::scratch)
      .def_readwrite("raw_frame_bytes", &pr::CalibPlan::raw_frame_bytes)
      .def_readwrite("out_frame_bytes", &pr::CalibPlan::out_frame_bytes)
      .def_readwrite("use_tiles", &pr::CalibPlan::use_tiles)
      .def_readwrite("tiles", &pr::CalibPlan::tiles)
      .def_readwrite("codes", &pr::CalibPlan::codes)
      .def_readwrite("n_tiles", &pr::CalibPlan::n_tiles)
      .def_readwrite("tiles_x", &pr::CalibPlan::tiles_x)
      .def_readwrite("img_h", &pr::CalibPlan::img_h)
      .def_readwrite("img_w", &pr::CalibPlan::img_w)
      .def_readwrite("img_desc", &pr::CalibPlan::img_desc)
      .def_readwrite("gap_runs", &pr::CalibPlan::gap_runs)
      .def_readwrite("n_gap_runs", &pr::CalibPlan::n_gap_runs);
  m.def("run_calib_plan",
        [](const pr::CalibPlan& plan, const std::vector<uint64_t>& in, const std::vector<uint64_t>& out,
           uint64_t stream, const std::vector<uint8_t>& plain) {
          pr::run_calib_plan(plan, in, out, stream, plain.empty() ? nullptr : &plain);
        },
        py::arg("plan"), py::arg("in_ptrs"), py::arg("out_ptrs"), py::arg("stream"),
        py::arg("plain") = std::vector<uint8_t>{});

  py::class_<pr::ProducerEngine>(m, "ProducerEngine")
      .def(py::init<pr::SlotPool*, int64_t, int, const pr::CalibPlan&, int, int, int64_t, int64_t, int, bool>(),
           py::arg("pool"), py::arg("slot_bytes"), py::arg("device"), py::arg("plan"),
           py::arg("chunk"), py::arg("n_raw_bufs"), py::arg("rank"), py::arg("size"),
           py::arg("copy_workgroups") = 32, py::arg("gpu_timing") = false, py::keep_alive<1, 2>())
      .def("set_cycled_source", &pr::ProducerEngine::set_cycled_source, py::arg("frames"), py::arg("photon_energy"))
      .def("start", &pr::ProducerEngine::start, py::arg("n_local_events"), py::arg("max_steps"), py::arg("k0") = 0)
      .def("set_file_source", &pr::ProducerEngine::set_file_source, py::arg("reader"), py::keep_alive<1, 2>())
      .def("set_header_rank", &pr::ProducerEngine::set_header_rank, py::arg("rank"))
      .def("set_fabric", &pr::ProducerEngine::set_fabric, py::arg("fabric").none(true))
      .def_property_readonly("direct_frames", &pr::ProducerEngine::direct_frames)
      .def("set_direct_headroom", &pr::ProducerEngine::set_direct_headroom, py::arg("slots"), py::arg("wait_s") = 0.002)
      .def_property_readonly("direct_wait_s", &pr::ProducerEngine::direct_wait_s)
      .def_property_readonly("direct_headroom", &pr::ProducerEngine::direct_headroom)
      .def("set_compute_streams", &pr::ProducerEngine::set_compute_streams, py::arg("n"), py::arg("kind") = 0)
      .def_property_readonly("compute_streams", &pr::ProducerEngine::compute_streams)
      .def("request_stop", &pr::ProducerEngine::request_stop)
      .def_property_readonly("device_resident", &pr::ProducerEngine::device_resident)
      .def("join", &pr::ProducerEngine::join, py::arg("timeout_s"), py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("running", &pr::ProducerEngine::running)
      .def_property_readonly("frames", &pr::ProducerEngine::frames)
      .def_property_readonly("completed", &pr::ProducerEngine::completed)
      .def(
          "completions",
          [](const pr::ProducerEngine& e, int64_t since) {
            int64_t first = 0;
            auto v = e.completions(since, &first);
            return py::make_tuple(first, v);
          },
          py::arg("since") = 0)
      .def("mark", &pr::ProducerEngine::mark, py::arg("stream"), py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("full_waits", &pr::ProducerEngine::full_waits)
      .def("error", &pr::ProducerEngine::error)
      .def("timing", &pr::ProducerEngine::timing)
      .def("gpu_timing", &pr::ProducerEngine::gpu_timing)
      .def("copy_stats", &pr::ProducerEngine::copy_stats)
      .def_property_readonly("gpu_timing_enabled", &pr::ProducerEngine::gpu_timing_enabled);

  py::class_<pr::MappedFile>(m, "MappedFile")
      .def(py::init<const std::string&, bool>(), py::arg("path"), py::arg("register_with_hip") = true,
           py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("ptr", &pr::MappedFile::ptr)
      .def_property_readonly("nbytes", &pr::MappedFile::bytes)
      .def_property_readonly("registered", &pr::MappedFile::registered)
      .def_property_readonly("register_s", &pr::MappedFile::register_s);

  py::class_<pr::Xtc2Index>(m, "Xtc2Index")
      .def_readonly("det_type", &pr::Xtc2Index::det_type)
      .def_readonly("shape", &pr::Xtc2Index::shape)
      .def_readonly("dtype", &pr::Xtc2Index::dtype)
      .def_readonly("frame_bytes", &pr::Xtc2Index::frame_bytes)
      .def_readonly("payload_off", &pr::Xtc2Index::payload_off)
      .def_readonly("gevt", &pr::Xtc2Index::gevt)
      .def_readonly("timestamp", &pr::Xtc2Index::timestamp)
      .def_readonly("photon_energy", &pr::Xtc2Index::photon_energy)
      .def_readonly("transitions", &pr::Xtc2Index::transitions)
      .def_readonly("walked", &pr::Xtc2Index::walked);
  m.def("xtc2_scan", &pr::xtc2_scan, py::arg("smd_path"), py::arg("big_path"), py::arg("det_name"),
        py::arg("array_name") = "raw", py::call_guard<py::gil_scoped_release>());

  py::class_<pr::RawRunReader>(m, "RawRunReader")
      .def(py::init<const std::string&, int>(), py::arg("path"), py::arg("n_threads") = 4)
      .def(py::init<const std::string&, int, std::vector<int64_t>, std::vector<int64_t>, std::vector<double>,
                    int64_t>(),
           py::arg("path"), py::arg("n_threads"), py::arg("payload_off"), py::arg("gevt"), py::arg("photon_energy"),
           py::arg("frame_bytes"))
      .def_property_readonly("indexed", &pr::RawRunReader::indexed)
      .def_property_readonly("n_events", &pr::RawRunReader::n_events)
      .def_property_readonly("frame_bytes", &pr::RawRunReader::frame_bytes)
      .def_property_readonly("record_bytes", &pr::RawRunReader::record_bytes)
      .def_property_readonly("header_bytes", &pr::RawRunReader::header_bytes)
      .def("read", &pr::RawRunReader::read, py::arg("events"), py::arg("dst_ptrs"),
           py::call_guard<py::gil_scoped_release>());
}
