// Host launchers of the gfx950 kernels (definitions in the .hip files).
#pragma once

#include <stddef.h>
#include <stdint.h>

#include "common.h"

namespace pr {
void launch_calib_basic(const FramePtrs& fp, int nframes, uint64_t ped, uint64_t gf, int64_t npix, int kind,
                        uint64_t stream);
void launch_calib_image(const FramePtrs& fp, int nframes, uint64_t ped, uint64_t gf, int64_t npix, int kind,
                        uint64_t idx, int64_t nout, uint64_t stream);
void launch_calib_cm(const FramePtrs& fp, int nframes, uint64_t ped, uint64_t gf, uint64_t elig, int kind,
                     int n_panels, int panel_rows, int panel_cols, int asic_rows, int asic_cols, float thr,
                     float maxcorr, int npix_min, int flags, int bank_cols, uint64_t stream,
                     uint64_t img_desc = 0, uint64_t gap_runs = 0,
                     int n_gap_runs = 0,    // img_desc: fused K-05 (ImgOut); gap runs zeroed by the same kernel
                     uint64_t ped_sg = 0,   // signed pedestal tables (eligibility in the sign bits), 0 = planes
                     uint64_t plain_mask = 0);  // bit f: plain (not streaming) stores for frame f
size_t cm_lds_bytes(int asic_rows, int asic_cols, int kind);
bool cm_signed_shape(int kind, int asic_rows, int asic_cols, int bank_cols);   // reads signed pedestal tables
void launch_image_tiles(const FramePtrs& fp, int nframes, bool calib, int kind, uint64_t ped, uint64_t gf,
                        int64_t npix, int panel_rows, int panel_cols, uint64_t tiles, int n_tiles, int tiles_x,
                        uint64_t codes, int img_h, int img_w, uint64_t stream);
int image_tile_h();
int image_tile_w();
int image_tile_stage();
int cm_tile_cols(int asic_rows, int asic_cols, int bank_cols, int max_cols, int kind);
void launch_convert_u16_f32(const FramePtrs& fp, int nframes, int64_t npix, uint64_t stream);
void launch_read_f32(const FramePtrs& fp, int nframes, int64_t npix, int k, bool nt, uint64_t sums, uint64_t stream);
void launch_xor_selftest(uint64_t out, uint64_t stream);
// diagnostic builds only (-DPR_CM_STAMPS=1): per-wave phase stamps of the epix10k2M CM kernel
void cm_set_stamp_buffer(uint64_t p);
void launch_fill_runs(const FramePtrs& fp, int nframes, uint64_t runs, int n_runs, uint64_t stream);
void launch_mask_frames(const FramePtrs& fp, int nframes, uint64_t zero, int64_t npix, uint64_t stream);
void launch_gather_frames(const FramePtrs& fp, int nframes, int64_t nelem, bool bf16, uint64_t stream);
// host (pinned / registered) -> HBM copy by a kernel; false = not applicable, use hipMemcpyAsync
bool launch_copy_h2d(uint64_t dst, uint64_t host_src, int64_t bytes, int workgroups, uint64_t stream);
// device -> device (incl. IPC-mapped peer HBM) copies of up to kMaxCopyRuns runs in ONE launch
// (queue fabric); fills cr.cstart, returns the grid size used
int launch_copy_runs(CopyRuns& cr, int workgroups, uint64_t stream);
void launch_assemble(const FramePtrs& fp, int nframes, uint64_t idx, int64_t nout, uint64_t omask,
                     uint64_t stream);
// scratch: 0, or a zero-initialised PfScratch block (kPfScratchBytes) reused by every launch on one
// stream: counts / summary then need no zeroing before the launch (csrc/peakfind.hip)
// The block also holds each workgroup's candidate SPILL list (hit-rich frames): candidates beyond the
// kPfCandCap parked in LDS go to the workgroup's kPfSpillCap entries here and are tested after the
// stream like the parked ones (only past both does a candidate get tested inline in the stream).
constexpr int kPfScratchHeader = 1024;                 // PfScratch (counters), padded
// The grid is one resident wave of workgroups (768 for radius 1, 512 for radius 2 on 256 CUs), so
// 1024 lists of 4096 entries cover every workgroup with 4x the round-3 depth: on a 2 %-candidate
// batch the in-stream path no longer runs (11.2 -> 7.4 us/frame, profiles/r4/README.md section 4).
#ifndef PR_PF_SPILL_WGS
#define PR_PF_SPILL_WGS 1024
#endif
constexpr int kPfSpillWgs = PR_PF_SPILL_WGS;                    // workgroups with a spill list
constexpr int kPfSpillCap = (4096 / kPfSpillWgs) * 1024;        // entries each (same block size)
constexpr int64_t kPfScratchBytes = kPfScratchHeader + (int64_t)kPfSpillWgs * kPfSpillCap * 4;
void launch_peakfind(const FramePtrs& fp, int nframes, int n_panels, int rows, int cols, float thr_peak,
                     float son_min, int radius, int max_peaks, uint64_t peaks, uint64_t counts,
                     uint64_t summary, uint64_t total, uint64_t stream,
                     uint64_t scratch = 0);
}  // namespace pr
