// Host-only stand-ins for the GPU kernel launchers the host runtime links against, for the
// sanitizer build of tests/cpp/slotpool_stress.cpp (tools/sanitize_host.sh): that build compiles no
// device code and runs host pools only (device < 0), so a launcher is never reached.
#include "kernels.h"
#include "verify.h"

namespace pr {
int launch_copy_runs(CopyRuns&, int, uint64_t) {
  check(false, "launch_copy_runs: the host-only sanitizer build has no GPU kernels");
  return 0;
}
}  // namespace pr

namespace pr {
// verify.hip launchers: the host-only sanitizer build runs host (CPU) rings only
void launch_frame_checksums(const CkFrames&, int, int64_t, uint64_t, uint64_t, uint64_t) {
  check(false, "launch_frame_checksums: the host-only sanitizer build has no GPU kernels");
}
void launch_acquire_fence(uint64_t) { check(false, "launch_acquire_fence: no GPU kernels in this build"); }
void launch_release_fence(uint64_t) { check(false, "launch_release_fence: no GPU kernels in this build"); }
}  // namespace pr
