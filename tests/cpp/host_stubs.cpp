// Host-only stand-ins for the GPU kernel launchers the host runtime links against, for the
// sanitizer build of tests/cpp/slotpool_stress.cpp (tools/sanitize_host.sh): that build compiles no
// device code and runs host pools only (device < 0), so a launcher is never reached.
#include "kernels.h"

namespace pr {
int launch_copy_runs(CopyRuns&, int, uint64_t) {
  check(false, "launch_copy_runs: the host-only sanitizer build has no GPU kernels");
  return 0;
}
}  // namespace pr
