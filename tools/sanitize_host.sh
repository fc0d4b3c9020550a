#!/bin/bash
# Build + run the host-side runtime stress test under a sanitizer (CPU only; no GPU needed).
#   tools/sanitize_host.sh thread|address [n_events]
# Host code only: no device code is compiled, so plain -fsanitize applies to the host build.
set -euo pipefail
SAN=${1:-thread}
N=${2:-20000}
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=${TMPDIR:-/tmp}/psana_ray_stress_$SAN
CXX=/opt/rocm/lib/llvm/bin/clang++
case $SAN in
  thread) FLAGS="-fsanitize=thread" ;;
  address) FLAGS="-fsanitize=address,undefined -fno-sanitize-recover=undefined -fno-omit-frame-pointer" ;;
  *) echo "unknown sanitizer $SAN" >&2; exit 2 ;;
esac
# the runtime sources include the HIP headers (as in the real build): compile them as HIP, HOST
# side only, with the sanitizer on the host pass and never on a GPU pass
$CXX -x hip --offload-host-only --offload-arch=gfx950 -fno-gpu-sanitize -std=c++17 -O1 -g $FLAGS \
  -I"$R/csrc" \
  "$R/tests/cpp/slotpool_stress.cpp" "$R/csrc/runtime.cpp" "$R/csrc/fabric.cpp" "$R/csrc/lifecycle.cpp" "$R/csrc/verify.cpp" "$R/csrc/trace.cpp" \
  "$R/csrc/streams.cpp" "$R/tests/cpp/host_stubs.cpp" \
  -L/opt/rocm/lib -Wl,-rpath,/opt/rocm/lib -lamdhip64 -lpthread -lrt -o "$OUT"
"$OUT" "$N"
