# CM A/B (plain vs non-temporal raw loads) with pipeline benches, then the stamps build with the
# image-placement split
set -o pipefail
R=$GRAFT_REPO_ROOT
VARIANTS="rawplain" BENCH=1 bash $R/tools/gpu_cm_ab.sh || exit $?
bash $R/tools/gpu_cm_stamps.sh || exit $?
