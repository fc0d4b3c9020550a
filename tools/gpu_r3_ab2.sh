# CM A/B round 2: gap-fill fix in every build; plain vs non-temporal raw loads (pipeline benches,
# two interleaved rounds); VALU-sensitivity probe (row network twice, timing only); stamps
set -o pipefail
R=$GRAFT_REPO_ROOT
VARIANTS="rawplain rows2x" NOTEST="rows2x" BENCH=1 BENCH_ROUNDS=2 BENCH_VARIANTS="base rawplain" bash $R/tools/gpu_cm_ab.sh || exit $?
bash $R/tools/gpu_cm_stamps.sh || exit $?
