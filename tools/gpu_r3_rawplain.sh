# Plain vs non-temporal raw-word loads in the common-mode kernel: device-resident pipelines,
# three interleaved rounds on one box (kernel tests of the variant first)
set -o pipefail
R=$GRAFT_REPO_ROOT
VARIANTS="rawplain" TESTK="common_mode or image" BENCH=1 BENCH_ROUNDS=3 bash $R/tools/gpu_cm_ab.sh || exit $?
