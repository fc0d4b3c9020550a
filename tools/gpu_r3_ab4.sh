# VALU issue-rate probe; spread median-phase mapping (every wave an equal share) vs packed
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
O=$R/gpurun_out/ab4
mkdir -p $O
timeout -k 10 60 $R/tools/valu_rate_bin > $O/valu_rate.jsonl 2>&1 || exit $?
cat $O/valu_rate.jsonl
VARIANTS="spread" TESTK="common_mode or image" BENCH=1 BENCH_ROUNDS=2 bash $R/tools/gpu_cm_ab.sh || exit $?
bash $R/tools/gpu_r3_final.sh || exit $?
