# VALU issue rate per instruction form (1-4 waves per SIMD), then the round-3 final checkpoint
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
O=$R/gpurun_out/ab5
mkdir -p $O
timeout -k 10 120 $R/tools/valu_rate_bin > $O/valu_rate.jsonl 2>&1 || exit $?
cat $O/valu_rate.jsonl
bash $R/tools/gpu_r3_final.sh || exit $?
