# Round 4, common mode: the column-median probe (network vs LDS-histogram select vs count-bisection,
# bitwise-checked, tools/median_probe.hip), then the same-box A/B of the non-temporal output
# stores (variant ntst) with its CM tests, cm_probe rounds and device-resident bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/r4_cm
mkdir -p $O
timeout -k 10 180 $R/tools/median_probe_bin 16384 > $O/median_probe.json 2> $O/median_probe.err; rc=$?
cat $O/median_probe.json; [ $rc -eq 0 ] || { echo "median probe rc=$rc"; tail -5 $O/median_probe.err; }
[ $rc -le 1 ] || exit $rc
VARIANTS="ntst" BENCH=1 BENCH_ROUNDS=2 bash $R/tools/gpu_cm_ab.sh
