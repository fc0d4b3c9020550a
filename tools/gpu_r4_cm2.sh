# Round 4, common mode pass 2: the column-median probe (register- and LDS-resident forms of the
# histogram select and the count-bisection, bitwise and value checks), then same-box A/B rounds of
# the streaming-store / streaming-load variants with the device-resident pipeline (calib + image).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/r4_cm2
mkdir -p $O
for b in median_probe_bin median_probe_lds_bin; do
  timeout -k 10 180 $R/tools/$b 16384 > $O/$b.json 2> $O/$b.err; rc=$?
  cat $O/$b.json; echo "$b rc=$rc"
  [ $rc -le 1 ] || exit $rc
done
NOTEST="" VARIANTS="ntcal pfnt ntcalpf" TESTK="common_mode or peakfind" BENCH=1 BENCH_ROUNDS=2 bash $R/tools/gpu_cm_ab.sh
