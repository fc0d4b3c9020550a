# Exit-path check (GPU suite must exit 0 with the stream pool closed at exit), rocprofv3 kernel
# stats of both device-resident pipelines, then the fastdec A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
export PYTHONPATH=$R
O=$R/gpurun_out/r3_prof2
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest $R/tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -1 $O/tests.log; [ $rc -eq 0 ] || { tail -30 $O/tests.log; exit $rc; }
cd $R
for m in calib image; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$m -o run -- python3 bench.py --steps 40 --warmup 10 --source device --mode $m > $O/prof_$m.log 2>&1; rc=$?
  find $O/prof_$m -type f ! -name "*stats.csv" -delete 2>/dev/null
  tail -1 $O/prof_$m.log | cut -c1-150
  [ $rc -eq 0 ] || { tail -20 $O/prof_$m.log; exit $rc; }
done
du -sh $O
VARIANTS="fastdec" TESTK="common_mode or image" BENCH=1 BENCH_ROUNDS=2 bash $R/tools/gpu_cm_ab.sh || exit $?
