# rocprofv3 kernel stats of both device-resident pipelines on the final tree
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
export PYTHONPATH=$R
O=$R/gpurun_out/r3_prof3
mkdir -p $O
cd $R
for m in calib image; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$m -o run -- python3 bench.py --steps 40 --warmup 10 --source device --mode $m > $O/prof_$m.log 2>&1; rc=$?
  find $O/prof_$m -type f ! -name "*kernel_stats.csv" -delete 2>/dev/null
  tail -1 $O/prof_$m.log | cut -c1-150
  [ $rc -eq 0 ] || { tail -20 $O/prof_$m.log; exit $rc; }
done
du -sh $O
