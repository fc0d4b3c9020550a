# Round-4 checkpoint on a fresh box: full GPU suite, smoke(), the driver's bench line
# (20 and 200 steps), device-resident calib / image benches, then rocprofv3 kernel stats of the
# device-resident calib and image pipelines (stats CSVs + logs kept, per-dispatch traces dropped)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
export PYTHONPATH=$R
O=$R/gpurun_out/${OUT:-r4_checkpoint}
mkdir -p $O
timeout -k 10 900 python3 ${PYFLAGS:-} -u -m pytest $R/tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -1 $O/tests.log
[ $rc -eq 0 ] || { grep -n -A60 "Fatal Python error" $O/tests.log | head -150; exit $rc; }
cd $R && timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit $?
tail -1 $O/smoke.log
for s in 20 200; do
  timeout -k 10 300 python3 bench.py --steps $s --warmup 5 > $O/bench_host_$s.json 2> $O/bench_host_$s.err || exit $?
  cut -c1-150 $O/bench_host_$s.json
done
for m in calib image; do
  timeout -k 10 300 python3 bench.py --steps 200 --warmup 5 --source device --mode $m > $O/bench_dev_$m.json 2> $O/bench_dev_$m.err || exit $?
  cut -c1-150 $O/bench_dev_$m.json
done
for m in calib image; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$m -o run -- python3 bench.py --steps 200 --warmup 20 --source device --mode $m > $O/prof_$m.log 2>&1 || exit $?
  tail -1 $O/prof_$m.log | cut -c1-150
done
find $O -path "*prof_*" -type f ! -name "*stats.csv" ! -name "*.log" -delete
du -sh $O
