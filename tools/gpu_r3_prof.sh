# Round-3 final numbers (bench JSON lines) and rocprofv3 kernel stats of both device-resident
# pipelines; per-dispatch traces are deleted right after each profiled run (only *stats.csv kept)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
export PYTHONPATH=$R
O=$R/gpurun_out/r3_prof
mkdir -p $O
cd $R
for s in 20 200; do
  timeout -k 10 300 python3 bench.py --steps $s --warmup 5 > $O/bench_host_$s.json 2> $O/bench_host_$s.err || exit $?
  cut -c1-150 $O/bench_host_$s.json
done
for m in calib image; do
  timeout -k 10 300 python3 bench.py --steps 200 --warmup 5 --source device --mode $m > $O/bench_dev_$m.json 2> $O/bench_dev_$m.err || exit $?
  cut -c1-150 $O/bench_dev_$m.json
done
for m in calib image; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$m -o run -- python3 bench.py --steps 40 --warmup 10 --source device --mode $m > $O/prof_$m.log 2>&1 || exit $?
  find $O/prof_$m -type f ! -name "*stats.csv" -delete
  tail -1 $O/prof_$m.log | cut -c1-150
done
du -sh $O
timeout -k 10 120 $R/tools/valu_rate_bin > $O/valu_rate2.jsonl 2>&1 || exit $?
cat $O/valu_rate2.jsonl | grep -E "cvt|bfe|and_or|cndmask|mul|mov|xor|sub|perm"
VARIANTS="fastdec" TESTK="common_mode or image" BENCH=1 BENCH_ROUNDS=2 bash $R/tools/gpu_cm_ab.sh || exit $?
