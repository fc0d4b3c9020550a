# Kernel statistics of the 2-rank cross-process window on the one GPU of a box: both ranks of
# `bench.py --gpus 2` started by hand (rank env set, so bench.py does not self-launch), each under its
# own `rocprofv3 --kernel-trace --stats` (the profiled program is python3 itself, no launcher hop), a
# short headline window and a long route=remote_only window, so the cross window dominates the trace.
#   OUT=r6_profx gpurun -- bash tools/gpu_prof_cross.sh
# Outputs: gpurun_out/${OUT:-profx}/rank{0,1}/run_kernel_stats.csv, bench.json (rank 0's line).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
O=$R/gpurun_out/${OUT:-profx}
mkdir -p $O
PORT=$((29500 + RANDOM % 2000))
pids=()
for r in 0 1; do
  RANK=$r WORLD_SIZE=2 LOCAL_RANK=$r LOCAL_WORLD_SIZE=2 MASTER_ADDR=127.0.0.1 MASTER_PORT=$PORT PYTHONPATH=$R \
    timeout -k 10 ${STEP_TIMEOUT:-300} rocprofv3 --kernel-trace --stats --output-format csv -d $O/rank$r -o run -- \
    python3 $R/bench.py --gpus 2 --steps ${STEPS:-20} --cross-steps ${CROSS_STEPS:-400} --warmup 5 --source device \
    ${BENCH_ARGS:-} > $O/rank$r.out 2> $O/rank$r.err &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait $p || rc=$?; done
[ $rc -eq 0 ] || { tail -20 $O/rank0.err $O/rank1.err; exit $rc; }
grep '"metric"' $O/rank0.out > $O/bench.json || exit 1
for r in 0 1; do echo "rank $r"; head -6 $O/rank$r/run_kernel_stats.csv | cut -c1-150; done
