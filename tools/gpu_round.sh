# one GPU round: tests, per-kernel device times (graph-replayed), pipeline bench
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench/kernels.py ${KOPTS:-} --json-out gpurun_out/kernels.jsonl > gpurun_out/kernels.log 2>&1 || exit $?
grep -v warning gpurun_out/kernels.log | cut -c1-200
timeout -k 10 300 python bench.py --steps 60 --warmup 10 > gpurun_out/bench_host.log 2>&1 || exit $?
tail -1 gpurun_out/bench_host.log | cut -c1-400
