set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
timeout -k 10 900 python -m pytest tests -m gpu -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -4 gpurun_out/pytest_gpu.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --source device > gpurun_out/bench_dev.log 2>&1 || exit $?
tail -1 gpurun_out/bench_dev.log | cut -c1-200
timeout -k 10 300 python bench.py > gpurun_out/bench_default.log 2>&1 || exit $?
tail -1 gpurun_out/bench_default.log | cut -c1-200
