set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
timeout -k 10 500 python -m pytest tests/test_loopback.py -m gpu -x -q -s > gpurun_out/pytest_loopback.log 2>&1; rc=$?; tail -5 gpurun_out/pytest_loopback.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 60 --warmup 10 --loopback > gpurun_out/bench_loopback.log 2>&1 || exit $?
tail -1 gpurun_out/bench_loopback.log | cut -c1-1400
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --loopback --source device > gpurun_out/bench_loopback_dev.log 2>&1 || exit $?
tail -1 gpurun_out/bench_loopback_dev.log | cut -c1-1400
