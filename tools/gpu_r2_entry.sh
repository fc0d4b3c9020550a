# Round-2 entry check: GPU tests, smoke, default bench, device-resident bench, rocprofv3 kernel stats
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
export TMPDIR=/tmp
mkdir -p gpurun_out/r2e
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2e/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/r2e/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > gpurun_out/r2e/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/r2e/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/r2e/bench_default.log 2>&1 || exit $?
tail -1 gpurun_out/r2e/bench_default.log | cut -c1-300
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --source device > gpurun_out/r2e/bench_dev.log 2>&1 || exit $?
tail -1 gpurun_out/r2e/bench_dev.log | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r2e/prof_dev -o run -- python bench.py --steps 100 --warmup 10 --source device > gpurun_out/r2e/prof_dev.log 2>&1 || exit $?
tail -1 gpurun_out/r2e/prof_dev.log | cut -c1-300
