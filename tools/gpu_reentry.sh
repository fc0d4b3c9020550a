# Re-entry check after a container rebuild: GPU tests, smoke, default bench (1 GPU)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
mkdir -p gpurun_out/re
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/re/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/re/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > gpurun_out/re/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/re/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/re/bench_default.log 2>&1 || exit $?
tail -1 gpurun_out/re/bench_default.log | cut -c1-300
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --source device > gpurun_out/re/bench_dev.log 2>&1 || exit $?
tail -1 gpurun_out/re/bench_dev.log | cut -c1-300
