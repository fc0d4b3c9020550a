# Round 2: elastic fabric on one GPU (IPC between processes), full GPU suite, headline bench, IPC throughput
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
export TMPDIR=/tmp
mkdir -p gpurun_out/r2f
timeout -k 10 300 python -u -m pytest tests/test_elastic_gpu.py -x -v --timeout 150 --timeout-method thread > gpurun_out/r2f/elastic_gpu.log 2>&1; rc=$?; tail -5 gpurun_out/r2f/elastic_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench/fabric_ipc.py --frames 4000 --log-dir gpurun_out/r2f --json-out gpurun_out/r2f/fabric_ipc.json > gpurun_out/r2f/fabric_ipc.log 2>&1; rc=$?; tail -2 gpurun_out/r2f/fabric_ipc.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/r2f/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/r2f/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/r2f/bench_default.log 2>&1 || exit $?
tail -1 gpurun_out/r2f/bench_default.log | cut -c1-400
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --source device > gpurun_out/r2f/bench_dev.log 2>&1 || exit $?
tail -1 gpurun_out/r2f/bench_dev.log | cut -c1-300
