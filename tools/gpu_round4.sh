set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
timeout -k 10 700 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -15 gpurun_out/pytest_gpu.log | cut -c1-600; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench/kernels.py --only peakfind --json-out gpurun_out/kernels_pf.jsonl > gpurun_out/kernels_pf.log 2>&1 || exit $?
grep -v warning gpurun_out/kernels_pf.log | cut -c1-220
timeout -k 10 300 python bench/kernels.py --detector jungfrau16M --frames 8 --iters 5 --only calib_basic,calib_cm,peakfind --json-out gpurun_out/kernels_jf.jsonl > gpurun_out/kernels_jf.log 2>&1 || exit $?
grep -v warning gpurun_out/kernels_jf.log | cut -c1-220
timeout -k 10 300 python bench.py --steps 60 --warmup 10 > gpurun_out/bench_host.log 2>&1 || exit $?
tail -1 gpurun_out/bench_host.log | cut -c1-300
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --source device > gpurun_out/bench_dev.log 2>&1 || exit $?
tail -1 gpurun_out/bench_dev.log | cut -c1-300
