# Peak finder: tests, kernel A/B (grid variants), device-resident pipeline bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py tests/test_pipeline_gpu.py -x -q -k "peakfind or peakfinder" > gpurun_out/pytest_pf.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_pf.log | cut -c1-600; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench/kernels.py --only peakfind --json-out gpurun_out/kernels_pf.jsonl > gpurun_out/kernels_pf.log 2>&1 || exit $?
grep -v warning gpurun_out/kernels_pf.log | cut -c1-180
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --source device > gpurun_out/bench_dev_pf.log 2>&1 || exit $?
tail -1 gpurun_out/bench_dev_pf.log | cut -c1-200
PSANA_RAY_PF_BLOCKS=0 timeout -k 10 300 python bench.py --steps 100 --warmup 10 --source device > gpurun_out/bench_dev_pf0.log 2>&1 || exit $?
tail -1 gpurun_out/bench_dev_pf0.log | cut -c1-200
