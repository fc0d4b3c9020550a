set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -x -q -k "common_mode" > gpurun_out/pytest_cm.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_cm.log | cut -c1-600; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench/kernels.py --detector jungfrau16M --frames 8 --iters 5 --only calib_basic,calib_cm,peakfind --json-out gpurun_out/kernels_jf.jsonl > gpurun_out/kernels_jf.log 2>&1 || exit $?
grep -v warning gpurun_out/kernels_jf.log | cut -c1-160
