set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -x -q -k "common_mode or image" > gpurun_out/pytest_cm.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_cm.log | cut -c1-600; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench/kernels.py --only calib_cm_ab,calib_cm --json-out gpurun_out/kernels_cm.jsonl > gpurun_out/kernels_cm.log 2>&1 || exit $?
grep -v warning gpurun_out/kernels_cm.log | cut -c1-160
