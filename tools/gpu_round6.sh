set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
timeout -k 10 700 python -m pytest tests/test_kernels_gpu.py -x -q -k "image" > gpurun_out/pytest_img.log 2>&1; rc=$?; tail -15 gpurun_out/pytest_img.log | cut -c1-600; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench/kernels.py --only calib_image --json-out gpurun_out/kernels_img.jsonl > gpurun_out/kernels_img.log 2>&1 || exit $?
grep -v warning gpurun_out/kernels_img.log | cut -c1-250
