set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
timeout -k 10 600 python -m pytest tests/test_pipeline_gpu.py tests/test_kernels_gpu.py -x -q -k "pipeline or resident or peakfind" > gpurun_out/pytest_q.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_q.log | cut -c1-600; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_profile.sh
