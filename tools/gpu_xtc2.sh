# XTC2 source on the GPU: engine e2e test, then file-source throughput for both on-disk formats.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_xtc2.py tests/test_pipeline_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_xtc2.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_xtc2.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
for f in xtc2 praw; do
  timeout -k 10 300 python bench/file_source.py --format $f --frames 1024 > gpurun_out/file_source_$f.log 2>&1 || exit $?
  tail -1 gpurun_out/file_source_$f.log | cut -c1-400
done
