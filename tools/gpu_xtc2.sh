# File sources on the GPU: engine e2e tests (pread staging and zero-copy mapping), then file-source
# throughput for both on-disk formats, zero-copy (default) and pread (PSANA_RAY_FILE_ZEROCOPY=0).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_xtc2.py tests/test_pipeline_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_xtc2.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_xtc2.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
for f in xtc2 praw; do
  for z in 1 0; do
    PSANA_RAY_FILE_ZEROCOPY=$z timeout -k 10 300 python bench/file_source.py --format $f --frames 3072 > gpurun_out/file_source_${f}_zc$z.log 2>&1 || exit $?
    tail -1 gpurun_out/file_source_${f}_zc$z.log | cut -c1-330
  done
done
