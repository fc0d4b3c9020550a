# Exactness on both staging paths, then a rocprofv3 kernel trace of the headline with the copy kernel.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
mkdir -p gpurun_out/ck4
timeout -k 10 300 python -u -m pytest tests/test_pipeline_gpu.py tests/test_xtc2.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/ck4/pytest.log 2>&1; rc=$?; tail -2 gpurun_out/ck4/pytest.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_ck -o run -- python3 $R/bench.py --steps 100 --warmup 10 > $R/gpurun_out/ck4/prof_host.log 2>&1 || exit $?
grep '^{' $R/gpurun_out/ck4/prof_host.log | cut -c1-160
python3 $R/tools/rocpd_summary.py /tmp/prof_ck > $R/gpurun_out/ck4/prof_host.md || exit $?
head -8 $R/gpurun_out/ck4/prof_host.md
