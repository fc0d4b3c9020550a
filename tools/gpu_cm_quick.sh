# Common-mode kernel iteration: bit-exact GPU kernel tests, then per-phase timing
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
export PYTHONPATH=$R
mkdir -p $R/gpurun_out/cmq
timeout -k 10 300 python3 -u -m pytest $R/tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > $R/gpurun_out/cmq/kernels_gpu.log 2>&1; rc=$?; tail -3 $R/gpurun_out/cmq/kernels_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 $R/tools/cm_probe.py --repeat ${REPEAT:-2} --json-out $R/gpurun_out/cmq/probe.jsonl > $R/gpurun_out/cmq/probe.log 2>&1 || exit $?
grep round $R/gpurun_out/cmq/probe.log
