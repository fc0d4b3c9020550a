# A/B of the transport drivers on one GPU (loopback: every frame goes through the control round
# and an RCCL send/recv to self): native C++ engine (shared-memory control plane) vs the python
# thread (gloo all-gather).  Each GPU step has its own time limit; stops at the first failure.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_loopback.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_loopback.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_loopback.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
for x in native python; do
  PSANA_RAY_XPORT=$x timeout -k 10 300 python bench.py --loopback --steps 100 --warmup 10 > gpurun_out/bench_loopback_$x.log 2>&1 || exit $?
  tail -1 gpurun_out/bench_loopback_$x.log | cut -c1-200
done
