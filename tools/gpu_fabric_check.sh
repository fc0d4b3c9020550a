# Fabric on the GPU after a fabric change: IPC elastic tests, producer->consumer process bench,
# and the 2-rank bench rehearsal on one GPU
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
export PYTHONPATH=$R
O=$R/gpurun_out/fab
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest $R/tests/test_elastic_gpu.py $R/tests/test_pipeline_gpu.py -x -q --timeout 180 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -1 $O/tests.log; [ $rc -eq 0 ] || exit $rc
cd $R && timeout -k 10 300 python3 bench/fabric_ipc.py > $O/fabric_ipc.log 2>&1 || exit $?
tail -1 $O/fabric_ipc.log | cut -c1-300
bash tools/gpu_bench_2rank_1gpu.sh
