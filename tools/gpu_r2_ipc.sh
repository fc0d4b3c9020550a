set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
mkdir -p gpurun_out/r2i
timeout -k 10 200 python -u bench/fabric_ipc.py --frames 2000 --log-dir gpurun_out/r2i --json-out gpurun_out/r2i/fabric_ipc.json > gpurun_out/r2i/fabric_ipc.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/r2i/fabric_ipc.log | tail -5; exit $rc
