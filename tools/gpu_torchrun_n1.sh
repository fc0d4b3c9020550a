# Driver-shaped launch rehearsal on one GPU: torch.distributed.run with one rank (RCCL world of 1)
# plus the N>1 per-rank transport path on one GPU
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
mkdir -p gpurun_out/trun
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 1 --steps 60 --warmup 10 > gpurun_out/trun/torchrun_n1.log 2>&1 || exit $?
grep '"metric"' gpurun_out/trun/torchrun_n1.log | cut -c1-200
timeout -k 10 300 python bench.py --steps 60 --warmup 10 --transport > gpurun_out/trun/transport.log 2>&1 || exit $?
grep '"metric"' gpurun_out/trun/transport.log | cut -c1-200
