# Driver-shaped launch rehearsal on one GPU: torch.distributed.run with one rank, exactly as the
# driver launches bench.py for N>1.  With one rank the bench runs in single-process mode (no queue
# session, no fabric links: WORLD_SIZE=1), so this checks env detection, the launcher and the
# result line; the multi-rank session + fabric path is rehearsed on the CPU (8 ranks,
# tests/test_bench_rehearsal.py) and on the GPU by the IPC tests (tests/test_elastic_gpu.py).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
mkdir -p gpurun_out/trun
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 1 --steps 60 --warmup 10 > gpurun_out/trun/torchrun_n1.log 2>&1 || exit $?
grep '"metric"' gpurun_out/trun/torchrun_n1.log | cut -c1-200
