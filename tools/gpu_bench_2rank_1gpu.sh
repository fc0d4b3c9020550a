# Rehearsal of the driver's N>1 launch on ONE GPU: two ranks share cuda:0 (device = local_rank %
# device_count), so the queue session, the HIP IPC links between the two processes, the headline
# window and the route=spread window all run on the GPU.  Rates are not N>1 numbers (one GPU's
# compute and HBM shared by both ranks).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
mkdir -p gpurun_out/b2
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29613 bench.py --gpus 2 --steps 40 --warmup 10 $EXTRA > gpurun_out/b2/host.log 2>&1 || exit $?
grep "\"metric\"" gpurun_out/b2/host.log | python -c "import json,sys;r=json.loads(sys.stdin.read());print(r[\"value\"], json.dumps(r[\"extra\"][\"xgmi_phase\"])[:300])"
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29614 bench.py --gpus 2 --steps 100 --warmup 20 --source device $EXTRA > gpurun_out/b2/dev.log 2>&1 || exit $?
grep '"metric"' gpurun_out/b2/dev.log > gpurun_out/b2/dev.json
python -c "import json;r=json.load(open('gpurun_out/b2/dev.json'));print(r['value'], json.dumps(r['extra']['xgmi_phase'])[:400], r['extra'].get('links_rank0'))"
