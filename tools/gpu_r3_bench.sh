# Round-3 bench check on one MI355X: sustained-rate windows (20 vs 200 steps, host-staged and
# device-resident, calib and image), then the driver's N>1 launch rehearsed with 2 ranks on the one
# GPU (remote_only cross window over HIP IPC, self-validation: exit 4 if < 90 % crossed)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/r3_bench
mkdir -p $O
for s in 20 200; do
  timeout -k 10 300 python3 bench.py --steps $s --warmup 5 > $O/host_$s.json 2> $O/host_$s.err || exit $?
  timeout -k 10 300 python3 bench.py --steps $s --warmup 5 --source device > $O/dev_$s.json 2> $O/dev_$s.err || exit $?
  timeout -k 10 300 python3 bench.py --steps $s --warmup 5 --source device --mode image > $O/devimg_$s.json 2> $O/devimg_$s.err || exit $?
done
for f in $O/*.json; do python3 -c "import json,sys;d=json.load(open('$f'));e=d['extra'];print('$f', d['value'], e['production_frames_per_s'], e['consumer_frames_per_s'])"; done
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29613 bench.py --gpus 2 --steps 20 --warmup 5 > $O/n2_host.log 2>&1 || exit $?
grep '"metric"' $O/n2_host.log > $O/n2_host.json
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29614 bench.py --gpus 2 --steps 100 --warmup 20 --source device > $O/n2_dev.log 2>&1 || exit $?
grep '"metric"' $O/n2_dev.log > $O/n2_dev.json
for f in $O/n2_host.json $O/n2_dev.json; do python3 -c "import json;r=json.load(open('$f'));x=r['extra']['xgmi_phase'];print('$f', r['value'], x['frames_per_s'], x['cross_gpu_fraction'], x['received_cross_per_consumed'], x['cross_gpu_GB_per_s'], r['extra']['validation'])"; done
