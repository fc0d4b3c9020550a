# Same-box A/B of the 2-rank host-staged rehearsal: the round-3 tree (variants/r3tree, built from
# commit 4ebc405) against this tree, interleaved, to tell a regression of the balanced window from
# box / start-up variance.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4_r3ab
mkdir -p $O
run() {  # name, tree, port, args
  ( cd $2 && PYTHONPATH=$2 timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $3 bench.py --gpus 2 ${@:4} > $O/$1.log 2>&1 ) || { tail -20 $O/$1.log; return 1; }
  grep '"metric"' $O/$1.log > $O/$1.json
  python -c "
import json; r=json.load(open('$O/$1.json')); x=r['extra']['xgmi_phase']
print('$1', r['value'], x['frames_per_s'], r['extra']['production_frames_per_s'], r['extra']['consumer_frames_per_s'], r['extra'].get('producer_host_s_stage_acquire_launch_commit_total'), flush=True)"
}
p=29850
for rnd in 1 2 3; do
  p=$((p+1)); run r3_host_$rnd $R/variants/r3tree $p --steps 40 --warmup 10 || exit $?
  p=$((p+1)); run r4_host_$rnd $R $p --steps 40 --warmup 10 || exit $?
done
for rnd in 1 2; do
  p=$((p+1)); run r3_dev_$rnd $R/variants/r3tree $p --steps 100 --warmup 20 --source device || exit $?
  p=$((p+1)); run r4_dev_$rnd $R $p --steps 100 --warmup 20 --source device || exit $?
done
