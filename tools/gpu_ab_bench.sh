set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
mkdir -p gpurun_out/ab
run() { name=$1; shift; timeout -k 10 200 python bench.py --steps 100 --warmup 10 "$@" --json-out gpurun_out/ab/$name.json > gpurun_out/ab/$name.log 2>&1 || return $?; python3 -c "
import json,sys; d=json.load(open('gpurun_out/ab/$name.json')); e=d['extra']; print('$name', d['value'], e['consumed_frames_per_s'], e['produced_frames_per_s'], e['queue_full_waits_rank0'], e['producer_host_s_stage_acquire_launch_commit_total'])"; }
run c16 && run c32 --chunk 32 && run c32b64 --chunk 32 --batch 64 && run c24 --chunk 24 && \
GPU_MAX_HW_QUEUES=8 run c16_hwq8 && GPU_MAX_HW_QUEUES=8 run c32_hwq8 --chunk 32 && run c16_dev --source device --steps 200 && run c32_dev --chunk 32 --source device --steps 200 && run c16_again
