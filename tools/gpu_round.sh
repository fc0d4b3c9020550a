export PYTHONUNBUFFERED=1
timeout -k 10 400 python -m pytest tests -m gpu -q -x 2>&1 | tail -2
for v in "" "--common-mode off" "--consumer none" "--chunk 32" ""; do
  timeout -k 10 200 python bench.py --steps 60 --warmup 10 $v > gpurun_out/sweep.log 2>&1 || { echo "fail: $v"; break; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/sweep.log').read().strip().splitlines()[-1]); print('$v', d['value'], d['extra']['producer_frames_per_s_rank0'], d['extra']['producer_host_s_stage_acquire_launch_commit_total'])"
done
