# copy engine x transport path (N>1 per-rank paths on one GPU)
mkdir -p gpurun_out/bx
for cfg in "t_blit:--transport --copy-engine blit" "t_sdma:--transport --copy-engine sdma" "l_blit:--loopback --copy-engine blit" "l_sdma:--loopback --copy-engine sdma"; do
  n=${cfg%%:*}; a=${cfg#*:}
  timeout -k 10 200 python bench.py --steps 200 $a --json-out gpurun_out/bx/$n.json > gpurun_out/bx/$n.log 2>&1 || exit $?
  python -c "
import json; d=json.load(open('gpurun_out/bx/$n.json')); e=d['extra']
print('$n', d['value'], e['consumed_frames_per_s'], e['transport_round_ms_rank0'], e['producer_host_s_stage_acquire_launch_commit_total'])"
done
