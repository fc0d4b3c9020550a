# per-rank cost of the N>1 transport path on one GPU: local route vs transport rounds with all
# frames routed to this rank (N>1 symmetric steady state) vs loopback (every frame through RCCL)
mkdir -p gpurun_out/xport
for r in 0 1; do
  for m in local transport loopback; do
    a=""; [ $m = transport ] && a="--transport"; [ $m = loopback ] && a="--loopback"
    timeout -k 10 200 python bench.py --steps 200 $a --json-out gpurun_out/xport/${m}_r$r.json > gpurun_out/xport/${m}_r$r.log 2>&1 || exit $?
    python -c "
import json; d=json.load(open('gpurun_out/xport/${m}_r$r.json')); e=d['extra']
print('$m r$r', d['value'], e['consumed_frames_per_s'], e['transport_driver'], e['transport_rounds_rank0'], e['transport_round_ms_rank0'], e['transport_ctrl_ms_rank0'])"
  done
done
for r in 0; do
  for m in local transport; do
    a=""; [ $m = transport ] && a="--transport"
    timeout -k 10 200 python bench.py --steps 300 --source device $a --json-out gpurun_out/xport/dev_${m}_r$r.json > gpurun_out/xport/dev_${m}_r$r.log 2>&1 || exit $?
    python -c "
import json; d=json.load(open('gpurun_out/xport/dev_${m}_r$r.json')); e=d['extra']
print('device $m r$r', d['value'], e['consumed_frames_per_s'], e['transport_driver'], e['transport_rounds_rank0'], e['transport_round_ms_rank0'])"
  done
done
