# copy engine A/B for the host-staged headline: SDMA (default) vs blit-kernel copies (HSA_ENABLE_SDMA=0)
mkdir -p gpurun_out/sdma
timeout -k 10 120 python bench/h2d.py > gpurun_out/sdma/h2d_sdma1.log 2>&1 || exit $?
grep '"chunk_frames": 32, "streams": 1' gpurun_out/sdma/h2d_sdma1.log
HSA_ENABLE_SDMA=0 timeout -k 10 120 python bench/h2d.py > gpurun_out/sdma/h2d_sdma0.log 2>&1 || exit $?
grep '"chunk_frames": 32' gpurun_out/sdma/h2d_sdma0.log
for r in 0 1; do
  for e in 1 0; do
    HSA_ENABLE_SDMA=$e timeout -k 10 200 python bench.py --steps 200 --json-out gpurun_out/sdma/e${e}_r$r.json > gpurun_out/sdma/e${e}_r$r.log 2>&1 || exit $?
    python -c "
import json; d=json.load(open('gpurun_out/sdma/e${e}_r$r.json')); e=d['extra']
print('sdma=$e r$r', d['value'], e['consumed_frames_per_s'], e['producer_host_s_stage_acquire_launch_commit_total'])"
  done
done
for r in 0 1; do
  for e in blit sdma; do
    timeout -k 10 200 python bench.py --steps 200 --copy-engine $e --json-out gpurun_out/sdma/flag_${e}_r$r.json > gpurun_out/sdma/flag_${e}_r$r.log 2>&1 || exit $?
    python -c "
import json; d=json.load(open('gpurun_out/sdma/flag_${e}_r$r.json')); e=d['extra']
print('flag $e r$r', d['value'], e['copy_engine'])"
  done
done
