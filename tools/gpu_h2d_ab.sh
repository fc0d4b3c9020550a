mkdir -p gpurun_out/ab
export PSANA_RAY_ENGINE_GPU_TIMING=1
for cfg in "a:--steps 200" "b:--steps 60" "c:--steps 200 --consumer none" "d:--steps 200 --common-mode off" "e:--steps 200 --mode image" "f:--steps 200"; do
  n=${cfg%%:*}; args=${cfg#*:}
  timeout -k 10 200 python bench.py $args --json-out gpurun_out/ab/$n.json > gpurun_out/ab/$n.log 2>&1 || exit $?
  python -c "
import json,sys; d=json.load(open('gpurun_out/ab/$n.json')); e=d['extra']
print('$n', '$args', d['value'], e['consumed_frames_per_s'], e['producer_gpu_ms_h2d_chunks_calib_chunks'], e['producer_host_s_stage_acquire_launch_commit_total'])"
done
