# same box: isolated H2D copy rate vs the pipeline's event-timed H2D and its delivered rate
mkdir -p gpurun_out/diag
timeout -k 10 120 python bench/h2d.py > gpurun_out/diag/h2d.log 2>&1 || exit $?
grep '"chunk_frames": 32' gpurun_out/diag/h2d.log
for r in 0 1; do
  PSANA_RAY_ENGINE_GPU_TIMING=1 timeout -k 10 200 python bench.py --steps 200 --json-out gpurun_out/diag/b$r.json > gpurun_out/diag/b$r.log 2>&1 || exit $?
  python -c "
import json; d=json.load(open('gpurun_out/diag/b$r.json')); e=d['extra']
print('bench r$r', d['value'], e['producer_gpu_ms_h2d_chunks_calib_chunks'], e['producer_host_s_stage_acquire_launch_commit_total'], e.get('numa_node'))"
done
