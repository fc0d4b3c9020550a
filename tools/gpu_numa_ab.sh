# NUMA binding A/B on one box (host-staged headline), interleaved
mkdir -p gpurun_out/numa
python -c "import os; print('cpus allowed', len(os.sched_getaffinity(0)), sorted(os.sched_getaffinity(0))[:64])"
cat /sys/devices/system/node/node*/cpulist 2>/dev/null | head -4
for r in 0 1; do
  for b in 1 0; do
    PSANA_RAY_NUMA_BIND=$b PSANA_RAY_ENGINE_GPU_TIMING=1 timeout -k 10 200 python bench.py --steps 200 --json-out gpurun_out/numa/b${b}_r$r.json > gpurun_out/numa/b${b}_r$r.log 2>&1 || exit $?
    python -c "
import json; d=json.load(open('gpurun_out/numa/b${b}_r$r.json')); e=d['extra']
print('bind=$b r$r', d['value'], e['numa_node'], e['cpus_allowed'], e['producer_gpu_ms_h2d_chunks_calib_chunks'], e['producer_host_s_stage_acquire_launch_commit_total'])"
  done
done
