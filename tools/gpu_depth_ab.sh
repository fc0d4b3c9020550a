# producer engine H2D prefetch depth A/B (host-staged headline), interleaved rounds
mkdir -p gpurun_out/depth
timeout -k 10 400 python -u -m pytest tests/test_pipeline_gpu.py tests/test_rawfile.py tests/test_xtc2.py tests/test_resume_metrics.py tests/test_panel_shards.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/depth/pytest.log 2>&1 || { tail -20 gpurun_out/depth/pytest.log; exit 1; }
tail -1 gpurun_out/depth/pytest.log
for r in 0 1 2; do
  for d in 1 3; do
    PSANA_RAY_STAGE_DEPTH=$d timeout -k 10 200 python bench.py --steps 200 --json-out gpurun_out/depth/d${d}_r$r.json > gpurun_out/depth/d${d}_r$r.log 2>&1 || exit $?
    python -c "
import json; d=json.load(open('gpurun_out/depth/d${d}_r$r.json')); e=d['extra']
print('depth $d round $r', d['value'], e['producer_host_s_stage_acquire_launch_commit_total'])"
  done
done
