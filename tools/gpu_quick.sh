set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
timeout -k 10 600 python -m pytest tests/test_pipeline_gpu.py -x -q > gpurun_out/pytest_q.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_q.log | cut -c1-600; [ $rc -eq 0 ] || exit $rc
PSANA_RAY_ENGINE_GPU_TIMING=1 timeout -k 10 300 python bench.py > gpurun_out/bench_t.log 2>&1 || exit $?
grep '^{' gpurun_out/bench_t.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['extra']['producer_gpu_ms_h2d_chunks_calib_chunks'])"
timeout -k 10 300 python bench.py > gpurun_out/bench_nt.log 2>&1 || exit $?
grep '^{' gpurun_out/bench_nt.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'])"
