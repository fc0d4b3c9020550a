export PYTHONUNBUFFERED=1
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1; echo pytest_rc=$? >> gpurun_out/pytest_gpu.log; tail -4 gpurun_out/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; echo smoke_rc=$?; tail -1 gpurun_out/smoke.log
timeout -k 10 240 python bench.py > gpurun_out/bench4.log 2>&1; echo bench_rc=$?; tail -1 gpurun_out/bench4.log | cut -c1-300
