export PYTHONUNBUFFERED=1
timeout -k 10 400 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1; echo pytest_rc=$? >> gpurun_out/pytest_gpu.log; tail -4 gpurun_out/pytest_gpu.log
timeout -k 10 200 python bench/kernels.py --only calib_basic,calib_cm,peakfind > gpurun_out/kernels2.log 2>&1; grep kernel gpurun_out/kernels2.log
timeout -k 10 240 python bench.py --steps 60 --warmup 10 > gpurun_out/bench2.log 2>&1; echo bench_rc=$?; tail -3 gpurun_out/bench2.log
timeout -k 10 240 python bench.py --steps 60 --warmup 10 --source device > gpurun_out/bench2d.log 2>&1; tail -1 gpurun_out/bench2d.log
