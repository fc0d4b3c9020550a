export PYTHONUNBUFFERED=1
timeout -k 10 400 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1; echo pytest_rc=$? >> gpurun_out/pytest_gpu.log; tail -4 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench/kernels.py --only calib_cm_ab,calib_basic,calib_cm,peakfind,calib_image > gpurun_out/kernels3.log 2>&1; grep kernel gpurun_out/kernels3.log | cut -c1-200
timeout -k 10 240 python bench.py --steps 60 --warmup 10 > gpurun_out/bench3.log 2>&1; echo bench_rc=$?; tail -1 gpurun_out/bench3.log | cut -c1-400
timeout -k 10 240 python bench.py --steps 60 --warmup 10 --source device > gpurun_out/bench3d.log 2>&1; tail -1 gpurun_out/bench3d.log | cut -c1-400
