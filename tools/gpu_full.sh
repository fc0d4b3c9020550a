# Full GPU pass: tests, smoke, per-kernel device times, pipeline benches (1 GPU)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
mkdir -p gpurun_out/full
timeout -k 10 900 python -m pytest tests -m gpu -q > gpurun_out/full/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/full/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.build(); g.smoke(); print('SMOKE_OK')" > gpurun_out/full/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/full/smoke.log
timeout -k 10 600 python bench/kernels.py --json-out gpurun_out/full/kernels.jsonl > gpurun_out/full/kernels.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --json-out gpurun_out/full/bench_n1_host.json > gpurun_out/full/bench_host.log 2>&1 || exit $?
tail -1 gpurun_out/full/bench_host.log | cut -c1-200
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --source device --json-out gpurun_out/full/bench_n1_device.json > gpurun_out/full/bench_dev.log 2>&1 || exit $?
tail -1 gpurun_out/full/bench_dev.log | cut -c1-200
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --mode image --json-out gpurun_out/full/bench_n1_image.json > gpurun_out/full/bench_img.log 2>&1 || exit $?
tail -1 gpurun_out/full/bench_img.log | cut -c1-200
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --mode image --source device --json-out gpurun_out/full/bench_n1_image_device.json > gpurun_out/full/bench_img_dev.log 2>&1 || exit $?
tail -1 gpurun_out/full/bench_img_dev.log | cut -c1-200
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --loopback --json-out gpurun_out/full/bench_n1_loopback.json > gpurun_out/full/bench_lb.log 2>&1 || exit $?
tail -1 gpurun_out/full/bench_lb.log | cut -c1-200
timeout -k 10 600 python bench.py --detector jungfrau16M --queue-size 400000 --steps 150 --warmup 40 --batch 8 --chunk 8 --pool-frames 16 --json-out gpurun_out/full/bench_jf16m.json > gpurun_out/full/bench_jf.log 2>&1 || exit $?
tail -1 gpurun_out/full/bench_jf.log | cut -c1-200
timeout -k 10 120 python bench/config1_cpu_queue.py > gpurun_out/full/config1.json 2>&1 || exit $?
cat gpurun_out/full/config1.json
