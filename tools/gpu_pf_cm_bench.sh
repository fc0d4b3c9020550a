# Kernel tests, peak-finder + common-mode probes, device-resident pipeline benches (calib, image)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
export PYTHONPATH=$R
O=$R/gpurun_out/pcb
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest $R/tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > $O/kernels_gpu.log 2>&1; rc=$?; tail -1 $O/kernels_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 $R/tools/pf_probe.py --repeat 2 > $O/pf.log 2>&1 || exit $?
grep us_per_frame $O/pf.log
timeout -k 10 200 python3 $R/tools/cm_probe.py --repeat 1 > $O/cm.log 2>&1 || exit $?
grep round $O/cm.log
cd $R
timeout -k 10 300 python3 bench.py --steps 300 --warmup 30 --source device > $O/bench_dev.json 2> $O/bench_dev.err || exit $?
cut -c1-200 $O/bench_dev.json
timeout -k 10 300 python3 bench.py --steps 300 --warmup 30 --source device --mode image > $O/bench_dev_image.json 2> $O/bench_dev_image.err || exit $?
cut -c1-200 $O/bench_dev_image.json
