# Peak-finder scratch path: kernel tests + device-resident and host-staged benches
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
export PYTHONPATH=$R
O=$R/gpurun_out/pfq
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest $R/tests/test_kernels_gpu.py $R/tests/test_pipeline_gpu.py -x -q --timeout 120 --timeout-method thread -k "peakfind or pipeline or consumer" > $O/tests.log 2>&1; rc=$?; tail -1 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 $R/bench.py --steps 200 --warmup 20 --source device > $O/bench_dev.json 2> $O/bench_dev.err || exit $?
tail -1 $O/bench_dev.json | cut -c1-140
timeout -k 10 200 python3 $R/bench.py --steps 60 --warmup 10 > $O/bench_host.json 2> $O/bench_host.err || exit $?
tail -1 $O/bench_host.json | cut -c1-140
