# Self-resetting peak-finder outputs: kernel + pipeline tests, then the steady-state kernel census
# of the device-resident bench (only pr:: kernels expected)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
export PYTHONPATH=$R
O=$R/gpurun_out/pf
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest $R/tests/test_kernels_gpu.py $R/tests/test_pipeline_gpu.py -x -q --timeout 120 --timeout-method thread -k "peakfind or pipeline or consumer" > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $R/bench.py --steps 60 --warmup 10 --source device > $O/bench.json 2> $O/bench.err || exit $?
tail -1 $O/bench.json | cut -c1-160
