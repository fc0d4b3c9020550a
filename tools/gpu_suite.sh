# Full GPU test suite, then the steady-state kernel census of the device-resident bench
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
export PYTHONPATH=$R
O=$R/gpurun_out/suite
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest $R/tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $R/bench.py --steps 60 --warmup 10 --source device > $O/bench.json 2> $O/bench.err || exit $?
tail -1 $O/bench.json | cut -c1-160
