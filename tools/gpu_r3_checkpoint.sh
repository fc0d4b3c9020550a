# Round-3 checkpoint on a fresh box: full GPU suite, smoke(), the driver's default bench line,
# device-resident calib / image benches
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
export PYTHONPATH=$R
O=$R/gpurun_out/${CKPT:-r3_ckpt}
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest $R/tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -1 $O/tests.log; [ $rc -eq 0 ] || exit $rc
cd $R && timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit $?
tail -1 $O/smoke.log
timeout -k 10 300 python3 bench.py > $O/bench_default.json 2> $O/bench_default.err || exit $?
cut -c1-140 $O/bench_default.json
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || exit $?
cut -c1-140 $O/bench_driver.json
timeout -k 10 300 python3 bench.py --steps 200 --warmup 5 --source device > $O/bench_dev.json 2> $O/bench_dev.err || exit $?
cut -c1-140 $O/bench_dev.json
timeout -k 10 300 python3 bench.py --steps 200 --warmup 5 --source device --mode image > $O/bench_dev_image.json 2> $O/bench_dev_image.err || exit $?
cut -c1-140 $O/bench_dev_image.json
