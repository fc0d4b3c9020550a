# Final tree check: full GPU suite (must exit 0), smoke, peak finder at default and hit-rich
# thresholds, fused image kernel, device-resident benches, the driver's N=1 line
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
export PYTHONPATH=$R
O=$R/gpurun_out/r3_final2
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest $R/tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -1 $O/tests.log; [ $rc -eq 0 ] || { tail -40 $O/tests.log; exit $rc; }
cd $R
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit $?
tail -1 $O/smoke.log
for t in 20 8; do
  timeout -k 10 200 python3 tools/pf_probe.py --repeat 1 --thr $t > $O/pf_thr$t.log 2>&1 || exit $?
  tail -1 $O/pf_thr$t.log
done
timeout -k 10 200 python3 tools/cm_image_probe.py > $O/image_probe.log 2>&1 || exit $?
tail -1 $O/image_probe.log | cut -c1-120
for m in calib image; do
  timeout -k 10 300 python3 bench.py --steps 200 --warmup 5 --source device --mode $m > $O/bench_dev_$m.json 2> $O/bench_dev_$m.err || exit $?
  cut -c1-130 $O/bench_dev_$m.json
done
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench_host_20.json 2> $O/bench_host_20.err || exit $?
cut -c1-130 $O/bench_host_20.json
