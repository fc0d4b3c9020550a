# Round-3 entry check: GPU tests, smoke(), and the sustained-rate bench at short and long windows
# (--steps 20 and --steps 200 must agree within 2%; host-staged <= the H2D ceiling)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
export PYTHONPATH=$R
O=$R/gpurun_out/r3_entry
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest $R/tests -m gpu -x -q --timeout 180 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -1 $O/tests.log; [ $rc -eq 0 ] || exit $rc
cd $R && timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit $?
tail -1 $O/smoke.log
timeout -k 10 120 python3 bench/h2d.py > $O/h2d.jsonl 2>&1 || exit $?
for s in 20 200; do
  w=$((s / 4)); [ $w -gt 20 ] && w=20
  timeout -k 10 300 python3 bench.py --steps $s --warmup 5 > $O/host_$s.json 2> $O/host_$s.err || exit $?
  cut -c1-120 $O/host_$s.json
  timeout -k 10 300 python3 bench.py --steps $s --warmup 5 --source device > $O/dev_$s.json 2> $O/dev_$s.err || exit $?
  cut -c1-120 $O/dev_$s.json
done
timeout -k 10 300 python3 bench.py --steps 200 --warmup 5 --source device --mode image > $O/dev_image_200.json 2> $O/dev_image_200.err || exit $?
cut -c1-120 $O/dev_image_200.json
