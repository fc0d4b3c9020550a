# Peak-finder A/B (tools/pf_probe.py variants), then the device-resident pipeline bench
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
export PYTHONPATH=$R
O=$R/gpurun_out/pfab
mkdir -p $O
timeout -k 10 200 python3 $R/tools/pf_probe.py --repeat 2 --frames ${PF_FRAMES:-32} > $O/pf.log 2>&1 || exit $?
grep us_per_frame $O/pf.log
cd $R
for cfg in ${BENCH_CFGS:-}; do
  c=${cfg%x*}; b=${cfg#*x}
  timeout -k 10 200 python3 bench.py --steps 300 --warmup 30 --source device --chunk $c --batch $b > $O/c${c}_b${b}.json 2> $O/c${c}_b${b}.err || exit $?
  echo "chunk $c batch $b $(cut -c90-140 $O/c${c}_b${b}.json)"
done
