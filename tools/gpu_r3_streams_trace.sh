# Kernel traces of the device-resident pipeline at 1 / 2 / 3 producer compute streams: hardware
# queue and stream of every kernel family, and how the common-mode launches overlap.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
export PYTHONPATH=$R
O=$R/gpurun_out/r3_strace
mkdir -p $O
for cs in ${CS:-1 2 3}; do
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/s$cs -o run -- python3 $R/bench.py --steps 60 --warmup 5 --source device --compute-streams $cs > $O/dev_s$cs.json 2> $O/dev_s$cs.err || exit $?
  python3 $R/tools/stream_trace.py $O/s$cs > $O/s$cs.summary.json || exit $?
  echo "s$cs $(grep -o '"value": [0-9.]*' $O/dev_s$cs.json)"
  cat $O/s$cs.summary.json
done
