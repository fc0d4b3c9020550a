# Kernel traces of the device-resident pipeline per (producer compute streams, stream kind):
# hardware queue and stream of every kernel family, and how the common-mode launches overlap.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
export PYTHONPATH=$R
O=$R/gpurun_out/r3_strace2
mkdir -p $O
for cfg in ${CFGS:-"1 shared" "1 dedicated" "2 dedicated" "3 dedicated"}; do
  set -- $cfg
  t=s$1_$2
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/$t -o run -- python3 $R/bench.py --steps 60 --warmup 5 --source device --compute-streams $1 --stream-kind $2 > $O/dev_$t.json 2> $O/dev_$t.err || exit $?
  python3 $R/tools/stream_trace.py $O/$t > $O/$t.summary.json || exit $?
  python3 - $O/$t.summary.json $O/dev_$t.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); v = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])["value"]
print(sys.argv[1].split("/")[-1], round(v), {k: x for k, x in d.items() if k != "placement"})
for p in d["placement"]:
    if p["kernel"] in ("calib_cm", "peakfind"):
        print("   ", p)
PY
done
