# Pipeline sweep: bench.py runs over a list of argument sets, interleaved over ROUNDS rounds so clock
# and thermal drift hits every set alike.  SETS: ';'-separated "name:args" entries (leading
# NAME=VALUE tokens of args are the run's environment), e.g.
#   SETS="cs4:--compute-streams 4;cs5:--compute-streams 5;img:--mode image" ROUNDS=3 \
#   gpurun -- bash tools/gpu_sweep.sh
# Every set shares BASE (default: the device-resident pipeline, 200 steps).  One JSON per run under
# gpurun_out/${OUT:-sweep}/, one "name round value" line each.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=$R/gpurun_out/${OUT:-sweep}
mkdir -p $O
BASE=${BASE:---steps 200 --warmup 5 --source device}
IFS=';' read -ra SS <<< "${SETS:-default:}"
for r in $(seq 1 ${ROUNDS:-1}); do
  for s in "${SS[@]}"; do
    name=${s%%:*}; args=${s#*:}
    envs=(); rest=()   # leading NAME=VALUE tokens of a set are environment for its run
    for t in $args; do if [[ $t =~ ^[A-Z_][A-Z0-9_]*= ]]; then envs+=("$t"); else rest+=("$t"); fi; done
    env "${envs[@]}" timeout -k 10 300 python3 bench.py $BASE "${rest[@]}" > $O/${name}_$r.json 2> $O/${name}_$r.err || { tail -20 $O/${name}_$r.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/${name}_$r.json'));print('$name', $r, d['value'])"
  done
done
