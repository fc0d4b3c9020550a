# Round 4: device-resident calib pipeline -- consumer batch 64 and producer compute-stream count.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=$R/gpurun_out/r4_sweep2
mkdir -p $O
b() {
  timeout -k 10 300 python bench.py --steps 200 --warmup 5 --source device "${@:2}" > $O/$1.json 2> $O/$1.err || { tail -20 $O/$1.err; return 1; }
  python -c "import json;d=json.load(open('$O/$1.json'));print('$1', d['value'])"
}
for r in 1 2; do
  b base_$r && b b64_$r --batch 64 && b cs2_$r --compute-streams 2 && b cs4_$r --compute-streams 4 || exit 1
done
