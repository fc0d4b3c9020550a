# Round 4: consumer (peak-finder) stream count 2 vs 3 at the new defaults (interleaved).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=$R/gpurun_out/r4_sweep5
mkdir -p $O
b() {
  timeout -k 10 300 python bench.py --steps 200 --warmup 5 --source device "${@:2}" > $O/$1.json 2> $O/$1.err || { tail -20 $O/$1.err; return 1; }
  python -c "import json;d=json.load(open('$O/$1.json'));print('$1', d['value'])"
}
for r in 1 2 3; do
  b c2_$r && b c3_$r --consumer-streams 3 || exit 1
done
