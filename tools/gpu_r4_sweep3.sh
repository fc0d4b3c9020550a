# Round 4: interleaved A/B (4 rounds) of the device-resident calib pipeline: shipped vs 4 producer
# compute streams vs consumer batch 64 vs both.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=$R/gpurun_out/r4_sweep3
mkdir -p $O
b() {
  timeout -k 10 300 python bench.py --steps 200 --warmup 5 --source device "${@:2}" > $O/$1.json 2> $O/$1.err || { tail -20 $O/$1.err; return 1; }
  python -c "import json;d=json.load(open('$O/$1.json'));print('$1', d['value'])"
}
for r in 1 2 3 4; do
  b base_$r && b cs4_$r --compute-streams 4 && b b64_$r --batch 64 && b both_$r --compute-streams 4 --batch 64 || exit 1
done
for r in 1 2; do
  b img_base_$r --mode image && b img_cs4_$r --mode image --compute-streams 4 || exit 1
done
