# Round 4: device-resident calib pipeline at 64-frame consumer batches: 4 / 5 / 6 producer compute
# streams (interleaved), image mode at 4 / 6.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=$R/gpurun_out/r4_sweep6
mkdir -p $O
b() {
  timeout -k 10 300 python bench.py --steps 200 --warmup 5 --source device "${@:2}" > $O/$1.json 2> $O/$1.err || { tail -20 $O/$1.err; return 1; }
  python -c "import json;d=json.load(open('$O/$1.json'));print('$1', d['value'])"
}
for r in 1 2 3; do
  b cs4_$r && b cs5_$r --compute-streams 5 && b cs6_$r --compute-streams 6 || exit 1
done
for r in 1 2; do
  b img4_$r --mode image && b img6_$r --mode image --compute-streams 6 || exit 1
done
