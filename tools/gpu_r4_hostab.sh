# Round 4: host-staged headline, consumer batch 32 vs 64, interleaved, the driver's default window
# (no flags = 20 steps) and 200 steps.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=$R/gpurun_out/r4_hostab
mkdir -p $O
b() {
  timeout -k 10 300 python bench.py "${@:2}" > $O/$1.json 2> $O/$1.err || { tail -20 $O/$1.err; return 1; }
  python -c "import json;d=json.load(open('$O/$1.json'));print('$1', d['value'], d['steps'])"
}
for r in 1 2 3; do
  b d64_$r && b d32_$r --batch 32 && b l64_$r --steps 200 && b l32_$r --steps 200 --batch 32 || exit 1
done
