# Round 4: host-staged headline at consumer batch 32 vs 64 (interleaved), device-resident calib /
# image at 4 compute streams + batch 64 vs the round-3 shape.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=$R/gpurun_out/r4_sweep4
mkdir -p $O
b() {
  timeout -k 10 300 python bench.py --steps 200 --warmup 5 "${@:2}" > $O/$1.json 2> $O/$1.err || { tail -20 $O/$1.err; return 1; }
  python -c "import json;d=json.load(open('$O/$1.json'));print('$1', d['value'])"
}
for r in 1 2 3; do
  b host32_$r && b host64_$r --batch 64 || exit 1
done
for r in 1 2; do
  b img_base_$r --source device --mode image && b img_new_$r --source device --mode image --compute-streams 4 --batch 64 || exit 1
done
