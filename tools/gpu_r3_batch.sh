# Consumer batch 32 vs 64 frames per peak-finder launch (bench --batch), interleaved, same box
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=$R/gpurun_out/batch
mkdir -p $O
for r in 1 2; do
  for b in 32 64; do
    for src in device host; do
      timeout -k 10 300 python3 bench.py --steps 100 --warmup 5 --source $src --batch $b > $O/${src}_b${b}_$r.json 2> $O/${src}_b${b}_$r.err || exit $?
      python3 -c "import json;d=json.load(open('$O/${src}_b${b}_$r.json'));print('$src b$b r$r', d['value'])"
    done
    timeout -k 10 300 python3 bench.py --steps 100 --warmup 5 --source device --mode image --batch $b > $O/img_b${b}_$r.json 2> $O/img_b${b}_$r.err || exit $?
    python3 -c "import json;d=json.load(open('$O/img_b${b}_$r.json'));print('img b$b r$r', d['value'])"
  done
done
