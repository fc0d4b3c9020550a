# Device-resident pipeline A/B over the peak finder's grid size (PSANA_RAY_PF_BLOCKS), interleaved.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
mkdir -p gpurun_out/pfpipe
for rnd in 0 1; do
  for b in 0 1024 2048 4096 8192; do
    PSANA_RAY_PF_BLOCKS=$b timeout -k 10 200 python bench.py --steps 100 --warmup 10 --source device \
      --json-out gpurun_out/pfpipe/b${b}_r${rnd}.json > gpurun_out/pfpipe/b${b}_r${rnd}.log 2>&1 || exit $?
    python -c "import json;d=json.load(open('gpurun_out/pfpipe/b${b}_r${rnd}.json'));print('blocks=$b r$rnd',d['value'])"
  done
done
