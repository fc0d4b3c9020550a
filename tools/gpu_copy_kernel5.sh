# --transport (N>1 per-rank steady state): copy kernel vs runtime blit copies, interleaved x3.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
mkdir -p gpurun_out/ck5
for rnd in 0 1 2; do
  for w in 32 0; do
    PSANA_RAY_COPY_KERNEL=$w timeout -k 10 240 python bench.py --transport --json-out gpurun_out/ck5/t_w${w}_r${rnd}.json > gpurun_out/ck5/t_w${w}_r${rnd}.log 2>&1 || exit $?
    python -c "import json;d=json.load(open('gpurun_out/ck5/t_w${w}_r${rnd}.json'));print('transport wgs=$w r$rnd',d['value'],d['extra']['queue_full_waits_rank0'])"
  done
done
