# Device-resident pipeline vs producer chunk / consumer batch: does a smaller hand-off (the
# consumer's peak finder reading frames the producer just wrote, still in the 256 MiB Infinity
# Cache) beat the 64-frame chunk?  One bench per config, each under its own limit.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/r3_chunks
mkdir -p $O
for cfg in ${CFGS:-"64 32" "32 32" "16 16" "8 8" "16 32" "8 32"}; do
  set -- $cfg
  for mode in ${MODES:-calib}; do
    timeout -k 10 240 python3 bench.py --source device --mode $mode --chunk $1 --batch $2 --steps ${STEPS:-200} --warmup 5 \
      > $O/${mode}_c$1_b$2.json 2> $O/${mode}_c$1_b$2.err || exit $?
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1].split('/')[-1], round(d['value']), d['ms_per_step'])" $O/${mode}_c$1_b$2.json
  done
done
