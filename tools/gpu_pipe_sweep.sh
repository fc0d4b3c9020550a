# Device-resident pipeline sweep: producer chunk / consumer batch sizes (does the consumer's read of
# a just-written batch hit the 256-MB Infinity Cache when the batch fits?), producer-only rate
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=$R/gpurun_out/sweep
mkdir -p $O
for cfg in "32 32" "16 16" "8 8" "16 32" "32 16"; do
  set -- $cfg
  timeout -k 10 200 python3 bench.py --steps 300 --warmup 30 --source device --chunk $1 --batch $2 > $O/c$1_b$2.json 2> $O/c$1_b$2.err || exit $?
  echo "chunk $1 batch $2 $(cut -c1-120 $O/c$1_b$2.json)"
done
timeout -k 10 200 python3 bench.py --steps 300 --warmup 30 --source device --consumer none > $O/nocons.json 2> $O/nocons.err || exit $?
echo "no consumer $(cut -c1-120 $O/nocons.json)"
