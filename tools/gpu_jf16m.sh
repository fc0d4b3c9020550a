# BASELINE config 4: Jungfrau-16M (32 x 512 x 1024) frames, queue_size 400000 (logical; physical HBM
# slots capped by free memory), host-staged and device-resident, per producer chunk
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=$R/gpurun_out/jf16m
mkdir -p $O
for c in ${CHUNKS:-8 16}; do
  timeout -k 10 240 python3 bench.py --detector jungfrau16M --queue-size 400000 --batch 8 --chunk $c --steps 150 --warmup 40 > $O/host_c$c.json 2> $O/host_c$c.err || exit $?
  echo "host chunk $c $(cut -c90-140 $O/host_c$c.json)"
  timeout -k 10 240 python3 bench.py --detector jungfrau16M --queue-size 400000 --batch 8 --chunk $c --steps 150 --warmup 40 --source device --pool-frames 16 > $O/dev_c$c.json 2> $O/dev_c$c.err || exit $?
  echo "device chunk $c $(cut -c90-140 $O/dev_c$c.json)"
done
