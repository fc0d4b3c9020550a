# A/B of the producer's compute streams (ProducerEngine.set_compute_streams) on one box:
# device-resident calib / image pipelines and the host-staged headline, rounds interleaved.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/r3_streams
mkdir -p $O
one() {  # tag, args...
  local tag=$1; shift
  timeout -k 10 240 python3 bench.py --steps ${STEPS:-200} --warmup 5 "$@" > $O/$tag.json 2> $O/$tag.err || return $?
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1].split('/')[-1], round(d['value']), d['ms_per_step'])" $O/$tag.json
}
for r in 1 2; do
  for cs in ${CS:-1 2 3}; do
    one dev_c64_s${cs}_r$r --source device --chunk 64 --compute-streams $cs || exit $?
    one dev_c32_s${cs}_r$r --source device --chunk 32 --compute-streams $cs || exit $?
    one img_c64_s${cs}_r$r --source device --mode image --chunk 64 --compute-streams $cs || exit $?
  done
done
for cs in 1 2; do one host_s${cs} --compute-streams $cs || exit $?; done
