# A/B of the producer's compute streams x stream kind on one box (device-resident calib / image
# pipelines; host-staged headline last), rounds interleaved.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/r3_streams2
mkdir -p $O
one() {  # tag, args...
  local tag=$1; shift
  timeout -k 10 240 python3 bench.py --steps ${STEPS:-200} --warmup 5 "$@" > $O/$tag.json 2> $O/$tag.err || return $?
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1].split('/')[-1], round(d['value']), d['ms_per_step'])" $O/$tag.json
}
for r in 1 2 3; do
  for cfg in ${CFGS:-"1 shared" "1 dedicated" "2 dedicated" "3 dedicated"}; do
    set -- $cfg
    one dev_s$1_$2_r$r --source device --compute-streams $1 --stream-kind $2 || exit $?
    one img_s$1_$2_r$r --source device --mode image --compute-streams $1 --stream-kind $2 || exit $?
  done
done
for cfg in ${HCFGS:-"1 shared" "2 dedicated"}; do
  set -- $cfg
  one host_s$1_$2 --compute-streams $1 --stream-kind $2 || exit $?
done
