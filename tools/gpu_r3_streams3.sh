# Host-staged headline and device-resident pipelines per (compute streams, stream kind), with the
# staging stream placed like the compute streams; rounds interleaved.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/r3_streams3
mkdir -p $O
one() {  # tag, args...
  local tag=$1; shift
  timeout -k 10 240 python3 bench.py --steps ${STEPS:-200} --warmup 5 "$@" > $O/$tag.json 2> $O/$tag.err || return $?
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1].split('/')[-1], round(d['value']), d['ms_per_step'], d['extra'].get('producer_host_s_stage_acquire_launch_commit_total'))" $O/$tag.json
}
for r in 1 2; do
  for cfg in "1 shared" "3 dedicated" "2 dedicated" "1 dedicated"; do
    set -- $cfg
    one host_s$1_$2_r$r --steps 60 --compute-streams $1 --stream-kind $2 || exit $?
  done
  for cfg in "3 dedicated" "4 dedicated" "3 high"; do
    set -- $cfg
    one dev_s$1_$2_r$r --source device --compute-streams $1 --stream-kind $2 || exit $?
    one img_s$1_$2_r$r --source device --mode image --compute-streams $1 --stream-kind $2 || exit $?
  done
done
