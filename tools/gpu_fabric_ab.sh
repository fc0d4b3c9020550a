# 2-rank fabric A/B on the one GPU of a box: bench.py --gpus 2 (self-launched, both windows:
# headline + route=remote_only cross window) for every CASE, rounds interleaved so drift hits every
# case alike.  A CASE is name:variant:ENV=VAL,ENV=VAL[:--bench-arg,value] (variant "base" = the
# shipped .so, else variants/_C_<variant>.so from tools/build_variant.py).
#   CASES="base:base: norel:norel: noacq:base:PSANA_RAY_AMD_FABRIC_ACQUIRE=0" SRC=device \
#   OUT=r6_fab gpurun -- bash tools/gpu_fabric_ab.sh
# Outputs: gpurun_out/${OUT:-fabric_ab}/<case>_<round>.json + summary.txt.  Each run has its own
# timeout; a failure ends the script.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
O=$R/gpurun_out/${OUT:-fabric_ab}
mkdir -p $O
SO=psana_ray_amd/_C.cpython-310-x86_64-linux-gnu.so
CASES=${CASES:-"base:base:"}
for c in $CASES; do
  v=$(echo $c | cut -d: -f2)
  T=/tmp/tree_$v
  [ -d $T ] && continue
  cp -r $R $T || exit 1
  [ $v = base ] || cp $R/variants/_C_$v.so $T/$SO || exit 1
done
for r in $(seq 1 ${ROUNDS:-2}); do
  for c in $CASES; do
    n=$(echo $c | cut -d: -f1); v=$(echo $c | cut -d: -f2); e=$(echo $c | cut -d: -f3 | tr ',' ' ')
    a=$(echo $c | cut -s -d: -f4 | tr ',' ' ')
    cd /tmp/tree_$v || exit 1
    env $e timeout -k 10 300 python3 bench.py --gpus 2 --steps ${STEPS:-100} --warmup 5 --source ${SRC:-device} \
      --mode ${MODE:-calib} ${BENCH_ARGS:-} $a > $O/${n}_$r.json 2> $O/${n}_$r.err || { tail -20 $O/${n}_$r.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$O/${n}_$r.json')); x=d['extra']; c=x['xgmi_phase']; f=x['frame_checks']
print('$n round $r: headline', d['value'], 'cross', c['frames_per_s'], 'direct', c.get('frames_direct_per_rank'),
      'sent', c.get('frames_sent_per_rank'), 'verified', f['frames_verified'], 'mismatched', f['frames_mismatched'],
      'valid', x['validation'])" | tee -a $O/summary.txt
  done
done
