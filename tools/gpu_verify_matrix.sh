# Frame-check matrix on the one GPU of a box: bench.py --gpus 2 (two processes, device-resident, every
# VERIFY_EVERY-th routed frame checksummed and re-summed by its consumer) for each CASE
# (name:variant:ENV=VAL,...; variant "base" = the shipped .so, else variants/_C_<variant>.so).
# A run that reports mismatches exits 4; the matrix records it and goes on (only a crash or a
# timeout ends the script).  Outputs: gpurun_out/${OUT:-verify}/<case>.json + summary.txt.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
O=$R/gpurun_out/${OUT:-verify}
mkdir -p $O
SO=psana_ray_amd/_C.cpython-310-x86_64-linux-gnu.so
for c in $CASES; do
  v=$(echo $c | cut -d: -f2)
  T=/tmp/tree_$v
  [ -d $T ] && continue
  cp -r $R $T || exit 1
  [ $v = base ] || cp $R/variants/_C_$v.so $T/$SO || exit 1
done
for c in $CASES; do
  n=$(echo $c | cut -d: -f1); v=$(echo $c | cut -d: -f2); e=$(echo $c | cut -d: -f3 | tr ',' ' ')
  cd /tmp/tree_$v || exit 1
  env PSANA_RAY_AMD_VERIFY_EVERY=${VERIFY_EVERY:-4} $e timeout -k 10 200 python3 bench.py --gpus 2 --steps ${STEPS:-40} \
    --warmup 3 --source ${SRC:-device} --mode ${MODE:-calib} --gate-max-s 3 ${BENCH_ARGS:-} > $O/$n.json 2> $O/$n.err
  rc=$?
  case $rc in 0|4) ;; *) echo "$n: rc $rc"; tail -20 $O/$n.err; exit $rc;; esac
  python3 -c "
import json; d=json.load(open('$O/$n.json')); x=d['extra']; c=x['xgmi_phase']; f=x['frame_checks']
print('$n rc $rc: headline', d['value'], 'cross', c['frames_per_s'], 'direct', c.get('frames_direct_per_rank'),
      'verified', f['verified_per_rank'], 'mismatched', f['mismatched_per_rank'], 'last bad', f['last_bad_gevt_per_rank'],
      'acq', f['acquires_per_rank'])" | tee -a $O/summary.txt
done
