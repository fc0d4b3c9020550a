# Soak of the cross-process path on the one GPU of a box: 2 self-launched ranks, raw pool in HBM,
# EVERY frame that crosses processes checksummed by its producer and re-summed by its consumer
# (PSANA_RAY_AMD_VERIFY_EVERY=1), calib then image mode.  Any mismatch fails the run (exit 4).
#   OUT=r6_soak2 STEPS=6000 gpurun -- bash tools/gpu_soak.sh
# ALLOW_MISMATCH=1: a run that found mismatches (exit 4) is reported and the script goes on.
# Outputs: gpurun_out/${OUT:-soak}/{calib,image}.json + .err + summary.txt.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
O=$R/gpurun_out/${OUT:-soak}
mkdir -p $O
export PSANA_RAY_AMD_VERIFY_EVERY=1
for m in ${MODES:-calib image}; do
  n=${STEPS:-6000}
  [ $m = image ] && n=$((n / 2))
  timeout -k 10 ${STEP_TIMEOUT:-400} python3 bench.py --gpus 2 --steps $n --cross-steps $n --warmup 10 --source device \
    --mode $m > $O/$m.json 2> $O/$m.err
  rc=$?
  # rc 4 = the run completed and found mismatching frames (reported below); anything else ends here
  [ $rc -eq 0 ] || { [ $rc -eq 4 ] && [ -n "${ALLOW_MISMATCH:-}" ]; } || { tail -20 $O/$m.err; exit 1; }
  python3 -c "
import json
d = json.load(open('$O/$m.json')); x = d['extra']; c = x['xgmi_phase']; f = x['frame_checks']
print('$m', d['value'], 'cross', c['frames_per_s'], 'verified', f['frames_verified'], 'mismatched',
      f['frames_mismatched'], 'direct', c['frames_direct_per_rank'], 'sent', c['frames_sent_per_rank'], x['validation'])
" | tee -a $O/summary.txt
done
