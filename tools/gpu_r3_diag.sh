# Round-3 diagnosis call: CM phase stamps (stamps build), peak finder with / without the running
# total, then the full GPU suite under faulthandler (LAST: a crash at interpreter exit ends the call)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
O=$R/gpurun_out/r3_diag
mkdir -p $O
bash $R/tools/gpu_cm_stamps.sh || exit $?
for t in "" "--total"; do
  PYTHONPATH=$R timeout -k 10 200 python3 $R/tools/pf_probe.py --repeat 2 $t > $O/pf$t.log 2>&1 || exit $?
  echo "pf $t: $(tail -1 $O/pf$t.log)"
done
PYTHONPATH=$R timeout -k 10 900 python3 -X faulthandler -u -m pytest $R/tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -5 $O/tests.log
grep -n -A40 "Fatal Python error" $O/tests.log | head -80
exit $rc
