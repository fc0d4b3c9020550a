# Round 4, peak finder on hit-rich frames: same-box A/B of peak-finder builds (tests of each, then
# tools/pf_probe.py at the default threshold and at thr 5 = 2 % candidates, interleaved rounds).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
O=$R/gpurun_out/${OUT:-r4_pf}
mkdir -p $O
SO=psana_ray_amd/_C.cpython-310-x86_64-linux-gnu.so
VS="base ${VARIANTS:-}"
for v in $VS; do
  T=/tmp/tree_$v
  rm -rf $T && cp -r $R $T || exit 1
  [ $v = base ] || cp $R/variants/_C_$v.so $T/$SO || exit 1
  case " ${NOTEST:-} " in *" $v "*) echo "$v: timing probe, no tests"; continue;; esac
  PYTHONPATH=$T timeout -k 10 300 python3 -u -m pytest $T/tests/test_kernels_gpu.py $T/tests/test_production_shapes_gpu.py -x -q --timeout 180 --timeout-method thread -k "peakfind" > $O/tests_$v.log 2>&1; rc=$?; echo "$v tests: $(tail -1 $O/tests_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
for r in 1 2; do
  for v in $VS; do
    for thr in default 5; do
      A=""; [ $thr = default ] || A="--thr $thr"
      PYTHONPATH=/tmp/tree_$v timeout -k 10 200 python3 /tmp/tree_$v/tools/pf_probe.py --repeat 2 --total $A > $O/pf_${v}_${thr}_$r.log 2>&1 || exit $?
      echo "$v thr=$thr r$r $(grep -o '"same_counts.*' $O/pf_${v}_${thr}_$r.log | tail -1)"
    done
  done
done
