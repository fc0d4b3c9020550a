# Same-box A/B of common-mode builds: each variant's bit-exact CM tests, then cm_probe rounds
# interleaved across variants (base, v1, v2, base, v1, v2, ...) so clock / thermal drift hits all
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
O=$R/gpurun_out/cm_ab
mkdir -p $O
SO=psana_ray_amd/_C.cpython-310-x86_64-linux-gnu.so
VS="base ${VARIANTS:-}"
for v in $VS; do
  T=/tmp/tree_$v
  rm -rf $T && cp -r $R $T || exit 1
  [ $v = base ] || cp $R/variants/_C_$v.so $T/$SO || exit 1
  case " ${NOTEST:-} " in *" $v "*) echo "$v: timing probe, no tests"; continue;; esac
  PYTHONPATH=$T timeout -k 10 300 python3 -u -m pytest $T/tests/test_kernels_gpu.py -x -q --timeout 180 --timeout-method thread -k "${TESTK:-common_mode}" > $O/tests_$v.log 2>&1; rc=$?; echo "$v tests: $(tail -1 $O/tests_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
for r in 1 2 3; do
  for v in $VS; do
    PYTHONPATH=/tmp/tree_$v timeout -k 10 200 python3 /tmp/tree_$v/tools/cm_probe.py --frames ${FRAMES:-64} > $O/probe_${v}_$r.log 2>&1 || exit $?
    echo "$v r$r $(grep -o 'flags0.*' $O/probe_${v}_$r.log)"
  done
done
if [ -n "${BENCH:-}" ]; then
  for br in $(seq 1 ${BENCH_ROUNDS:-1}); do
  for v in ${BENCH_VARIANTS:-$VS}; do
    cd /tmp/tree_$v
    for m in calib image; do
      PYTHONPATH=/tmp/tree_$v timeout -k 10 300 python3 bench.py --steps 200 --warmup 5 --source device --mode $m > $O/dev_${m}_${v}_$br.json 2> $O/dev_${m}_${v}_$br.err || exit $?
      python3 -c "import json;d=json.load(open('$O/dev_${m}_${v}_$br.json'));print('$v dev $m r$br', d['value'])"
    done
  done
  done
fi
