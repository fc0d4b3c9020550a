# Same-box A/B of extension builds (replaces the per-round cm_ab / variants scripts).
#
# The shipped .so ("base") and every variants/_C_<name>.so (tools/build_variant.py: one source
# recompiled with a -D constant or a compiler flag) each get a copy of the tree; then, per variant:
#   1. bit-exact kernel tests (TESTK, default common_mode; NOTEST="v1 v2" skips them for a variant);
#   2. PROBE rounds interleaved across variants (base, v1, ..., base, v1, ...) so clock / thermal
#      drift hits every build alike (PROBE default tools/cm_probe.py, ROUNDS default 3);
#   3. PMC=1: one counter pass per variant over `cm_probe.py --pmc-pass` (VALU / LDS / conflicts);
#   4. PMCW=1: WRITE_SIZE and FETCH_SIZE passes per variant (HBM bytes per phase);
#   5. BENCH=1: device-resident calib + image pipelines per variant (BENCH_ROUNDS rounds).
# Outputs: gpurun_out/${OUT:-ab}/.  Every GPU step has its own timeout; a failure ends the script.
#   VARIANTS="net0" PMC=1 BENCH=1 gpurun -- bash tools/gpu_ab.sh
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
O=$R/gpurun_out/${OUT:-ab}
mkdir -p $O
SO=psana_ray_amd/_C.cpython-310-x86_64-linux-gnu.so
VS="base ${VARIANTS:-}"
PROBE=${PROBE:-tools/cm_probe.py}
for v in $VS; do
  T=/tmp/tree_$v
  rm -rf $T && cp -r $R $T || exit 1
  [ $v = base ] || cp $R/variants/_C_$v.so $T/$SO || exit 1
  case " ${NOTEST:-} " in *" $v "*) echo "$v: no tests"; continue;; esac
  PYTHONPATH=$T timeout -k 10 300 python3 -u -m pytest $T/tests/test_kernels_gpu.py -x -q --timeout 180 --timeout-method thread -k "${TESTK:-common_mode}" > $O/tests_$v.log 2>&1; rc=$?
  echo "$v tests: $(tail -1 $O/tests_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
for r in $(seq 1 ${ROUNDS:-3}); do
  for v in $VS; do
    PYTHONPATH=/tmp/tree_$v timeout -k 10 200 python3 /tmp/tree_$v/$PROBE ${PROBE_ARGS:---frames 64} > $O/probe_${v}_$r.log 2>&1 || exit $?
    echo "$v r$r $(grep -v -i warn $O/probe_${v}_$r.log | tail -1 | cut -c1-220)"
  done
done
if [ -n "${PMC:-}" ]; then
  for v in $VS; do
    timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE \
      --output-format csv -d $O/pmc_$v -o run -- python3 /tmp/tree_$v/tools/cm_probe.py --pmc-pass > $O/pmc_$v.log 2>&1 || { tail -5 $O/pmc_$v.log; exit 1; }
    python3 $R/tools/pmc_table.py --cm-phases $O/pmc_$v > $O/pmc_$v.txt 2>&1 || { cat $O/pmc_$v.txt; exit 1; }
    echo "$v pmc:"; cat $O/pmc_$v.txt
  done
fi
if [ -n "${PMCW:-}" ]; then   # HBM traffic per phase: WRITE_SIZE (2 TCC slots) and FETCH_SIZE (3) in separate passes
  for v in $VS; do
    for c in WRITE_SIZE FETCH_SIZE; do
      timeout -s KILL 90 rocprofv3 --pmc $c GRBM_GUI_ACTIVE --output-format csv -d $O/pmc${c}_$v -o run -- python3 /tmp/tree_$v/tools/cm_probe.py --pmc-pass > $O/pmc${c}_$v.log 2>&1 || { tail -5 $O/pmc${c}_$v.log; exit 1; }
      python3 $R/tools/pmc_table.py --cm-phases $O/pmc${c}_$v > $O/pmc${c}_$v.txt 2>&1 || { cat $O/pmc${c}_$v.txt; exit 1; }
      echo "$v $c:"; grep -v GRBM $O/pmc${c}_$v.txt
    done
  done
fi
if [ -n "${BENCH:-}" ]; then
  for br in $(seq 1 ${BENCH_ROUNDS:-1}); do
    for v in ${BENCH_VARIANTS:-$VS}; do
      cd /tmp/tree_$v
      for m in ${BENCH_MODES:-calib image}; do
        PYTHONPATH=/tmp/tree_$v timeout -k 10 300 python3 bench.py --steps 200 --warmup 5 --source device --mode $m > $O/dev_${m}_${v}_$br.json 2> $O/dev_${m}_${v}_$br.err || exit $?
        python3 -c "import json;d=json.load(open('$O/dev_${m}_${v}_$br.json'));print('$v dev $m r$br', d['value'])"
      done
    done
  done
fi
