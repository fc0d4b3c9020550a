# A/B of extension builds: the shipped .so and each variants/_C_<name>.so (built here with a
# different compile-time constant), each in its own copy of the tree: image-mode kernel tests,
# then the probe given in PROBE (default: tools/cm_image_probe.py)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
O=$R/gpurun_out/variants
mkdir -p $O
SO=psana_ray_amd/_C.cpython-310-x86_64-linux-gnu.so
PROBE=${PROBE:-tools/cm_image_probe.py}
for v in base ${VARIANTS:-}; do
  T=/tmp/tree_$v
  rm -rf $T && cp -r $R $T || exit 1
  [ $v = base ] || cp $R/variants/_C_$v.so $T/$SO || exit 1
  export PYTHONPATH=$T
  timeout -k 10 200 python3 -u -m pytest $T/tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "${TESTK:-image}" > $O/tests_$v.log 2>&1; rc=$?; echo "$v tests: $(tail -1 $O/tests_$v.log)"; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 200 python3 $T/$PROBE > $O/probe_$v.log 2>&1 || exit $?
  echo "$v $(grep -v warning $O/probe_$v.log | tail -2)"
done
