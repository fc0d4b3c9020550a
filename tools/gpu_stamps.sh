# Phase stamps of the epix10k2M common-mode kernel: the stamps build (variants/_C_stamps.so, built
# beforehand: python tools/build_variant.py stamps common_mode.hip -DPR_CM_STAMPS=1) in a copy of
# the tree, its bit-exact CM tests, then tools/cm_stamps.py (per-wave phase durations).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
O=$R/gpurun_out/${OUT:-cm_stamps}
mkdir -p $O
SO=psana_ray_amd/_C.cpython-310-x86_64-linux-gnu.so
T=/tmp/tree_stamps
rm -rf $T && cp -r $R $T && cp $R/variants/_C_stamps.so $T/$SO || exit 1
PYTHONPATH=$T timeout -k 10 300 python3 -u -m pytest $T/tests/test_kernels_gpu.py -x -q --timeout 180 --timeout-method thread -k common_mode > $O/tests.log 2>&1; rc=$?; echo "stamps tests: $(tail -1 $O/tests.log)"; [ $rc -eq 0 ] || exit $rc
PYTHONPATH=$T timeout -k 10 200 python3 $T/tools/cm_stamps.py --frames ${FRAMES:-64} --json-out $O/stamps.json > $O/stamps.log 2>&1 || exit $?
cat $O/stamps.log
