# Fused common-mode -> image kernel: bit-exact image tests + kernel timings
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
export PYTHONPATH=$R
O=$R/gpurun_out/cmimg
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest $R/tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "image" > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 $R/bench/kernels.py --only calib_cm,calib_cm_image --json-out $O/kernels.jsonl > $O/kernels.log 2>&1 || exit $?
cat $O/kernels.jsonl | cut -c1-120
