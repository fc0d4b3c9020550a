# Round-3 queue semantics + production shapes on one MI355X: item-granular read-ahead, hand-back
# on close, keeper crash persistence, bit-exact 64/37-frame launches, peak-finder overflow
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
export PYTHONPATH=$R
O=$R/gpurun_out/r3_queue
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest $R/tests/test_production_shapes_gpu.py $R/tests/test_kernels_gpu.py $R/tests/test_pipeline_gpu.py -x -v --timeout 240 --timeout-method thread > $O/shapes.log 2>&1; rc=$?; tail -3 $O/shapes.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python3 -u -m pytest $R/tests/test_elastic_gpu.py -x -v --timeout 240 --timeout-method thread > $O/elastic.log 2>&1; rc=$?; tail -3 $O/elastic.log; [ $rc -eq 0 ] || exit $rc
