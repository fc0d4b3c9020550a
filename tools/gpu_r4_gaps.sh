# Round 4: zero-filled HBM rings -- the image pipeline skips the per-frame gap fill.  Tests first
# (bit-exact image frames through the engine with ring reuse), then a same-box A/B of the
# device-resident image pipeline with and without the skip (interleaved), plus calib as a control.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=$R/gpurun_out/r4_gaps
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_production_shapes_gpu.py tests/test_pipeline_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -1
b() {
  timeout -k 10 300 python bench.py --steps 200 --warmup 5 --source device "${@:2}" > $O/$1.json 2> $O/$1.err || { tail -20 $O/$1.err; return 1; }
  python -c "import json;d=json.load(open('$O/$1.json'));print('$1', d['value'])"
}
for r in 1 2 3; do
  b img_skip_$r --mode image && b img_fill_$r --mode image --gap-fill || exit 1
done
b calib_1 || exit 1
