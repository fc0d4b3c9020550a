# Image write-out rework (full chunks / ragged ends / preloaded gap table): CM + image tests, the
# production-shape tests, kernel probes (frame + image), pipeline benches; VALU probe w3busy (idle
# fourth wave busy during the row phase, timing only); stamps
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
O=$R/gpurun_out/ab3
mkdir -p $O
timeout -k 10 60 $R/tools/valu_rate_bin > $O/valu_rate.jsonl 2>&1 || exit $?
cat $O/valu_rate.jsonl
PYTHONPATH=$R timeout -k 10 400 python3 -u -m pytest $R/tests/test_production_shapes_gpu.py -x -q --timeout 240 --timeout-method thread > $O/shapes.log 2>&1; rc=$?; echo "shapes: $(tail -1 $O/shapes.log)"; [ $rc -eq 0 ] || exit $rc
PYTHONPATH=$R timeout -k 10 200 python3 $R/tools/cm_image_probe.py > $O/image_probe.log 2>&1 || exit $?
tail -1 $O/image_probe.log
VARIANTS="w3busy" NOTEST="w3busy" TESTK="common_mode or image" BENCH=1 BENCH_VARIANTS="base" bash $R/tools/gpu_cm_ab.sh || exit $?
bash $R/tools/gpu_cm_stamps.sh || exit $?
