# Common-mode iteration: bit-exact CM tests (unit + production launch shapes), cm_probe, device-
# resident pipelines (calib, image)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
export PYTHONPATH=$R
O=$R/gpurun_out/r3_cm
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest $R/tests/test_kernels_gpu.py $R/tests/test_production_shapes_gpu.py -x -q --timeout 180 --timeout-method thread -k "common_mode or image or production" > $O/tests.log 2>&1; rc=$?; tail -1 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 $R/tools/cm_probe.py --repeat 2 > $O/probe.log 2>&1 || exit $?
grep us_per $O/probe.log
timeout -k 10 200 python3 $R/tools/cm_image_probe.py > $O/image_probe.log 2>&1 || exit $?
grep -v warn $O/image_probe.log | tail -3
cd $R
for m in calib image; do
  timeout -k 10 300 python3 bench.py --steps 200 --warmup 5 --source device --mode $m > $O/dev_$m.json 2> $O/dev_$m.err || exit $?
  python3 -c "import json;d=json.load(open('$O/dev_$m.json'));e=d['extra'];print('dev $m', d['value'], e['production_frames_per_s'], e['consumer_frames_per_s'])"
done
