# Round-3 kernel iteration: peak-finder consumer on two alternating streams (tests + device-resident
# benches), then the common-mode scheduler-strategy variants (bit-exact tests + cm_probe)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
export PYTHONPATH=$R
O=$R/gpurun_out/r3_kernels
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest $R/tests/test_pipeline_gpu.py $R/tests/test_kernels_gpu.py -x -q --timeout 180 --timeout-method thread -k "peakfind or pipeline or consumer" > $O/tests.log 2>&1; rc=$?; tail -1 $O/tests.log; [ $rc -eq 0 ] || exit $rc
cd $R
for m in calib image; do
  timeout -k 10 300 python3 bench.py --steps 200 --warmup 5 --source device --mode $m > $O/dev_$m.json 2> $O/dev_$m.err || exit $?
  python3 -c "import json;d=json.load(open('$O/dev_$m.json'));e=d['extra'];print('dev $m', d['value'], e['production_frames_per_s'], e['consumer_frames_per_s'])"
done
VARIANTS="maxilp maxmem" PROBE=tools/cm_probe.py TESTK=common_mode bash tools/gpu_variants.sh
