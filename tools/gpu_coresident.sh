# Producer/consumer kernel co-residency A/B: the shipped build (common mode at 4 workgroups per CU)
# against variants (e.g. cm3: 3 per CU, a quarter of every CU left for the consumer's peak finder):
# common-mode bit-exact tests, cm_probe (the kernel alone), device-resident pipeline (calib, image)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
O=$R/gpurun_out/coresident
mkdir -p $O
SO=psana_ray_amd/_C.cpython-310-x86_64-linux-gnu.so
for v in base ${VARIANTS:-cm3}; do
  T=/tmp/tree_$v
  rm -rf $T && cp -r $R $T || exit 1
  [ $v = base ] || cp $R/variants/_C_$v.so $T/$SO || exit 1
  export PYTHONPATH=$T
  timeout -k 10 300 python3 -u -m pytest $T/tests/test_kernels_gpu.py $T/tests/test_production_shapes_gpu.py -x -q --timeout 180 --timeout-method thread -k "common_mode" > $O/tests_$v.log 2>&1; rc=$?; echo "$v tests: $(tail -1 $O/tests_$v.log)"; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 200 python3 $T/tools/cm_probe.py > $O/probe_$v.log 2>&1 || exit $?
  echo "$v $(grep us_per $O/probe_$v.log | tail -1)"
  cd $T
  for m in calib image; do
    timeout -k 10 300 python3 bench.py --steps 200 --warmup 5 --source device --mode $m > $O/dev_${m}_$v.json 2> $O/dev_${m}_$v.err || exit $?
    python3 -c "import json;d=json.load(open('$O/dev_${m}_$v.json'));e=d['extra'];print('$v dev $m', d['value'], e['production_frames_per_s'], e['consumer_frames_per_s'])"
  done
  cd /tmp
done
