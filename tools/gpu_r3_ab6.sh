# Fused CM -> image: lean placement loop (PR_CM_PLACE2) vs shipped -- CM + image tests, the
# production-shape tests, interleaved image-kernel probes, image pipeline benches
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
O=$R/gpurun_out/ab6
mkdir -p $O
SO=psana_ray_amd/_C.cpython-310-x86_64-linux-gnu.so
for v in base place2; do
  T=/tmp/tree_$v
  rm -rf $T && cp -r $R $T || exit 1
  [ $v = base ] || cp $R/variants/_C_$v.so $T/$SO || exit 1
  PYTHONPATH=$T timeout -k 10 400 python3 -u -m pytest $T/tests/test_kernels_gpu.py $T/tests/test_production_shapes_gpu.py -x -q --timeout 240 --timeout-method thread -k "common_mode or image or production" > $O/tests_$v.log 2>&1; rc=$?; echo "$v tests: $(tail -1 $O/tests_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
for r in 1 2; do
  for v in base place2; do
    PYTHONPATH=/tmp/tree_$v timeout -k 10 200 python3 /tmp/tree_$v/tools/cm_image_probe.py > $O/img_${v}_$r.log 2>&1 || exit $?
    echo "$v r$r $(tail -1 $O/img_${v}_$r.log | cut -c1-80)"
  done
done
for r in 1 2; do
  for v in base place2; do
    cd /tmp/tree_$v
    PYTHONPATH=/tmp/tree_$v timeout -k 10 300 python3 bench.py --steps 200 --warmup 5 --source device --mode image > $O/dev_image_${v}_$r.json 2> $O/dev_image_${v}_$r.err || exit $?
    python3 -c "import json;d=json.load(open('$O/dev_image_${v}_$r.json'));print('$v dev image r$r', d['value'])"
  done
done
# peak finder at rising candidate densities (thr_peak lowered): the overflow path's cost
cd $R
for t in 20 8 5 3; do
  PYTHONPATH=$R timeout -k 10 200 python3 tools/pf_probe.py --repeat 1 --thr $t > $O/pf_thr$t.log 2>&1 || exit $?
  tail -1 $O/pf_thr$t.log
done
