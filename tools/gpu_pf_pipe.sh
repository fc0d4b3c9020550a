# Peak-finder kernel tests + probe, then device-resident / host-staged pipeline benches per chunk x batch
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
export PYTHONPATH=$R
O=$R/gpurun_out/pfpipe
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest $R/tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > $O/kernels_gpu.log 2>&1; rc=$?; tail -1 $O/kernels_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 $R/tools/pf_probe.py --repeat 2 --frames 32 > $O/pf32.log 2>&1 || exit $?
timeout -k 10 200 python3 $R/tools/pf_probe.py --repeat 2 --frames 64 > $O/pf64.log 2>&1 || exit $?
grep us_per_frame $O/pf32.log $O/pf64.log
cd $R
for cfg in ${DEV_CFGS:-64x32}; do
  c=${cfg%x*}; b=${cfg#*x}
  timeout -k 10 200 python3 bench.py --steps 300 --warmup 30 --source device --chunk $c --batch $b > $O/dev_c${c}_b${b}.json 2> $O/dev_c${c}_b${b}.err || exit $?
  echo "device chunk $c batch $b $(cut -c90-140 $O/dev_c${c}_b${b}.json)"
done
for cfg in ${IMG_CFGS:-}; do
  c=${cfg%x*}; b=${cfg#*x}
  timeout -k 10 200 python3 bench.py --steps 300 --warmup 30 --source device --mode image --chunk $c --batch $b > $O/img_c${c}_b${b}.json 2> $O/img_c${c}_b${b}.err || exit $?
  echo "image chunk $c batch $b $(cut -c90-140 $O/img_c${c}_b${b}.json)"
done
for c in ${HOST_CHUNKS:-}; do
  timeout -k 10 200 python3 bench.py --chunk $c > $O/host_c${c}.json 2> $O/host_c${c}.err || exit $?
  echo "host chunk $c $(cut -c90-140 $O/host_c${c}.json)"
done
