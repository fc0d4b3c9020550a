# Kernel trace of the device-resident pipeline per build: does the consumer's peak finder run
# concurrently with the producer's common mode (co-residency)?
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
O=$R/gpurun_out/overlap
mkdir -p $O
SO=psana_ray_amd/_C.cpython-310-x86_64-linux-gnu.so
for v in base ${VARIANTS:-cm3}; do
  T=/tmp/tree_$v
  rm -rf $T && cp -r $R $T || exit 1
  [ $v = base ] || cp $R/variants/_C_$v.so $T/$SO || exit 1
  export PYTHONPATH=$T
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o run -- python3 $T/bench.py --steps 100 --warmup 5 --source device > $O/dev_$v.json 2> $O/dev_$v.err || exit $?
  echo "$v $(python3 $R/tools/kernel_overlap.py $O/$v) $(cut -c1-100 $O/dev_$v.json | grep -o 'value.: [0-9.]*')"
done
