# Copy kernel as the default staging path: full GPU suite, headline (kernel vs blit, interleaved),
# file sources (zero-copy mapping and pread staging).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
mkdir -p gpurun_out/ck2
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/ck2/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/ck2/pytest_gpu.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/ck2/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/ck2/smoke.log
for rnd in 0 1; do
  for w in 32 0; do
    PSANA_RAY_COPY_KERNEL=$w timeout -k 10 200 python bench.py --json-out gpurun_out/ck2/host_w${w}_r${rnd}.json > gpurun_out/ck2/host_w${w}_r${rnd}.log 2>&1 || exit $?
    python -c "import json;d=json.load(open('gpurun_out/ck2/host_w${w}_r${rnd}.json'));print('host wgs=$w r$rnd',d['value'])"
  done
done
PSANA_RAY_COPY_KERNEL=32 timeout -k 10 200 python bench.py --mode image --json-out gpurun_out/ck2/image_w32.json > gpurun_out/ck2/image_w32.log 2>&1 || exit $?
python -c "import json;d=json.load(open('gpurun_out/ck2/image_w32.json'));print('image wgs=32',d['value'])"
timeout -k 10 200 python bench.py --loopback --json-out gpurun_out/ck2/loopback_w32.json > gpurun_out/ck2/loopback_w32.log 2>&1 || exit $?
python -c "import json;d=json.load(open('gpurun_out/ck2/loopback_w32.json'));print('loopback wgs=32',d['value'])"
for f in xtc2; do
  for z in 1 0; do
    for w in 32 0; do
      PSANA_RAY_COPY_KERNEL=$w PSANA_RAY_FILE_ZEROCOPY=$z timeout -k 10 300 python bench/file_source.py --format $f --frames 3072 > gpurun_out/ck2/file_${f}_zc${z}_w${w}.log 2>&1 || exit $?
      echo "file $f zc=$z wgs=$w: $(tail -1 gpurun_out/ck2/file_${f}_zc${z}_w${w}.log | cut -c1-200)"
    done
  done
done
