# Host->HBM staging copies by our own kernel (PSANA_RAY_COPY_KERNEL=<workgroups>) vs the runtime's
# blit copies: exactness first, then the headline bench interleaved.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
mkdir -p gpurun_out/ck
PSANA_RAY_COPY_KERNEL=64 timeout -k 10 300 python -m pytest tests/test_pipeline_gpu.py tests/test_cli_gpu.py -x -q > gpurun_out/ck/pytest.log 2>&1; rc=$?; tail -2 gpurun_out/ck/pytest.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
for rnd in 0 1; do
  for w in 0 32 64 128 256; do
    PSANA_RAY_COPY_KERNEL=$w timeout -k 10 200 python bench.py --json-out gpurun_out/ck/w${w}_r${rnd}.json > gpurun_out/ck/w${w}_r${rnd}.log 2>&1 || exit $?
    python -c "import json;d=json.load(open('gpurun_out/ck/w${w}_r${rnd}.json'));print('wgs=$w r$rnd',d['value'],d['extra']['produced_frames_per_s'])"
  done
done
PSANA_RAY_COPY_KERNEL=64 timeout -k 10 200 python bench.py --copy-engine sdma --json-out gpurun_out/ck/w64_sdma.json > gpurun_out/ck/w64_sdma.log 2>&1 || exit $?
python -c "import json;d=json.load(open('gpurun_out/ck/w64_sdma.json'));print('wgs=64 sdma-env',d['value'])"
