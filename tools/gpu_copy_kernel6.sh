# Isolated host->HBM rates: hipMemcpyAsync (blit / SDMA) vs copy_h2d_kernel (U=4 / U=8), then the
# headline with U=8.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
mkdir -p gpurun_out/ck6
HSA_ENABLE_SDMA=0 timeout -k 10 200 python bench/h2d.py > gpurun_out/ck6/h2d_blit_u4.log 2>&1 || exit $?
grep '^{' gpurun_out/ck6/h2d_blit_u4.log | grep -E '"chunk_frames": 32, "streams": 1|copy_kernel'
PSANA_RAY_COPY_KERNEL_U=8 HSA_ENABLE_SDMA=0 timeout -k 10 200 python bench/h2d.py > gpurun_out/ck6/h2d_blit_u8.log 2>&1 || exit $?
grep '^{' gpurun_out/ck6/h2d_blit_u8.log | grep copy_kernel | sed 's/^/U8 /'
timeout -k 10 200 python bench/h2d.py > gpurun_out/ck6/h2d_sdma.log 2>&1 || exit $?
grep '^{' gpurun_out/ck6/h2d_sdma.log | grep -E '"chunk_frames": 32, "streams": 1' | sed 's/^/SDMA /'
for rnd in 0 1; do
  for u in 8 4; do
    PSANA_RAY_COPY_KERNEL_U=$u timeout -k 10 200 python bench.py --json-out gpurun_out/ck6/host_u${u}_r${rnd}.json > gpurun_out/ck6/host_u${u}_r${rnd}.log 2>&1 || exit $?
    python -c "import json;d=json.load(open('gpurun_out/ck6/host_u${u}_r${rnd}.json'));print('headline U=$u r$rnd',d['value'])"
  done
done
