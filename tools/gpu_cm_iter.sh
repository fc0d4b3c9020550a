# Common-mode kernel iteration: bit-exact GPU kernel tests, per-phase timing, one PMC pass
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
export PYTHONPATH=$R
mkdir -p $R/gpurun_out/cm
timeout -k 10 300 python3 -u -m pytest $R/tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > $R/gpurun_out/cm/kernels_gpu.log 2>&1; rc=$?; tail -3 $R/gpurun_out/cm/kernels_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 $R/tools/cm_probe.py --repeat 1 --json-out $R/gpurun_out/cm/probe.jsonl > $R/gpurun_out/cm/probe.log 2>&1 || exit $?
tail -1 $R/gpurun_out/cm/probe.log
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT --kernel-trace --output-format csv -d $R/gpurun_out/cm/pmc -o run -- python3 $R/tools/cm_probe.py --pmc-pass > $R/gpurun_out/cm/pmc.log 2>&1 || exit $?
tail -1 $R/gpurun_out/cm/pmc.log
