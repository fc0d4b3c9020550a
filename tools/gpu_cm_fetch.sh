set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
export PYTHONPATH=$R
mkdir -p $R/gpurun_out/cm
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE SQ_WAVES --kernel-trace --output-format csv -d $R/gpurun_out/cm/fetch -o run -- python3 $R/tools/cm_probe.py --pmc-pass > $R/gpurun_out/cm/fetch.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d $R/gpurun_out/cm/write -o run -- python3 $R/tools/cm_probe.py --pmc-pass > $R/gpurun_out/cm/write.log 2>&1 || exit $?
tail -1 $R/gpurun_out/cm/write.log
