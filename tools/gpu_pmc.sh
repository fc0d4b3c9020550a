# PMC passes over the hot kernels (tools/pmc_kernels.py); each pass within the per-block slot limits
# (TCC: FETCH_SIZE 3 / WRITE_SIZE 2 of 4 slots -> separate passes), kernel trace only, no sys/runtime trace.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
export PYTHONPATH=$R
pass() { name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $R/gpurun_out/pmc_$name -o run -- python3 $R/tools/pmc_kernels.py > $R/gpurun_out/pmc_$name.log 2>&1 || return $?
  tail -1 $R/gpurun_out/pmc_$name.log
}
pass a FETCH_SIZE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES && \
pass b WRITE_SIZE SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU && \
pass c TCC_HIT_sum TCC_MISS_sum SQ_WAIT_ANY SQ_ACTIVE_INST_ANY && \
python3 $R/tools/pmc_summary.py $R/gpurun_out/pmc_a $R/gpurun_out/pmc_b $R/gpurun_out/pmc_c > $R/gpurun_out/pmc_kernels.md && head -20 $R/gpurun_out/pmc_kernels.md
