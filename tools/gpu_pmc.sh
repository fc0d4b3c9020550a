# Counter table of the shipped kernels in production form (tools/pmc_workload.py: common mode calib /
# image, peak finder, host->HBM copy, fabric copy; 64 epix10k2M frames per launch): one
# --kernel-trace --stats pass for durations, then --pmc passes within the per-block counter limits
# (FETCH_SIZE and WRITE_SIZE in separate passes), kernel trace only, each under its own kill timeout.
# Table: gpurun_out/${OUT:-pmc}/pmc_kernels.md (tools/pmc_table.py).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
export PYTHONPATH=$R
O=$R/gpurun_out/${OUT:-pmc}
mkdir -p $O
timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/tools/pmc_workload.py --phases $O/phases.json > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
pass() { name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $O/$name -o run -- python3 $R/tools/pmc_workload.py > $O/$name.log 2>&1 || { tail -20 $O/$name.log; return 1; }
  echo "pass $name ok"
}
pass a FETCH_SIZE GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAVES && \
pass b WRITE_SIZE SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES && \
python3 $R/tools/pmc_table.py $O/phases.json $O/trace $O/a $O/b > $O/pmc_kernels.md && head -12 $O/pmc_kernels.md
