# Round-final rocprofv3 kernel stats of the headline bench (1 GPU) from the rebuilt tree
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
export TMPDIR=/tmp
mkdir -p gpurun_out/fprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/fprof/host -o run -- python3 bench.py --steps 60 --warmup 10 > gpurun_out/fprof/host.log 2>&1 || exit $?
tail -1 gpurun_out/fprof/host.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/fprof/device -o run -- python3 bench.py --steps 200 --warmup 20 --source device > gpurun_out/fprof/device.log 2>&1 || exit $?
tail -1 gpurun_out/fprof/device.log | cut -c1-200
# keep the stats and logs only (the per-dispatch traces exceed what comes back)
find gpurun_out/fprof -type f ! -name "*stats.csv" ! -name "*.log" -delete
du -sh gpurun_out/fprof
