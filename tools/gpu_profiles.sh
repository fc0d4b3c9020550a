# Profiles for profiles/r2: kernel stats of the host-staged and device-resident benches, and an HBM
# traffic pass (FETCH_SIZE / WRITE_SIZE) over the kernel micro-benchmarks
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
export PYTHONPATH=$R
O=$R/gpurun_out/prof2
mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/host -o run -- python3 $R/bench.py --steps 60 --warmup 10 > $O/host.json 2> $O/host.err || exit $?
echo host done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/dev -o run -- python3 $R/bench.py --steps 100 --warmup 20 --source device > $O/dev.json 2> $O/dev.err || exit $?
echo dev done
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/hbm_r -o run -- python3 $R/bench/kernels.py --only calib_basic,calib_cm,peakfind,calib_cm_image --iters 3 > $O/hbm_r.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/hbm_w -o run -- python3 $R/bench/kernels.py --only calib_basic,calib_cm,peakfind,calib_cm_image --iters 3 > $O/hbm_w.log 2>&1 || exit $?
echo hbm done
