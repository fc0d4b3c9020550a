set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
timeout -k 10 400 python bench.py --detector jungfrau16M --queue-size 400000 --steps 20 --warmup 4 --batch 8 --chunk 8 --pool-frames 16 > gpurun_out/bench_jf16m.log 2>&1 || exit $?
tail -1 gpurun_out/bench_jf16m.log | cut -c1-1500
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --marker-trace --kernel-trace --stats -d $R/gpurun_out/prof_marker -o run -- python3 $R/bench.py --steps 30 --warmup 5 > $R/gpurun_out/prof_marker.log 2>&1 || exit $?
tail -1 $R/gpurun_out/prof_marker.log | cut -c1-300
find $R/gpurun_out/prof_marker | head -20
