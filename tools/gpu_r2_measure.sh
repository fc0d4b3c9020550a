# Round-2 measurement pass: kernel micro-benchmarks, CM wave-state counters, headline bench
# (host source), device-resident calib and image benches.  Every GPU step has its own time limit.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
export PYTHONPATH=$R
O=$R/gpurun_out/r2m
mkdir -p $O
timeout -k 10 240 python3 $R/bench/kernels.py --json-out $O/kernels.jsonl > $O/kernels.log 2>&1 || exit $?
echo kernels done
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS --kernel-trace --output-format csv -d $O/pmc_wave -o run -- python3 $R/tools/cm_probe.py --pmc-pass > $O/pmc_wave.log 2>&1 || exit $?
echo pmc done
timeout -k 10 200 python3 $R/bench.py --steps 60 --warmup 10 > $O/bench_host.json 2> $O/bench_host.err || exit $?
tail -1 $O/bench_host.json
timeout -k 10 200 python3 $R/bench.py --steps 200 --warmup 20 --source device > $O/bench_dev.json 2> $O/bench_dev.err || exit $?
tail -1 $O/bench_dev.json
timeout -k 10 200 python3 $R/bench.py --steps 200 --warmup 20 --source device --mode image > $O/bench_dev_image.json 2> $O/bench_dev_image.err || exit $?
tail -1 $O/bench_dev_image.json
