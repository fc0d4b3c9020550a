# Round-3 end rehearsal on the final tree: the driver's N>1 launch with 2 ranks on one GPU (both
# windows, links, teardown), then the driver's own N=1 line and smoke()
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=$R/gpurun_out/r3_end
mkdir -p $O
bash $R/tools/gpu_bench_2rank_1gpu.sh > $O/n2.txt 2>&1; rc=$?; cat $O/n2.txt; [ $rc -eq 0 ] || { tail -30 gpurun_out/b2/*.log; exit $rc; }
cp gpurun_out/b2/*.log gpurun_out/b2/*.json $O/ 2>/dev/null
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit $?
tail -1 $O/smoke.log
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench_n1.json 2> $O/bench_n1.err || exit $?
cut -c1-160 $O/bench_n1.json
