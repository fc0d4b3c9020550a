# Round 4, second fabric pass: the N=1 headline (unaffected by the fabric), then the 2-rank-on-one-GPU
# rehearsal -- copy stream placement A/B (dedicated vs shared hardware queue), the runtime engine,
# BASELINE config 3's shape (1 producer, 1 consumer-only rank) after the starving-consumer fix --
# then the peak finder's spill path and its probe at ~2 % candidate density.  Every step prints
# as it goes (no pipes into tail: a silent step looks hung).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=$R/gpurun_out/r4_fabric2
mkdir -p $O
summ() {
  python - $1 <<'PY'
import json, sys
r = json.load(open(sys.argv[1])); e = r["extra"]; x = e.get("xgmi_phase") or {}
d = x.get("copy_dispatch_per_rank") or [{}]
print(sys.argv[1].split("/")[-1], "value", r["value"], "remote_only", x.get("frames_per_s"),
      "ratio", round(x["frames_per_s"] / r["value"], 3) if x else None, "fabric_copy", x.get("fabric_copy"),
      "dev_ms_p50", [c.get("dev_ms_p50") for c in d], "ms/64 p50", [c.get("ms_per_64_frames_dev_p50") for c in d],
      "GB/s", [c.get("dev_GB_per_s") for c in d], "recv_share", e.get("recv_cross_per_consumed_per_rank"),
      "prod/cons", e["production_frames_per_s"], e["consumer_frames_per_s"], flush=True)
PY
}
run() {  # name, port, extra args
  timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $2 bench.py --gpus 2 ${@:3} > $O/$1.log 2>&1 || { tail -30 $O/$1.log; return 1; }
  grep '"metric"' $O/$1.log > $O/$1.json && summ $O/$1.json
}
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/n1_host.json 2> $O/n1_host.err || exit $?
summ $O/n1_host.json
run cfg3_host 29721 --steps 40 --warmup 10 --producers 1 && \
run cfg3_dev 29722 --steps 100 --warmup 20 --source device --producers 1 && \
run host_ded_a 29723 --steps 40 --warmup 10 --fabric-copy-stream dedicated && \
run host_sh_a 29724 --steps 40 --warmup 10 --fabric-copy-stream shared && \
run host_ded_b 29725 --steps 40 --warmup 10 --fabric-copy-stream dedicated && \
run host_sh_b 29726 --steps 40 --warmup 10 --fabric-copy-stream shared && \
run dev_ded 29727 --steps 100 --warmup 20 --source device --fabric-copy-stream dedicated && \
run dev_sh 29728 --steps 100 --warmup 20 --source device --fabric-copy-stream shared && \
run dev_ded_w256 29729 --steps 100 --warmup 20 --source device --fabric-copy-wgs 256 || exit $?
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_production_shapes_gpu.py -k peakfind > $O/pf_tests.log 2>&1 || { tail -30 $O/pf_tests.log; exit 1; }
grep -E "passed|failed" $O/pf_tests.log
timeout -k 10 200 python tools/pf_probe.py --repeat 3 --total > $O/pf_default.log 2>&1 || { tail -20 $O/pf_default.log; exit 1; }
cat $O/pf_default.log
timeout -k 10 200 python tools/pf_probe.py --repeat 3 --thr 5 --total > $O/pf_thr5.log 2>&1 || { tail -20 $O/pf_thr5.log; exit 1; }
cat $O/pf_thr5.log
