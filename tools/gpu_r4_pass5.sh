# Round 4, pass 5: the 2-rank-on-one-GPU rehearsal after the consumer-only low-water feed and the
# common window end of config-3 runs (producers < ranks), then the fabric's GPU tests.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=$R/gpurun_out/r4_pass5
mkdir -p $O
summ() {
  python - $1 <<'PY'
import json, sys
r = json.load(open(sys.argv[1])); e = r["extra"]; x = e.get("xgmi_phase") or {}
d = x.get("copy_dispatch_per_rank") or [{}]
print(sys.argv[1].split("/")[-1], "value", r["value"], "remote_only", x.get("frames_per_s"),
      "ratio", round(x["frames_per_s"] / r["value"], 3) if x else None,
      "cross", x.get("cross_gpu_fraction"), "ms/64 p50", [c.get("ms_per_64_frames_dev_p50") for c in d],
      "recv_share", e.get("recv_cross_per_consumed_per_rank"), "consumed", e.get("consumed_per_rank"),
      "prod/cons", e["production_frames_per_s"], e["consumer_frames_per_s"], flush=True)
PY
}
run() {
  timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $2 bench.py --gpus 2 ${@:3} > $O/$1.log 2>&1 || { tail -30 $O/$1.log; return 1; }
  grep '"metric"' $O/$1.log > $O/$1.json && summ $O/$1.json
}
run cfg3_host_a 29901 --steps 40 --warmup 10 --producers 1 && \
run cfg3_dev_a 29902 --steps 100 --warmup 20 --source device --producers 1 && \
run cfg3_host_b 29903 --steps 40 --warmup 10 --producers 1 && \
run cfg3_dev_b 29904 --steps 100 --warmup 20 --source device --producers 1 && \
run host 29905 --steps 40 --warmup 10 && \
run dev 29906 --steps 100 --warmup 20 --source device || exit 1
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_elastic_gpu.py > $O/elastic_tests.log 2>&1 || { tail -30 $O/elastic_tests.log; exit 1; }
grep -E "passed|failed" $O/elastic_tests.log
