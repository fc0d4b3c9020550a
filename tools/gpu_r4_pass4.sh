# Round 4, pass 4: the counter table of the shipped kernels (tools/gpu_r4_pmc.sh), then the
# 2-rank-on-one-GPU rehearsal after the consumer-only feeding rule and the adaptive copy grid.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
bash $R/tools/gpu_r4_pmc.sh || exit $?
cd $R
O=$R/gpurun_out/r4_pass4
mkdir -p $O
summ() {
  python - $1 <<'PY'
import json, sys
r = json.load(open(sys.argv[1])); e = r["extra"]; x = e.get("xgmi_phase") or {}
d = x.get("copy_dispatch_per_rank") or [{}]
print(sys.argv[1].split("/")[-1], "value", r["value"], "remote_only", x.get("frames_per_s"),
      "ratio", round(x["frames_per_s"] / r["value"], 3) if x else None, "fabric_copy", x.get("fabric_copy"),
      "cross", x.get("cross_gpu_fraction"), "ms/64 p50", [c.get("ms_per_64_frames_dev_p50") for c in d],
      "GB/s", [c.get("dev_GB_per_s") for c in d], "recv_share", e.get("recv_cross_per_consumed_per_rank"),
      "prod/cons", e["production_frames_per_s"], e["consumer_frames_per_s"], flush=True)
PY
}
run() {
  timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $2 bench.py --gpus 2 ${@:3} > $O/$1.log 2>&1 || { tail -30 $O/$1.log; return 1; }
  grep '"metric"' $O/$1.log > $O/$1.json && summ $O/$1.json
}
run host_a 29801 --steps 40 --warmup 10 && \
run host_b 29802 --steps 40 --warmup 10 && \
run dev_a 29803 --steps 100 --warmup 20 --source device && \
run dev_b 29804 --steps 100 --warmup 20 --source device && \
run cfg3_host 29805 --steps 40 --warmup 10 --producers 1 && \
run cfg3_dev 29806 --steps 100 --warmup 20 --source device --producers 1 && \
run img_dev 29807 --steps 100 --warmup 20 --source device --mode image
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_production_shapes_gpu.py tests/test_kernels_gpu.py -k "peakfind" > $O/pf_tests.log 2>&1 || { tail -30 $O/pf_tests.log; exit 1; }
grep -E "passed|failed" $O/pf_tests.log
timeout -k 10 200 python tools/pf_probe.py --repeat 3 --total > $O/pf_default.log 2>&1 || { tail -20 $O/pf_default.log; exit 1; }
grep us_per_frame $O/pf_default.log
timeout -k 10 200 python tools/pf_probe.py --repeat 3 --thr 5 --total > $O/pf_thr5.log 2>&1 || { tail -20 $O/pf_thr5.log; exit 1; }
grep us_per_frame $O/pf_thr5.log
