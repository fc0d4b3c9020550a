# Round 4: the fabric copy path.  Elastic GPU tests (bit-exact multi-process frames through the
# new copy kernel), then the 2-rank-on-one-GPU rehearsal (both windows) with the kernel engine and
# the round-3 runtime engine, host-staged and device-resident.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=$R/gpurun_out/r4_fabric
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_elastic_gpu.py tests/test_psana_wrapper.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k copy_runs > $O/copy_tests.log 2>&1 || { tail -30 $O/copy_tests.log; exit 1; }
tail -2 $O/copy_tests.log
run() {  # name, port, extra args
  timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $2 bench.py --gpus 2 ${@:3} > $O/$1.log 2>&1 || { tail -30 $O/$1.log; return 1; }
  grep '"metric"' $O/$1.log > $O/$1.json
  python - $O/$1.json <<'PY'
import json, sys
r = json.load(open(sys.argv[1])); x = r["extra"]["xgmi_phase"]
e = r["extra"]
print(sys.argv[1].split("/")[-1], "balanced", r["value"], "remote_only", x["frames_per_s"], "ratio", round(x["frames_per_s"] / r["value"], 3),
      "GB/s", x["cross_gpu_GB_per_s"], x["copy_dispatch_per_rank"], x["copy_ms_per_batch_per_rank"], e["producer_host_s_stage_acquire_launch_commit_total"],
      "recv_share", e.get("recv_cross_per_consumed_per_rank"), "prod/cons", e["production_frames_per_s"], e["consumer_frames_per_s"])
PY
}
run host_kernel 29711 --steps 40 --warmup 10 --fabric-copy kernel && \
run host_runtime 29712 --steps 40 --warmup 10 --fabric-copy runtime && \
run dev_kernel 29713 --steps 100 --warmup 20 --source device --fabric-copy kernel && \
run dev_runtime 29714 --steps 100 --warmup 20 --source device --fabric-copy runtime && \
run host_kernel_b 29715 --steps 40 --warmup 10 --fabric-copy kernel && \
run cfg3_host 29716 --steps 40 --warmup 10 --producers 1 && \
run cfg3_dev 29717 --steps 100 --warmup 20 --source device --producers 1
# peak finder: the spill path (hit-rich frames) against the golden model, then the probe at the
# default threshold and at ~2 % candidate density
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_production_shapes_gpu.py -k peakfind > $O/pf_tests.log 2>&1 || { tail -30 $O/pf_tests.log; exit 1; }
tail -2 $O/pf_tests.log
timeout -k 10 200 python tools/pf_probe.py --repeat 3 --total > $O/pf_default.log 2>&1 || { tail -20 $O/pf_default.log; exit 1; }
tail -2 $O/pf_default.log
timeout -k 10 200 python tools/pf_probe.py --repeat 3 --thr 5 --total > $O/pf_thr5.log 2>&1 || { tail -20 $O/pf_thr5.log; exit 1; }
tail -2 $O/pf_thr5.log
