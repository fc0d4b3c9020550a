# Round 4, fabric pass 3: copy-kernel grid x copy-stream placement on the 2-rank-on-one-GPU
# rehearsal (device-resident, where the copies are the bottleneck), then host-staged at the pick.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=$R/gpurun_out/r4_fabric3
mkdir -p $O
summ() {
  python - $1 <<'PY'
import json, sys
r = json.load(open(sys.argv[1])); e = r["extra"]; x = e.get("xgmi_phase") or {}
d = x.get("copy_dispatch_per_rank") or [{}]
print(sys.argv[1].split("/")[-1], "value", r["value"], "remote_only", x.get("frames_per_s"),
      "ratio", round(x["frames_per_s"] / r["value"], 3) if x else None, "fabric_copy", x.get("fabric_copy"),
      "cross", x.get("cross_gpu_fraction"), "ms/64 p50", [c.get("ms_per_64_frames_dev_p50") for c in d],
      "p99", [c.get("dev_ms_p99") for c in d], "GB/s", [c.get("dev_GB_per_s") for c in d],
      "prod/cons", e["production_frames_per_s"], e["consumer_frames_per_s"], flush=True)
PY
}
run() {
  timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $2 bench.py --gpus 2 ${@:3} > $O/$1.log 2>&1 || { tail -30 $O/$1.log; return 1; }
  grep '"metric"' $O/$1.log > $O/$1.json && summ $O/$1.json
}
p=29740
for rnd in 1 2; do
  for st in dedicated shared; do
    for w in 128 256 512; do
      p=$((p+1))
      run dev_${st}_${w}_r$rnd $p --steps 100 --warmup 20 --source device --fabric-copy-stream $st --fabric-copy-wgs $w || exit $?
    done
  done
done
run host_ded_256 29790 --steps 40 --warmup 10 --fabric-copy-stream dedicated --fabric-copy-wgs 256 && \
run host_sh_256 29791 --steps 40 --warmup 10 --fabric-copy-stream shared --fabric-copy-wgs 256 && \
run host_ded_256_long 29792 --steps 200 --warmup 10 --preroll-s 3 --fabric-copy-stream dedicated --fabric-copy-wgs 256
for b in median_probe_bin median_probe_lds_bin; do
  timeout -k 10 180 $R/tools/$b 16384 > $O/$b.json 2> $O/$b.err; rc=$?
  cat $O/$b.json; echo "$b rc=$rc"
  [ $rc -le 1 ] || exit $rc
done
