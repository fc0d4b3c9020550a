# Copy kernel vs runtime copies on the N>1 per-rank paths (transport rounds, loopback) and on
# Jungfrau-16M frames; interleaved on one box.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
mkdir -p gpurun_out/ck3
run() { name=$1; w=$2; shift 2
  PSANA_RAY_COPY_KERNEL=$w timeout -k 10 240 python bench.py "$@" --json-out gpurun_out/ck3/${name}_w${w}.json > gpurun_out/ck3/${name}_w${w}.log 2>&1 || return $?
  python -c "import json;d=json.load(open('gpurun_out/ck3/${name}_w${w}.json'));print('$name wgs=$w',d['value'],d['extra'].get('transport_round_ms_rank0'))"
}
run transport 32 --transport && run transport 0 --transport && run loopback 0 --loopback && run loopback 32 --loopback \
  && run jf16m 32 --detector jungfrau16M --queue-size 400000 --batch 8 --chunk 8 --steps 150 --warmup 40 \
  && run jf16m 0 --detector jungfrau16M --queue-size 400000 --batch 8 --chunk 8 --steps 150 --warmup 40
