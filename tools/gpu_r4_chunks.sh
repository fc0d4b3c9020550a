# Round 4: device-resident pipeline vs producer chunk / consumer batch (MALL reuse of the peak
# finder's reads needs the frames it reads to be recent: smaller chunks keep less data in flight).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=$R/gpurun_out/r4_chunks
mkdir -p $O
b() {
  timeout -k 10 300 python bench.py --steps 200 --warmup 5 --source device "${@:2}" > $O/$1.json 2> $O/$1.err || { tail -20 $O/$1.err; return 1; }
  python -c "import json;d=json.load(open('$O/$1.json'));print('$1', d['value'])"
}
for r in 1 2; do
  b c64b32_$r --chunk 64 --batch 32 && b c32b32_$r --chunk 32 --batch 32 && b c16b16_$r --chunk 16 --batch 16 && \
  b c8b8_$r --chunk 8 --batch 8 && b c32b16_$r --chunk 32 --batch 16 || exit 1
done
