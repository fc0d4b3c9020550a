# Round checkpoint on a fresh box (replaces the per-round gpu_r*_checkpoint / final scripts).
#
# STAGES (default "tests smoke bench dev rehearsal prof"), each step under its own timeout, a
# failure ends the script:
#   tests      the full `pytest -m gpu` suite (PYFLAGS: interpreter flags)
#   smoke      __graft_entry__.smoke()
#   bench      the driver's line: bench.py --steps 20 --warmup 5 (and --steps 200)
#   dev        device-resident calib / image pipelines, 200 steps
#   rehearsal  the driver's N>1 launch on this one GPU, 2 ranks: plain `bench.py --gpus 2` (self-
#              launched) host-staged, torch.distributed.run device-resident (links, both windows,
#              gate, topology record, frame checks, teardown)
#   prof       rocprofv3 --kernel-trace --stats of both device-resident pipelines (stats CSVs kept)
#   configs    BASELINE config 4 (Jungfrau-16M, queue_size 400000; host-staged / device-resident,
#              rocprofv3 stats) and config 1 (256x256, in-process CPU queue)
#   jfcm       Jungfrau-16M device-resident with common mode ON (the Jungfrau CM kernel) + its stats
#   rehearsal4 4 ranks on the one GPU (the shared-GPU pipeline shape; `mpirun -n 4` on fewer GPUs)
# Outputs: gpurun_out/${OUT:-checkpoint}/
#   OUT=r5_cp STAGES="tests smoke bench" gpurun -- bash tools/gpu_checkpoint.sh
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
export PYTHONPATH=$R
O=$R/gpurun_out/${OUT:-checkpoint}
mkdir -p $O
has() { case " ${STAGES:-tests smoke bench dev rehearsal prof} " in *" $1 "*) return 0;; esac; return 1; }
line() { python3 -c "import json,sys;d=json.load(open('$1'));x=d['extra'];print('$2', d['value'], 'gate', (x.get('steady_gate') or {}).get('iterations'), (x.get('steady_gate') or {}).get('converged'))"; }
if has tests; then
  timeout -k 10 900 python3 ${PYFLAGS:-} -u -m pytest $R/tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1; rc=$?
  tail -1 $O/tests.log
  [ $rc -eq 0 ] || { grep -n -B5 -A40 "Error\|FAILED" $O/tests.log | head -120; exit $rc; }
fi
cd $R
if has smoke; then
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
  tail -1 $O/smoke.log
fi
if has bench; then
  for s in 20 200; do
    timeout -k 10 300 python3 bench.py --steps $s --warmup 5 > $O/bench_host_$s.json 2> $O/bench_host_$s.err || { tail $O/bench_host_$s.err; exit 1; }
    line $O/bench_host_$s.json "host $s"
  done
fi
if has dev; then
  for m in calib image; do
    timeout -k 10 300 python3 bench.py --steps 200 --warmup 5 --source device --mode $m > $O/bench_dev_$m.json 2> $O/bench_dev_$m.err || { tail $O/bench_dev_$m.err; exit 1; }
    line $O/bench_dev_$m.json "device $m"
  done
fi
if has rehearsal; then
  for src in host device; do
    # host: the driver's plain command (bench.py self-launches its ranks); device: under torchrun
    if [ $src = host ]; then
      timeout -k 10 300 python3 bench.py --gpus 2 --steps 40 --warmup 10 --source $src > $O/n2_$src.log 2>&1 || { tail -30 $O/n2_$src.log; exit 1; }
    else
      timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $((29600 + RANDOM % 300)) \
        bench.py --gpus 2 --steps 40 --warmup 10 --source $src > $O/n2_$src.log 2>&1 || { tail -30 $O/n2_$src.log; exit 1; }
    fi
    grep '"metric"' $O/n2_$src.log > $O/n2_$src.json
    python3 -c "import json;d=json.load(open('$O/n2_$src.json'));x=d['extra'];c=x['xgmi_phase'];print('n2 $src', d['value'], 'n_gpus', d['n_gpus'], 'n_ranks', d['n_ranks'], 'cross', c['frames_per_s'], c['cross_gpu_fraction'], 'checks', x['frame_checks']['frames_verified'], x['frame_checks']['frames_mismatched'], 'gate', x['steady_gate'], 'links', x['topology']['outgoing_links_per_rank'])"
  done
fi
if has prof; then
  for m in calib image; do
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$m -o run -- python3 bench.py --steps 200 --warmup 20 --source device --mode $m > $O/prof_$m.log 2>&1 || { tail $O/prof_$m.log; exit 1; }
    head -4 $O/prof_$m/run_kernel_stats.csv | cut -c1-160
  done
fi
if has configs; then
  for src in host device; do
    extra=""; [ $src = device ] && extra="--pool-frames 16"
    timeout -k 10 300 python3 bench.py --detector jungfrau16M --queue-size 400000 --batch 8 --chunk 8 --steps 150 --warmup 40 --source $src $extra > $O/jf16m_$src.json 2> $O/jf16m_$src.err || { tail $O/jf16m_$src.err; exit 1; }
    line $O/jf16m_$src.json "jf16m $src"
  done
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_jf16m -o run -- python3 bench.py --detector jungfrau16M --queue-size 400000 --batch 8 --chunk 8 --steps 150 --warmup 40 --source device --pool-frames 16 > $O/prof_jf16m.log 2>&1 || { tail $O/prof_jf16m.log; exit 1; }
  head -4 $O/prof_jf16m/run_kernel_stats.csv | cut -c1-160
  timeout -k 10 300 python3 bench/config1_cpu_queue.py > $O/config1.json 2> $O/config1.err || { tail $O/config1.err; exit 1; }
  cut -c1-200 $O/config1.json
fi
if has jfcm; then
  timeout -k 10 300 python3 bench.py --detector jungfrau16M --queue-size 400000 --batch 8 --chunk 8 --steps 150 --warmup 40 --source device --pool-frames 16 --common-mode default > $O/jf16m_cm_device.json 2> $O/jf16m_cm_device.err || { tail $O/jf16m_cm_device.err; exit 1; }
  line $O/jf16m_cm_device.json "jf16m cm device"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_jf16m_cm -o run -- python3 bench.py --detector jungfrau16M --queue-size 400000 --batch 8 --chunk 8 --steps 150 --warmup 40 --source device --pool-frames 16 --common-mode default > $O/prof_jf16m_cm.log 2>&1 || { tail $O/prof_jf16m_cm.log; exit 1; }
  head -4 $O/prof_jf16m_cm/run_kernel_stats.csv | cut -c1-160
fi
if has rehearsal4; then
  timeout -k 10 400 python3 bench.py --gpus 4 --steps 40 --warmup 10 --source device > $O/n4_device.log 2>&1 || { tail -30 $O/n4_device.log; exit 1; }
  grep '"metric"' $O/n4_device.log > $O/n4_device.json
  python3 -c "import json;d=json.load(open('$O/n4_device.json'));x=d['extra'];c=x['xgmi_phase'];print('n4 device', d['value'], 'rpg', d['config']['ranks_per_gpu'], 'batch', d['config']['global_batch'], 'streams', x['producer_streams'], 'cross', c['frames_per_s'], c['cross_gpu_fraction'], 'gate', x['steady_gate']['iterations'], x['steady_gate']['converged'])"
fi
find $O -path "*prof_*" -type f ! -name "*stats.csv" ! -name "*.log" -delete 2>/dev/null
du -sh $O
