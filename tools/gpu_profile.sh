# rocprofv3 kernel + roctx marker trace of the headline bench (host-staged) and of the device-sourced
# pipeline; summaries only come back (the databases stay on the box)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
prof() { name=$1; shift
  timeout -k 10 300 rocprofv3 --marker-trace --kernel-trace --stats -d /tmp/prof_$name -o run -- python3 $R/bench.py "$@" > $R/gpurun_out/prof_$name.log 2>&1 || return $?
  tail -1 $R/gpurun_out/prof_$name.log | cut -c1-200
  python3 $R/tools/rocpd_summary.py /tmp/prof_$name > $R/gpurun_out/prof_$name.md || return $?
  rm -rf /tmp/prof_$name
}
prof host --steps 100 --warmup 10 && prof dev --steps 200 --warmup 10 --source device
