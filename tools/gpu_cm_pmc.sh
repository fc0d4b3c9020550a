# Counter passes over the common-mode kernel (cm_probe --pmc-pass: flags 0,1,2,3 x 3 launches each,
# 32 epix10k2M frames): what bounds it (VALU issue, LDS, waits, clock)?  One pass per counter set,
# kernel trace only.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
export PYTHONPATH=$R
O=$R/gpurun_out/cm_pmc
mkdir -p $O
timeout -k 10 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
pass() { name=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d $O/$name -o run -- python3 $R/tools/cm_probe.py --pmc-pass > $O/$name.log 2>&1
  echo "pass $name rc=$?"
}
pass a SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE
pass b SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA GRBM_COUNT
python3 - <<'PY'
import csv, glob, collections, os
O = os.environ["GRAFT_REPO_ROOT"] + "/gpurun_out/cm_pmc"
for p in ("a", "b"):
    rows = [r for f in glob.glob(f"{O}/{p}/**/*counter_collection.csv", recursive=True) for r in csv.DictReader(open(f))]
    agg = collections.OrderedDict()
    for r in rows:
        if "calib_cm" not in r.get("Kernel_Name", ""):
            continue
        key = (int(r["Dispatch_Id"]), r["Counter_Name"])
        agg[key] = agg.get(key, 0.0) + float(r["Counter_Value"])
    disp = sorted({k[0] for k in agg})
    names = sorted({k[1] for k in agg})
    print("pass", p, "dispatches", len(disp))
    for i, d in enumerate(disp):
        print(d, " ".join(f"{n}={agg[(d, n)]:.4g}" for n in names))
PY
