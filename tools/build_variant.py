#!/usr/bin/env python3
"""Build an A/B variant of the native extension: ONE source recompiled with extra flags (e.g. a
scheduler strategy or a -D constant), linked with the shipped objects into variants/_C_<name>.so.

    python tools/build_variant.py maxilp common_mode.hip -mllvm -amdgpu-sched-strategy=max-ilp
    VARIANTS="maxilp" PROBE=tools/cm_probe.py gpurun -- bash tools/gpu_variants.sh
"""
import subprocess
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from psana_ray_amd import _build  # noqa: E402


def main():
    if len(sys.argv) < 3:
        raise SystemExit(__doc__)
    name, src_names, extra = sys.argv[1], set(sys.argv[2].split(",")), sys.argv[3:]   # sources: a,b,...
    _build.build()                      # the shipped objects are current
    inc, common = _build._flags()
    hipcc = _build._hipcc()
    out_dir = _build.REPO / "variants"
    out_dir.mkdir(exist_ok=True)
    objs = []
    for src in _build._sources():
        obj = _build.BUILD_DIR / (src.name + ".o")
        if src.name in src_names:
            obj = out_dir / f"{src.name}.{name}.o"
            lang = ["-x", "hip"] if src.suffix == ".hip" else []
            cmd = [hipcc, *common, *extra, *inc, *lang, "-c", str(src), "-o", str(obj)]
            r = subprocess.run(cmd, capture_output=True, text=True)
            if r.returncode != 0:
                raise SystemExit(f"compile failed:\n{r.stderr}")
        objs.append(str(obj))
    target = out_dir / f"_C_{name}.so"
    link = [hipcc, "-shared", f"--offload-arch={_build.ARCH}", "-fPIC", *objs, "-o", str(target)]
    tlib = _build._torch_lib_dir()
    if tlib:
        link += [f"-L{tlib}", f"-Wl,-rpath,{tlib}"]
    link += ["-lamdhip64", "-lpthread", "-ldl", "-lrt"]
    r = subprocess.run(link, capture_output=True, text=True)
    if r.returncode != 0:
        raise SystemExit(f"link failed:\n{r.stderr}")
    print(target)


if __name__ == "__main__":
    main()
