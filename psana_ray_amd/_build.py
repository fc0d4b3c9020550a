"""In-tree build of the native extension ``psana_ray_amd._C`` for gfx950.

Every ``csrc/*.hip`` / ``csrc/*.cpp`` file is compiled with ``hipcc --offload-arch=gfx950``
(in parallel) and linked into ``psana_ray_amd/_C<EXT_SUFFIX>``.  The build is incremental: a
stamp file records a hash of the sources + flags, and nothing is rebuilt when it matches.
No torch C++ headers are used, so the module builds here (no GPU) and on the GPU box alike.

Usage:  ``python -m psana_ray_amd._build [--force] [--verbose]``
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import hashlib
import os
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path

PKG_DIR = Path(__file__).resolve().parent
REPO = PKG_DIR.parent
CSRC = REPO / "csrc"
BUILD_DIR = REPO / "build" / "native"
EXT_SUFFIX = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
TARGET = PKG_DIR / f"_C{EXT_SUFFIX}"
STAMP = PKG_DIR / "_C.build-stamp"
ARCH = os.environ.get("PSANA_RAY_AMD_ARCH", "gfx950")


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (is ROCm installed at /opt/rocm?)")


def _torch_lib_dir() -> str | None:
    """torch ships its own libamdhip64.so.7; link/rpath against it so exactly ONE HIP
    runtime is loaded in a process that imports torch and this extension."""
    try:
        import importlib.util

        spec = importlib.util.find_spec("torch")
        if spec and spec.origin:
            lib = Path(spec.origin).parent / "lib"
            if (lib / "libamdhip64.so").exists():
                return str(lib)
    except Exception:  # pragma: no cover
        pass
    return None


def _flags():
    import pybind11

    inc = [f"-I{CSRC}", f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}"]
    common = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-ffp-contract=off",
              "-Wno-unused-result", "-fvisibility=hidden"]
    return inc, common


def _sources():
    return sorted(list(CSRC.glob("*.hip")) + list(CSRC.glob("*.cpp")))


def _stamp(srcs, inc, common) -> str:
    h = hashlib.sha256()
    for p in srcs + sorted(CSRC.glob("*.h")):
        h.update(p.name.encode())
        h.update(p.read_bytes())
    # the tree's own location is not part of the build (a copy of the tree elsewhere -- a GPU box's
    # scratch path, an A/B variant tree -- has the same extension)
    h.update(" ".join([f.replace(str(CSRC), "<csrc>") for f in inc] + common + [ARCH]).encode())
    return h.hexdigest()


def build(force: bool = False, verbose: bool = False, jobs: int | None = None) -> Path:
    srcs = _sources()
    inc, common = _flags()
    stamp = _stamp(srcs, inc, common)
    # the stamp sits NEXT TO the extension, so the pair travels together (a snapshot of the tree
    # without build/ -- a GPU box -- loads the extension as built instead of recompiling it)
    stamp_file = STAMP
    if not force and TARGET.exists() and stamp_file.exists() and stamp_file.read_text() == stamp:
        return TARGET
    BUILD_DIR.mkdir(parents=True, exist_ok=True)
    hipcc = _hipcc()

    def compile_one(src: Path) -> Path:
        obj = BUILD_DIR / (src.name + ".o")
        lang = ["-x", "hip"] if src.suffix == ".hip" else []
        cmd = [hipcc, *common, *inc, *lang, "-c", str(src), "-o", str(obj)]
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"compile failed for {src.name}:\n{r.stdout}\n{r.stderr}")
        if verbose and r.stderr.strip():
            print(r.stderr, flush=True)
        return obj

    jobs = jobs or min(len(srcs), max(1, (os.cpu_count() or 4)), 8)
    with cf.ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(compile_one, srcs))
    link = [hipcc, "-shared", f"--offload-arch={ARCH}", "-fPIC", *map(str, objs), "-o", str(TARGET) + ".tmp"]
    tlib = _torch_lib_dir()
    if tlib:
        link += [f"-L{tlib}", f"-Wl,-rpath,{tlib}"]
    link += ["-lamdhip64", "-lpthread", "-ldl", "-lrt"]
    if verbose:
        print(" ".join(link), flush=True)
    r = subprocess.run(link, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
    os.replace(str(TARGET) + ".tmp", TARGET)
    stamp_file.write_text(stamp)
    return TARGET


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--verbose", action="store_true")
    a = ap.parse_args(argv)
    out = build(force=a.force, verbose=a.verbose)
    print(out)


if __name__ == "__main__":
    sys.exit(main())
