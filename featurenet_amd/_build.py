"""In-tree build of the native libraries (no JIT cache, no pip install).

Two shared objects are produced next to this file:

* ``_C``  -- the gfx950 HIP kernel library (hipcc ``--offload-arch=gfx950``),
  exposed to Python through pybind11 (``csrc/kernels/bind.cpp``).
* ``_rt`` -- the host-side native runtime (C++17, no GPU): the PLEDGE-style
  SAT sampler / diversity EA, the SPLOT feature-model parser and the voxel
  data pipeline (``csrc/runtime``).

Object files are cached under ``build/obj`` and rebuilt when a source or any
header in its directory is newer than the object.  ``python -m
featurenet_amd._build`` builds everything; ``__graft_entry__.build()`` calls
:func:`build_all`.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import subprocess
import sys
import sysconfig
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
OBJ = ROOT / "build" / "obj"
ARCH = os.environ.get("FEATURENET_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
EXT = sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def _py_includes() -> list[str]:
    import pybind11

    return [f"-I{sysconfig.get_paths()['include']}", f"-I{pybind11.get_include()}"]


def _newer(src: Path, obj: Path) -> bool:
    if not obj.exists():
        return True
    t = obj.stat().st_mtime
    deps = [src] + [p for p in src.parent.glob("*.h")]
    return any(d.stat().st_mtime > t for d in deps)


def _run(cmd: list[str]) -> None:
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")


def _compile_many(jobs: list[tuple[list[str], Path]], workers: int) -> None:
    todo = [cmd for cmd, _ in jobs]
    if not todo:
        return
    with cf.ThreadPoolExecutor(max_workers=max(1, workers)) as ex:
        list(ex.map(_run, todo))


def build_kernels(force: bool = False, workers: int | None = None, verbose: bool = False) -> Path:
    src_dir = PKG / "csrc" / "kernels"
    out = PKG / f"_C{EXT}"
    OBJ.mkdir(parents=True, exist_ok=True)
    flags = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wno-unused-result"] + _py_includes()
    # FN_BUILD_EXPERIMENTS=1: also the measured-slower / timing-only kernel variants (the int8
    # fp8-stem instance, the FN_TILE_DBG / FN_F8_DBG timing instances) -- off by default (compile
    # time, code size, test surface)
    if os.environ.get("FN_BUILD_EXPERIMENTS", "0") == "1":
        flags.append("-DFN_EXPERIMENTS=1")
    stamp = OBJ / "kernel_flags.txt"
    if not stamp.exists() or stamp.read_text() != " ".join(flags):
        force = True                             # (a flag change rebuilds every object)
        stamp.write_text(" ".join(flags))
    srcs = sorted(src_dir.glob("*.hip")) + sorted(src_dir.glob("*.cpp"))
    jobs, objs = [], []
    for s in srcs:
        o = OBJ / f"k_{s.stem}.o"
        objs.append(o)
        if force or _newer(s, o):
            jobs.append(([HIPCC, *flags, "-c", str(s), "-o", str(o)], o))
    workers = workers or min(8, os.cpu_count() or 4)
    if verbose and jobs:
        print(f"[featurenet_amd] compiling {len(jobs)} kernel sources for {ARCH}", flush=True)
    _compile_many(jobs, workers)
    if jobs or force or not out.exists():
        _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *map(str, objs), "-o", str(out)])
    return out


def build_runtime(force: bool = False, workers: int | None = None, verbose: bool = False) -> Path | None:
    src_dir = PKG / "csrc" / "runtime"
    srcs = sorted(src_dir.glob("*.cpp"))
    if not srcs:
        return None
    out = PKG / f"_rt{EXT}"
    OBJ.mkdir(parents=True, exist_ok=True)
    cxx = os.environ.get("CXX", "g++")
    flags = ["-O3", "-std=c++17", "-fPIC", "-fvisibility=hidden", "-Wall", "-Wno-sign-compare"] + _py_includes()
    jobs, objs = [], []
    for s in srcs:
        o = OBJ / f"rt_{s.stem}.o"
        objs.append(o)
        if force or _newer(s, o):
            jobs.append(([cxx, *flags, "-c", str(s), "-o", str(o)], o))
    workers = workers or min(8, os.cpu_count() or 4)
    if verbose and jobs:
        print(f"[featurenet_amd] compiling {len(jobs)} runtime sources", flush=True)
    _compile_many(jobs, workers)
    if jobs or force or not out.exists():
        _run([cxx, "-shared", "-fPIC", *map(str, objs), "-o", str(out), "-lpthread"])
    return out


def build_runtime_sanitized(out_dir: str | Path | None = None, sanitizers: str = "address,undefined") -> Path:
    """The host runtime ``_rt`` built with -fsanitize (ASan + UBSan) into its own
    directory (sanitizers on host code; GPU sanitizers are not used).
    Load it in a fresh process with ``LD_PRELOAD=$(g++ -print-file-name=libasan.so)``."""
    src_dir = PKG / "csrc" / "runtime"
    out_dir = Path(out_dir or (ROOT / "build" / "asan"))
    out_dir.mkdir(parents=True, exist_ok=True)
    out = out_dir / f"_rt{EXT}"
    cxx = os.environ.get("CXX", "g++")
    flags = ["-O1", "-g", "-std=c++17", "-fPIC", f"-fsanitize={sanitizers}", "-fno-omit-frame-pointer",
             "-fno-sanitize-recover=undefined"] + _py_includes()
    srcs = sorted(src_dir.glob("*.cpp"))
    if not out.exists() or any(_newer(s, out) for s in srcs):
        _run([cxx, *flags, "-shared", *map(str, srcs), "-o", str(out), "-lpthread"])
    return out


def build_all(force: bool = False, verbose: bool = True) -> None:
    build_runtime(force=force, verbose=verbose)
    build_kernels(force=force, verbose=verbose)


if __name__ == "__main__":
    build_all(force="--force" in sys.argv)
