"""Build recipe for libmolclr_hip.so (gfx950, in-tree).

Every ``molclr_amd/csrc/*.hip`` file is compiled with ``hipcc
--offload-arch=gfx950`` into an object file under ``build/`` and linked into
``molclr_amd/libmolclr_hip.so``, the C-ABI library declared by
``include/molclr.h``.  Objects are rebuilt only when a source or header is
newer.  Run as ``python -m molclr_amd.build`` or call :func:`build`.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = PKG / "csrc"
INCLUDE = ROOT / "include"
BUILD = ROOT / "build" / "hip"
LIB = PKG / "libmolclr_hip.so"
ARCH = os.environ.get("MOLCLR_OFFLOAD_ARCH", "gfx950")

CXXFLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-fvisibility=hidden",
            "-mcode-object-version=5",
            "-Wall", "-Wno-unused-function"]


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and Path(cand).exists():
            return cand
    raise RuntimeError("hipcc not found (ROCm is required to build molclr_amd)")


def _headers() -> list[Path]:
    return list(CSRC.glob("*.h")) + list(INCLUDE.glob("*.h"))


def _stale(target: Path, deps: list[Path]) -> bool:
    if not target.exists():
        return True
    t = target.stat().st_mtime
    return any(d.stat().st_mtime > t for d in deps)


def build(verbose: bool = False, jobs: int | None = None) -> Path:
    hipcc = _hipcc()
    BUILD.mkdir(parents=True, exist_ok=True)
    sources = sorted(CSRC.glob("*.hip"))
    headers = _headers()
    objs = []
    todo = []
    for src in sources:
        obj = BUILD / (src.stem + ".o")
        objs.append(obj)
        if _stale(obj, [src] + headers):
            todo.append((src, obj))

    def compile_one(item):
        src, obj = item
        cmd = [hipcc, *CXXFLAGS, "-I", str(INCLUDE), "-c", str(src), "-o", str(obj)]
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed for {src.name}:\n{r.stdout}\n{r.stderr}")
        return src.name

    if todo:
        n = jobs or min(len(todo), max(1, min(8, os.cpu_count() or 1)))
        with cf.ThreadPoolExecutor(n) as ex:
            for name in ex.map(compile_one, todo):
                if verbose:
                    print(f"compiled {name}", flush=True)
    if todo or _stale(LIB, objs):
        tmp = LIB.with_suffix(".so.tmp")
        cmd = [hipcc, "-shared", "-fPIC", f"--offload-arch={ARCH}", *map(str, objs), "-o", str(tmp)]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
        os.replace(tmp, LIB)
        if verbose:
            print(f"linked {LIB}", flush=True)
    return LIB


if __name__ == "__main__":
    build(verbose="-v" in sys.argv)
