"""Build libspimdecon.so in-tree with hipcc for gfx950 (no JIT cache, no pip install).

    python -m spim_registration_amd.build [--force] [-j N]

Objects go to ``spim_registration_amd/_build/``; the shared library to
``spim_registration_amd/libspimdecon.so`` (git-ignored, shipped to the GPU box by
gpurun's snapshot).
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = PKG / "csrc"
BUILD = PKG / "_build"
LIB = PKG / "libspimdecon.so"
INCLUDE = ROOT / "include"
ROCM = Path(os.environ.get("ROCM_PATH", "/opt/rocm"))
ARCH = os.environ.get("SPIMDECON_ARCH", "gfx950")

CXXFLAGS = [
    "-O3", "-fPIC", "-std=c++17", f"--offload-arch={ARCH}",
    "-ffp-contract=off",            # keep the Java float op order (no FMA contraction)
    "-Wall", "-Wno-unused-function", "-Wno-unused-result",
    f"-I{INCLUDE}", f"-I{ROCM / 'include'}",
]
LDFLAGS = [f"-L{ROCM / 'lib'}", "-lrocfft", "-lrccl", f"-Wl,-rpath,{ROCM / 'lib'}"]


def hipcc() -> str:
    p = shutil.which("hipcc") or str(ROCM / "bin" / "hipcc")
    if not Path(p).exists():
        raise RuntimeError("hipcc not found; cannot build libspimdecon.so")
    return p


def _sources():
    return sorted(list(CSRC.glob("*.hip")) + list(CSRC.glob("*.cpp")))


def _headers():
    return list(CSRC.glob("*.hpp")) + list(CSRC.glob("*.inc")) + list(INCLUDE.glob("*.h"))


def _stale(obj: Path, src: Path, hdr_mtime: float) -> bool:
    if not obj.exists():
        return True
    m = obj.stat().st_mtime
    return src.stat().st_mtime > m or hdr_mtime > m


def _compile(src: Path, force: bool, hdr_mtime: float) -> Path:
    obj = BUILD / (src.name + ".o")
    if not force and not _stale(obj, src, hdr_mtime):
        return obj
    cmd = [hipcc(), *CXXFLAGS]
    if src.suffix == ".hip":
        cmd += ["-x", "hip"]
    cmd += ["-c", str(src), "-o", str(obj)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src.name}:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return obj


def build(force: bool = False, jobs: int | None = None, verbose: bool = True) -> Path:
    BUILD.mkdir(exist_ok=True)
    hdr_mtime = max((h.stat().st_mtime for h in _headers()), default=0.0)
    srcs = _sources()
    jobs = jobs or min(8, os.cpu_count() or 4)
    with cf.ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, force, hdr_mtime), srcs))
    newest = max(o.stat().st_mtime for o in objs)
    if force or not LIB.exists() or LIB.stat().st_mtime < newest:
        tmp = LIB.with_suffix(".so.tmp")
        cmd = [hipcc(), f"--offload-arch={ARCH}", "-shared", "-o", str(tmp), *map(str, objs), *LDFLAGS]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        os.replace(tmp, LIB)
        if verbose:
            print(f"[spimdecon] built {LIB}", file=sys.stderr)
    return LIB


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", type=int, default=None)
    a = ap.parse_args()
    build(force=a.force, jobs=a.j)


if __name__ == "__main__":
    main()
