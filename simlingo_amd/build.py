"""In-tree build of libslx_hip.so (gfx950) with hipcc — no cmake, no JIT cache.

`python -m simlingo_amd.build` compiles every csrc/*.hip to an object (in parallel, incremental
on mtime) and links the shared library next to the sources, so it travels with the repo snapshot
to the GPU box.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import subprocess
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent
CSRC = HERE / "csrc"
INCLUDE = HERE.parent / "include"
OUT = CSRC / "libslx_hip.so"
BUILD_DIR = CSRC / "build"
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("SLX_OFFLOAD_ARCH", "gfx950")
FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-munsafe-fp-atomics",
         f"-I{INCLUDE}", f"-I{CSRC}"]
# Per-source flags. attention.hip: no SLP packing of f32 math (v_pk_mul/add_f32 issue at ~5x the cost of the two
# scalar ops they replace when placed between MFMAs, MI355X_MICROARCH.md 'price of one filler beside MFMAs').
PER_FILE = {"attention.hip": ["-fno-slp-vectorize"]}


def _needs(obj: Path, deps: list[Path]) -> bool:
    if not obj.exists():
        return True
    deps = deps + [Path(__file__)]
    t = obj.stat().st_mtime
    return any(d.stat().st_mtime > t for d in deps)


def _compile(src: Path, extra: list[str]) -> Path:
    obj = BUILD_DIR / (src.stem + ".o")
    headers = list(CSRC.glob("*.h")) + list(INCLUDE.glob("*.h"))
    if _needs(obj, [src] + headers):
        cmd = [HIPCC, *FLAGS, *PER_FILE.get(src.name, []), *extra, "-c", str(src), "-o", str(obj)]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed for {src.name}:\n{r.stdout}\n{r.stderr}")
    return obj


def build(verbose: bool = True, jobs: int | None = None, extra: list[str] | None = None) -> Path:
    BUILD_DIR.mkdir(exist_ok=True)
    srcs = sorted(CSRC.glob("*.hip"))
    jobs = jobs or min(8, os.cpu_count() or 4)
    with cf.ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, extra or []), srcs))
    if _needs(OUT, objs):
        # hipBLASLt: slx_gemm_lt (csrc/blaslt.hip), the vendor library for the plain GEMMs it runs faster
        cmd = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", *map(str, objs), "-lhipblaslt", "-o", str(OUT)]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
    if verbose:
        print(f"[slx] built {OUT} ({len(srcs)} sources)")
    return OUT


if __name__ == "__main__":
    build()
    sys.exit(0)
