"""Build ``librtx_hip.so`` in-tree with hipcc for gfx950 (no JIT cache: the .so travels with the repo
snapshot to the GPU box)."""

from __future__ import annotations

import os
import shutil
import subprocess
from pathlib import Path

PKG = Path(__file__).resolve().parent
REPO = PKG.parent
SRC = PKG / "csrc" / "rtx_kernels.hip"
HDR = REPO / "include" / "rtx_hip.h"
LIB = PKG / "librtx_hip.so"

# -ffp-contract=off: NumPy never fuses a*b+c, and FMA contraction would move linspace / checker
# boundaries. No fast-math: sqrt and division stay correctly rounded.
HIPCC_FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fPIC", "-shared",
               "-Wall", "-Wno-unused-function", "-Wno-unused-result",
               # MachineLICM hoists the ocml sin polynomial constants out of the bounce loop into VGPRs,
               # which then spill at 128 VGPRs; A/B (profiles/r1_ab_variants.txt): faster on every config
               "-mllvm", "-disable-machine-licm"]


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and Path(cand).exists():
            return cand
    raise FileNotFoundError("hipcc not found (ROCm is required to build the HIP backend)")


def needs_build() -> bool:
    if not LIB.exists():
        return True
    t = LIB.stat().st_mtime
    return any(p.stat().st_mtime > t for p in (SRC, HDR, Path(__file__)))


def build_library(force: bool = False, extra_flags=(), out: Path | None = None, verbose: bool = False) -> Path:
    out = LIB if out is None else Path(out)
    if not force and out == LIB and not needs_build():
        return out
    cmd = [hipcc(), *HIPCC_FLAGS, *extra_flags, "-o", str(out), str(SRC)]
    if verbose:
        print(" ".join(cmd))
    tmp = out.with_suffix(".so.tmp")
    cmd[-2] = str(tmp)
    subprocess.run(cmd, check=True, cwd=str(REPO))
    os.replace(tmp, out)
    return out


if __name__ == "__main__":
    print(build_library(force=True, verbose=True))
