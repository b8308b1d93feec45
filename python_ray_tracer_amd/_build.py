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
SMALL_SRC = PKG / "csrc" / "rtx_small.hip"  # includes SRC's device code
TILES_SRC = PKG / "csrc" / "rtx_tiles.hip"  # host code: the row-tiled multi-GPU frame (RCCL at run time)
HDR = REPO / "include" / "rtx_hip.h"
LIB = PKG / "librtx_hip.so"
OPS_SRC = PKG / "csrc" / "rt_ops.cpp"
OPS_LIB = PKG / "librt_ops.so"

# -ffp-contract=off: NumPy never fuses a*b+c, and FMA contraction would move linspace / checker
# boundaries. No fast-math: sqrt and division stay correctly rounded.
HIPCC_FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fPIC",
               "-Wall", "-Wno-unused-function", "-Wno-unused-result",
               # MachineLICM hoists the ocml sin polynomial constants out of the bounce loop into VGPRs,
               # which then spill at 128 VGPRs; A/B (profiles/r1_ab_variants.txt): faster on every config
               "-mllvm", "-disable-machine-licm"]
# rtx_small.hip only (the TREE = false kernels). Round 3 built them with the max-ilp machine
# scheduler (profiles/r3_ab_variants.txt: C2 -0.5..-0.9%, C1 -2.4%); with the forward fold of round 5
# the default scheduler is the faster one (A/B r5i: C2 -0.8%, C1 -0.9%, C2main -0.4%). The unit
# stays separate so that its flags can differ from the culled kernels'.
SMALL_FLAGS: list = []


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and Path(cand).exists():
            return cand
    raise FileNotFoundError("hipcc not found (ROCm is required to build the HIP backend)")


def needs_build() -> bool:
    if not LIB.exists():
        return True
    t = LIB.stat().st_mtime
    return any(p.stat().st_mtime > t for p in (SRC, SMALL_SRC, TILES_SRC, HDR, Path(__file__)))


OBJ_CACHE = PKG / ".objcache"  # compiled units by content hash (a one-unit change rebuilds one unit)


def _unit_key(src: Path, flags) -> str:
    """Hash of a unit's text, the text of every file it #includes (recursively, quoted includes) and
    its compile command's flags."""
    import hashlib
    import re

    h = hashlib.sha256()
    seen, todo = set(), [src.resolve()]
    while todo:
        f = todo.pop()
        if f in seen or not f.exists():
            continue
        seen.add(f)
        text = f.read_bytes()
        h.update(str(f.name).encode() + b"\0" + text)
        todo += [(f.parent / m.decode()).resolve() for m in re.findall(rb'#include\s+"([^"]+)"', text)]
    h.update(repr([hipcc(), *flags]).encode())
    return h.hexdigest()[:32]


def compile_units(out: Path, main_src: Path, small_src: Path | None, extra_flags=(), verbose: bool = False,
                  small_flags=None) -> None:
    """Compile the library's translation units to objects (in parallel) and link ``out``: main_src
    with HIPCC_FLAGS, small_src (None: a single-unit source) with SMALL_FLAGS (or small_flags) added."""
    import tempfile

    sf = list(SMALL_FLAGS if small_flags is None else small_flags)
    units = [(main_src, [])] + ([(small_src, sf)] if small_src is not None else [])
    if small_src is not None and TILES_SRC.exists():  # (single-unit revisions of the A/B tool build alone)
        units.append((TILES_SRC, []))
    objs, procs = [], []
    # objects in a directory of this call's own: concurrent builds (several ranks importing on a
    # fresh checkout) cannot overwrite or delete each other's objects before the link
    objdir = Path(tempfile.mkdtemp(prefix=f".{out.stem}.", dir=str(out.parent)))
    try:
        OBJ_CACHE.mkdir(exist_ok=True)
        fresh = []
        for src, flags in units:
            allf = [*HIPCC_FLAGS, *flags, *extra_flags]
            cached = OBJ_CACHE / f"{src.stem}.{_unit_key(src, allf)}.o"
            if cached.exists():
                objs.append(cached)
                continue
            obj = objdir / f"{src.stem}.o"
            cmd = [hipcc(), *allf, "-c", "-o", str(obj), str(src)]
            if verbose:
                print(" ".join(cmd))
            objs.append(obj)
            fresh.append((obj, cached))
            procs.append((subprocess.Popen(cmd, cwd=str(REPO)), cmd))
        for proc, cmd in procs:
            if proc.wait() != 0:
                raise subprocess.CalledProcessError(proc.returncode, cmd)
        for obj, cached in fresh:  # keep the new objects (renamed whole: concurrent builds stay safe)
            tmp = cached.with_suffix(f".o.tmp{os.getpid()}")
            shutil.copyfile(obj, tmp)
            os.replace(tmp, cached)
        cmd = [hipcc(), "--offload-arch=gfx950", "-shared", "-fPIC", "-o", str(out), *map(str, objs), "-ldl"]
        if verbose:
            print(" ".join(cmd))
        subprocess.run(cmd, check=True, cwd=str(REPO))
    finally:
        for proc, _ in procs:
            proc.wait()
        shutil.rmtree(objdir, ignore_errors=True)


def build_library(force: bool = False, extra_flags=(), out: Path | None = None, verbose: bool = False) -> Path:
    out = LIB if out is None else Path(out)
    if not force and out == LIB and not needs_build():
        return out
    tmp = out.with_suffix(f".so.tmp{os.getpid()}")  # per process: concurrent builds each rename a whole file
    try:
        compile_units(tmp, SRC, SMALL_SRC, extra_flags, verbose)
        os.replace(tmp, out)
    finally:
        tmp.unlink(missing_ok=True)
    return out


def ops_flags() -> list:
    """Compile/link flags of the TORCH_LIBRARY(rt) op library against the installed torch (the
    include and library paths torch.utils.cpp_extension would use), linked to librtx_hip.so."""
    import torch
    import torch.utils.cpp_extension as ce

    inc = [f"-I{p}" for p in ce.include_paths(device_type="cuda")]
    libdirs = [p for p in ce.library_paths(device_type="cuda") if Path(p).exists()]
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return (["-O2", "-std=c++17", "-fPIC", "-shared", "-Wall", f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-DUSE_ROCM=1", "-D__HIP_PLATFORM_AMD__=1",
             "-Wno-unused-result", "-Wno-deprecated-declarations"] + inc + [f"-L{p}" for p in libdirs]
            + [f"-L{PKG}", "-lrtx_hip", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip",
               "-Wl,-rpath,$ORIGIN"] + [f"-Wl,-rpath,{p}" for p in libdirs])


def build_ops(force: bool = False, verbose: bool = False) -> Path:
    """librt_ops.so: the PyTorch custom ops rt::* (csrc/rt_ops.cpp) over the C ABI. Host code only,
    compiled by hipcc as C++ (HIP runtime headers for c10::hip)."""
    if not force and OPS_LIB.exists() and all(p.stat().st_mtime <= OPS_LIB.stat().st_mtime
                                              for p in (OPS_SRC, HDR, LIB, Path(__file__))):
        return OPS_LIB
    tmp = OPS_LIB.with_suffix(f".so.tmp{os.getpid()}")
    cmd = [hipcc(), "-x", "c++", *ops_flags(), "-o", str(tmp), str(OPS_SRC)]
    if verbose:
        print(" ".join(cmd))
    try:
        subprocess.run(cmd, check=True, cwd=str(REPO))
        os.replace(tmp, OPS_LIB)
    finally:
        tmp.unlink(missing_ok=True)
    return OPS_LIB


STUB_SRC = REPO / "tests" / "stub_rccl.cpp"  # test-only RCCL stand-in (world > 1 tiles plans on one GPU)
STUB_LIB = REPO / "tests" / "libstub_rccl.so"


def build_test_stub(force: bool = False, verbose: bool = False) -> Path:
    """tests/libstub_rccl.so: the test-only RCCL stand-in the world > 1 tiles tests bind through
    rtx_rccl_load(path) (host code; -Bsymbolic so its own calls never resolve to torch's librccl)."""
    if not force and STUB_LIB.exists() and STUB_SRC.stat().st_mtime <= STUB_LIB.stat().st_mtime:
        return STUB_LIB
    tmp = STUB_LIB.with_suffix(f".so.tmp{os.getpid()}")
    cmd = [hipcc(), "--offload-arch=gfx950", "-O2", "-std=c++17", "-fPIC", "-shared", "-Wall", "-Wl,-Bsymbolic",
           "-o", str(tmp), str(STUB_SRC)]
    if verbose:
        print(" ".join(cmd))
    try:
        subprocess.run(cmd, check=True, cwd=str(REPO))
        os.replace(tmp, STUB_LIB)
    finally:
        tmp.unlink(missing_ok=True)
    return STUB_LIB


if __name__ == "__main__":
    print(build_library(force=True, verbose=True))
    print(build_ops(force=True, verbose=True))
    print(build_test_stub(force=True, verbose=True))
