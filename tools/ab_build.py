"""Build librtx_hip.so variants for tools/ab.py (A/B timing on identical output).

    python tools/ab_build.py OUT.so [--set kName=VALUE ...] [--rev GIT_REV] [--patch FILE.py]

The shipped kernel has no tuning macros: its tuning values are ``constexpr`` lines in
``csrc/rtx_kernels.hip``. A variant rewrites those lines (``--set kFwdWavesPersist=5``), takes the
source of another revision (``--rev HEAD~3``: the baseline of an A/B), or applies a Python file
defining ``patch(src: str) -> str``, and compiles it with the library's own flags next to the
original (so its relative #include resolves). (Rounds 2-5 kept a set of named source patches,
tools/ab_patches.py; round 6 retired it with the experiments it served, whose results are in
profiles/ and DESIGN.md, and which stay in git history.)
"""

import argparse
import re
import runpy
import subprocess
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))

from python_ray_tracer_amd import _build  # noqa: E402


def trim(src: str, caps: set) -> str:
    """Instantiate only the capped fast kernels of `caps` (timing builds: other caps, unbounded
    renders and stats buffers then launch nothing)."""
    def sub(old, new):
        nonlocal src
        if old not in src:
            raise SystemExit(f"--only-b: pattern not found: {old!r}")
        src = src.replace(old, new)

    for b in range(6):
        if b not in caps:
            sub(f"    case {b}: launch_fast_b<{b}>(p, grid, s); break;\n", "")
    if 6 not in caps:
        sub("    default: launch_fast_b<6>(p, grid, s); break;", "    default: break;")
    sub("{ launch_fast_b<kDeepLevels, 1>(p, grid, s); }", "{}")
    sub("{ launch_fast_b<kDeepLevels, 2>(p, grid, s); }", "{}")
    sub("    launch_fast_lds_s<B, DEEP, LVL, true>(p, grid, s);", "    launch_fast_lds_s<B, DEEP, LVL, false>(p, grid, s);")
    return src


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--set", action="append", default=[], help="kName=VALUE (a constexpr tuning line)")
    ap.add_argument("--rev", default=None, help="git revision of csrc/rtx_kernels.hip to build")
    ap.add_argument("--patch", default=None, help="a python file defining patch(src) -> src")
    ap.add_argument("--flag", action="append", default=[], help="extra hipcc flag")
    ap.add_argument("--small-flag", action="append", default=None,
                    help="hipcc flag of the small-scene unit only (replaces _build.SMALL_FLAGS)")
    ap.add_argument("--only-b", default=None,
                    help="comma list of bounce caps to instantiate (A/B builds in ~1/10 of the time: no "
                         "other caps, no deep/unbounded kernels, no stats instantiations)")
    a = ap.parse_args()
    rel = _build.SRC.relative_to(REPO)
    if a.rev:
        src = subprocess.run(["git", "show", f"{a.rev}:{rel}"], cwd=REPO, check=True, capture_output=True,
                             text=True).stdout
    else:
        src = _build.SRC.read_text()
    for kv in a.set:
        name, val = kv.split("=", 1)
        pat = re.compile(rf"^(constexpr\s+\w+\s+{re.escape(name)}\s*=\s*)([^;]+)(;)", re.M)
        src, n = pat.subn(lambda m: m.group(1) + val + m.group(3), src)
        if n != 1:
            raise SystemExit(f"--set {name}: {n} matching constexpr lines")
    if a.patch:
        src = runpy.run_path(a.patch)["patch"](src)
    if a.only_b is not None:
        src = trim(src, {int(b) for b in a.only_b.split(",") if b})
    tmp = _build.SRC.with_name(f"_ab_{Path(a.out).stem}.hip")
    tmp.write_text(src)
    # sources split in two units (RTX_DEVICE_CODE_ONLY: rtx_small.hip includes the kernel file) get
    # the small unit too, including the variant's text; older single-unit revisions build alone
    small = None
    if "RTX_DEVICE_CODE_ONLY" in src:
        small_src = (subprocess.run(["git", "show", f"{a.rev}:{_build.SMALL_SRC.relative_to(REPO)}"], cwd=REPO,
                                    check=True, capture_output=True, text=True).stdout
                     if a.rev else _build.SMALL_SRC.read_text())
        small = _build.SRC.with_name(f"_ab_{Path(a.out).stem}_small.hip")
        small.write_text(small_src.replace('#include "rtx_kernels.hip"', f'#include "{tmp.name}"'))
    try:
        out = Path(a.out).resolve()
        out.parent.mkdir(parents=True, exist_ok=True)
        _build.compile_units(out, tmp, small, a.flag, small_flags=a.small_flag)
    finally:
        tmp.unlink(missing_ok=True)
        if small is not None:
            small.unlink(missing_ok=True)
    print(out)


if __name__ == "__main__":
    main()
