"""Registers, spills and scratch of every k_render_fast instantiation, from hipcc's
-Rpass-analysis=kernel-resource-usage remarks (no GPU needed).

    python tools/resource_usage.py [SOURCE.hip ...]      (default: csrc/rtx_kernels.hip)

Compiles each source for gfx950 with the library's flags (device only, in parallel) and prints one
row per instantiation: template arguments <B, LDS, DEEP, LVL, STATS, TP, IMG, NSPH[, WAVES]>, VGPRs, VGPR spills, scratch
bytes per lane and occupancy, side by side for the sources given (A/B variants of the kernel file
must sit next to it, e.g. csrc/_ab_x.hip, so that its relative #include resolves).
"""

from __future__ import annotations

import re
import subprocess
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))

from python_ray_tracer_amd import _build  # noqa: E402

FLAGS = [f for f in _build.HIPCC_FLAGS if f not in ("-fPIC", "-shared")]


def demangle_args(name: str) -> str:
    # <B, LDS, DEEP (bool before round 6's split, int 0/1/2 since), LVL, STATS, TP, IMG[, NSPH[, WAVES]]>
    m = re.search(r"k_render_fastILi(\d+)ELb(\d)EL[bi](\d)ELb(\d)ELb(\d)ELi(\d)ELb(\d)E(?:Li(\d+)E)?(?:Li(\d+)E)?", name)
    if not m:
        return name
    g = [x for x in m.groups() if x is not None]
    return "<" + ",".join(g) + ">"


def usage(text: str) -> dict:
    out, cur = {}, None
    for line in text.splitlines():
        m = re.search(r"remark: Function Name: (\S+)", line)
        if m:
            cur = m.group(1) if "k_render_fast" in m.group(1) else None
            if cur:
                out[cur] = {}
            continue
        m = re.search(r"remark:\s+([A-Za-z /\[\]]+?):\s+(\S+) \[", line)
        if cur and m:
            out[cur][m.group(1).strip()] = m.group(2)
    return out


def main():
    # default: the library's two units (the small-scene kernels live in rtx_small.hip, built with
    # _build.SMALL_FLAGS); each source is a column
    srcs = [Path(s) for s in sys.argv[1:]] or [_build.SRC, _build.SMALL_SRC]
    procs = [subprocess.Popen([_build.hipcc(), *FLAGS, *(_build.SMALL_FLAGS if "small" in s.name else []),
                               "--cuda-device-only", "-c",
                               "-Rpass-analysis=kernel-resource-usage", "-o", "/dev/null", str(s)],
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True) for s in srcs]
    res = [usage(p.communicate()[0]) for p in procs]
    names = sorted(set().union(*res), key=demangle_args)
    print("instantiation".ljust(18) + "".join(f"| {s.stem[:22]:22s} vgpr spill scr occ " for s in srcs))
    for n in names:
        row = demangle_args(n).ljust(18)
        for r in res:
            u = r.get(n, {})
            row += "| {:22s} {:>4} {:>5} {:>3} {:>3} ".format("", u.get("VGPRs", "-"), u.get("VGPRs Spill", "-"),
                                                             u.get("ScratchSize [bytes/lane]", "-"),
                                                             u.get("Occupancy [waves/SIMD]", "-"))
        print(row)


if __name__ == "__main__":
    main()
