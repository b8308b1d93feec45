"""Static instruction budget of one kernel in a gfx950 assembly dump, by source function.

    hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -mllvm -disable-machine-licm \
          -gline-tables-only --cuda-device-only -S -o rtx.s python_ray_tracer_amd/csrc/rtx_kernels.hip
    python tools/isa_budget.py rtx.s '_ZN12_GLOBAL__N_113k_render_fastILi3ELb1ELb0ELb1ELb0EEEvNS_6ParamsE'

Every instruction is attributed to the innermost source line of its `.loc` (inlined helpers keep
their own lines) and that line to the enclosing function of rtx_kernels.hip; instructions are
classified (f64 arithmetic, f64 transcendental, compares, 64-bit selects, moves, other VALU, SALU,
scalar/vector/LDS memory, scratch, waitcnt, branches). Static counts: a loop body counts once. The
register/spill metadata of the kernel is printed too.
"""

from __future__ import annotations

import re
import sys
from collections import Counter, defaultdict
from pathlib import Path

SRC = Path(__file__).resolve().parent.parent / "python_ray_tracer_amd" / "csrc" / "rtx_kernels.hip"

CLASSES = ("f64", "f64_trans", "cmp", "cndmask", "mov", "valu_other", "salu", "smem", "lds", "vmem", "scratch",
           "waitcnt", "branch", "other")


def classify(op: str) -> str:
    if op.startswith("v_"):
        if op in ("v_rcp_f64", "v_rsq_f64", "v_sqrt_f64", "v_rcp_f64_e32", "v_rsq_f64_e32", "v_sqrt_f64_e32"):
            return "f64_trans"
        base = op.replace("_e32", "").replace("_e64", "")
        if base.endswith("_f64") and not base.startswith(("v_cmp", "v_cvt", "v_readlane", "v_mov")):
            return "f64"
        if base.startswith(("v_cmp", "v_cmpx")):
            return "cmp"
        if base.startswith("v_cndmask"):
            return "cndmask"
        if base.startswith(("v_mov", "v_readfirstlane", "v_readlane", "v_writelane", "v_accvgpr")):
            return "mov"
        return "valu_other"
    if op.startswith("s_waitcnt"):
        return "waitcnt"
    if op.startswith(("s_cbranch", "s_branch", "s_setpc", "s_swappc", "s_endpgm")):
        return "branch"
    if op.startswith(("s_load", "s_buffer_load", "s_store", "s_buffer_store", "s_dcache")):
        return "smem"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith("scratch_"):
        return "scratch"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "vmem"
    return "other"


def source_functions(path: Path):
    """[(first_line, last_line, name)] of the top-level functions of the .hip source."""
    lines = path.read_text().splitlines()
    out = []
    start = None
    name = None
    depth = 0
    for i, line in enumerate(lines, 1):
        if depth == 0 and start is None:
            m = re.match(r"^(?:template\s*<.*>\s*)?(?:__host__\s+)?(?:__global__|__device__|static|int|void|size_t|"
                         r"dim3|WsLayout|int64_t|inline|constexpr)\b.*?\b(\w+)\s*\(", line)
            if m and not line.rstrip().endswith(";"):
                start, name = i, m.group(1)
        if re.match(r"^(namespace\b.*\{|\}\s*//\s*namespace|extern \"C\" \{|\}\s*//\s*extern)", line):
            continue  # namespace / extern "C" braces do not nest functions
        depth += line.count("{") - line.count("}")
        if start is not None and depth == 0 and "{" in "".join(lines[start - 1:i]):
            out.append((start, i, name))
            start = None
    return out


def _chain(comment: str):
    """Source lines of a .loc comment's inline chain, innermost first (file rtx_kernels.hip)."""
    return [int(m) for m in re.findall(r"rtx_kernels\.hip:(\d+):\d+", comment)]


def stages(asm_path: str, symbol: str, root_line: int, outer: tuple, inner: tuple | None = None):
    """Per-stage static budget of the code inlined at kernel line ``root_line`` (one fast_tile call
    site): an instruction's stage is the line of its inline chain that lies in ``outer`` (first,
    last source line: the function whose call sites name the stages, e.g. fast_tile); inside
    ``inner`` (e.g. shade) it is refined by the line there."""
    out = defaultdict(Counter)
    inside = False
    chain = []
    with open(asm_path) as f:
        for raw in f:
            if not inside:
                if raw.startswith(symbol + ":"):
                    inside = True
                continue
            s = raw.strip()
            if s.startswith(".Lfunc_end") or s.startswith("; -- End function"):
                break
            if s.startswith(".loc"):
                chain = _chain(s)
                continue
            if not s or s.startswith((".", ";", "//")) or s.endswith(":"):
                continue
            if not chain or chain[-1] != root_line:
                continue
            st = next((ln for ln in chain if outer[0] <= ln <= outer[1]), None)
            key = f"L{st}" if st is not None else "kernel"
            if inner is not None:
                sub = next((ln for ln in chain if inner[0] <= ln <= inner[1]), None)
                if sub is not None:
                    key += f"/L{sub}"
            out[key][classify(s.split()[0])] += 1
    return out


def main(asm_path: str, symbol: str) -> None:
    funcs = source_functions(SRC)

    def func_of(line: int) -> str:
        for a, b, n in funcs:
            if a <= line <= b:
                return n
        return f"line{line}"

    by_func = defaultdict(Counter)
    by_line = defaultdict(Counter)
    meta = {}
    # the .file index of rtx_kernels.hip (0 when it is the compiled unit; rtx_small.hip includes it)
    kfile = "0"
    with open(asm_path) as f:
        for raw in f:
            m = re.match(r'\s*\.file\s+(\d+)\s+"[^"]*"(?:\s+"([^"]*)")?', raw)
            if m and (m.group(2) or "").endswith(SRC.name) or (m and m.group(2) is None and SRC.name in raw):
                kfile = m.group(1)
                break
    inside = False
    cur = ("?", 0)
    with open(asm_path) as f:
        for raw in f:
            if not inside:
                if raw.startswith(symbol + ":"):
                    inside = True
                continue
            s = raw.strip()
            if s.startswith(".Lfunc_end") or s.startswith("; -- End function"):
                break
            if s.startswith(".loc"):
                parts = s.split()
                cur = (parts[1], int(parts[2]))
                continue
            if not s or s.startswith((".", ";", "//")) or s.endswith(":"):
                continue
            op = s.split()[0]
            c = classify(op)
            key = func_of(cur[1]) if cur[0] == kfile else f"hdr{cur[0]}"
            by_func[key][c] += 1
            by_line[cur][c] += 1
    # kernel resource metadata (the .amdhsa block after the function)
    text = Path(asm_path).read_text(errors="replace")
    i = text.find(f".amdhsa_kernel {symbol}")
    if i >= 0:
        blk = text[i:text.find(".end_amdhsa_kernel", i)]
        for k in ("amdhsa_next_free_vgpr", "amdhsa_accum_offset", "amdhsa_private_segment_fixed_size",
                  "amdhsa_group_segment_fixed_size"):
            m = re.search(rf"\.{k}\s+(\d+)", blk)
            if m:
                meta[k] = int(m.group(1))
    j = text.find(f"; -- End function", text.find(symbol + ":"))
    tail = text[j - 4000:j] if j > 0 else ""
    for k in ("NumVgprs", "NumAgprs", "ScratchSize", "Occupancy", "SGPRBlocks", "NumSgprs"):
        m = re.search(rf"; {k}: (\d+)", tail)
        if m:
            meta[k] = int(m.group(1))
    total = Counter()
    for c in by_func.values():
        total.update(c)
    print(f"kernel {symbol}")
    print("metadata:", meta)
    hdr = f"{'function':28s}" + "".join(f"{c:>10s}" for c in CLASSES) + f"{'total':>8s}"
    print(hdr)
    for name, c in sorted(by_func.items(), key=lambda kv: -sum(kv[1].values())):
        print(f"{name:28s}" + "".join(f"{c[k]:10d}" for k in CLASSES) + f"{sum(c.values()):8d}")
    print(f"{'TOTAL':28s}" + "".join(f"{total[k]:10d}" for k in CLASSES) + f"{sum(total.values()):8d}")
    print(f"\ntop source lines (file {kfile} = rtx_kernels.hip):")
    for (fi, ln), c in sorted(by_line.items(), key=lambda kv: -sum(kv[1].values()))[:40]:
        src = SRC.read_text().splitlines()[ln - 1].strip()[:70] if fi == kfile and ln > 0 else ""
        print(f"  {fi}:{ln:5d} {sum(c.values()):5d}  {dict(c.most_common(4))}  {src}")


def print_stages(asm_path: str, symbol: str, root_line: int, outer: tuple, inner: tuple | None = None) -> None:
    lines = SRC.read_text().splitlines()
    st = stages(asm_path, symbol, root_line, outer, inner)
    total = Counter()
    print(f"stages of the code inlined at line {root_line} (stage = call line in {outer}, refined in {inner})")
    print(f"{'stage':16s}" + "".join(f"{c:>9s}" for c in CLASSES) + f"{'total':>7s}  source")
    for key in sorted(st, key=lambda k: [int(x[1:]) if x[1:].isdigit() else 0 for x in k.split("/")]):
        c = st[key]
        total.update(c)
        ln = int(key.split("/")[-1][1:]) if key != "kernel" else 0
        src = lines[ln - 1].strip()[:60] if ln else ""
        print(f"{key:16s}" + "".join(f"{c[k]:9d}" for k in CLASSES) + f"{sum(c.values()):7d}  {src}")
    print(f"{'TOTAL':16s}" + "".join(f"{total[k]:9d}" for k in CLASSES) + f"{sum(total.values()):7d}")


if __name__ == "__main__":
    if len(sys.argv) > 3:  # asm symbol root_line outer_a outer_b [inner_a inner_b]
        a = [int(v) for v in sys.argv[3:]]
        print_stages(sys.argv[1], sys.argv[2], a[0], (a[1], a[2]), (a[3], a[4]) if len(a) > 4 else None)
    else:
        main(sys.argv[1], sys.argv[2])
