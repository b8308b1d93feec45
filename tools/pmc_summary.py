"""Summarise rocprofv3 --pmc counter_collection.csv files per kernel.

    python tools/pmc_summary.py gpurun_out/<tag> [--kernel k_render_fast] [--json profiles/x.json]

Per kernel name: dispatch count and the mean per-dispatch value of every counter found in the
<tag>/*/run_counter_collection.csv files. HBM traffic per launch follows MI355X_MICROARCH.md §HBM:
FETCH_SIZE and WRITE_SIZE are KiB; on gfx950 FETCH_SIZE reports half the bytes of a wide coalesced
read stream, so the read side is reported both raw and x2 (the write side is exact for 16-B stores;
our stores are 4-B per lane, uncalibrated).
"""

from __future__ import annotations

import argparse
import csv
import json
from collections import defaultdict
from pathlib import Path


def load(root: Path):
    acc = defaultdict(lambda: defaultdict(list))
    for f in sorted(root.glob("*/run_counter_collection.csv")):
        with f.open() as fh:
            for row in csv.DictReader(fh):
                acc[row["Kernel_Name"]][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return acc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--kernel", default="k_render_fast")
    ap.add_argument("--json", default=None)
    ap.add_argument("--config", default="C2")
    args = ap.parse_args()
    acc = load(Path(args.root))
    out = {}
    for name, ctrs in acc.items():
        short = name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        out[short] = {k: sum(v) / len(v) for k, v in ctrs.items()}
        out[short]["_dispatches"] = max(len(v) for v in ctrs.values())
    for k, v in sorted(out.items(), key=lambda kv: kv[0]):
        print(k)
        for c, val in sorted(v.items()):
            print(f"    {c:28s} {val:,.1f}")
    sel = [k for k in out if args.kernel in k]
    if sel:
        k = sel[0]
        v = out[k]
        rd = v.get("FETCH_SIZE")
        wr = v.get("WRITE_SIZE")
        res = {"kernel": k, "counters": v}
        if rd is not None and wr is not None:
            res["fetch_bytes_raw"] = rd * 1024
            res["fetch_bytes_x2"] = rd * 2048
            res["write_bytes"] = wr * 1024
            res["hbm_bytes_per_launch"] = rd * 2048 + wr * 1024
        f64 = sum(v.get(c, 0) for c in ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_TRANS_F64"))
        if f64:
            res["valu_f64_wave_insts"] = f64 + v.get("SQ_INSTS_VALU_FMA_F64", 0)
            res["valu_f64_flops_executed"] = 64 * (f64 + 2 * v.get("SQ_INSTS_VALU_FMA_F64", 0))
        print(json.dumps({kk: vv for kk, vv in res.items() if kk != "counters"}, indent=1))
        if args.json:
            p = Path(args.json)
            d = json.loads(p.read_text()) if p.exists() else {}
            d[args.config] = res
            p.write_text(json.dumps(d, indent=1))


if __name__ == "__main__":
    main()
