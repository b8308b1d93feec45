"""profiles/pmc_traffic.json from the ``pmc:C`` steps of a tools/session.sh session (before round 6:
tools/gpu_pmc.sh, in git history): HBM bytes per k_render_fast launch
per config (median over the timed instantiation's dispatches; FETCH_SIZE x2 + WRITE_SIZE, the
calibration of profiles/r2_traffic_calibration.txt), which bench.py reports as roofline.traffic.

    python tools/pmc_traffic_json.py gpurun_out/<tag> [--out profiles/pmc_traffic.json]
"""

from __future__ import annotations

import argparse
import csv
import json
import statistics
from pathlib import Path

FRAME_PX = {"C1": 960 * 540, "C2": 1920 * 1080, "C2main": 1920 * 1080, "C3": 3840 * 2160, "C4": 7680 * 4320,
            "C5": 32 * 1920 * 1080}


def per_launch(d: Path, counter: str) -> float | None:
    vals = []
    for f in d.glob("**/run_counter_collection.csv"):
        with f.open() as fh:
            for row in csv.DictReader(fh):
                name = row["Kernel_Name"]
                tmpl = name.split("k_render_fast<", 1)[-1].split(">", 1)[0] if "k_render_fast<" in name else ""
                args = [t.strip() for t in tmpl.split(",")]
                if len(args) >= 5 and args[4] == "false" and row["Counter_Name"] == counter:  # STATS = false
                    vals.append(float(row["Counter_Value"]))
    return statistics.median(vals) if vals else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--out", default="profiles/pmc_traffic.json")
    ap.add_argument("--keep", default="", help="configs whose previous entries stay (kernel unchanged since)")
    a = ap.parse_args()
    root = Path(a.root)
    out = Path(a.out)
    old = json.loads(out.read_text()) if out.exists() else {}
    keep = set(a.keep.split(",")) if a.keep else set()
    res = {k: v for k, v in old.items() if k.startswith("_") or k in keep}
    res["_source"] = (f"median per k_render_fast launch (timed instantiation, STATS=false), rocprofv3 --pmc "
                      f"FETCH_SIZE / WRITE_SIZE in separate runs of bench.py, {root}")
    for c, px in FRAME_PX.items():
        rd = per_launch(root / f"{c}_fetch", "FETCH_SIZE") or per_launch(root / f"pmc_{c}" / "fetch", "FETCH_SIZE")
        wr = per_launch(root / f"{c}_write", "WRITE_SIZE") or per_launch(root / f"pmc_{c}" / "write", "WRITE_SIZE")
        if rd is None or wr is None:
            continue
        frame = 12 * px
        res[c] = {"kernel": "k_render_fast (timed instantiation)", "fetch_bytes_raw": round(rd * 1024),
                  "fetch_bytes_x2": round(rd * 2048), "write_bytes": round(wr * 1024),
                  "hbm_bytes_per_launch": round(rd * 2048 + wr * 1024), "frame_bytes": frame,
                  "traffic_over_frame": round((rd * 2048 + wr * 1024) / frame, 3)}
    out.write_text(json.dumps(res, indent=1))
    for c in FRAME_PX:
        if c in res:
            print(c, res[c]["hbm_bytes_per_launch"], res[c]["traffic_over_frame"])


if __name__ == "__main__":
    main()
