"""Per-launch k_render_fast durations from a rocprofv3 --kernel-trace run of bench.py, split into
warm-up, timed region and the bench's extra launches (the counter launch and the output-path
renders), to compare with the bench line's live ``roofline.kernel_ms``.

    python tools/rocprof_summary.py gpurun_out/<tag>/prof --warmup 10 --steps 100 [--ramp 1700]
    python tools/rocprof_summary.py gpurun_out/<tag>/prof --log gpurun_out/<tag>/rocprof.log

``--log``: the profiled bench.py's output, whose JSON line gives the clock-ramp launches (bench.py
--ramp-ms runs untimed steps before the warm-up), the warm-up and the timed steps.
"""

import argparse
import csv
import statistics
from pathlib import Path


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("prof_dir")
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--kernel", default="k_render_fast")
    ap.add_argument("--prof-every", type=int, default=10, help="bench.py's sampling stride")
    ap.add_argument("--ramp", type=int, default=0, help="launches of bench.py's clock ramp (before the warm-up)")
    ap.add_argument("--log", default=None, help="bench.py's output: ramp, warm-up and steps from its JSON line")
    a = ap.parse_args()
    if a.log:
        import json

        for line in open(a.log, errors="replace"):
            if line.startswith("{") and '"metric"' in line:
                d = json.loads(line)
                a.warmup, a.steps = d["warmup"], d["steps"]
                a.ramp = d.get("ramp", {}).get("steps", 0)
    rows = [r for r in csv.DictReader(open(Path(a.prof_dir) / "run_kernel_trace.csv")) if a.kernel in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
    if a.ramp:  # the clock ramp's launches precede the warm-up
        print(f"clock ramp: {a.ramp} launches, mean {statistics.mean(d[:a.ramp]):.2f} us, last 10 mean "
              f"{statistics.mean(d[max(0, a.ramp - 10):a.ramp]):.2f} us")
        rows, d = rows[a.ramp:], d[a.ramp:]
    timed = d[a.warmup:a.warmup + a.steps]
    print(f"kernel {rows[0]['Kernel_Name']}")
    print(f"launches: {len(d)} (warm-up {a.warmup}, timed {len(timed)}, after {len(d) - a.warmup - len(timed)})")
    print(f"timed region: mean {statistics.mean(timed):.2f} us, median {statistics.median(timed):.2f} us, "
          f"min {min(timed):.2f}, max {max(timed):.2f}")
    e = a.prof_every
    samp = [timed[k] for k in range(e - 1, len(timed), e)]
    print(f"launches bench.py times live ({e - 1}, {2 * e - 1}, ... of the timed region): mean "
          f"{statistics.mean(samp):.2f} us over {len(samp)}")
    print(f"all launches: mean {statistics.mean(d):.2f} us (includes the cold first launch and the counter launch)")
    print("warm-up:", [round(x, 1) for x in d[:a.warmup]])
    print("after the timed region:", [round(x, 1) for x in d[a.warmup + a.steps:]])
    timeline(Path(a.prof_dir) / "run_kernel_trace.csv", rows[a.warmup:a.warmup + a.steps])


def timeline(csv_path, fast):
    """Where a step's stream time goes: from one timed k_render_fast start to the next, the fast
    kernel itself, the other kernels in between, and the idle gaps between kernel boundaries."""
    allk = sorted(csv.DictReader(open(csv_path)), key=lambda r: int(r["Start_Timestamp"]))
    spans = {"fast kernel": [], "other kernels": [], "idle gaps": []}
    names = set()
    for f0, f1 in zip(fast, fast[1:]):
        s0, s1 = int(f0["Start_Timestamp"]), int(f1["Start_Timestamp"])
        inside = [r for r in allk if s0 <= int(r["Start_Timestamp"]) < s1]
        busy = other = 0
        end = s0
        for r in inside:
            b, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            busy += max(0, min(e, s1) - max(b, end))
            end = max(end, e)
            if b != s0:
                other += e - b
                names.add(r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "")[:50])
        spans["fast kernel"].append((int(f0["End_Timestamp"]) - s0) / 1e3)
        spans["other kernels"].append(other / 1e3)
        spans["idle gaps"].append((s1 - s0 - busy) / 1e3)
    print(f"step timeline over {len(spans['idle gaps'])} timed steps (start of one fast launch to the next), mean us:")
    for k, v in spans.items():
        print(f"  {k:14s} {statistics.mean(v):8.2f}")
    print("  other kernels:", sorted(names))


if __name__ == "__main__":
    main()
