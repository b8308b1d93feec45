"""Per-tile timeline of k_render_fast (the ``tile_trace`` instrument of tools/ab_patches.py).

    python tools/ab_build.py ab/trace.so --patch tile_trace --only-b 3,5
    python tools/tile_trace.py ab/trace.so --config C4 --parts 8 --part 0 [--launches 3]

Renders the configuration's frame (or one interleaved row tile of it) with a library built with
the instrument, reads every wave's (start, end) per tile and prints one JSON line: the launch span,
how many tiles are in flight over time (the fill and the drain), per-tile duration quantiles, the
mean duration by tile-row band, per-XCD busy time, and a list-scheduling estimate of the span with
the tiles handed out in their observed order and longest first (what a cost-ordered fetch could
save; durations are measured under the launch's own contention, so this is an estimate).
"""

from __future__ import annotations

import argparse
import ctypes
import heapq
import json
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "tools"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from ab import open_lib  # noqa: E402
from python_ray_tracer_amd import scenes, tiling  # noqa: E402
from python_ray_tracer_amd.infrastructure.hip import _lib as L  # noqa: E402
from python_ray_tracer_amd.infrastructure.hip.scene_pack import pack_scene  # noqa: E402

WORDS = 4


def list_schedule(durs, slots):
    """Makespan of greedy list scheduling of `durs` (in order) on `slots` identical workers."""
    heap = [0.0] * slots
    for d in durs:
        t = heapq.heappop(heap)
        heapq.heappush(heap, t + d)
    return max(heap)


def analyse(rec, persistent, n_tiles_x, bands=16, bins=40):
    t0 = rec[:, 0].astype(np.float64) / 100.0  # 100 MHz -> us
    t1 = rec[:, 1].astype(np.float64) / 100.0
    base = t0.min()
    t0 -= base
    t1 -= base
    span = float(t1.max())
    dur = t1 - t0
    ident = rec[:, 2]
    hw = rec[:, 3]
    xcc = (hw >> 32) & 0xF
    edges = np.linspace(0.0, span, bins + 1)
    mid = 0.5 * (edges[1:] + edges[:-1])
    inflight = [int(((t0 <= m) & (t1 > m)).sum()) for m in mid]
    peak = max(inflight)
    # drain: from the last time the in-flight count was >= 90% of its peak to the end
    ev = np.concatenate([np.stack([t0, np.ones_like(t0)], 1), np.stack([t1, -np.ones_like(t1)], 1)])
    ev = ev[np.argsort(ev[:, 0], kind="stable")]
    level = np.cumsum(ev[:, 1])
    above = np.nonzero(level >= 0.9 * level.max())[0]
    drain_start = float(ev[above[-1], 0]) if len(above) else 0.0
    fill = np.nonzero(level >= 0.9 * level.max())[0]
    fill_end = float(ev[fill[0], 0]) if len(fill) else 0.0
    out = {
        "tiles": int(len(rec)), "span_us": round(span, 2), "peak_in_flight": peak,
        "fill_to_90pct_us": round(fill_end, 2), "drain_from_90pct_us": round(span - drain_start, 2),
        "in_flight": inflight,
        "dur_us": {q: round(float(np.quantile(dur, v)), 2) for q, v in
                   (("p10", .1), ("p50", .5), ("p90", .9), ("p99", .99), ("max", 1.0))},
        "dur_mean_us": round(float(dur.mean()), 3),
        "busy_over_slots": round(float(dur.sum()) / max(peak, 1), 2),
    }
    if persistent:
        tile = (ident & 0xFFFFFFFF).astype(np.int64)
        pw = (ident >> 32) & 0x7FFFFFFF
        slots = int(len(np.unique(pw)))
        row = tile // n_tiles_x
        nrows = int(row.max()) + 1
        band = (row * bands) // nrows
        out["slots"] = slots
        out["dur_by_row_band_us"] = [round(float(dur[band == b].mean()), 2) if (band == b).any() else None
                                     for b in range(bands)]
        order = np.argsort(t0, kind="stable")
        out["sim_observed_order_us"] = round(list_schedule(dur[order], slots), 2)
        out["sim_longest_first_us"] = round(list_schedule(np.sort(dur)[::-1], slots), 2)
        out["lower_bound_us"] = round(max(float(dur.sum()) / slots, float(dur.max())), 2)
        # the tiles still running in the last 10% of the span: their rows and durations
        late = t1 > 0.9 * span
        out["late_tiles"] = {"count": int(late.sum()), "mean_dur_us": round(float(dur[late].mean()), 2),
                             "rows": sorted({int(v) for v in row[late]})[:40]}
        # how long a tile of each row takes at most (the deepest chains)
        out["max_dur_by_row_band_us"] = [round(float(dur[band == b].max()), 2) if (band == b).any() else None
                                         for b in range(bands)]
    xs = {}
    for x in np.unique(xcc):
        m = xcc == x
        xs[int(x)] = {"tiles": int(m.sum()), "busy_us": round(float(dur[m].sum()), 1),
                      "end_us": round(float(t1[m].max()), 2)}
    out["per_xcc"] = xs
    return out, dur, t0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib")
    ap.add_argument("--config", default="C4")
    ap.add_argument("--parts", type=int, default=1)
    ap.add_argument("--part", type=int, default=0)
    ap.add_argument("--row-block", type=int, default=8)
    ap.add_argument("--launches", type=int, default=3)
    ap.add_argument("--ramp-ms", type=float, default=300.0)
    ap.add_argument("--dump", default=None, help="save the raw records of the last launch (.npy)")
    a = ap.parse_args()
    spec, B = scenes.CONFIGS[a.config]()
    scene = scenes.build_scene(spec)
    blob_np = pack_scene(scene)
    dev = torch.device("cuda", 0)
    blob = torch.from_numpy(blob_np).to(dev)
    S = int(blob_np[L.H_NSPH])
    W, H = spec["camera"]["width"], spec["camera"]["height"]
    rows = tiling.n_local_rows(H, a.row_block, a.parts, a.part)
    n = W * rows
    lib = open_lib(a.lib)
    lib.rtx_trace_set.restype = ctypes.c_int
    lib.rtx_trace_set.argtypes = [ctypes.c_void_p]
    out = torch.empty(3 * n, dtype=torch.float32, device=dev)
    ws = torch.zeros(int(lib.rtx_workspace_bytes(n, B)), dtype=torch.uint8, device=dev)
    cap = (n + 63) // 64 + 4096
    buf = torch.zeros(8 + WORDS * cap, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream

    def launch():
        rc = lib.rtx_render_camera(blob.data_ptr(), S, W, H, a.row_block, a.parts, a.part, rows, B, out.data_ptr(),
                                   L.OUT_F32_SOA, ws.data_ptr(), ws.numel(), None, stream)
        assert rc == 0, lib.rtx_last_error()

    lib.rtx_trace_set(None)
    launch()
    torch.cuda.synchronize()
    t_end = time.perf_counter() + a.ramp_ms / 1e3
    while time.perf_counter() < t_end:
        for _ in range(8):
            launch()
        torch.cuda.synchronize()
    persistent = S >= 32
    res = []
    for _ in range(a.launches):
        buf.zero_()
        buf[1] = cap
        lib.rtx_trace_set(ctypes.c_void_p(buf.data_ptr()))
        launch()
        lib.rtx_trace_set(None)
        torch.cuda.synchronize()
        rec = buf[8:8 + WORDS * cap].view(-1, WORDS).cpu().numpy().view(np.uint64)
        rec = rec[rec[:, 1] != 0]  # the slots of rendered tiles / waves
        cnt = len(rec)
        r, dur, t0 = analyse(rec, persistent, (W + 7) // 8)
        r["records"] = cnt
        res.append(r)
        if a.dump:
            np.save(a.dump, rec)
        for _ in range(8):  # untraced launches between traced ones (steady clocks)
            launch()
        torch.cuda.synchronize()
    line = {"config": a.config, "width": W, "height": H, "parts": a.parts, "part": a.part, "rows": rows,
            "bounces": B, "spheres": S, "lib": Path(a.lib).name, "launches": res}
    print(json.dumps(line))


if __name__ == "__main__":
    main()
