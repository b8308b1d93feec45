"""Diagnostic: per-wave start/end times of k_render_fast (library built with -DRTX_WAVE_TIMES).

    python tools/wave_times.py build/ab/wavetimes.so --config C2 [--out gpurun_out/wt.npz]

Renders the config's frame a few times and keeps the last launch's per-wave [start, end] pairs
(s_memrealtime, 100 MHz), indexed by (block y, block x, wave); prints the launch span, the
distribution of wave durations and when the last-finishing waves started.
"""

import argparse
import ctypes
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from python_ray_tracer_amd import scenes  # noqa: E402
from python_ray_tracer_amd.infrastructure.hip import _lib as L  # noqa: E402
from python_ray_tracer_amd.infrastructure.hip.scene_pack import pack_scene  # noqa: E402
from tools.ab import open_lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib")
    ap.add_argument("--config", default="C2")
    ap.add_argument("--out", default=None)
    ap.add_argument("--bounces", type=int, default=None, help="override the config's bounce cap")
    ap.add_argument("--block-waves", type=int, default=4, help="RTX_BLOCK_WAVES of the library")
    a = ap.parse_args()
    spec, B = scenes.CONFIGS[a.config]()
    if a.bounces is not None:
        B = a.bounces
    blob_np = pack_scene(scenes.build_scene(spec))
    dev = torch.device("cuda", 0)
    blob = torch.from_numpy(blob_np).to(dev)
    S = int(blob_np[L.H_NSPH])
    W, H = spec["camera"]["width"], spec["camera"]["height"]
    n = W * H
    lib = open_lib(a.lib)
    bw = a.block_waves
    tw, th = (8, 8) if bw == 1 else (16, 8) if bw == 2 else (16, 16)
    tx, ty = (W + tw - 1) // tw, (H + th - 1) // th
    nw = tx * ty * bw
    out = torch.empty(3 * n * 4, dtype=torch.uint8, device=dev)
    ws = torch.zeros(int(lib.rtx_workspace_bytes(n, B)), dtype=torch.uint8, device=dev)
    st = torch.zeros(L.S_WORDS + 2 * nw, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    for k in range(5):
        if k == 4:
            ev0.record()
        rc = lib.rtx_render_camera(blob.data_ptr(), S, W, H, 1, 1, 0, H, B, out.data_ptr(), L.OUT_F32_SOA,
                                   ws.data_ptr(), ws.numel(), ctypes.c_void_p(st.data_ptr()), stream)
        assert rc == 0
    ev1.record()
    torch.cuda.synchronize()
    wall_us = ev0.elapsed_time(ev1) * 1e3
    t = st[L.S_WORDS:].cpu().numpy().reshape(ty, tx, bw, 2).astype(np.int64)
    t0 = t[..., 0].min()
    ticks = t[..., 1].max() - t0
    tpu = ticks / wall_us  # clock ticks per us, calibrated on the launch's event time (upper bound)
    print(f"last launch: {wall_us:.1f} us by events, {ticks} ticks -> >= {tpu:.1f} ticks/us")
    start = (t[..., 0] - t0) / tpu  # us
    end = (t[..., 1] - t0) / tpu
    dur = end - start
    span = end.max()
    print(f"{a.config} B={B}: launch span {span:.1f} us, waves {nw}")
    print("wave duration us: p50 %.2f p90 %.2f p99 %.2f max %.2f mean %.2f" % (
        np.percentile(dur, 50), np.percentile(dur, 90), np.percentile(dur, 99), dur.max(), dur.mean()))
    busy = dur.sum()
    print(f"sum of wave durations {busy:.0f} us; concurrency = sum / span = {busy / span:.0f} waves")
    rows = dur.mean(axis=(1, 2))
    print("mean wave duration per tile row (top->bottom, every 8th):", np.round(rows[::8], 2).tolist())
    last = np.argsort(end.ravel())[-20:]
    for k in last[::-1][:10]:
        y, x, w = np.unravel_index(k, end.shape)
        print(f"  late wave tile ({y},{x}) w{w}: start {start[y, x, w]:.1f} end {end[y, x, w]:.1f} dur {dur[y, x, w]:.1f}")
    # concurrency over time
    edges = np.linspace(0, span, 21)
    act = [((start.ravel() < b) & (end.ravel() > a_)).sum() for a_, b in zip(edges[:-1], edges[1:])]
    print("active waves per 5% of the span:", act)
    if a.out:
        np.savez(a.out, start=start, end=end)


if __name__ == "__main__":
    main()
