"""Diagnostic: per-tile (8x8 wave tile) start/end times of k_render_fast, for the one-tile-per-block
grid and the persistent-wave launch alike (library built with -DRTX_WAVE_TIMES).

    python tools/tile_times.py build/ab/wt.so --config C2

Prints the launch span, the sum of tile durations over the span (= mean concurrently busy waves),
the tile duration distribution and the busy-wave count over time.
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
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--config", default="C2")
    a = ap.parse_args()
    spec, B = scenes.CONFIGS[a.config]()
    blob_np = pack_scene(scenes.build_scene(spec))
    dev = torch.device("cuda", 0)
    blob = torch.from_numpy(blob_np).to(dev)
    S = int(blob_np[L.H_NSPH])
    W, H = spec["camera"]["width"], spec["camera"]["height"]
    n = W * H
    nt = ((W + 7) // 8) * ((H + 7) // 8)
    stream = torch.cuda.current_stream(dev).cuda_stream
    for path in a.libs:
        lib = open_lib(path)
        out = torch.empty(3 * n * 4, dtype=torch.uint8, device=dev)
        ws = torch.zeros(int(lib.rtx_workspace_bytes(n, B)), dtype=torch.uint8, device=dev)
        st = torch.zeros(L.S_WORDS + 4 * nt + 4096, dtype=torch.int64, device=dev)  # block-grid slots pad rows
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
        t = st[L.S_WORDS:].cpu().numpy().reshape(-1, 2).astype(np.int64)
        t = t[t[:, 1] > 0]
        t0 = t[:, 0].min()
        start = (t[:, 0] - t0) / 100.0  # s_memrealtime: 100 MHz
        end = (t[:, 1] - t0) / 100.0
        dur = end - start
        span = end.max()
        print(f"== {Path(path).name} {a.config}: {len(t)} tiles, span {span:.1f} us (events {wall_us:.1f} us)")
        print("   tile us: p50 %.2f p90 %.2f p99 %.2f max %.2f mean %.2f; sum/span = %.0f busy waves" % (
            np.percentile(dur, 50), np.percentile(dur, 90), np.percentile(dur, 99), dur.max(), dur.mean(),
            dur.sum() / span))
        edges = np.linspace(0, span, 21)
        act = [int(((start < b) & (end > a_)).sum()) for a_, b in zip(edges[:-1], edges[1:])]
        print("   busy waves per 5% of the span:", act)
        first = np.sort(start)
        print("   tiles started by 1/2/5/10 us:", [int((first < x).sum()) for x in (1, 2, 5, 10)])


if __name__ == "__main__":
    main()
