"""Probe: per-frame time of back-to-back single-frame renders with 1, 2 or 3 frames in flight
(round-robin over that many HIP streams, each with its own workspace and output), against one
stream. Overlapping one frame's drain with the next one's ramp-up is what a multi-frame launch
gets inside one kernel.

    python tools/stream_probe.py --config C2 --iters 200
"""

import argparse
import ctypes
import statistics
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

import torch  # noqa: E402

from python_ray_tracer_amd import scenes  # noqa: E402
from python_ray_tracer_amd.infrastructure.hip import _lib as L  # noqa: E402
from python_ray_tracer_amd.infrastructure.hip.scene_pack import pack_scene  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C2")
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    spec, B = scenes.CONFIGS[a.config]()
    blob_np = pack_scene(scenes.build_scene(spec))
    dev = torch.device("cuda", 0)
    blob = torch.from_numpy(blob_np).to(dev)
    S = int(blob_np[L.H_NSPH])
    W, H = spec["camera"]["width"], spec["camera"]["height"]
    n = W * H
    lib = L.load()
    res = {}
    for depth in (1, 2, 3):
        streams = [torch.cuda.Stream(dev) for _ in range(depth)]
        outs = [torch.empty(3 * n, dtype=torch.float32, device=dev) for _ in range(depth)]
        wss = [torch.zeros(int(lib.rtx_workspace_bytes(n, B)), dtype=torch.uint8, device=dev) for _ in range(depth)]

        def launch(k):
            s = streams[k % depth]
            rc = lib.rtx_render_camera(blob.data_ptr(), S, W, H, 1, 1, 0, H, B, outs[k % depth].data_ptr(),
                                       L.OUT_F32_SOA, wss[k % depth].data_ptr(), wss[k % depth].numel(), None,
                                       s.cuda_stream)
            assert rc == 0

        for k in range(20):
            launch(k)
        torch.cuda.synchronize()
        per = []
        for _ in range(a.rounds):
            ev0 = torch.cuda.Event(enable_timing=True)
            ev1 = torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            ev0.record()
            for s in streams:
                s.wait_event(ev0)
            for k in range(a.iters):
                launch(k)
            for s in streams:
                ev = torch.cuda.Event()
                ev.record(s)
                torch.cuda.current_stream().wait_event(ev)
            ev1.record()
            torch.cuda.synchronize()
            per.append(ev0.elapsed_time(ev1) / a.iters * 1e3)
        res[depth] = statistics.median(per)
        print(f"{a.config}: {depth} stream(s): {res[depth]:8.2f} us/frame  ({n / res[depth]:9.1f} Mpix/s)")


if __name__ == "__main__":
    main()
