"""A/B timing of librtx_hip.so variants in ONE process, interleaved rounds (guide §5.4 rule 24).

    python tools/ab.py --config C2 --rounds 10 --iters 50 lib_a.so lib_b.so ...

Each variant renders the same packed scene with rtx_render_camera into its own output; per round
and variant, `iters` launches are timed with HIP events (rtx_profile_* of that library). Prints the
median and min per-launch kernel time, and checks every variant's output against the first.
A variant `lib.so@NAME=VALUE+...` packs its own scene with those scene_pack constants set (host
packer A/B: e.g. `ab/x.so@SHGRID_CELLS=48+SHGRID_MAX_VOXELS=65536`).
"""

import argparse
import ast
import ctypes
import statistics
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

import torch  # noqa: E402

from python_ray_tracer_amd import scenes  # noqa: E402
from python_ray_tracer_amd.infrastructure.hip import _lib as L  # noqa: E402
from python_ray_tracer_amd.infrastructure.hip.scene_pack import pack_scene  # noqa: E402


def open_lib(path):
    lib = ctypes.CDLL(str(Path(path).resolve()))
    for name, (res, args) in L._SIGS.items():
        if not hasattr(lib, name):  # older builds lack newer entry points
            continue
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--config", default="C2")
    ap.add_argument("--rounds", type=int, default=10)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--out", default="f32", choices=["f32", "f64", "u8"])
    ap.add_argument("--no-events", action="store_true", help="end-to-end only: no per-launch kernel events")
    ap.add_argument("--bvh-leaf", type=int, default=None, help="override scene_pack.BVH_LEAF (spheres per leaf)")
    ap.add_argument("--bounces", type=int, default=None, help="override the config's bounce cap (-1: unbounded)")
    ap.add_argument("--spheres", type=int, default=None, help="a seeded random scene of this many spheres at the config's size")
    a = ap.parse_args()
    spec, B = scenes.CONFIGS[a.config]()
    if a.bounces is not None:
        B = a.bounces
    if a.spheres is not None:
        spec = scenes.random_spec(a.spheres, 0, spec["camera"]["width"], spec["camera"]["height"])
    if a.bvh_leaf is not None:
        from python_ray_tracer_amd.infrastructure.hip import scene_pack

        scene_pack.BVH_LEAF = a.bvh_leaf
    from python_ray_tracer_amd.infrastructure.hip import scene_pack

    scene = scenes.build_scene(spec)
    dev = torch.device("cuda", 0)

    def pack(overrides):
        saved = {k: getattr(scene_pack, k) for k in overrides}
        try:
            for k, v in overrides.items():
                setattr(scene_pack, k, ast.literal_eval(v))
            scene_pack._pack_static.cache_clear()
            return pack_scene(scene)
        finally:
            for k, v in saved.items():
                setattr(scene_pack, k, v)
            scene_pack._pack_static.cache_clear()

    paths, blobs = [], []
    for arg in a.libs:
        path, _, ov = arg.partition("@")
        paths.append(path)
        blobs.append(torch.from_numpy(pack(dict(kv.split("=") for kv in ov.split("+") if kv))).to(dev))
    S = int(blobs[0][L.H_NSPH].item())
    W, H = spec["camera"]["width"], spec["camera"]["height"]
    n = W * H
    kind = {"f32": L.OUT_F32_SOA, "f64": L.OUT_F64_SOA, "u8": L.OUT_U8_HWC}[a.out]
    libs = [open_lib(p) for p in paths]
    outs, wss = [], []
    for lib in libs:
        outs.append(torch.empty(3 * n * (8 if a.out == "f64" else 4 if a.out == "f32" else 1), dtype=torch.uint8,
                                device=dev))
        wss.append(torch.zeros(int(lib.rtx_workspace_bytes(n, B)), dtype=torch.uint8, device=dev))
    stream = torch.cuda.current_stream(dev).cuda_stream

    def launch(k):
        rc = libs[k].rtx_render_camera(blobs[k].data_ptr(), S, W, H, 1, 1, 0, H, B, outs[k].data_ptr(), kind,
                                       wss[k].data_ptr(), wss[k].numel(), None, stream)
        assert rc == 0, libs[k].rtx_last_error()

    for k in range(len(libs)):
        for _ in range(5):
            launch(k)
    torch.cuda.synchronize()
    times = [[] for _ in libs]
    e2e = [[] for _ in libs]
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    for _ in range(a.rounds):
        for k, lib in enumerate(libs):
            lib.rtx_profile_enable(0 if a.no_events else a.iters)
            ev0.record()
            for _ in range(a.iters):
                launch(k)
            ev1.record()
            ms = ctypes.c_double()
            cnt = ctypes.c_int()
            lib.rtx_profile_collect(ctypes.byref(ms), ctypes.byref(cnt))
            lib.rtx_profile_enable(0)
            torch.cuda.synchronize()
            times[k].append(ms.value / max(cnt.value, 1) * 1e3)
            e2e[k].append(ev0.elapsed_time(ev1) / a.iters * 1e3)
    torch.cuda.synchronize()
    for k, p in enumerate(a.libs):
        same = torch.equal(outs[k], outs[0])
        t = times[k]
        km = statistics.median(t)
        print(f"{Path(p.partition('@')[0]).name + p.partition('@')[1] + p.partition('@')[2]:28s} median {km:9.2f} us  min {min(t):9.2f} us  "
              f"Mpix/s(kernel) {n / km if km else float('nan'):10.1f}  e2e/frame {statistics.median(e2e[k]):9.2f} us  "
              f"equal_to_first={same}")


if __name__ == "__main__":
    main()
