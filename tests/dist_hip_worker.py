"""Worker of tests/test_gpu_distributed.py: one rank of a torchrun job whose ranks share one GPU
over gloo (the box has one GPU; RCCL needs one GPU per rank). Every rank renders its HipRenderer
row tile; rank 0 checks the gathered frame against its own single-GPU render.

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port P \
        tests/dist_hip_worker.py OUTDIR
"""

import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    outdir = Path(sys.argv[1])
    from python_ray_tracer_amd import scenes
    from python_ray_tracer_amd.application import render_frame_distributed, render_image_pipeline
    from python_ray_tracer_amd.distributed import TileGather
    from python_ray_tracer_amd.infrastructure.hip import HipRenderer

    dist.init_process_group("gloo")
    rank = dist.get_rank()
    torch.cuda.set_device(0)
    try:
        results = {}
        for name, spec, B, dtype in (("readme", scenes.readme_spec(320, 181), 3, torch.float64),
                                     ("c4like", scenes.random_spec(64, 0, 256, 97), 5, torch.float32),
                                     ("main_unbounded", scenes.main_spec(240, 135), None, torch.float64)):
            scene = scenes.build_scene(spec)
            r = HipRenderer(max_bounces=B, color_dtype=dtype)
            frame = render_frame_distributed(scene, r, row_block=8)
            frame_u8 = render_frame_distributed(scene, r, row_block=8, gather="u8")
            if rank == 0:
                full = r.render(scene).data
                results[f"{name}_color"] = bool(torch.equal(frame, full))
                results[f"{name}_u8"] = bool(torch.equal(frame_u8, r.quantize(r.render(scene), scene.camera)))
            else:
                results[f"{name}_none"] = frame is None and frame_u8 is None
        # PNG through render_image_pipeline on both ranks (colour gather: save_image quantises the
        # host-assembled frame on the device) against the single-rank pipeline's PNG
        spec = scenes.main_spec(200, 113)
        scene = scenes.build_scene(spec)
        r = HipRenderer()
        render_image_pipeline(scene, outdir / "multi.png", r)
        render_image_pipeline(scene, outdir / "multi_u8.png", r, gather="u8")
        # pipelined frames (bench.py --mode tiles): two orbit frames in flight
        spec = scenes.random_spec(16, 0, 192, 108)
        frames = [scenes.build_scene(scenes.with_camera(spec, scenes.orbit_position(k, 256))) for k in (0, 37)]
        r3 = HipRenderer(max_bounces=3, color_dtype=torch.float32)
        tg = TileGather(r3, 192, 108, row_block=8, slots=2)
        tg.submit(frames[0], 0)
        tg.submit(frames[1], 1)
        f0, f1 = tg.finish(0), tg.finish(1)
        if rank == 0:
            results["pipe0"] = bool(torch.equal(f0, r3.render(frames[0]).data))
            results["pipe1"] = bool(torch.equal(f1, r3.render(frames[1]).data))
        dist.barrier()
        if rank == 0:
            dist.destroy_process_group()
            # the single-rank pipeline, the reference's three calls (application.py:48-52)
            from python_ray_tracer_amd.application import render_image_pipeline as rip

            rip(scene, outdir / "single.png", HipRenderer())
            from PIL import Image

            a = np.asarray(Image.open(outdir / "single.png"))
            results["png_color"] = bool(np.array_equal(np.asarray(Image.open(outdir / "multi.png")), a))
            results["png_u8"] = bool(np.array_equal(np.asarray(Image.open(outdir / "multi_u8.png")), a))
        (outdir / f"rank{rank}.txt").write_text(repr(results))
        ok = all(results.values())
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    main()
