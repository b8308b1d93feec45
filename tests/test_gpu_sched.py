"""Longest-first dispatch of camera launches (rtx_render_camera_sched, HipRenderer._sched_plan).

A scene of >= 32 spheres renders as persistent waves fetching 8x8 wave tiles, smaller scenes as one
block tile per block. HipRenderer records every unit's render time on the first launch of a
(scene, tile, cap) and hands the units out longest first from then on. The order changes when a
unit is rendered, never what it renders: the frames must equal those of a renderer that keeps the
bottom-up order, bit for bit, and the oracle.
"""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


def test_learnt_order_leaves_frames_unchanged():
    """Persistent (40 spheres), small (README, TREE = false) and culled one-block-per-tile (16
    spheres) launches, capped and unbounded, whole frames and row tiles."""
    dev = _dev()
    from python_ray_tracer_amd import scenes

    for spec, Bs in ((scenes.random_spec(40, 7, 200, 131), (3, 5, None)), (scenes.readme_spec(203, 117), (3, None)),
                     (scenes.random_spec(16, 2, 150, 97), (4,))):
        _check(spec, Bs, dev)


def _check(spec, Bs, dev):
    from oracle import numpy_oracle as O
    from python_ray_tracer_amd import scenes
    from python_ray_tracer_amd.infrastructure.hip import HipRenderer

    scene = scenes.build_scene(spec)
    for B in Bs:
        plain = HipRenderer(max_bounces=B, color_dtype=torch.float64, device=dev, learn_tile_order=False)
        learn = HipRenderer(max_bounces=B, color_dtype=torch.float64, device=dev)
        want = plain.render_tile(scene)
        for rb, parts, part in ((1, 1, 0), (8, 3, 1)):
            ref = plain.render_tile(scene, rb, parts, part)
            got = [learn.render_tile(scene, rb, parts, part).clone() for _ in range(4)]
            torch.cuda.synchronize()
            got.append(learn.render_tile(scene, rb, parts, part))
            assert any(isinstance(v, torch.Tensor) for v in learn._sched.values()), learn._sched
            for g in got:
                assert torch.equal(g, ref), (B, rb, parts, part)
        # the learnt order is a permutation of the launch's units
        for st in learn._sched.values():
            if st is not None:
                o = st.cpu().numpy()
                assert np.array_equal(np.sort(o), np.arange(len(o)))
        if B == Bs[0]:
            ora = O.render(O.scene_from_spec(spec), B)
            assert float(np.abs(learn.render_tile(scene).cpu().numpy() - ora).max()) <= 1e-12
            assert torch.equal(learn.render_tile(scene), want)


def test_bench_line_contract(tmp_path):
    """bench.py at N = 1 prints ONE JSON line with the driver's contract fields, the roofline and
    the top-level strong_scaling object (the row-tiled C4 frame on a one-rank loopback plan, its
    gather labelled as HBM, not xGMI); a short run, CPU baseline skipped."""
    import json
    import subprocess
    import sys
    from pathlib import Path

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    repo = Path(__file__).resolve().parent.parent
    out = tmp_path / "line.json"
    p = subprocess.run([sys.executable, str(repo / "bench.py"), "--steps", "5", "--warmup", "1", "--ramp-ms", "10",
                        "--cpu-seconds", "0", "--json-out", str(out)], cwd=str(repo), capture_output=True, text=True,
                       timeout=110)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [s for s in p.stdout.splitlines() if s.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    d = json.loads(lines[0])
    assert d == json.loads(out.read_text())
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 5 and d["warmup"] == 1 and d["value"] > 0 and d["higher_is_better"]
    assert d["scaling"] == "weak" and d["vs_baseline"] is None and d["dtype"] == "f64"
    assert d["config"]["workload"].startswith("C2") and d["config"]["width"] == 1920
    r = d["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in r, k
    assert 0 < r["frac"] < 1 and abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-3
    ss = d["strong_scaling"]
    assert ss["n_gpus"] == 1 and ss["speedup_vs_1gpu"] > 0 and ss["single_gpu_ms_per_step"] > 0
    assert ss["gather"]["link"] == "loopback (HBM)" and ss["gather"]["xgmi_GBps_per_peer"] is None
    assert ss["xgmi_GBps"]["measured"] is None and ss["xgmi_GBps"]["assumed"] > 0
