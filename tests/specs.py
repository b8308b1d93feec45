"""Scene specs shared by the CPU packer tests and the GPU parity tests."""

from python_ray_tracer_amd import scenes

# layouts of huge spheres (radius > scene_pack.HUGE_RADIUS) for RTX_H_NBEAM: (small spheres, huge
# spheres inserted before the ground, index of one more huge sphere among the small ones or None,
# ground first instead of last, expected NBEAM)
HUGE_LAYOUTS = {
    "tail_at_64": (64, 5, None, False, 64),     # 70 spheres: the tail fills the second frustum pass
    "tail_below_64": (60, 10, None, False, 60),  # the tail starts inside the first pass
    "tail_above_64": (70, 3, None, False, 70),   # the second pass tests spheres 64..69
    "huge_inside": (64, 0, 10, False, 65),       # a huge sphere among the small ones; the tail: the ground
    "ground_first": (64, 0, None, True, 0),      # the last sphere is small: no tail
}


def huge_tail_spec(layout: str, width: int, height: int, seed: int = 5):
    """random_spec's small spheres and ground, with huge spheres inserted before the ground (the
    fuzz generators' radius-150 'big' spheres, behind the small ones) or at one index among them."""
    n_small, n_huge, inside, ground_first, _ = HUGE_LAYOUTS[layout]
    spec = scenes.random_spec(n_small, seed, width, height)
    ground = spec["spheres"][-1]
    proto = spec["spheres"][0]

    def big(k):
        return dict(proto, center=[-240.0 + 90.0 * k, -150.5, 180.0 + 40.0 * k], radius=150.0)

    small = spec["spheres"][:-1]
    spec["spheres"] = ([ground] + small) if ground_first else (small + [big(k) for k in range(n_huge)] + [ground])
    if inside is not None:
        spec["spheres"].insert(inside, big(0))
    return spec
