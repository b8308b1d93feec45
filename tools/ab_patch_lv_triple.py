"""A/B patch: ab_patch_lv_together + ab_patch_self_triple."""
import runpy
from pathlib import Path

_HERE = Path(__file__).resolve().parent


def patch(src: str) -> str:
    for name in ("ab_patch_lv_together.py", "ab_patch_self_triple.py"):
        src = runpy.run_path(str(_HERE / name))["patch"](src)
    return src
