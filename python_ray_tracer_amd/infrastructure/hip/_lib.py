"""ctypes binding of the C ABI in ``include/rtx_hip.h`` (``librtx_hip.so``, built in-tree).

There is no fallback: if the library is missing or was built for a different layout, importing the
HIP backend raises. ``torch`` is imported first so the library binds to the HIP runtime torch has
already loaded (one runtime per process; both are ``libamdhip64.so.7``).
"""

from __future__ import annotations

import ctypes
import os
from pathlib import Path

import torch  # noqa: F401  (loads the HIP runtime the library links against)

PKG_DIR = Path(__file__).resolve().parent.parent.parent
LIB_PATH = Path(os.environ.get("RTX_HIP_LIB", PKG_DIR / "librtx_hip.so"))

# mirrors of include/rtx_hip.h (checked against the library at load time)
ABI_VERSION = 1
HDR_WORDS = 64
GEOM_WORDS = 8
MAT_WORDS = 24
MAX_DOMES = 8
S_WORDS = 266
WS_HDR_BYTES = 256
FAST_MAX_BOUNCES = 6
UNBOUNDED_LEVELS = 333
MAX_SPHERES = 1024
MAGIC = 5527384.0
UNBOUNDED = -1

TEX_CONST, TEX_CHECKER, TEX_IMAGE = 0.0, 1.0, 2.0
MAX_TEXELS = 1 << 20

OUT_F32_SOA = 0
OUT_F64_SOA = 1
OUT_U8_HWC = 2

ST_STACK_OVERFLOW = 1
ST_LIST_OVERFLOW = 2
ST_BAD_SCENE = 4
ST_UNRENDERED = 8  # RTX_F_NO_GENERAL render deferred rays: those pixels are unwritten

F_NO_GENERAL = 1  # rtx_render_camera_ex flags
F_IMAGES = 2  # RTX_F_IMAGES: the texturing build of the fast kernel (scenes with image textures)
F_RESERVE_SHIFT = 4  # RTX_F_RESERVE(n) = (n & 0xFFF) << 4

# header words
H_MAGIC, H_NSPH, H_CAM, H_LIGHT, H_DOMEC, H_NDOME, H_DOMEI = 0, 1, 2, 5, 8, 11, 12
H_XSTART, H_XSTEP, H_XSTOP, H_XFIX = 20, 21, 22, 23
H_YSTART, H_YSTEP, H_YSTOP, H_YFIX = 24, 25, 26, 27
H_VZ, H_VZ2, H_W, H_H, H_CAMOO = 28, 29, 30, 31, 32
H_NNODES, H_NALWAYS, H_NODES, H_CGEO, H_TAME, H_MAT0, H_SHGRID, H_SINRED, H_NBEAM, H_SBOX = (
    33, 34, 35, 36, 37, 38, 39, 40, 41, 42)
SIN_TFT_MAX = 2.0 ** 20 / (10.0 * 3.141592653589793 * 1.001)  # thin-film thickness bound of RTX_H_SINRED
SHGRID_WORDS = 13
TAME_BOUND = 2.0 ** 60
# geometry words
G_CX, G_CY, G_CZ, G_CC, G_RR, G_INVR, G_C0, G_IDX = 0, 1, 2, 3, 4, 5, 6, 7
# culling-tree node words
NODE_WORDS = 12
N_LOX, N_LOY, N_LOZ, N_HIX, N_HIY, N_HIZ, N_FIRST, N_COUNT, N_SKIP, N_MARGIN = range(10)
# material words
(M_G, M_DG, M_TEX, M_TR, M_TG, M_TB, M_A2, M_A2M1, M_1MA2, M_F0, M_1MF0, M_IG, M_TFW, M_TFT, M_HS, M_1MHS,
 M_ROUGH, M_REFL, M_IOR, M_TFIOR) = range(20)
# stats words
S_TESTS, S_NODES, S_TESTS1, S_NODES1, S_BEAMW, S_BOXES, S_BEAMT = 3, 4, 5, 6, 7, 264, 265
S_PIXELS, S_DEFERRED, S_TIES, S_RAYS, S_HITS, S_LEVELS, S_WTRACE, S_WSHADE = 0, 1, 2, 8, 72, 64, 136, 200

EXPORTS = (
    "rtx_abi_version",
    "rtx_last_error",
    "rtx_workspace_bytes",
    "rtx_render_camera",
    "rtx_render_camera_ex",
    "rtx_render_frames",
    "rtx_trace_rays",
    "rtx_ray_directions",
    "rtx_sphere_intersect",
    "rtx_quantize_u8",
    "rtx_profile_enable",
    "rtx_profile_collect",
    "rtx_profile_sample",
    "rtx_selftest_math",
    "rtx_assemble_rows",
    "rtx_shade_hits",
    "rtx_assemble_runs",
    "rtx_sched_tiles",
    "rtx_render_camera_sched",
    "rtx_rccl_load",
    "rtx_comm_unique_id",
    "rtx_comm_init",
    "rtx_comm_destroy",
    "rtx_tiles_create",
    "rtx_tiles_submit",
    "rtx_tiles_finish",
    "rtx_tiles_destroy",
    "rtx_tiles_timing",
)

TILES_MAX_SLOTS = 4
TILES_LOOPBACK = 1  # rtx_tiles_create flags
TILES_ROWS = 2
TILES_TIMED = 4
UNIQUE_ID_BYTES = 128  # ncclUniqueId

_c_void_p = ctypes.c_void_p
_i32 = ctypes.c_int
_i64 = ctypes.c_int64
_size = ctypes.c_size_t

_SIGS = {
    "rtx_abi_version": (_i32, [ctypes.POINTER(_i32), _i32]),
    "rtx_last_error": (ctypes.c_char_p, []),
    "rtx_workspace_bytes": (_size, [_i64, _i32]),
    "rtx_render_camera": (_i32, [_c_void_p, _i32, _i32, _i32, _i32, _i32, _i32, _i32, _i32, _c_void_p, _i32,
                                 _c_void_p, _size, _c_void_p, _c_void_p]),
    "rtx_render_camera_ex": (_i32, [_c_void_p, _i32, _i32, _i32, _i32, _i32, _i32, _i32, _i32, _c_void_p, _i32,
                                    _c_void_p, _size, _c_void_p, _c_void_p, ctypes.c_uint, _c_void_p]),
    "rtx_render_frames": (_i32, [_c_void_p, _i64, _i32, _i32, _i32, _i32, _i32, _c_void_p, _i32, _c_void_p, _size,
                                 _c_void_p, _c_void_p]),
    "rtx_trace_rays": (_i32, [_c_void_p, _i32, _c_void_p, _i64, _c_void_p, _i64, _i32, _c_void_p, _i32, _c_void_p,
                              _size, _c_void_p, _c_void_p]),
    "rtx_ray_directions": (_i32, [_c_void_p, _i32, _i32, _i32, _i32, _i32, _i32, _c_void_p, _c_void_p]),
    "rtx_sphere_intersect": (_i32, [_c_void_p, _c_void_p, _i64, _c_void_p, _i64, _c_void_p, _c_void_p]),
    "rtx_quantize_u8": (_i32, [_c_void_p, _i32, _i64, _c_void_p, _c_void_p]),
    "rtx_profile_enable": (_i32, [_i32]),
    "rtx_profile_collect": (_i32, [ctypes.POINTER(ctypes.c_double), ctypes.POINTER(_i32)]),
    "rtx_profile_sample": (_i32, [_i32]),
    "rtx_selftest_math": (_i32, [_c_void_p, _c_void_p, _i64, _c_void_p, _c_void_p]),
    "rtx_shade_hits": (_i32, [_c_void_p, _i32, _i32, _c_void_p, _i64, _c_void_p, _c_void_p, _i64, _i32, _c_void_p,
                              _i32, _c_void_p, _size, _c_void_p, _c_void_p]),
    "rtx_assemble_rows": (_i32, [_c_void_p, _i64, _i32, _i32, _i32, _i32, _i32, _c_void_p, _c_void_p]),
    "rtx_rccl_load": (_i32, [ctypes.c_char_p]),
    "rtx_comm_unique_id": (_i32, [_c_void_p]),
    "rtx_comm_init": (_i32, [_c_void_p, _i32, _i32, _i32, ctypes.POINTER(_c_void_p)]),
    "rtx_comm_destroy": (_i32, [_c_void_p]),
    "rtx_tiles_create": (_i32, [_c_void_p, _i32, _i32, _i32, _i32, _i32, _i32, _i32, _i32, ctypes.POINTER(_c_void_p),
                                ctypes.POINTER(_c_void_p), _i64, _i32, _i32, ctypes.c_uint, ctypes.POINTER(_c_void_p)]),
    "rtx_assemble_runs": (_i32, [_c_void_p, _i64, _i32, _i32, _i32, _i32, _i32, _i32, _i32, _c_void_p, _c_void_p]),
    "rtx_tiles_submit": (_i32, [_c_void_p, _i32, _c_void_p, _i32, _i32, _c_void_p, _size, ctypes.c_uint, _c_void_p,
                                _c_void_p, _c_void_p, _c_void_p, _c_void_p]),
    "rtx_sched_tiles": (_i32, [_i32, _i32, _i32, ctypes.POINTER(_i64)]),
    "rtx_render_camera_sched": (_i32, [_c_void_p, _i32, _i32, _i32, _i32, _i32, _i32, _i32, _i32, _i32, _c_void_p, _i32,
                                       _c_void_p, _size, _c_void_p, _c_void_p, ctypes.c_uint, _c_void_p, _c_void_p,
                                       _c_void_p]),
    "rtx_tiles_finish": (_i32, [_c_void_p, _i32, _c_void_p]),
    "rtx_tiles_destroy": (_i32, [_c_void_p]),
    "rtx_tiles_timing": (_i32, [_c_void_p, _i32, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_float)]),
}

_lib = None


class RtxError(RuntimeError):
    """A C-ABI entry point returned an error code."""


def load():
    """Load and check ``librtx_hip.so``; raises (ImportError/RuntimeError) if unusable."""
    global _lib
    if _lib is not None:
        return _lib
    if not LIB_PATH.exists():
        raise ImportError(
            f"librtx_hip.so not found at {LIB_PATH}; build it with `python -c 'import __graft_entry__ as g; g.build()'`"
            " (the HIP backend has no CPU fallback)")
    lib = ctypes.CDLL(str(LIB_PATH))
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    layout = (_i32 * 8)()
    ver = lib.rtx_abi_version(layout, 8)
    want = [HDR_WORDS, GEOM_WORDS, MAT_WORDS, MAX_DOMES, S_WORDS, WS_HDR_BYTES, FAST_MAX_BOUNCES, UNBOUNDED_LEVELS]
    if ver != ABI_VERSION or list(layout) != want:
        raise ImportError(f"librtx_hip.so ABI mismatch: version {ver}, layout {list(layout)} != {want}")
    _lib = lib
    return lib


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = _lib.rtx_last_error().decode(errors="replace") if _lib is not None else ""
        raise RtxError(f"{what} failed ({rc}): {msg}")


def profile_enable(max_launches: int) -> None:
    check(load().rtx_profile_enable(int(max_launches)), "rtx_profile_enable")


def profile_sample(every: int) -> None:
    """Record one render launch in ``every`` while profiling is enabled (rtx_profile_sample)."""
    check(load().rtx_profile_sample(int(every)), "rtx_profile_sample")


def profile_collect() -> tuple[float, int]:
    """(summed ms of the dominant render kernel, launches) since profile_enable; synchronises."""
    ms = ctypes.c_double()
    n = _i32()
    check(load().rtx_profile_collect(ctypes.byref(ms), ctypes.byref(n)), "rtx_profile_collect")
    return ms.value, n.value


def stream_handle(stream=None) -> int:
    """hipStream_t of a torch stream (default: the current stream of the current device)."""
    if stream is None:
        stream = torch.cuda.current_stream()
    return int(stream.cuda_stream)


def rccl_load() -> None:
    """Bind the row-tiled frame's RCCL calls to the librccl torch loaded (one RCCL instance per
    process: a communicator must be driven by the library that created it)."""
    path = Path(torch.__file__).resolve().parent / "lib" / "librccl.so"
    check(load().rtx_rccl_load(str(path).encode() if path.exists() else None), "rtx_rccl_load")
