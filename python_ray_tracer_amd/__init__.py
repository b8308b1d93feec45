"""MI355X-native backend for the python_ray_tracer render path.

The product is ``HipRenderer`` (``python_ray_tracer_amd.infrastructure.hip``), a drop-in for the
reference's ``NumpyRenderer`` behind the same ``Renderer`` / ``render_image_pipeline`` surface
(``/root/reference/ray_tracer/application.py:7-52``), driving hand-written HIP kernels for gfx950
through the C-ABI library ``librtx_hip.so`` (``include/rtx_hip.h``).
"""

__version__ = "0.1.0"
