"""Materials — ``Texture``, ``TextureChecker``, ``HipShader`` (reference ``shader.py:13-54``).

On this backend a shader is a parameter record: ``HipRenderer`` packs its fields into the scene blob
(``scene_pack.py``) and the render kernel evaluates ``NumpyShader.create`` (``shader.py:63-112``)
per hit; ``HipShader.create`` itself runs that evaluation for a caller-given batch of hits
(``rtx_shade_hits``). The constructor signature, defaults and the four hard-wired physical constants
(``specular_ior=1.5``, ``thin_film_weight=0.1``, ``thin_film_thickness=0.3``, ``thin_film_ior=1.4``,
``shader.py:51-54``) match the reference, and are writable like there.
"""

from __future__ import annotations

from python_ray_tracer_amd.application import Shader

from .base import HipRGBColor


class Texture:
    """Constant colour (shader.py:13-19)."""

    def __init__(self, color=None) -> None:
        self.color = color if color is not None else HipRGBColor(1, 1, 1)

    def get_color(self, intersection_point):
        return self.color


class TextureChecker(Texture):
    """White x checker mask ((int(2Px) % 2) == (int(2Pz) % 2)); its own colour is ignored
    (shader.py:22-32)."""

    def get_color(self, intersection_point):
        import numpy as np

        x = np.asarray(intersection_point.x, dtype=np.float64)
        z = np.asarray(intersection_point.z, dtype=np.float64)
        checker = ((x * 2).astype(int) % 2) == ((z * 2).astype(int) % 2)
        return HipRGBColor(1 * checker, 1 * checker, 1 * checker)


class ImageTexture(Texture):
    """An image as a diffuse texture, looked up per hit point at the spherical coordinates of the
    reference's ``NumpyTexturedSphere.diffusecolor`` (shape.py:66-79) about the hit sphere's
    centre. ``image``: a path (loaded like shape.py:64-65, ``np.asarray(Image.open(p).convert("RGB"))
    / 255.0``), an (H, W, 3) uint8 array (divided by 255.0 the same way) or an (H, W, 3) float array
    of texel colours. The reference class averages the texels of all points handed to one call into a
    single colour (shape.py:81-90), which makes it depend on how rays are batched, and cannot render
    at all (its shader is a colour, shape.py:64); this is the per-point lookup it evidently intends.
    At most 2^20 texels."""

    def __init__(self, image) -> None:
        import hashlib

        import numpy as np

        if isinstance(image, (str, bytes)) or hasattr(image, "__fspath__"):
            from PIL import Image

            arr = np.asarray(Image.open(image).convert("RGB")) / 255.0  # shape.py:64-65
        else:
            arr = np.asarray(image)
            arr = arr / 255.0 if arr.dtype == np.uint8 else arr.astype(np.float64)
        if arr.ndim != 3 or arr.shape[2] < 3 or arr.shape[0] < 1 or arr.shape[1] < 1:
            raise ValueError(f"image texture: need an (H, W, 3) image, got shape {arr.shape}")
        self.texels = np.ascontiguousarray(arr[:, :, :3], dtype=np.float64)
        if self.texels.shape[0] * self.texels.shape[1] > (1 << 20):
            raise ValueError("image texture: at most 2^20 texels")
        self.digest = hashlib.blake2b(self.texels.tobytes() + repr(self.texels.shape).encode(),
                                      digest_size=16).hexdigest()
        super().__init__(HipRGBColor(1, 1, 1))

    def get_color(self, intersection_point):
        raise NotImplementedError("ImageTexture is evaluated per hit inside the HipRenderer kernel")


class HipShader(Shader):
    """NumpyShader parameters (shader.py:36-54)."""

    def __init__(self, reflection_gain: float, specular_gain: float, specular_roughness: float,
                 iridescence_gain: float, diffuse_gain: float, diffuse_color: Texture) -> None:
        self.reflection_gain = reflection_gain  # stored, never read by the reference (shader.py:45)
        self.specular_gain = specular_gain
        self.specular_roughness = specular_roughness
        self.iridescence_gain = iridescence_gain
        self.diffuse_gain = diffuse_gain
        self.diffuse_color = diffuse_color
        self.specular_ior = 1.5
        self.thin_film_weight = 0.1
        self.thin_film_thickness = 0.3
        self.thin_film_ior = 1.4

    def create(self, shape, scene, ray_origin, normalized_ray_direction, distance, ray_tracer=None):
        """NumpyShader.create (shader.py:63-112) on the GPU: the colour of the rays (origin,
        direction) that hit ``shape`` at ``distance`` — shadow, diffuse, dome, specular,
        iridescence and the reflection recursion (shader.py:143-161), one ``rtx_shade_hits``
        launch. ``ray_tracer``: the HipRenderer whose bounce cap the reflections follow (the
        reference re-enters ``ray_tracer.raytrace_scene``); any other value uses an unbounded
        HipRenderer, as the reference NumpyRenderer recursion is. Called on another shape's
        shader, the hits are shaded with this shader's parameters on ``shape``'s geometry and the
        reflections are traced through the unchanged scene, as in the reference (shader.py:73-112,
        :152). Returns a HipRGBColor over a [3, n] device tensor."""
        from .base import HipRenderer, HipRGBColor

        r = ray_tracer if isinstance(ray_tracer, HipRenderer) else HipRenderer()
        return HipRGBColor.from_tensor(r.shade_hits(shape, scene, ray_origin, normalized_ray_direction, distance,
                                                    shader=self))
