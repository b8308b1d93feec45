// rt_ops.cpp — the PyTorch-ROCm custom-op surface of the render path:
// TORCH_LIBRARY(rt, m) over the C ABI of librtx_hip.so (include/rtx_hip.h).
//
//   rt::render_tile   <- NumpyRenderer.get_ray_directions + raytrace_scene, fused, for one interleaved
//                        row tile of the scene camera's frame (base.py:91-141, shader.py:63-161)
//   rt::trace         <- NumpyRenderer.raytrace_scene(O, D, scene) on arbitrary rays (base.py:91-121)
//   rt::intersect     <- NumpySphere.intersect (shape.py:28-51)
//   rt::quantize_u8   <- save_image's (255*clip(c,0,1)).astype(uint8) (base.py:143-151)
//   rt::assemble_rows <- the multi-GPU frame's row un-permute (application.render_frame_distributed)
//   rt::workspace_bytes
//
// Conventions (those of a TORCH_CHECKed op): tensors must live on the GPU, be contiguous and have
// the documented dtype, or the op raises RuntimeError; outputs are allocated by the caching
// allocator on the input's device and returned; work is enqueued on the current HIP stream of that
// device (c10::hip::getCurrentHIPStream) and is asynchronous. The ops keep no state: the caller
// owns the workspace (zero-filled once, left zeroed by every call) and the optional stats buffer.
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <torch/library.h>

#include "../../include/rtx_hip.h"

namespace {

void check_rc(int rc, const char* what) {
  TORCH_CHECK(rc == RTX_OK, what, " failed (", rc, "): ", rtx_last_error());
}

void check_gpu(const at::Tensor& t, const char* name, at::ScalarType dtype) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor, got one on ", t.device());
  TORCH_CHECK(t.scalar_type() == dtype, name, " must be ", dtype, ", got ", t.scalar_type());
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
}

void check_same_device(const at::Tensor& a, const at::Tensor& b, const char* name) {
  TORCH_CHECK(a.device() == b.device(), name, " is on ", b.device(), ", the scene on ", a.device());
}

void* stream_of(const at::Tensor& t) { return c10::hip::getCurrentHIPStream(t.device().index()).stream(); }

void check_scene(const at::Tensor& scene, int64_t n_spheres) {
  check_gpu(scene, "scene", at::kDouble);
  TORCH_CHECK(scene.dim() == 1, "scene must be the 1-D packed blob (scene_pack.pack_scene)");
  TORCH_CHECK(n_spheres >= 1 && n_spheres <= RTX_MAX_SPHERES, "n_spheres out of range: ", n_spheres);
  TORCH_CHECK(scene.numel() >= RTX_HDR_WORDS + n_spheres * (RTX_GEOM_WORDS + RTX_MAT_WORDS),
              "scene blob too short for ", n_spheres, " spheres");
}

int64_t tile_rows(int64_t height, int64_t row_block, int64_t n_parts, int64_t part) {
  const int64_t cycle = row_block * n_parts, q = height / cycle, rem = height % cycle - part * row_block;
  return q * row_block + (rem < 0 ? 0 : rem > row_block ? row_block : rem);
}

at::Tensor new_output(const at::Tensor& like, int64_t n, int64_t rows, int64_t width, int64_t out_kind) {
  auto o = like.options();
  if (out_kind == RTX_OUT_F32_SOA) return at::empty({3, n}, o.dtype(at::kFloat));
  if (out_kind == RTX_OUT_F64_SOA) return at::empty({3, n}, o.dtype(at::kDouble));
  TORCH_CHECK(out_kind == RTX_OUT_U8_HWC, "bad out_kind ", out_kind);
  return rows >= 0 ? at::empty({rows, width, 3}, o.dtype(at::kByte)) : at::empty({n, 3}, o.dtype(at::kByte));
}

void check_workspace(const at::Tensor& ws, const at::Tensor& scene, int64_t n, int64_t max_bounces) {
  check_gpu(ws, "workspace", at::kByte);
  check_same_device(scene, ws, "workspace");
  const size_t need = rtx_workspace_bytes(n, (int)max_bounces);
  TORCH_CHECK((size_t)ws.numel() >= need, "workspace too small: ", ws.numel(), " < ", need,
              " bytes (rt::workspace_bytes)");
}

uint64_t* stats_ptr(const std::optional<at::Tensor>& stats, const at::Tensor& scene) {
  if (!stats.has_value()) return nullptr;
  check_gpu(*stats, "stats", at::kLong);
  check_same_device(scene, *stats, "stats");
  TORCH_CHECK(stats->numel() >= RTX_S_WORDS, "stats needs ", RTX_S_WORDS, " int64 words");
  return (uint64_t*)stats->data_ptr();
}

at::Tensor render_tile(const at::Tensor& scene, int64_t n_spheres, int64_t width, int64_t height, int64_t row_block,
                       int64_t n_parts, int64_t part, int64_t max_bounces, int64_t out_kind, at::Tensor& workspace,
                       const std::optional<at::Tensor>& stats) {
  check_scene(scene, n_spheres);
  TORCH_CHECK(width > 0 && height > 0 && row_block > 0 && n_parts > 0 && part >= 0 && part < n_parts,
              "bad frame/tile geometry");
  TORCH_CHECK(max_bounces >= RTX_UNBOUNDED, "max_bounces must be >= 0, or -1 (unbounded)");
  const int64_t rows = tile_rows(height, row_block, n_parts, part);
  const int64_t n = width * rows;
  check_workspace(workspace, scene, n, max_bounces);
  at::Tensor out = new_output(scene, n, rows, width, out_kind);
  check_rc(rtx_render_camera(scene.data_ptr<double>(), (int)n_spheres, (int)width, (int)height, (int)row_block,
                             (int)n_parts, (int)part, (int)rows, (int)max_bounces, out.data_ptr(), (int)out_kind,
                             workspace.data_ptr(), (size_t)workspace.numel(), stats_ptr(stats, scene), stream_of(scene)),
           "rtx_render_camera");
  return out;
}

at::Tensor trace(const at::Tensor& scene, int64_t n_spheres, const at::Tensor& origins, const at::Tensor& dirs,
                 int64_t max_bounces, int64_t out_kind, at::Tensor& workspace, const std::optional<at::Tensor>& stats) {
  check_scene(scene, n_spheres);
  check_gpu(origins, "origins", at::kDouble);
  check_gpu(dirs, "dirs", at::kDouble);
  check_same_device(scene, origins, "origins");
  check_same_device(scene, dirs, "dirs");
  TORCH_CHECK(dirs.dim() == 2 && dirs.size(0) == 3, "dirs must be [3, n]");
  const int64_t n = dirs.size(1);
  int64_t stride;
  if (origins.dim() == 1) {
    TORCH_CHECK(origins.numel() == 3, "a shared origin is 3 doubles");
    stride = 0;
  } else {
    TORCH_CHECK(origins.dim() == 2 && origins.size(0) == 3 && origins.size(1) == n, "origins must be [3] or [3, n]");
    stride = n;
  }
  TORCH_CHECK(max_bounces >= RTX_UNBOUNDED, "max_bounces must be >= 0, or -1 (unbounded)");
  TORCH_CHECK(out_kind == RTX_OUT_F32_SOA || out_kind == RTX_OUT_F64_SOA, "trace returns colour: out_kind 0 or 1");
  check_workspace(workspace, scene, n, max_bounces);
  at::Tensor out = new_output(scene, n, -1, 0, out_kind);
  check_rc(rtx_trace_rays(scene.data_ptr<double>(), (int)n_spheres, origins.data_ptr<double>(), stride,
                          dirs.data_ptr<double>(), n, (int)max_bounces, out.data_ptr(), (int)out_kind,
                          workspace.data_ptr(), (size_t)workspace.numel(), stats_ptr(stats, scene), stream_of(scene)),
           "rtx_trace_rays");
  return out;
}

at::Tensor intersect(const at::Tensor& sphere, const at::Tensor& origins, const at::Tensor& dirs) {
  check_gpu(sphere, "sphere", at::kDouble);
  TORCH_CHECK(sphere.numel() >= RTX_GEOM_WORDS, "sphere: ", RTX_GEOM_WORDS, " geometry words");
  check_gpu(origins, "origins", at::kDouble);
  check_gpu(dirs, "dirs", at::kDouble);
  check_same_device(sphere, origins, "origins");
  check_same_device(sphere, dirs, "dirs");
  TORCH_CHECK(dirs.dim() == 2 && dirs.size(0) == 3, "dirs must be [3, n]");
  const int64_t n = dirs.size(1);
  const int64_t stride = origins.dim() == 1 ? 0 : n;
  TORCH_CHECK(stride == 0 ? origins.numel() == 3 : (origins.size(0) == 3 && origins.size(1) == n),
              "origins must be [3] or [3, n]");
  at::Tensor t = at::empty({n}, dirs.options());
  check_rc(rtx_sphere_intersect(sphere.data_ptr<double>(), origins.data_ptr<double>(), stride,
                                dirs.data_ptr<double>(), n, t.data_ptr<double>(), stream_of(dirs)),
           "rtx_sphere_intersect");
  return t;
}

at::Tensor quantize_u8(const at::Tensor& color) {
  TORCH_CHECK(color.is_cuda() && color.is_contiguous(), "color must be a contiguous GPU tensor");
  TORCH_CHECK(color.dim() == 2 && color.size(0) == 3, "color must be [3, n]");
  int kind;
  if (color.scalar_type() == at::kFloat) {
    kind = RTX_OUT_F32_SOA;
  } else {
    TORCH_CHECK(color.scalar_type() == at::kDouble, "color must be float32 or float64");
    kind = RTX_OUT_F64_SOA;
  }
  const int64_t n = color.size(1);
  at::Tensor out = at::empty({n, 3}, color.options().dtype(at::kByte));
  check_rc(rtx_quantize_u8(color.data_ptr(), kind, n, (uint8_t*)out.data_ptr(), stream_of(color)), "rtx_quantize_u8");
  return out;
}

at::Tensor assemble_rows(const at::Tensor& tiles, int64_t width, int64_t height, int64_t row_block, int64_t out_kind) {
  TORCH_CHECK(tiles.is_cuda() && tiles.is_contiguous() && tiles.dim() == 2, "tiles must be a contiguous [P, L] GPU tensor");
  const int64_t P = tiles.size(0);
  at::Tensor out;
  if (out_kind == RTX_OUT_U8_HWC) {
    TORCH_CHECK(tiles.scalar_type() == at::kByte, "uint8 tiles for out_kind 2");
    out = at::empty({height, width, 3}, tiles.options());
  } else {
    TORCH_CHECK((out_kind == RTX_OUT_F32_SOA && tiles.scalar_type() == at::kFloat) ||
                    (out_kind == RTX_OUT_F64_SOA && tiles.scalar_type() == at::kDouble),
                "tiles dtype does not match out_kind");
    out = at::empty({3, height * width}, tiles.options());
  }
  check_rc(rtx_assemble_rows(tiles.data_ptr(), tiles.stride(0) * (int64_t)tiles.element_size(), (int)P, (int)width,
                             (int)height, (int)row_block, (int)out_kind, out.data_ptr(), stream_of(tiles)),
           "rtx_assemble_rows");
  return out;
}

int64_t workspace_bytes(int64_t n_rays, int64_t max_bounces) {
  return (int64_t)rtx_workspace_bytes(n_rays, (int)max_bounces);
}

}  // namespace

TORCH_LIBRARY(rt, m) {
  m.def("render_tile(Tensor scene, int n_spheres, int width, int height, int row_block, int n_parts, int part, "
        "int max_bounces, int out_kind, Tensor(a!) workspace, Tensor? stats=None) -> Tensor");
  m.def("trace(Tensor scene, int n_spheres, Tensor origins, Tensor dirs, int max_bounces, int out_kind, "
        "Tensor(a!) workspace, Tensor? stats=None) -> Tensor");
  m.def("intersect(Tensor sphere, Tensor origins, Tensor dirs) -> Tensor");
  m.def("quantize_u8(Tensor color) -> Tensor");
  m.def("assemble_rows(Tensor tiles, int width, int height, int row_block, int out_kind) -> Tensor");
  m.def("workspace_bytes(int n_rays, int max_bounces) -> int", &workspace_bytes);
}

TORCH_LIBRARY_IMPL(rt, CUDA, m) {
  m.impl("render_tile", &render_tile);
  m.impl("trace", &trace);
  m.impl("intersect", &intersect);
  m.impl("quantize_u8", &quantize_u8);
  m.impl("assemble_rows", &assemble_rows);
}

// Host tensors reach the same functions, whose checks raise RuntimeError ("must be a GPU tensor")
// instead of the dispatcher's "no kernel for CPU".
TORCH_LIBRARY_IMPL(rt, CPU, m) {
  m.impl("render_tile", &render_tile);
  m.impl("trace", &trace);
  m.impl("intersect", &intersect);
  m.impl("quantize_u8", &quantize_u8);
  m.impl("assemble_rows", &assemble_rows);
}
