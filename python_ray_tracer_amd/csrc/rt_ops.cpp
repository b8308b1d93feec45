// rt_ops.cpp — the PyTorch-ROCm custom-op surface of the render path:
// TORCH_LIBRARY(rt, m) over the C ABI of librtx_hip.so (include/rtx_hip.h).
//
//   rt::render_tile   <- NumpyRenderer.get_ray_directions + raytrace_scene, fused, for one interleaved
//                        row tile of the scene camera's frame, or a run of part_run parts (a rank's
//                        weighted share: rtx_render_camera_sched) (base.py:91-141, shader.py:63-161)
//   rt::render_frames <- F x render_image_pipeline's render step in one launch (application.py:43-52)
//   rt::trace         <- NumpyRenderer.raytrace_scene(O, D, scene) on arbitrary rays (base.py:91-121)
//   rt::shade_hits    <- NumpyShader.create(shape, scene, O, D, t, renderer) (shader.py:63-112)
//   rt::intersect     <- NumpySphere.intersect (shape.py:28-51)
//   rt::quantize_u8   <- save_image's (255*clip(c,0,1)).astype(uint8) (base.py:143-151)
//   rt::assemble_rows <- the multi-GPU frame's row un-permute (application.render_frame_distributed),
//                        equal shares or weighted ones (root_run / run: rtx_assemble_runs)
//   rt::status        <- reads and clears the workspace's sticky RTX_ST_* flags
//   rt::comm_unique_id, rt::comm_init, rt::comm_destroy, rt::tiles_create, rt::tiles_submit,
//   rt::tiles_finish, rt::tiles_destroy
//                     <- the row-tiled multi-GPU frame of render_frame_distributed, one native call
//                        per frame and rank (rtx_tiles_*: render, RCCL gather to the root, assembly)
//   rt::workspace_bytes
//
// Conventions (those of a TORCH_CHECKed op): tensors must live on the GPU, be contiguous and have
// the documented dtype, or the op raises RuntimeError; every op runs under a device guard of its
// input's device (so the occupancy query, the CU count and the launch all see that device, whatever
// the current device is); outputs are allocated by the caching allocator on the input's device and
// returned; work is enqueued on the current HIP stream of that device and is asynchronous, except
// for the error channel below. The ops keep no state: the caller owns the workspace (zero-filled
// once, its counters left zeroed by every call) and the optional stats buffer (accumulated into).
//
// Error channel of the render ops (render_tile, render_frames, trace, shade_hits), check=True (the
// default), mirroring HipRenderer:
//   * before the first launch on a blob (and again after any in-place write to it), the blob's
//     header (magic, sphere count) is read back to the host — one small synchronous copy — and a
//     blob that disagrees with n_spheres raises RuntimeError (the kernel would refuse it,
//     RTX_ST_BAD_SCENE, and render nothing); later calls on the same blob do not synchronise;
//   * after a launch that can defer chains beyond the fast kernel's levels (max_bounces -1 or above
//     RTX_FAST_MAX_BOUNCES), the workspace's status word is read back (a synchronisation) and
//     cleared; RTX_ST_STACK_OVERFLOW raises RuntimeError("maximum recursion depth exceeded ...",
//     where HipRenderer raises RecursionError), any other flag raises RuntimeError.
// check=False keeps the op fully asynchronous (no host synchronisation): the caller reads and clears the
// flags later with rt::status(workspace).
#include <ATen/ATen.h>
#include <ATen/DeviceGuard.h>
#include <c10/hip/HIPStream.h>
#include <torch/library.h>

#include <mutex>
#include <vector>

#include "../../include/rtx_hip.h"

namespace {

void check_rc(int rc, const char* what) {
  TORCH_CHECK(rc == RTX_OK, what, " failed (", rc, "): ", rtx_last_error());
}

bool on_gpu(const at::Tensor& t) { return t.is_cuda(); }

void check_gpu(const at::Tensor& t, const char* name, at::ScalarType dtype) {
  TORCH_CHECK(on_gpu(t), name, " must be a GPU tensor, got one on ", t.device());
  TORCH_CHECK(t.scalar_type() == dtype, name, " must be ", dtype, ", got ", t.scalar_type());
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
}

void check_same_device(const at::Tensor& a, const at::Tensor& b, const char* name) {
  TORCH_CHECK(a.device() == b.device(), name, " is on ", b.device(), ", the scene on ", a.device());
}

void* stream_of(const at::Tensor& t) { return c10::hip::getCurrentHIPStream(t.device().index()).stream(); }

void check_scene_shape(const at::Tensor& scene, int64_t n_spheres) {
  TORCH_CHECK(scene.dim() == 1, "scene must be the 1-D packed blob (scene_pack.pack_scene)");
  TORCH_CHECK(n_spheres >= 1 && n_spheres <= RTX_MAX_SPHERES, "n_spheres out of range: ", n_spheres);
  TORCH_CHECK(scene.numel() >= RTX_HDR_WORDS + n_spheres * (RTX_GEOM_WORDS + RTX_MAT_WORDS),
              "scene blob too short for ", n_spheres, " spheres");
}

void check_scene(const at::Tensor& scene, int64_t n_spheres) {
  check_gpu(scene, "scene", at::kDouble);
  check_scene_shape(scene, n_spheres);
}

// Blobs whose headers passed, keyed by the tensor object (held weakly: a live entry cannot be a freed
// tensor's address reused by a new one), its data pointer, size and version counter (bumped by every
// in-place write): a blob is read back once per content version, not on every call, so repeated
// renders of one scene stay asynchronous.
struct CheckedBlob {
  c10::weak_intrusive_ptr<c10::TensorImpl, c10::UndefinedTensorImpl> impl{
      c10::weak_intrusive_ptr<c10::TensorImpl, c10::UndefinedTensorImpl>::reclaim(
          c10::UndefinedTensorImpl::singleton())};
  const void* data = nullptr;
  int64_t numel = -1, version = -1, n_spheres = -1;
  bool matches(const at::Tensor& t, int64_t ns) const {
    return !impl.expired() && impl._unsafe_get_target() == t.unsafeGetTensorImpl() && data == t.data_ptr() &&
           numel == t.numel() && version == version_of(t) && n_spheres == ns;
  }
  // inference tensors keep no version counter (_version() throws): they are keyed on the object, its
  // storage and size alone (a blob rewritten in place under inference_mode is caught by the kernel's
  // own header test, RTX_ST_BAD_SCENE, which renders nothing)
  static int64_t version_of(const at::Tensor& t) { return t.is_inference() ? -2 : (int64_t)t._version(); }
};
constexpr int kCheckedBlobs = 32;
std::mutex g_checked_mu;
CheckedBlob g_checked[kCheckedBlobs];
int g_checked_next = 0;

// The header words of F blobs (rows of a [F, L] tensor, or one 1-D blob) against n_spheres: the
// host-side form of the kernel's RTX_ST_BAD_SCENE test (one synchronous copy of 2 words per blob,
// once per blob content: see CheckedBlob).
void check_headers(const at::Tensor& blobs, int64_t n_spheres) {
  {
    std::lock_guard<std::mutex> lock(g_checked_mu);
    for (const CheckedBlob& c : g_checked)
      if (c.matches(blobs, n_spheres)) return;
  }
  const at::Tensor head = (blobs.dim() == 1 ? blobs.narrow(0, 0, 2).unsqueeze(0) : blobs.narrow(1, 0, 2)).to(at::kCPU);
  const auto h = head.contiguous();
  const double* w = h.data_ptr<double>();
  for (int64_t f = 0; f < h.size(0); ++f) {
    TORCH_CHECK(w[2 * f + RTX_H_MAGIC] == RTX_MAGIC, "scene blob ", f, " is not a packed scene (bad magic)");
    TORCH_CHECK(w[2 * f + RTX_H_NSPH] == (double)n_spheres, "n_spheres=", n_spheres, " but scene blob ", f,
                " holds ", w[2 * f + RTX_H_NSPH], " spheres");
  }
  std::lock_guard<std::mutex> lock(g_checked_mu);
  CheckedBlob& c = g_checked[g_checked_next];
  g_checked_next = (g_checked_next + 1) % kCheckedBlobs;
  c.impl = c10::weak_intrusive_ptr<c10::TensorImpl, c10::UndefinedTensorImpl>(blobs.getIntrusivePtr());
  c.data = blobs.data_ptr();
  c.numel = blobs.numel();
  c.version = CheckedBlob::version_of(blobs);
  c.n_spheres = n_spheres;
}

// After a launch: read and clear the sticky status flags when the launch can set them (chains
// deferred beyond the fast kernel's levels); raise on any.
void check_status_after(at::Tensor& ws, int64_t max_bounces) {
  if (max_bounces >= 0 && max_bounces <= RTX_FAST_MAX_BOUNCES) return;
  at::Tensor word = ws.narrow(0, 4 * RTX_WS_STATUS, 4);
  const int32_t st = word.view(at::kInt).item<int32_t>();
  if (st == 0) return;
  word.zero_();
  TORCH_CHECK(!(st & RTX_ST_STACK_OVERFLOW), "maximum recursion depth exceeded (reflection chain > ",
              RTX_UNBOUNDED_LEVELS, " levels; HipRenderer raises RecursionError)");
  TORCH_CHECK(!(st & RTX_ST_BAD_SCENE), "the scene blob's header disagrees with n_spheres: nothing was rendered");
  TORCH_CHECK(!(st & RTX_ST_UNRENDERED), "a render passed RTX_F_NO_GENERAL but deferred rays: pixels unwritten");
  TORCH_CHECK(false, "render status flags ", st, " (RTX_ST_LIST_OVERFLOW: deferred list full)");
}

// local rows of the run of `run` parts from `part` (tiling.n_local_rows)
int64_t tile_rows(int64_t height, int64_t row_block, int64_t n_parts, int64_t part, int64_t run = 1) {
  const int64_t cycle = row_block * n_parts, own = row_block * run, q = height / cycle,
                rem = height % cycle - part * row_block;
  return q * own + (rem < 0 ? 0 : rem > own ? own : rem);
}

void check_tile(int64_t width, int64_t height, int64_t row_block, int64_t n_parts, int64_t part, int64_t part_run) {
  TORCH_CHECK(width > 0 && height > 0 && row_block > 0 && n_parts > 0 && part >= 0 && part_run >= 1 &&
                  part + part_run <= n_parts,
              "bad frame/tile geometry (part ", part, ", part_run ", part_run, " of ", n_parts, " parts)");
}

// frames: 0 = a single output, F > 0 = [F, ...] outputs of F frames
at::Tensor new_output(const at::Tensor& like, int64_t n, int64_t rows, int64_t width, int64_t out_kind,
                      int64_t frames = 0) {
  auto o = like.options();
  std::vector<int64_t> shape;
  if (frames > 0) shape.push_back(frames);
  if (out_kind == RTX_OUT_F32_SOA || out_kind == RTX_OUT_F64_SOA) {
    shape.push_back(3);
    shape.push_back(n);
    return at::empty(shape, o.dtype(out_kind == RTX_OUT_F32_SOA ? at::kFloat : at::kDouble));
  }
  TORCH_CHECK(out_kind == RTX_OUT_U8_HWC, "bad out_kind ", out_kind);
  if (rows >= 0) {
    shape.push_back(rows);
    shape.push_back(width);
  } else {
    shape.push_back(n);
  }
  shape.push_back(3);
  return at::empty(shape, o.dtype(at::kByte));
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

void check_bounces(int64_t max_bounces) {
  TORCH_CHECK(max_bounces >= RTX_UNBOUNDED, "max_bounces must be >= 0, or -1 (unbounded)");
}

// origins [3] (shared, stride 0) or [3, n]; returns the stride
int64_t check_rays(const at::Tensor& scene, const at::Tensor& origins, const at::Tensor& dirs) {
  check_gpu(origins, "origins", at::kDouble);
  check_gpu(dirs, "dirs", at::kDouble);
  check_same_device(scene, origins, "origins");
  check_same_device(scene, dirs, "dirs");
  TORCH_CHECK(dirs.dim() == 2 && dirs.size(0) == 3, "dirs must be [3, n]");
  const int64_t n = dirs.size(1);
  if (origins.dim() == 1) {
    TORCH_CHECK(origins.numel() == 3, "a shared origin is 3 doubles");
    return 0;
  }
  TORCH_CHECK(origins.dim() == 2 && origins.size(0) == 3 && origins.size(1) == n, "origins must be [3] or [3, n]");
  return n;
}

// ---- ops ---------------------------------------------------------------------------------------

at::Tensor render_tile(const at::Tensor& scene, int64_t n_spheres, int64_t width, int64_t height, int64_t row_block,
                       int64_t n_parts, int64_t part, int64_t max_bounces, int64_t out_kind, at::Tensor& workspace,
                       const std::optional<at::Tensor>& stats, bool check, int64_t part_run) {
  check_scene(scene, n_spheres);
  const at::OptionalDeviceGuard guard(at::device_of(scene));
  check_tile(width, height, row_block, n_parts, part, part_run);
  check_bounces(max_bounces);
  const int64_t rows = tile_rows(height, row_block, n_parts, part, part_run);
  const int64_t n = width * rows;
  check_workspace(workspace, scene, n, max_bounces);
  if (check) check_headers(scene, n_spheres);
  at::Tensor out = new_output(scene, n, rows, width, out_kind);
  // a run of parts (a rank's weighted share, distributed.ROOT_SHARES) in one launch; bottom-up order
  check_rc(rtx_render_camera_sched(scene.data_ptr<double>(), (int)n_spheres, (int)width, (int)height, (int)row_block,
                                   (int)n_parts, (int)part, (int)part_run, (int)rows, (int)max_bounces, out.data_ptr(),
                                   (int)out_kind, workspace.data_ptr(), (size_t)workspace.numel(),
                                   stats_ptr(stats, scene), stream_of(scene), 0u, nullptr, nullptr, nullptr),
           "rtx_render_camera_sched");
  if (check) check_status_after(workspace, max_bounces);
  return out;
}

at::Tensor render_frames(const at::Tensor& scenes, int64_t n_spheres, int64_t width, int64_t height,
                         int64_t max_bounces, int64_t out_kind, at::Tensor& workspace,
                         const std::optional<at::Tensor>& stats, bool check) {
  check_gpu(scenes, "scenes", at::kDouble);
  TORCH_CHECK(scenes.dim() == 2, "scenes must be [F, L]: one packed blob per frame (rows padded to one length)");
  const int64_t F = scenes.size(0);
  TORCH_CHECK(F >= 1 && F <= 65535, "1 to 65535 frames per launch, got ", F);
  TORCH_CHECK(n_spheres >= 1 && n_spheres <= RTX_MAX_SPHERES, "n_spheres out of range: ", n_spheres);
  TORCH_CHECK(scenes.size(1) >= RTX_HDR_WORDS + n_spheres * (RTX_GEOM_WORDS + RTX_MAT_WORDS),
              "scene blobs too short for ", n_spheres, " spheres");
  const at::OptionalDeviceGuard guard(at::device_of(scenes));
  TORCH_CHECK(width > 0 && height > 0, "bad frame geometry");
  check_bounces(max_bounces);
  const int64_t n = width * height;
  check_workspace(workspace, scenes, F * n, max_bounces);
  if (check) check_headers(scenes, n_spheres);
  at::Tensor out = new_output(scenes, n, height, width, out_kind, F);
  check_rc(rtx_render_frames(scenes.data_ptr<double>(), scenes.stride(0), (int)F, (int)n_spheres, (int)width,
                             (int)height, (int)max_bounces, out.data_ptr(), (int)out_kind, workspace.data_ptr(),
                             (size_t)workspace.numel(), stats_ptr(stats, scenes), stream_of(scenes)),
           "rtx_render_frames");
  if (check) check_status_after(workspace, max_bounces);
  return out;
}

at::Tensor trace(const at::Tensor& scene, int64_t n_spheres, const at::Tensor& origins, const at::Tensor& dirs,
                 int64_t max_bounces, int64_t out_kind, at::Tensor& workspace, const std::optional<at::Tensor>& stats,
                 bool check) {
  check_scene(scene, n_spheres);
  const at::OptionalDeviceGuard guard(at::device_of(scene));
  const int64_t stride = check_rays(scene, origins, dirs);
  const int64_t n = dirs.size(1);
  check_bounces(max_bounces);
  TORCH_CHECK(out_kind == RTX_OUT_F32_SOA || out_kind == RTX_OUT_F64_SOA, "trace returns colour: out_kind 0 or 1");
  check_workspace(workspace, scene, n, max_bounces);
  if (check) check_headers(scene, n_spheres);
  at::Tensor out = new_output(scene, n, -1, 0, out_kind);
  check_rc(rtx_trace_rays(scene.data_ptr<double>(), (int)n_spheres, origins.data_ptr<double>(), stride,
                          dirs.data_ptr<double>(), n, (int)max_bounces, out.data_ptr(), (int)out_kind,
                          workspace.data_ptr(), (size_t)workspace.numel(), stats_ptr(stats, scene), stream_of(scene)),
           "rtx_trace_rays");
  if (check) check_status_after(workspace, max_bounces);
  return out;
}

at::Tensor shade_hits(const at::Tensor& scene, int64_t n_spheres, int64_t shape, const at::Tensor& origins,
                      const at::Tensor& dirs, const at::Tensor& t, int64_t max_bounces, int64_t out_kind,
                      at::Tensor& workspace, const std::optional<at::Tensor>& stats, bool check) {
  check_scene(scene, n_spheres);
  const at::OptionalDeviceGuard guard(at::device_of(scene));
  const int64_t stride = check_rays(scene, origins, dirs);
  const int64_t n = dirs.size(1);
  check_gpu(t, "t", at::kDouble);
  check_same_device(scene, t, "t");
  TORCH_CHECK(t.dim() == 1 && t.size(0) == n, "t must be [n]: one hit distance per ray");
  TORCH_CHECK(shape >= 0 && shape < n_spheres, "shape index out of range: ", shape,
              " (NumpyShader.create raises ValueError for a shape not in scene.shapes)");
  check_bounces(max_bounces);
  TORCH_CHECK(out_kind == RTX_OUT_F32_SOA || out_kind == RTX_OUT_F64_SOA, "shade_hits returns colour: out_kind 0 or 1");
  check_workspace(workspace, scene, n, max_bounces);
  if (check) check_headers(scene, n_spheres);
  at::Tensor out = new_output(scene, n, -1, 0, out_kind);
  check_rc(rtx_shade_hits(scene.data_ptr<double>(), (int)n_spheres, (int)shape, origins.data_ptr<double>(), stride,
                          dirs.data_ptr<double>(), t.data_ptr<double>(), n, (int)max_bounces, out.data_ptr(),
                          (int)out_kind, workspace.data_ptr(), (size_t)workspace.numel(), stats_ptr(stats, scene),
                          stream_of(scene)),
           "rtx_shade_hits");
  if (check) check_status_after(workspace, max_bounces);
  return out;
}

at::Tensor intersect(const at::Tensor& sphere, const at::Tensor& origins, const at::Tensor& dirs) {
  check_gpu(sphere, "sphere", at::kDouble);
  TORCH_CHECK(sphere.numel() >= RTX_GEOM_WORDS, "sphere: ", RTX_GEOM_WORDS, " geometry words");
  const at::OptionalDeviceGuard guard(at::device_of(sphere));
  const int64_t stride = check_rays(sphere, origins, dirs);
  const int64_t n = dirs.size(1);
  at::Tensor t = at::empty({n}, dirs.options());
  check_rc(rtx_sphere_intersect(sphere.data_ptr<double>(), origins.data_ptr<double>(), stride,
                                dirs.data_ptr<double>(), n, t.data_ptr<double>(), stream_of(dirs)),
           "rtx_sphere_intersect");
  return t;
}

at::Tensor quantize_u8(const at::Tensor& color) {
  TORCH_CHECK(on_gpu(color) && color.is_contiguous(), "color must be a contiguous GPU tensor");
  TORCH_CHECK(color.dim() == 2 && color.size(0) == 3, "color must be [3, n]");
  int kind;
  if (color.scalar_type() == at::kFloat) {
    kind = RTX_OUT_F32_SOA;
  } else {
    TORCH_CHECK(color.scalar_type() == at::kDouble, "color must be float32 or float64");
    kind = RTX_OUT_F64_SOA;
  }
  const at::OptionalDeviceGuard guard(at::device_of(color));
  const int64_t n = color.size(1);
  at::Tensor out = at::empty({n, 3}, color.options().dtype(at::kByte));
  check_rc(rtx_quantize_u8(color.data_ptr(), kind, n, (uint8_t*)out.data_ptr(), stream_of(color)), "rtx_quantize_u8");
  return out;
}

at::Tensor assemble_out(const at::Tensor& tiles, int64_t width, int64_t height, int64_t out_kind) {
  TORCH_CHECK(tiles.is_contiguous() && tiles.dim() == 2, "tiles must be a contiguous [P, L] GPU tensor");
  if (out_kind == RTX_OUT_U8_HWC) {
    TORCH_CHECK(tiles.scalar_type() == at::kByte, "uint8 tiles for out_kind 2");
    return at::empty({height, width, 3}, tiles.options());
  }
  TORCH_CHECK((out_kind == RTX_OUT_F32_SOA && tiles.scalar_type() == at::kFloat) ||
                  (out_kind == RTX_OUT_F64_SOA && tiles.scalar_type() == at::kDouble),
              "tiles dtype does not match out_kind");
  return at::empty({3, height * width}, tiles.options());
}

at::Tensor assemble_rows(const at::Tensor& tiles, int64_t width, int64_t height, int64_t row_block, int64_t out_kind,
                         int64_t root_run, int64_t run) {
  TORCH_CHECK(on_gpu(tiles), "tiles must be a contiguous [P, L] GPU tensor");
  TORCH_CHECK(root_run >= 1 && run >= 1, "root_run and run must be >= 1");
  const at::OptionalDeviceGuard guard(at::device_of(tiles));
  at::Tensor out = assemble_out(tiles, width, height, out_kind);
  // rank i's tile at row i (its run of parts: rank 0 parts [0, root_run), rank i >= 1 the run
  // [root_run + (i - 1) run, + run) of the root_run + (P - 1) run interleave); equal runs of one
  // part are rtx_assemble_rows
  check_rc(rtx_assemble_runs(tiles.data_ptr(), tiles.stride(0) * (int64_t)tiles.element_size(), (int)tiles.size(0),
                             (int)root_run, (int)run, (int)width, (int)height, (int)row_block, (int)out_kind,
                             out.data_ptr(), stream_of(tiles)),
           "rtx_assemble_runs");
  return out;
}

int64_t status(at::Tensor& workspace) {
  check_gpu(workspace, "workspace", at::kByte);
  TORCH_CHECK(workspace.numel() >= RTX_WS_HDR_BYTES, "workspace shorter than its header");
  const at::OptionalDeviceGuard guard(at::device_of(workspace));
  at::Tensor word = workspace.narrow(0, 4 * RTX_WS_STATUS, 4);
  const int32_t st = word.view(at::kInt).item<int32_t>();
  if (st) word.zero_();
  return st;
}

int64_t workspace_bytes(int64_t n_rays, int64_t max_bounces) {
  return (int64_t)rtx_workspace_bytes(n_rays, (int)max_bounces);
}

// ---- the row-tiled multi-GPU frame (rtx_tiles_*, rtx_comm_*; csrc/rtx_tiles.hip) ---------------
// Handles are plain int64: a communicator from comm_init, a plan from tiles_create. The caller keeps
// the plan's buffers (send / recv, the workspace, the frame) alive until tiles_destroy, as the C ABI
// asks. These are what distributed.TileGather drives through ctypes; an integrator binding only the
// ops gets the same overlapped native gather.

void* as_ptr(int64_t h) { return reinterpret_cast<void*>(static_cast<intptr_t>(h)); }
int64_t as_handle(void* p) { return static_cast<int64_t>(reinterpret_cast<intptr_t>(p)); }

struct DeviceScope {  // the current device set to `device` (>= 0) for the scope
  int prev = -1;
  explicit DeviceScope(int64_t device) {
    if (device >= 0) {
      TORCH_CHECK(hipGetDevice(&prev) == hipSuccess, "hipGetDevice failed");
      TORCH_CHECK(hipSetDevice((int)device) == hipSuccess, "hipSetDevice(", device, ") failed");
    }
  }
  ~DeviceScope() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

at::Tensor comm_unique_id() {
  check_rc(rtx_rccl_load(nullptr), "rtx_rccl_load");
  at::Tensor id = at::empty({128}, at::TensorOptions().dtype(at::kByte));
  check_rc(rtx_comm_unique_id(id.data_ptr()), "rtx_comm_unique_id");
  return id;
}

int64_t comm_init(const at::Tensor& unique_id, int64_t world, int64_t rank, int64_t device, int64_t max_ctas) {
  TORCH_CHECK(!unique_id.is_cuda() && unique_id.scalar_type() == at::kByte && unique_id.numel() == 128 &&
                  unique_id.is_contiguous(),
              "unique_id must be the 128-byte host uint8 tensor comm_unique_id returned (broadcast to every rank)");
  check_rc(rtx_rccl_load(nullptr), "rtx_rccl_load");
  DeviceScope scope(device);
  void* comm = nullptr;
  check_rc(rtx_comm_init(unique_id.data_ptr(), (int)world, (int)rank, (int)max_ctas, &comm), "rtx_comm_init");
  return as_handle(comm);
}

void comm_destroy(int64_t comm) { check_rc(rtx_comm_destroy(as_ptr(comm)), "rtx_comm_destroy"); }

int64_t tiles_create(int64_t comm, int64_t world, int64_t rank, int64_t root, int64_t width, int64_t height,
                     int64_t row_block, int64_t out_kind, int64_t slots, at::TensorList send, at::TensorList recv,
                     int64_t part_bytes, int64_t root_run, int64_t run, int64_t flags, int64_t device) {
  TORCH_CHECK(slots >= 1 && slots <= RTX_TILES_MAX_SLOTS, "slots must be in 1..", RTX_TILES_MAX_SLOTS);
  TORCH_CHECK(send.empty() || (int64_t)send.size() == slots, "send: one buffer per slot, or none");
  TORCH_CHECK(recv.empty() || (int64_t)recv.size() == slots, "recv: one buffer per slot, or none");
  std::vector<void*> sp, rp;
  for (const at::Tensor& t : send) {
    check_gpu(t, "send buffer", at::kByte);
    TORCH_CHECK(t.numel() >= part_bytes, "a send buffer must hold part_bytes");
    sp.push_back(t.data_ptr());
  }
  for (const at::Tensor& t : recv) {
    check_gpu(t, "recv buffer", at::kByte);
    TORCH_CHECK(t.numel() >= world * part_bytes, "a recv buffer must hold world * part_bytes");
    rp.push_back(t.data_ptr());
  }
  DeviceScope scope(device);
  void* plan = nullptr;
  check_rc(rtx_tiles_create(as_ptr(comm), (int)world, (int)rank, (int)root, (int)width, (int)height, (int)row_block,
                            (int)out_kind, (int)slots, sp.empty() ? nullptr : sp.data(),
                            rp.empty() ? nullptr : rp.data(), part_bytes, (int)root_run, (int)run,
                            (unsigned)flags, &plan),
           "rtx_tiles_create");
  return as_handle(plan);
}

void tiles_submit(int64_t plan, int64_t slot, const at::Tensor& scene, int64_t n_spheres, int64_t max_bounces,
                  at::Tensor& workspace, const std::optional<at::Tensor>& frame, int64_t flags) {
  check_scene(scene, n_spheres);
  const at::OptionalDeviceGuard guard(at::device_of(scene));
  check_bounces(max_bounces);
  check_gpu(workspace, "workspace", at::kByte);
  check_same_device(scene, workspace, "workspace");
  if (frame) {
    TORCH_CHECK(frame->is_cuda() && frame->is_contiguous(), "frame must be a contiguous GPU tensor");
    check_same_device(scene, *frame, "frame");
  }
  check_rc(rtx_tiles_submit(as_ptr(plan), (int)slot, scene.data_ptr<double>(), (int)n_spheres, (int)max_bounces,
                            workspace.data_ptr(), (size_t)workspace.numel(), (unsigned)flags, nullptr, nullptr,
                            nullptr, frame ? frame->data_ptr() : nullptr, stream_of(scene)),
           "rtx_tiles_submit");
}

void tiles_finish(int64_t plan, int64_t slot, int64_t device) {
  TORCH_CHECK(device >= 0, "tiles_finish needs the plan's device index");
  check_rc(rtx_tiles_finish(as_ptr(plan), (int)slot, c10::hip::getCurrentHIPStream((int)device).stream()),
           "rtx_tiles_finish");
}

void tiles_destroy(int64_t plan) { check_rc(rtx_tiles_destroy(as_ptr(plan)), "rtx_tiles_destroy"); }

// ---- fake (Meta) kernels: output shapes only, for tracing (torch.compile / FakeTensor) ----------

at::Tensor render_tile_meta(const at::Tensor& scene, int64_t n_spheres, int64_t width, int64_t height,
                            int64_t row_block, int64_t n_parts, int64_t part, int64_t, int64_t out_kind, at::Tensor&,
                            const std::optional<at::Tensor>&, bool, int64_t part_run) {
  check_scene_shape(scene, n_spheres);
  check_tile(width, height, row_block, n_parts, part, part_run);
  const int64_t rows = tile_rows(height, row_block, n_parts, part, part_run);
  return new_output(scene, width * rows, rows, width, out_kind);
}

at::Tensor render_frames_meta(const at::Tensor& scenes, int64_t, int64_t width, int64_t height, int64_t,
                              int64_t out_kind, at::Tensor&, const std::optional<at::Tensor>&, bool) {
  TORCH_CHECK(scenes.dim() == 2, "scenes must be [F, L]");
  return new_output(scenes, width * height, height, width, out_kind, scenes.size(0));
}

at::Tensor trace_meta(const at::Tensor& scene, int64_t, const at::Tensor&, const at::Tensor& dirs, int64_t,
                      int64_t out_kind, at::Tensor&, const std::optional<at::Tensor>&, bool) {
  TORCH_CHECK(dirs.dim() == 2 && dirs.size(0) == 3, "dirs must be [3, n]");
  return new_output(scene, dirs.size(1), -1, 0, out_kind);
}

at::Tensor shade_hits_meta(const at::Tensor& scene, int64_t, int64_t, const at::Tensor&, const at::Tensor& dirs,
                           const at::Tensor&, int64_t, int64_t out_kind, at::Tensor&,
                           const std::optional<at::Tensor>&, bool) {
  TORCH_CHECK(dirs.dim() == 2 && dirs.size(0) == 3, "dirs must be [3, n]");
  return new_output(scene, dirs.size(1), -1, 0, out_kind);
}

at::Tensor intersect_meta(const at::Tensor&, const at::Tensor&, const at::Tensor& dirs) {
  TORCH_CHECK(dirs.dim() == 2 && dirs.size(0) == 3, "dirs must be [3, n]");
  return at::empty({dirs.size(1)}, dirs.options());
}

at::Tensor quantize_u8_meta(const at::Tensor& color) {
  TORCH_CHECK(color.dim() == 2 && color.size(0) == 3, "color must be [3, n]");
  return at::empty({color.size(1), 3}, color.options().dtype(at::kByte));
}

at::Tensor assemble_rows_meta(const at::Tensor& tiles, int64_t width, int64_t height, int64_t, int64_t out_kind,
                              int64_t root_run, int64_t run) {
  TORCH_CHECK(root_run >= 1 && run >= 1, "root_run and run must be >= 1");
  return assemble_out(tiles, width, height, out_kind);
}

}  // namespace

TORCH_LIBRARY(rt, m) {
  m.def("render_tile(Tensor scene, int n_spheres, int width, int height, int row_block, int n_parts, int part, "
        "int max_bounces, int out_kind, Tensor(a!) workspace, Tensor(b!)? stats=None, bool check=True, "
        "int part_run=1) -> Tensor");
  m.def("render_frames(Tensor scenes, int n_spheres, int width, int height, int max_bounces, int out_kind, "
        "Tensor(a!) workspace, Tensor(b!)? stats=None, bool check=True) -> Tensor");
  m.def("trace(Tensor scene, int n_spheres, Tensor origins, Tensor dirs, int max_bounces, int out_kind, "
        "Tensor(a!) workspace, Tensor(b!)? stats=None, bool check=True) -> Tensor");
  m.def("shade_hits(Tensor scene, int n_spheres, int shape, Tensor origins, Tensor dirs, Tensor t, int max_bounces, "
        "int out_kind, Tensor(a!) workspace, Tensor(b!)? stats=None, bool check=True) -> Tensor");
  m.def("intersect(Tensor sphere, Tensor origins, Tensor dirs) -> Tensor");
  m.def("quantize_u8(Tensor color) -> Tensor");
  m.def("assemble_rows(Tensor tiles, int width, int height, int row_block, int out_kind, int root_run=1, "
        "int run=1) -> Tensor");
  m.def("status(Tensor(a!) workspace) -> int");
  m.def("workspace_bytes(int n_rays, int max_bounces) -> int", &workspace_bytes);
  // the row-tiled multi-GPU frame (one native call per frame and rank; handles are int64)
  m.def("comm_unique_id() -> Tensor", &comm_unique_id);
  m.def("comm_init(Tensor unique_id, int world, int rank, int device=-1, int max_ctas=0) -> int", &comm_init);
  m.def("comm_destroy(int comm) -> ()", &comm_destroy);
  m.def("tiles_create(int comm, int world, int rank, int root, int width, int height, int row_block, int out_kind, "
        "int slots, Tensor[] send, Tensor[] recv, int part_bytes, int root_run=1, int run=1, int flags=0, "
        "int device=-1) -> int",
        &tiles_create);
  m.def("tiles_submit(int plan, int slot, Tensor scene, int n_spheres, int max_bounces, Tensor(a!) workspace, "
        "Tensor(b!)? frame=None, int flags=0) -> ()",
        &tiles_submit);
  m.def("tiles_finish(int plan, int slot, int device) -> ()", &tiles_finish);
  m.def("tiles_destroy(int plan) -> ()", &tiles_destroy);
}

TORCH_LIBRARY_IMPL(rt, CUDA, m) {
  m.impl("render_tile", &render_tile);
  m.impl("render_frames", &render_frames);
  m.impl("trace", &trace);
  m.impl("shade_hits", &shade_hits);
  m.impl("intersect", &intersect);
  m.impl("quantize_u8", &quantize_u8);
  m.impl("assemble_rows", &assemble_rows);
  m.impl("status", &status);
}

// Host tensors reach the same functions, whose checks raise RuntimeError ("must be a GPU tensor")
// instead of the dispatcher's "no kernel for CPU".
TORCH_LIBRARY_IMPL(rt, CPU, m) {
  m.impl("render_tile", &render_tile);
  m.impl("render_frames", &render_frames);
  m.impl("trace", &trace);
  m.impl("shade_hits", &shade_hits);
  m.impl("intersect", &intersect);
  m.impl("quantize_u8", &quantize_u8);
  m.impl("assemble_rows", &assemble_rows);
  m.impl("status", &status);
}

TORCH_LIBRARY_IMPL(rt, Meta, m) {
  m.impl("render_tile", &render_tile_meta);
  m.impl("render_frames", &render_frames_meta);
  m.impl("trace", &trace_meta);
  m.impl("shade_hits", &shade_hits_meta);
  m.impl("intersect", &intersect_meta);
  m.impl("quantize_u8", &quantize_u8_meta);
  m.impl("assemble_rows", &assemble_rows_meta);
}
