/*
 * rtx_hip.h — C ABI of the MI355X (gfx950) render-path library  librtx_hip.so
 *
 * This is the drop-in boundary for the reference's NumPy render backend
 * (/root/reference/ray_tracer/infrastructure/numpy/). Every entry point below replaces one
 * reference interface; the Python host layer (python_ray_tracer_amd/infrastructure/hip/) calls
 * them through ctypes with device pointers owned by torch tensors. Signatures are plain C:
 * pointers, sizes and an opaque stream handle (a hipStream_t) — no torch types.
 *
 *   rtx_render_camera   <- NumpyRenderer.get_ray_directions + NumpyRenderer.raytrace_scene at
 *                          level 0 with the camera origin   (base.py:123-141, base.py:91-121,
 *                          and the recursion through shader.py:63-161), fused; also one row tile
 *                          of the frame for the multi-GPU path (application.py:43-52 gains it)
 *   rtx_trace_rays      <- NumpyRenderer.raytrace_scene(ray_origin, dirs, scene) for an arbitrary
 *                          batch of rays                      (base.py:91-121)
 *   rtx_shade_hits      <- NumpyShader.create (the Shader plugin, shader.py:63-112 / application.py:35-40)
 *   rtx_ray_directions  <- NumpyRenderer.get_ray_directions  (base.py:123-141)
 *   rtx_sphere_intersect<- NumpySphere.intersect             (shape.py:28-51)
 *   rtx_quantize_u8     <- NumpyRenderer.save_image's (255*clip(c,0,1)).astype(uint8)
 *                                                             (base.py:143-151)
 *
 * Conventions
 *  - All array pointers are DEVICE pointers (hipMalloc / torch caching allocator), read-only
 *    unless documented as output. Vectors are structure-of-arrays [3][n] float64, exactly the
 *    x/y/z arrays of the reference's NumpyVector3D. A shared origin (the reference passes the
 *    camera position as Python scalars at level 0) is origin_stride == 0 and 3 doubles.
 *  - Work is enqueued asynchronously on `stream` (hipStream_t; NULL = the null stream); the caller
 *    synchronises. Entry points never allocate and never synchronise, so they can be captured into
 *    a HIP graph (tools/graph_ab.py replays captured frames bit-identical to eager ones; the caller
 *    keeps the graph's buffers alive); replays are no faster than eager launches here.
 *  - Return 0 on success, a negative RTX_E_* code otherwise; rtx_last_error() gives a message
 *    (thread-local). The Python layer raises RuntimeError on non-zero, like TORCH_CHECK would.
 *  - Scene blob: float64 array built by the host packer (scene_pack.py), layout below. It holds
 *    everything the reference reads from Scene3D during a render.
 *  - Arithmetic is IEEE float64 with no contraction (built with -ffp-contract=off), in the
 *    reference's operation order; sin (<= 2 ulp) and pow (x^5, x^2.5 by multiplications and a
 *    square root) are the only operations that are not correctly rounded, as NumPy's SIMD sin and
 *    pow (~1 ulp) are not either.
 */
#ifndef RTX_HIP_H
#define RTX_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RTX_ABI_VERSION 1

/* ---- scene blob layout (float64 words) ---- */
enum {
  RTX_HDR_WORDS = 64,  /* header */
  RTX_GEOM_WORDS = 8,  /* per sphere, at RTX_HDR_WORDS + s*RTX_GEOM_WORDS            */
  RTX_MAT_WORDS = 24,  /* per sphere, at RTX_HDR_WORDS + S*RTX_GEOM_WORDS + s*MAT    */
  RTX_MAX_DOMES = 8,
  RTX_MAX_SPHERES = 1024
};

/* header words */
enum {
  RTX_H_MAGIC = 0,   /* RTX_MAGIC */
  RTX_H_NSPH = 1,    /* S */
  RTX_H_CAM = 2,     /* camera position x,y,z (also V target on every level, shader.py:76) */
  RTX_H_LIGHT = 5,   /* scene.lights[0].position (shader.py:75) */
  RTX_H_DOMEC = 8,   /* colour of the LAST DomeLight, white if none (shader.py:237-241) */
  RTX_H_NDOME = 11,  /* number of DomeLights */
  RTX_H_DOMEI = 12,  /* their intensities, scene order (RTX_MAX_DOMES words) */
  RTX_H_XSTART = 20, /* np.linspace(-1, 1, W): start, step, stop, (W > 1) endpoint fix */
  RTX_H_XSTEP = 21,
  RTX_H_XSTOP = 22,
  RTX_H_XFIX = 23,
  RTX_H_YSTART = 24, /* np.linspace(1/ar + .25, -1/ar + .25, H) */
  RTX_H_YSTEP = 25,
  RTX_H_YSTOP = 26,
  RTX_H_YFIX = 27,
  RTX_H_VZ = 28,     /* 0 - camera.z (base.py:141) */
  RTX_H_VZ2 = 29,    /* VZ*VZ */
  RTX_H_W = 30,
  RTX_H_H = 31,
  RTX_H_CAMOO = 32,  /* |camera|^2 = camera.dot(camera) (shape.py:35 with the level-0 origin) */
  /* optional culling hierarchy (RTX_H_NNODES == 0: none, every ray tests every sphere) */
  RTX_H_NNODES = 33, /* bounding-sphere tree nodes, depth-first order                        */
  RTX_H_NALWAYS = 34,/* leading entries of the culled geometry list tested by every ray (huge spheres) */
  RTX_H_NODES = 35,  /* word offset of the node array (RTX_NODE_WORDS each)                 */
  RTX_H_CGEO = 36,   /* word offset of the culled geometry list (S records, RTX_GEOM_WORDS)  */
  RTX_H_TAME = 37,   /* 1: every coordinate (centres, camera) and radius below 2^60 in magnitude, so
                        the fast kernel may use the half-b sphere test (rtx_kernels.hip SphTest); 0: the
                        reference expressions everywhere */
  RTX_H_MAT0 = 38,   /* rtx_shade_hits only: word offset of a material record (RTX_MAT_WORDS) that
                        replaces the shape's own at level 0 — NumpyShader.create called on another
                        shape's shader (shader.py:63-112 reads self.* for the hit, and traces the
                        reflections through the unchanged scene, :152); 0 = none */
  RTX_H_SHGRID = 39, /* optional shadow grid (scenes with a culling tree and at most 128 spheres): word
                        offset of its record, 0 = none. Record: lo x,y,z; 1/cell x,y,z; nx, ny, nz;
                        centre x,y,z and grown radius of the small spheres' bounding ball; then per
                        voxel (x fastest) two 64-bit masks stored as the bits of two doubles: bit j of
                        mask k set unless sphere 64k+j provably cannot shadow (shader.py:126-128 in its
                        any-hit form) a shadow ray whose nudged origin lies in the voxel; last, the
                        huge spheres' mask (rays outside the grid that miss the ball) */
  RTX_H_SINRED = 40, /* 1: every material's thin-film phase (shader.py:208, |phase| <= 10 pi |thickness|)
                        lies in the kernel sine's reduction range (|x| <= 2^20), so no lane needs a
                        range check; 0: checked per wave */
  RTX_H_NBEAM = 41,  /* culled scenes: spheres [NBEAM, S) are all huge (the culling tree's always-tested
                        ones, RTX_H_NALWAYS): the level-0 tile candidates and the reflected-ray beams take
                        them as candidates without a test; 0 = no such tail (older blobs) */
  RTX_H_SBOX = 42    /* culled scenes of at most 128 spheres: word offset of S records {x lo, x hi, y lo,
                        y hi}, each sphere's image-plane box for this camera: a camera ray through (x, y, 0)
                        outside it provably yields FARAWAY for that sphere (bounds may be infinite);
                        0 = none (the level-0 tile candidates then take the frustum-plane test) */
};
#define RTX_MAGIC 5527384.0 /* 'RTX1' */
#define RTX_SHGRID_WORDS 13 /* words of the shadow-grid record before its masks */

/* per-sphere geometry words */
enum {
  RTX_G_CX = 0, RTX_G_CY = 1, RTX_G_CZ = 2,
  RTX_G_CC = 3,    /* abs(position) = C.C                 (shape.py:35)  */
  RTX_G_RR = 4,    /* radius*radius                       (shape.py:36)  */
  RTX_G_INVR = 5,  /* 1.0/radius                          (shader.py:74) */
  RTX_G_C0 = 6,    /* c for the camera origin: ((C.C + O.O) - 2*C.O) - r*r, O = camera */
  RTX_G_IDX = 7    /* scene index of the sphere (culled geometry list only)              */
};

/* culling-tree node words. A node bounds all spheres below it with an axis-aligned box; the tree
 * is stored depth-first with a skip link, so a wave traverses it without a stack. A node is
 * entered when any lane's ray segment may meet the box expanded by the rounding margin of the
 * reference formula (conservative test, see rtx_kernels.hip: a skipped sphere is one the reference
 * formula provably reports as FARAWAY or beyond the current nearest distance); leaves list their
 * spheres as a range of the culled geometry list. */
enum {
  RTX_NODE_WORDS = 12,
  RTX_N_LOX = 0, RTX_N_LOY = 1, RTX_N_LOZ = 2,  /* box minimum */
  RTX_N_HIX = 3, RTX_N_HIY = 4, RTX_N_HIZ = 5,  /* box maximum */
  RTX_N_FIRST = 6,  /* leaf: first culled-geometry entry   */
  RTX_N_COUNT = 7,  /* leaf: sphere count (0: inner node)  */
  RTX_N_SKIP = 8,   /* node index after this subtree        */
  RTX_N_MARGIN = 9  /* 2e-7 * (3 (|Cn|+R)^2 + R^2 + 1), Cn/R: the box's bounding sphere (error budget) */
};

/* per-sphere material words (NumpyShader, shader.py:36-54; derived constants computed on the
 * host in Python with the reference's own expressions) */
enum {
  RTX_M_G = 0,       /* specular_gain                                      */
  RTX_M_DG = 1,      /* diffuse_gain                                       */
  RTX_M_TEX = 2,     /* RTX_TEX_CONST / _CHECKER / _IMAGE                  */
  RTX_M_TR = 3, RTX_M_TG = 4, RTX_M_TB = 5, /* Texture colour; IMAGE: texel table word offset in
                                               the blob, width, height (texels: float64 RGB, row-major) */
  RTX_M_A2 = 6,      /* alpha**2, alpha = specular_roughness**2 (:294-296) */
  RTX_M_A2M1 = 7,    /* alpha**2 - 1                                       */
  RTX_M_1MA2 = 8,    /* 1 - alpha**2                                       */
  RTX_M_F0 = 9,      /* ((ior-1)/(ior+1))**2                     (:290)    */
  RTX_M_1MF0 = 10,   /* 1 - F0                                             */
  RTX_M_IG = 11,     /* iridescence_gain                                   */
  RTX_M_TFW = 12,    /* thin_film_weight                                   */
  RTX_M_TFT = 13,    /* thin_film_thickness                                */
  RTX_M_HS = 14,     /* (thin_film_ior - 1.0)/2.0                (:215)    */
  RTX_M_1MHS = 15,   /* 1.0 - hue_shift                                    */
  RTX_M_ROUGH = 16,  /* specular_roughness (informational)                 */
  RTX_M_REFL = 17,   /* reflection_gain (stored, never read: shader.py:45) */
  RTX_M_IOR = 18,
  RTX_M_TFIOR = 19
};

/* texture kinds (RTX_M_TEX) */
#define RTX_TEX_CONST 0.0   /* Texture: constant colour (shader.py:13-19)                         */
#define RTX_TEX_CHECKER 1.0 /* TextureChecker (shader.py:22-32)                                  */
#define RTX_TEX_IMAGE 2.0   /* ImageTexture: per-point texel of NumpyTexturedSphere's mapping (shape.py:66-79) */
#define RTX_MAX_TEXELS (1 << 20) /* per image texture */

/* output kinds */
enum {
  RTX_OUT_F32_SOA = 0, /* float  [3][n]  unclipped colour                     */
  RTX_OUT_F64_SOA = 1, /* double [3][n]  unclipped colour (reference dtype)   */
  RTX_OUT_U8_HWC = 2   /* uint8  [n][3]  (255*clip(c,0,1)) truncated (base.py:147) */
};

#define RTX_UNBOUNDED (-1)       /* max_bounces: no cap, like the reference recursion */
#define RTX_UNBOUNDED_LEVELS 333 /* ~ Python's recursion limit / 3 frames per level */
#define RTX_FAST_MAX_BOUNCES 6   /* bounce caps served entirely by the register-resident kernel; a
                                    larger or no cap runs it for a few levels and defers the
                                    pixels whose chain goes on to the continuation passes and the
                                    depth-first kernel (caps 7-8 that way: 1.1-1.6x faster than
                                    the 7- and 8-level kernels, which spill) */

/* stats buffer (uint64 words, accumulated with atomics; pass NULL to disable) */
enum {
  RTX_S_PIXELS = 0,   /* rays started at level 0               */
  RTX_S_DEFERRED = 1, /* rays handed to the general (tie/deep) kernel */
  RTX_S_TIES = 2,     /* (ray, level) pairs with >1 nearest shape */
  RTX_S_TESTS = 3,    /* ray-sphere tests executed by live lanes (fast kernel; culling skips most) */
  RTX_S_NODES = 4,    /* culling-node (box) tests executed by live lanes (fast kernel)            */
  RTX_S_TESTS1 = 5,   /* ... of them, the sphere tests of reflected rays' nearest-hit searches (levels >= 1) */
  RTX_S_NODES1 = 6,   /* ... and their node tests (the culling tree's box tests where the beam was not used) */
  RTX_S_BEAMW = 7,    /* reflected-ray searches served by the wave's beam candidates (waves x levels) */
  RTX_S_LEVELS = 64,  /* levels recorded                        */
  RTX_S_RAYS = 8,     /* [8 .. 8+64): rays traced per level     */
  RTX_S_HITS = 72,    /* [72 .. 72+64): shaded hits (= shadow rays) per level */
  RTX_S_WTRACE = 136, /* [136 .. 136+64): waves that traced a level (any lane live), fast kernel */
  RTX_S_WSHADE = 200, /* [200 .. 200+64): waves that shaded a level (any lane hit), fast kernel  */
  RTX_S_BOXES = 264,  /* of RTX_S_NODES, the culling tree's box tests (the rest are frustum-plane, shadow-grid
                         and beam work priced as node tests)                                       */
  RTX_S_BEAMT = 265,  /* reflected-ray beam tests: one per live lane and beam pass (a lane's cone test of one
                         sphere; round 6, counted apart from the node tests they used to be priced as) */
  RTX_S_WORDS = 266
};

/* workspace: status words then deferred-ray list then per-worker frame stacks.
 * The workspace must be zero-filled before its first use; every call leaves the counters zeroed
 * again (no per-call memset). RTX_WS_STATUS flags are sticky: the caller reads and clears them. */
enum {
  RTX_WS_COUNT = 0,    /* uint32: deferred rays            */
  RTX_WS_STATUS = 1,   /* uint32: RTX_ST_* flags           */
  RTX_WS_DONE = 2,     /* uint32: finished blocks of the general kernel (reset by the last one) */
  RTX_WS_COUNT2 = 3,   /* uint32: rays deferred by the first continuation pass (caps above 8 or none) */
  RTX_WS_COUNT3 = 4,   /* uint32: rays deferred by the second continuation pass */
  RTX_WS_HDR_BYTES = 256
};
/* RTX_ST_BAD_SCENE: the scene blob's magic or sphere count (RTX_H_NSPH) disagrees with the
 * n_spheres argument; nothing was rendered. RTX_ST_UNRENDERED: a render passed RTX_F_NO_GENERAL
 * but deferred rays (a tie, an image-textured hit): those pixels were left unwritten. */
enum { RTX_ST_STACK_OVERFLOW = 1, RTX_ST_LIST_OVERFLOW = 2, RTX_ST_BAD_SCENE = 4, RTX_ST_UNRENDERED = 8 };

enum {
  RTX_OK = 0,
  RTX_E_ARG = -1,     /* bad argument (null pointer, size, kind)  */
  RTX_E_LAUNCH = -2,  /* HIP launch / runtime error               */
  RTX_E_WORKSPACE = -3, /* workspace too small                    */
  RTX_E_COMM = -4      /* RCCL missing, or an RCCL call failed      */
};

/* Library version (RTX_ABI_VERSION) and the layout constants above, for the host to verify:
 * writes up to n ints: {HDR_WORDS, GEOM_WORDS, MAT_WORDS, MAX_DOMES, S_WORDS, WS_HDR_BYTES,
 * FAST_MAX_BOUNCES, UNBOUNDED_LEVELS}; returns RTX_ABI_VERSION. */
int rtx_abi_version(int* layout, int n);
const char* rtx_last_error(void);

/* Bytes of workspace rtx_render_camera / rtx_trace_rays need for n rays at this bounce cap. */
size_t rtx_workspace_bytes(int64_t n_rays, int max_bounces);

/* Fused primary-ray generation + trace for the camera of `scene` (replaces
 * get_ray_directions + raytrace_scene, base.py:91-141). Renders the local rows of one
 * interleaved row tiling of the frame: local row lr is global row
 *   ((lr / row_block) * n_parts + part) * row_block + lr % row_block,
 * n_local_rows of them (1,1,0 with n_local_rows == height: the whole frame). Output holds
 * n = width * n_local_rows pixels in local row-major order, as out_kind says. */
int rtx_render_camera(const double* scene, int n_spheres, int width, int height,
                      int row_block, int n_parts, int part, int n_local_rows,
                      int max_bounces, void* out, int out_kind,
                      void* workspace, size_t workspace_bytes, uint64_t* stats, void* stream);

/* rtx_render_camera with options for callers that render the same frame repeatedly:
 *  - deferred_out (may be NULL): a device-accessible uint32 (device memory, or mapped host memory)
 *    that receives, in stream order, the number of rays the fast kernel deferred in this launch
 *    (ties, longer chains); written by the general kernel, so it is left untouched when that kernel
 *    is skipped;
 *  - flags RTX_F_NO_GENERAL: for a render whose identical earlier launch (same blob content, tile,
 *    cap) deferred no ray, the general kernel is not launched — nor, for an uncapped render, the
 *    continuation pass — (the render is deterministic, so it defers none again). Passing it for a
 *    render that does defer rays leaves those pixels unwritten and raises the sticky
 *    RTX_ST_UNRENDERED flag (the workspace counters stay clean, so later calls are unaffected). */
#define RTX_F_NO_GENERAL 1u
/* RTX_F_IMAGES: the scene has image-textured spheres (RTX_TEX_IMAGE). A capped render then runs the
 * fast kernel's texturing build, which shades those hits itself (the texel lookup compiled in);
 * without the flag they are deferred to k_render_general like ties (same colours either way; the
 * texturing build costs untextured scenes 3-7%, so it is opt-in). Uncapped renders ignore it. */
#define RTX_F_IMAGES 2u
/* RTX_F_RESERVE(n): a persistent launch (>= 32 spheres, one frame) sizes its grid n blocks below what
 * the device holds at once, leaving room for the kernels of a collective running beside it (the
 * row-tiled frame's RCCL gather of the previous frame: the persistent waves would otherwise hold
 * every slot until they finish). n < 4096. */
#define RTX_F_RESERVE_SHIFT 4
#define RTX_F_RESERVE(n) ((((unsigned)(n)) & 0xFFFu) << RTX_F_RESERVE_SHIFT)
int rtx_render_camera_ex(const double* scene, int n_spheres, int width, int height,
                         int row_block, int n_parts, int part, int n_local_rows,
                         int max_bounces, void* out, int out_kind,
                         void* workspace, size_t workspace_bytes, uint64_t* stats, void* stream,
                         unsigned flags, uint32_t* deferred_out);

/* rtx_render_camera_ex with a run of parts and a dispatch order.
 * part_run >= 1: the local rows of parts part .. part + part_run - 1 of the n_parts interleave as one
 * tile (part_run * row_block rows of every cycle of n_parts * row_block rows; local row lr is global
 * row (lr / (part_run row_block)) n_parts row_block + part row_block + lr % (part_run row_block)),
 * so a rank can take a larger or smaller share of the frame than 1 / n_parts.
 * A camera launch of one frame (or row tile) is
 * dispatched in units: scenes of >= 32 spheres run persistent waves fetching kWaveW x kWaveH (8 x 8)
 * wave tiles from counters; smaller scenes one block tile (4 waves) per block, blocks dispatched in
 * grid order. rtx_sched_tiles gives the number of units; unit t is column t % units_x, row
 * t / units_x counted from the bottom of the (local) frame, and the default order is t = 0, 1, 2, ...
 * (bottom-up rows: the ground and the spheres, whose pixels run long bounce chains, first).
 *  - tile_order (may be NULL): a permutation of the units, the order in which they are handed out.
 *    Longest first shortens the launch's drain, where a few long units (long reflection chains)
 *    would otherwise run alone at its end. Output does not depend on the order.
 *  - tile_cost (may be NULL; zero-filled): receives each unit's render time (s_memrealtime ticks,
 *    100 MHz; a block tile: its slowest wave) in this launch, from which a caller derives the order
 *    of the next identical launch. A recording launch runs the kernel build that carries the
 *    counters (slower; the records stay out of the timed build's registers), so record once. */
int rtx_sched_tiles(int width, int n_local_rows, int n_spheres, int64_t* n_tiles);
int rtx_render_camera_sched(const double* scene, int n_spheres, int width, int height,
                            int row_block, int n_parts, int part, int part_run, int n_local_rows,
                            int max_bounces, void* out, int out_kind,
                            void* workspace, size_t workspace_bytes, uint64_t* stats, void* stream,
                            unsigned flags, uint32_t* deferred_out, const uint32_t* tile_order,
                            uint32_t* tile_cost);

/* Animation / batch driver (the reference renders one frame per
 * render_image_pipeline call, application.py:43-52): n_frames whole frames of one size, sphere
 * count and bounce cap in ONE launch. Frame f reads the blob at scenes + f * scene_stride (words;
 * every blob is self-describing, so frames may differ in camera, spheres and lights) and writes
 * its width*height pixels at out + f * (one frame's output bytes for out_kind). Equivalent to
 * n_frames rtx_render_camera calls of whole frames. Workspace: rtx_workspace_bytes(n_frames *
 * width * height, max_bounces). */
int rtx_render_frames(const double* scenes, int64_t scene_stride, int n_frames, int n_spheres,
                      int width, int height, int max_bounces, void* out, int out_kind,
                      void* workspace, size_t workspace_bytes, uint64_t* stats, void* stream);

/* raytrace_scene(ray_origin, normalized_ray_direction, scene) for n rays (base.py:91-121),
 * including all reflection levels up to max_bounces. origins: [3][n] (origin_stride == n) or one
 * shared origin (origin_stride == 0, 3 doubles); dirs: [3][n]. */
int rtx_trace_rays(const double* scene, int n_spheres, const double* origins, int64_t origin_stride,
                   const double* dirs, int64_t n, int max_bounces, void* out, int out_kind,
                   void* workspace, size_t workspace_bytes, uint64_t* stats, void* stream);

/* NumpyShader.create(shape, scene, ray_origin, dirs, distance, ray_tracer) (shader.py:63-112): the
 * colour of n rays that hit sphere `shape` at distances t[n] — P = O + D*t, shadow, diffuse, dome,
 * specular, iridescence, and the reflection recursion through raytrace_scene up to max_bounces
 * (the reflected rays are level 1; -1 = unbounded). The shape is taken as hit whether or not it is
 * the nearest, as create shades what it is handed. A blob whose RTX_H_MAT0 word is set shades the
 * level-0 hits with that material record instead of the shape's own (create on another shape's
 * shader). Same origins/dirs layout as rtx_trace_rays; out_kind colour or u8; workspace
 * rtx_workspace_bytes(n, max_bounces). */
int rtx_shade_hits(const double* scene, int n_spheres, int shape, const double* origins, int64_t origin_stride,
                   const double* dirs, const double* t, int64_t n, int max_bounces, void* out, int out_kind,
                   void* workspace, size_t workspace_bytes, uint64_t* stats, void* stream);

/* get_ray_directions (base.py:123-141) for the same row tiling: dirs_out [3][width*n_local_rows]. */
int rtx_ray_directions(const double* scene, int width, int height, int row_block, int n_parts,
                       int part, int n_local_rows, double* dirs_out, void* stream);

/* NumpySphere.intersect (shape.py:28-51): t_out[i] = distance or 1e39 (FARAWAY).
 * sphere: RTX_GEOM_WORDS doubles (cx, cy, cz, C.C, r*r, ...). */
int rtx_sphere_intersect(const double* sphere, const double* origins, int64_t origin_stride,
                         const double* dirs, int64_t n, double* t_out, void* stream);

/* save_image's quantisation (base.py:143-151): color [3][n] (RTX_OUT_F32_SOA or _F64_SOA) ->
 * out [n][3] uint8 = (uint8)(255 * clip(c, 0, 1)). */
int rtx_quantize_u8(const void* color, int color_kind, int64_t n, uint8_t* out, void* stream);

/* Frame assembly of the multi-GPU path (render_image_pipeline's row-tile gather, SURVEY.md §8e;
 * the reference renders one process-local frame, application.py:43-52): `tiles` holds n_parts
 * gathered row tiles, part p at tiles + p * part_stride_bytes, each as rtx_render_camera wrote it
 * for (row_block, n_parts, p) with out_kind `kind` (SoA colour: [3][rows_p * width]; u8:
 * [rows_p][width][3]). Writes the whole frame to `out` in the layout of a whole-frame render
 * (SoA [3][height * width] or u8 [height][width][3]). part_stride_bytes must hold part 0's tile
 * (the largest). */
int rtx_assemble_rows(const void* tiles, int64_t part_stride_bytes, int n_parts, int width, int height,
                      int row_block, int kind, void* out, void* stream);
/* rtx_assemble_rows for ranks that render runs of parts (rtx_render_camera_sched part_run): rank 0
 * renders parts [0, root_run), rank i >= 1 parts [root_run + (i - 1) run, root_run + i run) of the
 * root_run + (n_ranks - 1) run interleave; rank i's tile at tiles + i * part_stride_bytes (which
 * must hold the longest run's tile). root_run == run == 1 is rtx_assemble_rows. */
int rtx_assemble_runs(const void* tiles, int64_t part_stride_bytes, int n_ranks, int root_run, int run, int width,
                      int height, int row_block, int kind, void* out, void* stream);

/* ---- the row-tiled multi-GPU frame, one call per frame and rank (csrc/rtx_tiles.hip) ----
 * The north star's "framebuffer row-tiles across the GPUs of one node with an RCCL gather over
 * xGMI": the reference renders one frame in one process (render_image_pipeline,
 * application.py:43-52); python_ray_tracer_amd.distributed.TileGather drives these entry points.
 * Every rank renders its interleaved row tile (as rtx_render_camera_ex with row_block, n_parts =
 * world, part = rank); the root receives every peer's tile with one ncclRecv per peer inside one
 * RCCL group (each peer's link carries its own bytes at once; a ring would be bound by one link)
 * and un-permutes the rows on the device (rtx_assemble_rows). RCCL is the process's own librccl,
 * resolved at run time (rtx_rccl_load): the library has no link-time RCCL dependency. */
#define RTX_TILES_MAX_SLOTS 4
/* dlopen the RCCL library at `path` (NULL: "librccl.so"), reusing it if the process already loaded
 * it (torch's), and resolve the calls used here. Idempotent. */
int rtx_rccl_load(const char* path);
/* ncclGetUniqueId into id_out (128 bytes): the root calls it, the host broadcasts the bytes. */
int rtx_comm_unique_id(void* id_out);
/* ncclCommInitRank over `world` ranks (collective: every rank calls it with the same id); the
 * communicator is bound to the current device. max_ctas > 0: ncclCommInitRankConfig with
 * maxCTAs = max_ctas, capping the blocks its kernels take from a render running beside them. */
int rtx_comm_init(const void* id, int world, int rank, int max_ctas, void** comm_out);
int rtx_comm_destroy(void* comm);
/* rtx_tiles_create flags. RTX_TILES_LOOPBACK: a one-rank plan whose tile still travels through
 * RCCL (sent to and received from itself, then assembled): the gather path on a single GPU.
 * RTX_F_RESERVE(n): every render of a plan that gathers (world > 1 or loopback) passes it, so that
 * frame k's RCCL kernels find free slots beside frame k+1's persistent render. */
#define RTX_TILES_LOOPBACK 1u
/* RTX_TILES_ROWS (uint8 frames): every row block travels on its own, straight into its rows of the
 * root's frame (one ncclSend / ncclRecv per block; the root's own blocks by one strided device
 * copy), so the root never runs the assembly pass (a read and a write of the whole frame in HBM,
 * beside its next render). recv[s] then holds the root's own tile only (part_bytes). */
#define RTX_TILES_ROWS 2u
/* RTX_TILES_TIMED: timing events on the plan's stream around each slot's RCCL group and the root's
 * assembly (plans that gather), read back by rtx_tiles_timing: the measured gather per frame and
 * rank (bench.py's secondary.c4_tiles.gather: bytes per peer and the achieved rate per link). */
#define RTX_TILES_TIMED 4u
/* Shares: rank 0 renders the run of parts [0, root_run) and rank i >= 1 the run [root_run + (i - 1)
 * run, root_run + i run) of the root_run + (world - 1) run interleave (rtx_render_camera_sched
 * part_run). root_run = run = 1 is the even split; a root_run below run leaves the root, which also
 * receives and assembles every frame, a smaller share (then the root must be rank 0). part_bytes must
 * hold the longest run's tile.
 * A plan for frames of width x height in row blocks of row_block, out_kind RTX_OUT_*, `slots`
 * frames in flight (<= RTX_TILES_MAX_SLOTS). Per slot s, caller-owned device buffers kept for the
 * plan's life: a peer's send[s] (part_bytes) and the root's recv[s] (world * part_bytes: part p at
 * p * part_bytes). part_bytes holds the longest run's tile, a multiple of 16. world == 1 needs
 * neither buffers nor a communicator (comm NULL): the single part is the frame (unless
 * RTX_TILES_LOOPBACK: then send and recv as a root and peer would). Creates the plan's own
 * collective stream on the current device. */
int rtx_tiles_create(void* comm, int world, int rank, int root, int width, int height, int row_block, int out_kind,
                     int slots, void* const* send, void* const* recv, int64_t part_bytes, int root_run, int run,
                     unsigned flags, void** plan_out);
/* Frame of slot `slot`: on `stream`, wait until the slot's previous frame has left its buffers, then
 * render this rank's tile (scene, n_spheres, max_bounces, workspace, flags, deferred_out, tile_order,
 * tile_cost as rtx_render_camera_sched); then, on the plan's stream after the render, the RCCL gather to the root
 * and (root) the assembly into `frame` (the root's whole frame, in a whole-frame render's layout;
 * ignored on peers). Asynchronous; never synchronises. */
int rtx_tiles_submit(void* plan, int slot, const double* scene, int n_spheres, int max_bounces, void* workspace,
                     size_t workspace_bytes, unsigned flags, uint32_t* deferred_out, const uint32_t* tile_order,
                     uint32_t* tile_cost, void* frame, void* stream);
/* Make `stream` wait until slot `slot`'s frame is complete (the root's frame is then valid in
 * stream order). */
int rtx_tiles_finish(void* plan, int slot, void* stream);
/* Waits for the plan's stream, then frees its stream and events (not the caller's buffers). */
int rtx_tiles_destroy(void* plan);
/* RTX_TILES_TIMED plans: waits for slot `slot`'s latest frame on the plan's stream, then gives
 * gather_ms, from the moment the plan's stream could start the gather (this rank's tile rendered)
 * to the completion of its RCCL group (a peer: its send delivered; the root: every peer's tile
 * received), and assemble_ms, the root's assembly after it (0 on peers). Synchronising: call it
 * outside a timed region. No replacement in the reference (one process, application.py:43-52). */
int rtx_tiles_timing(void* plan, int slot, float* gather_ms, float* assemble_ms);

/* Test hook: out[0:n] = the library's fast-path sqrt(a), out[n:2n] = the compiler's full sqrt(a),
 * out[2n:3n] = fast-path a/b, out[3n:4n] = full a/b, out[4n:5n] = the renormalisation factor of an
 * already-unit vector with |v|^2 = a (closed form when every lane of the wave has a within 2^-30
 * of 1), out[5n:6n] = 1/sqrt(a) by the full expansions (a == 0: 1). out holds 6n doubles. The
 * render kernels use the fast paths (correctly rounded sequences without operand scaling where it
 * is the identity); tests require each pair to agree bit for bit. */
int rtx_selftest_math(const double* a, const double* b, int64_t n, double* out, void* stream);

/* Live timing of the dominant render kernel (used by bench.py for the roofline): after
 * rtx_profile_enable(k), the next k render launches hand a hipEvent pair to the k_render_fast
 * dispatch itself (hipExtLaunchKernelGGL start/stop events: the kernel's own start and end, as
 * rocprofv3's kernel trace sees them). rtx_profile_collect waits for the recorded events and
 * returns the summed kernel time and the launch count, then resets. rtx_profile_enable(0)
 * disables. The profiling state is per calling thread (only that thread's launches are timed);
 * meant for benchmarks, not for graph capture. */
int rtx_profile_enable(int max_launches);
int rtx_profile_collect(double* total_ms, int* n_launches);
/* Time only one render launch in `every` (default 1: all), the every-th, 2*every-th, ... after
 * rtx_profile_enable (not the first: it follows an idle GPU). Timing a launch costs stream time
 * (1080p C2: 24.1 Gpix/s timing every launch against 26.0 timing one in 10); sampling keeps the
 * live kernel timing while leaving the timed region nearly unperturbed. Persists across
 * rtx_profile_enable calls. */
int rtx_profile_sample(int every);

#ifdef __cplusplus
}
#endif
#endif /* RTX_HIP_H */
