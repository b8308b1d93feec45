// rtx_kernels.hip — hand-written CDNA4 (gfx950) kernels for the python_ray_tracer render path,
// plus the extern "C" entry points declared in include/rtx_hip.h.
//
// One thread = one ray (one pixel in camera mode); 64-lane waves cover 8x8 pixel tiles so the
// rays of a wave stay coherent through the bounce chain. All geometry is float64 (SURVEY.md §7
// hard part 1: the R=99999 ground sphere flips checker cells in fp32) and every expression keeps
// the reference's operation order (file:line cited at each step); the library is compiled with
// -ffp-contract=off because NumPy never fuses a multiply into an add.
//
// Kernels
//   k_render_fast<B, LDS>  B <= RTX_FAST_MAX_BOUNCES. The reference's recursion
//                     raytrace_scene -> create -> _calculate_reflection -> raytrace_scene
//                     (base.py:91-121, shader.py:63-161) becomes an in-register loop over bounce
//                     levels. For every non-terminal level a compile-time-sized shift register keeps
//                     the INPUTS of that level's colour terms (max(N.L,0), the dome sum, the specular,
//                     N.V, the hit sphere and its checker bit: 4 doubles + 1 int); the fold from the
//                     deepest level recomputes A and I from them with the same instructions and
//                     applies the reference association
//                         col_k = ((A_k + (spec_k + col_{k+1}*0.5)*g_k) + I_k)      (shader.py:106-110)
//                     exactly. Sphere geometry is read by the wave-uniform loops through the scalar
//                     cache (s_load); the per-lane hit-sphere/material records come from an LDS copy
//                     of the scene table (LDS = S <= kLdsMaxSpheres). Scenes of >= 8 spheres carry
//                     a tree of boxes that the loops walk wave-uniformly (exact culling). Tile rows
//                     are dispatched bottom-up (longest work first). A ray that meets a tie (two
//                     shapes at the same nearest distance, base.py:103 — both get shaded and summed)
//                     or, under a cap above 8 or none, a chain longer than kDeepLevels levels is
//                     appended to a deferred list.
//   k_render_general  Any bounce cap, ties included: an explicit depth-first walk of the ray tree
//                     with per-worker frame stacks in the workspace (HBM). Renders the deferred
//                     list of k_render_fast from level 0. Its last block resets the list counter,
//                     so the workspace is left zeroed for the next call (no per-frame memset).
//   k_ray_dirs, k_intersect, k_quantize — the remaining boundary functions.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "../../include/rtx_hip.h"

#define FARAWAY 1.0e39  // base.py:12
#define RTX_PI 3.141592653589793  // np.pi

namespace {

constexpr int kBlock = 256;   // threads per block of the elementwise boundary kernels
// ---- tuning constants (each value chosen by an A/B on identical output, profiles/r1_ab_variants.txt;
// tools/ab_build.py builds variants by rewriting these lines) ----
constexpr int kWaveW = 8;       // pixels per wave row: a wave renders a kWaveW x (64 / kWaveW) tile
// ... in scenes below kTreeMinSpheres (the TREE = false kernels; A/B profiles/r3_ab_variants.txt r3x-r3z:
// C2 -0.8%, C2main -1.1%, C1 -6%; the culled kernels keep 8 x 8: C5 +0.6%, C4 +3% at 16 x 4, the
// wave frustum and beam bounds are tighter on square tiles)
constexpr int kWaveWSmall = 16;
constexpr int kFastWaves = 4;   // waves per k_render_fast block (1, 2 or 4) of the culled kernels
// ... and of the TREE = false kernels (scenes below kTreeMinSpheres): one wave per block, so the
// hardware hands out single 16x4 wave tiles in the learnt longest-first order (rtx_render_camera_sched;
// A/B r4f, C2: 52.8 against 54.5 us per frame with four-wave blocks, 54.7 / 55.7 without the order)
constexpr int kFastWavesSmall = 1;
// k_render_fast single-frame launches of scenes with at least this many spheres: persistent waves
// fetching wave tiles (A/B: 65 spheres -14%, 17 spheres +-0, 3-16 spheres without the culling tree
// +12%: their tiles are short, so the ramp-up of the fetch counters and the drain cost more than
// the balancing gains)
constexpr int kPersistMinSpheres = 32;
constexpr int kMaxFetch = 32;   // tile counters (one 128-byte line each) shared round-robin by the waves
// general-kernel threads: ties only (caps <= RTX_FAST_MAX_BOUNCES; an empty launch costs more with
// more blocks), or ties and deep chains (A/B for unbounded renders: 4096, 16384, 65536)
constexpr int kDeferredWorkers = 4096;
constexpr int kDeepWorkers = 16384;
constexpr bool kLevelsInLds = true;  // capped kernels with B <= kLevelsLdsMaxB keep their levels' colour inputs in LDS
constexpr int kLevelsLdsMaxB = 6;    // the deepest cap with LDS level slots
constexpr int kLevelsLdsSlots = 3;   // levels kept in LDS; deeper ones (B = 4) in a register slot
constexpr int kB5Slots = 2;          // LDS level slots of the B >= 5 kernels (the others in a register shift)
constexpr int kB5Waves = 4;          // their waves/SIMD
constexpr int kLvWaves = 5;          // waves/SIMD of the kernels with LDS level slots (96 VGPRs; 5 blocks fit up to 17 spheres)
constexpr int kLvWavesSmall = 5;     // ... and of their TREE = false instantiations (scenes below kTreeMinSpheres)
constexpr int kDeepLvMaxSpheres = 32;  // DEEP kernels with LDS level slots up to this many spheres (3 blocks of 54 KB per CU)
constexpr int kDeepWaves = 4;        // waves/SIMD of the persistent DEEP kernel (with the beam at 3 its persistent kernel takes
                                     // 134 VGPRs; at 4, 128: A/B r6ap, unbounded C4 -14%)
constexpr int kDeepWavesTile = 5;    // ... of the one-tile first passes (TP 1 and 0; A/B r6ar, unbounded: C3 -5.1%,
                                     // C2 -2.0%, C2main -5.0% against 4, the persistent C4 +-0)
constexpr int kFastWavesPerSimd = 4; // __launch_bounds__ min waves per SIMD otherwise: <=128 VGPRs (A/B: faster than 3 waves without spills)
// Capped kernels (B <= RTX_FAST_MAX_BOUNCES): the bounce chain's colour is accumulated forwards,
// col = sum_k T_k L_k with T_0 = 1, T_{k+1} = (T_k * 0.5) * g_k and L_k level k's colour with a
// black reflection, instead of storing every non-terminal level's colour inputs and folding them
// back from the deepest level (the reference's association, shader.py:106-110: col_k = ((A_k +
// (spec_k + col_{k+1} * 0.5) * g_k) + I_k)). Same terms, reassociated: the result moves by a few
// ulp of the colour (<= ~1e-13 absolute at the brightest unclipped values, under the 1e-12 parity
// bar), and no level's inputs live in LDS slots or registers across the chain: C4's B = 5 kernel
// kept three levels in a register shift (27 VGPRs, the bulk of its 41 spilled) beside two LDS slots.
// The DEEP kernels keep the backward fold (their resume records carry the levels' inputs).
// A/B r5c (one box, tools/ab.py, frames identical): C2 55.20 -> 52.94 us (-4.1%), C4 2,055 -> 1,874 us
// (-8.8%: 41 spilled VGPRs -> 0), C3 273.1 -> 265.7 us (-2.7%, at 5 waves/SIMD; 283.9 at 4)
constexpr bool kForwardFold = true;
constexpr int kFwdWavesPersist = 4;  // waves/SIMD of the forward-fold persistent kernels (TP 2; C4: 5 waves 2,025 us)
constexpr int kFwdWaves = 5;         // ... of the culled one-tile-per-block kernels (TP 1; C3: 4 waves 283.9 us)
// ... and of their launches of at least kWavesLargeMinPixels pixels (A/B r6aw, 6 waves against 5: C3 (8.3 M
// pixels) -3.3%, C5's 32-frame launches -3.5%, but one 1080p frame of C5's scene +4%: 80 VGPRs spill)
constexpr int kFwdWavesLarge = 6;
constexpr int64_t kWavesLargeMinPixels = int64_t(4) << 20;
constexpr int kFwdWavesSmall = 5;    // ... and of the TREE = false kernels (TP 0; C2: 6 waves 56.0 us, spills)
constexpr int kDeepLevels = 5;       // fast-kernel levels before a longer chain is deferred (A/B: 3, 5, 8; the
                                     // 8-level instantiation spills, 3 defers too many pixels)
constexpr int kCappedMax = RTX_FAST_MAX_BOUNCES;  // caps rendered entirely by k_render_fast<cap>
// shading-only terms (the view vector, the half vector and the specular's internal divisions and
// square roots; none of them decides a hit, a shadow, a checker cell or a reflected ray):
//   0 = the wave-uniform range-checked correctly rounded paths;
//   1 = the correctly rounded cores without range checks (operands in range by construction);
//   3 = the specular's divisions and square roots by shorter Newton sequences (within ~1 ulp,
//       tools/approx_probe), V and H normalised by the correctly rounded cores (A/B on identical
//       parity: C2 -6.4%, C2main -8.5%, C5 -2.9%, C3 -2.8% against 1);
//   2 / 4 = also V and H (2) or H (4) by rsq + Newton: N.V near grazing amplifies their rounding,
//       C4 and 1080p colour moved by 1.4e-12 (over the 1e-12 bar), not adopted.
constexpr int kShadeMath = 3;
// ---- derived ----
constexpr int kWaveH = 64 / kWaveW;
static_assert(kFastWaves == 1 || kFastWaves == 2 || kFastWaves == 4, "kFastWaves");
static_assert(kFastWavesSmall == 1 || kFastWavesSmall == 2 || kFastWavesSmall == 4, "kFastWavesSmall");
static_assert((kMaxFetch & (kMaxFetch - 1)) == 0, "kMaxFetch must be a power of two");
constexpr int kFastBlock = 64 * kFastWaves;
constexpr int kWavesX = kFastWavesSmall == 1 ? 1 : 2;  // block tile of the small kernels: kWavesX x kWavesY waves
constexpr int kWavesXTree = kFastWaves;  // ... of the culled kernels: one row of waves (A/B r3o: C5 -3.0%, C3 +-0.3%; C1 +9% for the small ones)
static_assert(kWaveWSmall > 0 && kWaveWSmall <= 64 && 64 % kWaveWSmall == 0, "kWaveWSmall");
template <bool TREE>
__host__ __device__ constexpr int wave_w() { return TREE ? kWaveW : kWaveWSmall; }
template <bool TREE>
__host__ __device__ constexpr int waves_x() { return TREE ? kWavesXTree : kWavesX; }
template <bool TREE>
__host__ __device__ constexpr int fast_waves() { return TREE ? kFastWaves : kFastWavesSmall; }
template <bool TREE>
__host__ __device__ constexpr int fast_block() { return 64 * fast_waves<TREE>(); }
static_assert(kFastWavesSmall % kWavesX == 0 && kFastWaves % kWavesXTree == 0, "block wave layout");
constexpr int kFrameWords = 20;  // general-kernel stack frame (float64 words)
constexpr int kFetchStride = 32;  // uint32 words between counters
constexpr int kSphWords = RTX_GEOM_WORDS + RTX_MAT_WORDS;
constexpr int kLdsMaxSpheres = 128;  // scene table staged in LDS up to this size (32 KiB)
// The colour inputs of the non-terminal levels (4 doubles + the key per level and lane) go to LDS
// slots indexed by the level instead of a register shift register (no moves per level, 27 fewer
// live VGPRs): [B][4][kFastBlock] doubles + [B][kFastBlock] ints after the scene table.
template <int B, bool LDS, bool DEEP>
constexpr bool levels_in_lds() { return kLevelsInLds && LDS && !DEEP && !kForwardFold && B > 0 && B <= kLevelsLdsMaxB; }
// the DEEP variant (3 waves/SIMD: 3 blocks per CU) keeps all its levels in LDS
template <bool DEEP = false>
__host__ __device__ constexpr int level_lds_slots(int B) {
  return DEEP || B < kLevelsLdsSlots ? B : B >= 5 ? kB5Slots : kLevelsLdsSlots;
}
template <bool DEEP = false, bool TREE = true>
__host__ __device__ constexpr size_t level_lds_bytes(int B) {
  return (size_t)level_lds_slots<DEEP>(B) * fast_block<TREE>() * (4 * 8 + 4);
}
// The one-tile culled kernels (TP 1, capped: the forward fold) accumulate the pixel colour in LDS
// after the scene table ([3][block] doubles, each lane its own slots) instead of three VGPR pairs:
// at 96 VGPRs (5 waves/SIMD) one of them spilled to scratch on every level (C3 traffic 1.5x).
constexpr size_t kColourLdsBytes = 3 * sizeof(double) * 256;
// the general kernel's nearest pass walks the culling tree from this many spheres on (A/B: 65
// spheres -11%, 17 spheres +2..6%: its depth-first lanes diverge, so a wave-uniform walk pays less)
constexpr int kGeneralTreeMin = 32;
// scenes of fewer spheres never carry a culling tree (scene_pack.BVH_MIN_SPHERES): the fast kernel's
// TREE = false instantiations serve them
constexpr int kTreeMinSpheres = 8;
constexpr size_t kLdsBytesPerCu = 160 * 1024;  // gfx950

// Wave-uniform loads through the scalar cache: the constant address space makes hipcc emit s_load
// even though the kernel also stores (it cannot prove the scene blob is not aliased otherwise).
typedef const double __attribute__((address_space(4))) cdouble;

struct Params {
  const double* scene;
  int nsph;
  int mode;  // 0: camera rays, 1: explicit rays, 2: continuation of deferred chains (in_list),
             // 3: explicit rays whose level-0 hit is given (hit_shape at hit_t: Shader.create)
  // camera mode: local rows of parts part .. part + part_run - 1 of the n_parts-way row interleave
  int width, height, row_block, n_parts, part, n_rows;
  int part_run = 1;
  // explicit-ray mode
  const double* org;
  int64_t org_stride;
  const double* dir;
  const double* hit_t;  // mode 3: level-0 distance per ray
  int hit_shape;        // mode 3: the shape every ray hit
  // common
  int64_t n;  // rays in this launch (= width * n_rows in camera mode)
  int max_bounces;
  void* out;
  int out_kind;
  uint8_t* ws;
  int64_t list_cap;  // capacity of each deferred list
  // Deferred lists (workspace). A launch appends to dlist (counter dcount); a chain deferred for
  // depth after level drec_level also gets a resume record (slot < rec_cap) in drec. The
  // continuation pass (mode 2) and the general kernel read in_list (counter in_count), whose deep
  // entries of level in_level resume from in_rec.
  uint64_t* dlist;
  uint32_t* dcount;
  double* drec;
  int drec_level;
  const uint64_t* in_list;
  const uint32_t* in_count;
  const double* in_rec;
  int in_level;
  int64_t rec_cap;     // records drec holds
  int64_t in_rec_cap;  // records in_rec holds
  double* stack;
  int64_t n_workers;
  int stack_levels;
  unsigned long long* stats;
  int n_tiles_x, n_tiles_y;  // persistent launch of k_render_fast (wave tiles; 0: one block tile per block)
  // persistent waves (n_fetch > 0): wave tiles (kWaveW x kWaveH) handed out by n_fetch counters
  uint32_t* fetch;
  int n_fetch;
  // multi-frame launch (rtx_render_frames): frame f reads scene + f * scene_stride and writes
  // out + f * (one frame's output); n counts the pixels of ONE frame
  int64_t scene_stride;
  int n_frames;
  int frame;  // set per block / per deferred ray (kernel side)
  uint32_t* deferred_out;  // the launch's deferred-ray count (rtx_render_camera_ex), or null
  int no_general;  // RTX_F_NO_GENERAL: no general kernel follows, so nothing may be deferred
  int images;      // RTX_F_IMAGES: the capped LDS kernels shade image-textured spheres themselves
  // camera launches of one frame (rtx_render_camera_sched): the dispatch units (the persistent
  // launch's wave tiles, else the grid's block tiles) in dispatch order (null: bottom-up row order),
  // and per-unit render times to record (s_memrealtime ticks), or null
  const uint32_t* tile_order;
  uint32_t* tile_cost;
  int reserve;  // RTX_F_RESERVE: block slots the persistent launch leaves free (host side only)
};

// Deferred-list entry (uint64): pixel | frame << 40 | (rays counted through level a) + 1 << 56 |
// (hits counted through level b) + 1 << 60. The general kernel re-renders the pixel from level 0
// and skips the per-level counts the fast kernel already made (a, b = -1: none).
constexpr int kFrameShift = 34;
constexpr int kRaysShift = 50;
constexpr int kHitsShift = 57;
constexpr int kLevelMask = 0x7F;  // 7-bit level fields (level + 1)
// Resume record of a pixel deferred for depth at level L = kDeepLevels: the next level's ray
// (origin, direction) and the colour inputs (dli, di, spec, va, key) of levels 0..L; the general
// kernel continues the chain at level L + 1 instead of re-rendering it from level 0.
constexpr int kRecLevelWords = 5;
// With the forward fold (kForwardFold) the DEEP kernels' record is the next ray, the colour
// accumulated through level L and the throughput of level L + 1: 10 words whatever L.
__host__ __device__ constexpr int rec_words(int level) {
  return kForwardFold ? 10 : 6 + kRecLevelWords * (level + 1);
}
// the first DEEP pass's record level (forward fold: a runtime level, no storage per level; A/B r5zo
// on unbounded renders end to end, 5 / 9 / 14 levels: C2 98.7 / 93.7 / 77.8 us, C3 378 / 367 / 326 us,
// C4 2,514 / 2,485 / 2,440 us; r5zp, 14 / 16 / 30 with the continuation pass to 60: C2 77.8 / 77.5 /
// 77.4, C3 327 / 310 / 304, C4 2,437 / 2,380 / 2,166 us)
constexpr int kFirstPassLevels = 30;
constexpr int kDeepLevel2 = 2 * kDeepLevels + 1;  // deferral level of the first continuation pass
constexpr int kDeepLevel3 = kForwardFold ? 60 : 3 * kDeepLevels + 2;  // ... and of the second (forward: the one)
static_assert(!kForwardFold || (kFirstPassLevels >= kDeepLevels && kFirstPassLevels < kDeepLevel3),
              "first-pass record level");
static_assert(kDeepLevel3 + 2 < kLevelMask, "deferred-entry level fields hold 7 bits");
// Resume-record capacities per deferral level (pass 0: the first pass's level kDeepLevels;
// 1, 2: the continuation passes'): at least 2^18 / 2^16 / 2^14, or one per 32 / 256 / 2048 pixels,
// whichever is more. Chains alive at level 5 are 0.2-1.4% of the pixels in the bench scenes (C4:
// 467,657 of 33.2 M), far fewer at 11 and 17. An entry beyond the capacity is re-rendered from
// level 0 by the general kernel: correct, but slow.
__host__ __device__ constexpr int64_t records_cap(int64_t n, int pass) {
  const int64_t lo = int64_t(1) << (18 - 2 * pass);
  const int64_t by_n = n / (int64_t(32) << (3 * pass));
  const int64_t want = by_n > lo ? by_n : lo;
  return n < want ? n : want;
}

// append one entry to the launch's deferred list; returns its slot (or -1 when the list is full).
// Under RTX_F_NO_GENERAL no general kernel follows: the entry is dropped and RTX_ST_UNRENDERED raised
// (the pixel stays unwritten, the list and its counter stay clean for the next call).
__device__ __forceinline__ int64_t append_deferred(const Params& p, uint64_t entry) {
  if (p.no_general) {
    atomicOr((uint32_t*)p.ws + RTX_WS_STATUS, (uint32_t)RTX_ST_UNRENDERED);
    return -1;
  }
  const uint32_t slot = atomicAdd(p.dcount, 1u);
  if ((int64_t)slot < p.list_cap) {
    p.dlist[slot] = entry;
    return slot;
  }
  atomicOr((uint32_t*)p.ws + RTX_WS_STATUS, (uint32_t)RTX_ST_LIST_OVERFLOW);
  return -1;
}
__device__ __forceinline__ uint64_t deferred_entry(int64_t i, int frame, int rays_through, int hits_through) {
  return (uint64_t)i | ((uint64_t)frame << kFrameShift) | ((uint64_t)(rays_through + 1) << kRaysShift) |
         ((uint64_t)(hits_through + 1) << kHitsShift);
}

__device__ __forceinline__ int64_t out_bytes_per_pixel(int kind) {
  return kind == RTX_OUT_F32_SOA ? 12 : kind == RTX_OUT_F64_SOA ? 24 : 3;
}

// Parameters of frame f of a multi-frame launch (the identity for f == 0).
__device__ __forceinline__ Params frame_view(const Params& p, int f) {
  Params q = p;
  q.scene = p.scene + (int64_t)f * p.scene_stride;
  q.out = (uint8_t*)p.out + (int64_t)f * p.n * out_bytes_per_pixel(p.out_kind);
  q.frame = f;
  return q;
}

// ------------------------------------------------------------------------------------------
// arithmetic helpers (reference semantics)
// ------------------------------------------------------------------------------------------

__device__ __forceinline__ double dot3(double ax, double ay, double az, double bx, double by, double bz) {
  return ((ax * bx) + (ay * by)) + (az * bz);  // NumpyVector3D.dot, base.py:34-35
}

// Correctly rounded sqrt and division, fast paths. LLVM lowers f64 sqrt / fdiv for gfx9 to a
// correctly rounded sequence (v_rsq_f64 / v_rcp_f64 + Newton-Raphson FMAs) wrapped in operand
// scaling (v_ldexp, v_div_scale) and special-value fix-ups (v_cmp_class, v_div_fixup). For operands
// where the scaling is provably the identity and no special value occurs, the cores below are the
// very same instruction sequence without the wrapping, hence bit-identical; every other operand
// takes the full expansion. (k_selftest_math checks both paths bit for bit on the device.)
__device__ __forceinline__ double sqrt_core(double x) {  // x in [2^-767, DBL_MAX]
  const double y = __builtin_amdgcn_rsq(x);
  double g = x * y;
  double h = y * 0.5;
  const double r = __builtin_fma(-h, g, 0.5);
  g = __builtin_fma(g, r, g);
  h = __builtin_fma(h, r, h);
  double d = __builtin_fma(-g, g, x);
  g = __builtin_fma(d, h, g);
  d = __builtin_fma(-g, g, x);
  return __builtin_fma(d, h, g);
}
__device__ __forceinline__ double sqrt_cr(double x) {
  // wave-uniform choice (one ballot): the fast core unless some active lane is out of range
  if (__ballot(!(x >= 0x1.0p-767 && x <= 0x1.fffffffffffffp+1023)) == 0) return sqrt_core(x);
  return __builtin_sqrt(x);
}
// a / b for a, b with |.| in [2^-300, 2^300] (v_div_scale leaves them unchanged and clears VCC, so
// v_div_fmas is a plain fma; the quotient is normal, so v_div_fixup returns it unchanged)
__device__ __forceinline__ double div_core(double a, double b) {
  double r = __builtin_amdgcn_rcp(b);
  double e = __builtin_fma(-b, r, 1.0);
  r = __builtin_fma(r, e, r);
  e = __builtin_fma(-b, r, 1.0);
  r = __builtin_fma(r, e, r);
  const double q = a * r;
  const double rem = __builtin_fma(-b, q, a);
  return __builtin_fma(rem, r, q);
}
__device__ __forceinline__ bool div_range(double x) {
  const double ax = fabs(x);
  return ax >= 0x1.0p-300 && ax <= 0x1.0p+300;
}
__device__ __forceinline__ double div_cr(double a, double b) {
  if (__ballot(!(div_range(b) && (a == 0.0 || div_range(a)))) == 0)  // wave-uniform choice
    return a == 0.0 ? a * __builtin_copysign(1.0, b) : div_core(a, b);
  return a / b;
}

// 1.0 / where(mag == 0, 1, mag) with mag = sqrt(d), d = |v|^2 (NumpyVector3D.norm, base.py:61-64).
// d in [2^-600, 2^600] puts sqrt's operand and the quotient's divisor (mag in [2^-300, 2^300],
// non-zero) in both cores' exact ranges: one wave-uniform check instead of three.
__device__ __forceinline__ double inv_mag(double d) {
  if (__ballot(!(d >= 0x1.0p-600 && d <= 0x1.0p+600)) == 0) return div_core(1.0, sqrt_core(d));
  const double mag = sqrt_cr(d);
  return div_cr(1.0, mag == 0.0 ? 1.0 : mag);
}

__device__ __forceinline__ void norm3(double& x, double& y, double& z) {
  // NumpyVector3D.norm, base.py:61-64: v * (1.0 / where(mag == 0, 1, mag))
  const double r = inv_mag(dot3(x, y, z, x, y, z));
  x = x * r;
  y = y * r;
  z = z * r;
}

// 1.0 / where(mag == 0, 1, mag), mag = sqrt(d), for d = |v|^2 within 2^-30 of 1: the norm of a
// vector that is already unit up to rounding (a direction normalised before, or the reflection of
// one). Write d = 1 + j 2^-53 (j an integer, even when positive). The correctly rounded sqrt(d) is
// 1 + floor(j/4) 2^-52 for j >= 0 and 1 - ceil(-j/2) 2^-53 for j < 0, and the correctly rounded
// reciprocal of either is 1 - floor(j/4) 2^-52: the second-order terms stay far below half an ulp
// for |j| <= 2^23. (d - 1) * 2^51 = j/4 exactly, floor is exact and so is the fma, so the result is
// bit-identical to div(1, sqrt(d)) (tests/test_unit_norm.py checks every such d against IEEE sqrt
// and division; k_selftest_math checks this path on the device).
__device__ __forceinline__ double inv_mag_near1(double d) {
  return __builtin_fma(-__builtin_floor((d - 1.0) * 0x1.0p51), 0x1.0p-52, 1.0);
}
__device__ __forceinline__ double inv_mag_unit(double d) {
  // wave-uniform: the closed form unless some active lane is out of its range
  if (__ballot(!(fabs(d - 1.0) <= 0x1.0p-30)) == 0) return inv_mag_near1(d);
  return inv_mag(d);
}
__device__ __forceinline__ void norm3_unit(double& x, double& y, double& z) {
  // NumpyVector3D.norm (base.py:61-64) of a vector expected to be unit up to rounding
  const double r = inv_mag_unit(dot3(x, y, z, x, y, z));
  x = x * r;
  y = y * r;
  z = z * r;
}

// np.clip(x, 0, 1) and np.maximum(x, 0) as v_max_f64 / v_min_f64. They differ from the reference
// only for NaN inputs and in the sign of a zero result, which never reaches the output: every such
// value is squared, scaled into a sum with the 0.004 ambient term, or compared with <= 0.
__device__ __forceinline__ double clip01(double x) { return __builtin_fmin(__builtin_fmax(x, 0.0), 1.0); }

__device__ __forceinline__ double max0(double x) { return __builtin_fmax(x, 0.0); }

__device__ __forceinline__ int trunc_parity(double x) {
  // (x).astype(int) % 2 (shader.py:30): truncation to int64, then floor-mod 2 == (k & 1).
  // |x| >= 2^53 doubles are even integers; NaN / |x| >= 2^63 convert to INT64_MIN (even).
  const double k = trunc(x);
  const double h = k * 0.5;
  return (x == x) && (h != trunc(h));
}

// b > 0 and c >= 0 (the sphere lies behind an origin outside it): the reference's root is never
// positive, so the test is FARAWAY without a square root. Proof: disc = fl(fl(b*b) - 4c) <= fl(b*b),
// and for b with b*b a normal double (1e-150 <= b <= 1e150) the correctly rounded sqrt(fl(b*b)) is b
// itself (b*b*(1 + 2^-53) has a root below b + ulp(b)/2), so sq <= b and s1 = (-b + sq) / 2 <= 0.
// Below 1e-150, b*b may round up by far more than an ulp in the subnormal range (b = 1.6e-162, c = 0:
// the reference reports a hit at 3.1e-163, tests/golden/intersect_kat.json), so those take the root.
__device__ __forceinline__ bool behind(double b, double c) {
  return b >= 1e-150 && c >= 0.0 && b <= 1e150;
}

// NumpySphere.intersect, shape.py:28-51, for a ray with precomputed oo = O.O.
// b = 2 * D.(O - C);  c = ((C.C + O.O) - 2 * C.O) - r*r;  disc = b^2 - 4c.
template <typename P>
__device__ __forceinline__ double isect(const P* g, double ox, double oy, double oz, double oo, double dx, double dy,
                                        double dz) {
  const double cx = g[RTX_G_CX], cy = g[RTX_G_CY], cz = g[RTX_G_CZ];
  const double b = 2.0 * dot3(dx, dy, dz, ox - cx, oy - cy, oz - cz);
  const double c = ((g[RTX_G_CC] + oo) - 2.0 * dot3(cx, cy, cz, ox, oy, oz)) - g[RTX_G_RR];
  const double disc = (b * b) - (4.0 * c);
  double t = FARAWAY;
  if (disc > 0.0 && !behind(b, c)) {  // np.where((disc > 0) & (sol > 0), sol, FARAWAY); sqrt(max(0, disc)) == sqrt(disc) here
    const double sq = sqrt_cr(disc);
    const double s0 = (-b - sq) * 0.5;  // == / 2 exactly
    const double s1 = (-b + sq) * 0.5;
    // (s0 > 0) & (s0 < s1) ? s0 : s1 — with sq > 0, s0 <= s1 and s0 == s1 only as equal values
    const double sol = s0 > 0.0 ? s0 : s1;
    if (sol > 0.0) t = sol;
  }
  return t;
}

// The same test split in two halves so that two spheres' dependency chains interleave (and their
// scalar loads share one wait): isect_disc computes the quadratic's coefficients, isect_sol the rest.
//
// Half-b form. With h = D.(O - C) the reference's b is 2h exactly, b*b = 4 fl(h*h), 4c is exact,
// disc = 4 fl(fl(h*h) - c) = 4q, sqrt(disc) = 2 sqrt(q) and its roots (-b -+ sqrt(disc)) / 2 are
// fl(-h -+ sqrt(q)): bit for bit the same numbers, four multiplications and the range checks
// fewer. Each step is an exact scaling by a power of two as long as nothing leaves the normal
// range: h*h must be normal and not overflow, 4c must not overflow. The host marks a scene "tame"
// (RTX_H_TAME) when every coordinate and radius is below 2^60, so that |O|, |O - C| stay below
// ~2^140 for every origin a hit can produce (t < FARAWAY ~ 2^130) and |h| < 2^141, |c| < 2^284;
// the lower end is checked per wave: |h| >= 2^-350 in every active lane. Then q is 0 or at least
// 2^-753 in magnitude (h*h >= 2^-700; a nonzero q = fl(h*h) - c is either above half of h*h or an
// exact Sterbenz difference, a multiple of ulp(h*h)/2), so q is inside sqrt_core's exact range,
// and -h -+ sqrt(q) is 0 or normal. Explicit-ray launches and untamed scenes, and any wave with a
// lane at |h| < 2^-350 (a ray at right angles to O - C, such as tests/golden/intersect_kat.json's
// b = 1.6e-162 case), evaluate the reference expressions instead.
struct SphTest {
  double h, d;  // h = D.(O - C); d: q (half) or the reference's disc = (2h)^2 - 4c
  bool skip;    // no hit in this lane: d <= 0, or the sphere lies behind the origin
  int half;     // wave-uniform (an int: a uniform bool carried across blocks costs VALU copies)
};
// h > 0 and c >= 0 (|h| >= 2^-350): q <= fl(h*h) and sqrt(fl(h*h)) == h, so -h + sqrt(q) <= 0
// tame: the lower bound 2^-350 in a tame launch, NaN otherwise (no |h| passes; a double threshold
// keeps the uniform flag out of lane-mask copies)
__device__ __forceinline__ SphTest sph_test(double h, double c, double tame) {
  SphTest t;
  t.half = __ballot(!(fabs(h) >= tame)) == 0 ? 1 : 0;
  t.h = h;
  if (t.half) {
    t.d = (h * h) - c;
    t.skip = !(t.d > 0.0) || (h > 0.0 && c >= 0.0);
  } else {
    const double b = 2.0 * h;  // b = 2.0 * D.(O - C), shape.py:33-37
    t.d = (b * b) - (4.0 * c);
    t.skip = !(t.d > 0.0) || behind(b, c);
  }
  return t;
}
template <typename P>
__device__ __forceinline__ SphTest isect_disc(const P* g, double ox, double oy, double oz, double oo, double dx,
                                              double dy, double dz, double tame) {
  const double cx = g[RTX_G_CX], cy = g[RTX_G_CY], cz = g[RTX_G_CZ];
  const double h = dot3(dx, dy, dz, ox - cx, oy - cy, oz - cz);
  const double c = ((g[RTX_G_CC] + oo) - 2.0 * dot3(cx, cy, cz, ox, oy, oz)) - g[RTX_G_RR];
  return sph_test(h, c, tame);
}
// level-0 camera origin: O - C from uniform values, c precomputed on the host (same expressions)
template <typename P>
__device__ __forceinline__ SphTest isect_disc_cam(const P* g, double ox, double oy, double oz, double dx, double dy,
                                                  double dz, double tame) {
  const double h = dot3(dx, dy, dz, ox - g[RTX_G_CX], oy - g[RTX_G_CY], oz - g[RTX_G_CZ]);
  return sph_test(h, g[RTX_G_C0], tame);
}
// The rest of the test, as a root and a validity flag instead of the FARAWAY sentinel (no f64
// selects of a non-inline constant): valid <=> the reference returns the root, not FARAWAY. With
// s0 <= s1 (rounding is monotone), (s0 > 0 ? s0 : s1) > 0 <=> s1 > 0. Lanes without a root take
// the square root of |disc|, a discarded dummy.
__device__ __forceinline__ double isect_sol(const SphTest& t, bool& valid) {
  if (t.half) {
    // s1 = fl(-h + sq) > 0 <=> sq > h and s0 > 0 <=> -h > sq (a sum of two doubles rounds to 0 only
    // when it is 0); the root is -h + (s0 > 0 ? -sq : sq), -sq by flipping the high word's sign.
    // (skip covers q <= 0; its other half, behind, implies s1 <= 0, so valid needs no q > 0 test.)
    const double sq = sqrt_core(fabs(t.d));
    valid = !t.skip && sq > t.h;
    const uint32_t hi = __double2hiint(sq), lo = __double2loint(sq);
    const uint32_t shi = (-t.h > sq) ? (hi ^ 0x80000000u) : hi;
    return -t.h + __hiloint2double(shi, lo);
  }
  const double b = 2.0 * t.h;
  const double sq = sqrt_cr(fabs(t.d));
  const double s0 = (-b - sq) * 0.5;  // == / 2 exactly
  const double s1 = (-b + sq) * 0.5;
  valid = !t.skip && s1 > 0.0;  // behind (in skip) implies s1 <= 0
  return s0 > 0.0 ? s0 : s1;
}
// One sphere / two spheres at once: the square roots run only if some lane may hit, and the
// consumer f(t, valid[, t1, valid1]) runs inside that branch, so an invalid root is never carried
// out of it (a placeholder root would cost a move per test; an uninitialised one would be
// undefined behaviour, which the compiler exploits by deleting the skip test). Lanes outside the
// branch have no valid root for either sphere.
template <typename F>
__device__ __forceinline__ void isect_one(const SphTest& a, F&& f) {
  if (!a.skip) {
    bool v;
    const double t = isect_sol(a, v);
    f(t, v);
  }
}
template <typename F>
__device__ __forceinline__ void isect_pair(const SphTest& a, const SphTest& b, F&& f) {
  if (!a.skip || !b.skip) {
    bool v0, v1;
    const double t0 = isect_sol(a, v0);
    const double t1 = isect_sol(b, v1);
    f(t0, v0, t1, v1);
  }
}
// isect (the reference's root or FARAWAY) through the split test
template <typename P>
__device__ __forceinline__ double isect_t(const P* g, double ox, double oy, double oz, double oo, double dx, double dy,
                                          double dz, double tame) {
  double r = FARAWAY;
  isect_one(isect_disc(g, ox, oy, oz, oo, dx, dy, dz, tame), [&](double t, bool v) {
    if (v) r = t;
  });
  return r;
}

// nearest-hit bookkeeping in scene order (base.py:97-103): the first strictly smaller t wins; an
// equal t marks a tie, which is cleared by any later strictly smaller t. tmin starts at FARAWAY and
// only decreases, so an invalid test (FARAWAY) never updates it. A valid root equal to FARAWAY
// itself would flag a tie here: the pixel then goes to the general kernel, which is exact.
__device__ __forceinline__ void nearest_update(bool valid, double t, int s, double& tmin, int& hit, bool& tie) {
  if (valid && t < tmin) {
    tmin = t;
    hit = s;
    tie = false;
  } else if (valid && t == tmin) {
    tie = true;
  }
}

// Executed-work counters of the stats launch (bench.py's executed-FLOP model): ray-sphere tests
// and culling-node tests performed by each live lane. Work<false> (the timed kernels) compiles to
// nothing.
template <bool ON>
struct Work {
  __device__ __forceinline__ void test(int) {}
  __device__ __forceinline__ void node() {}
  __device__ __forceinline__ void box() {}
  __device__ __forceinline__ void beam() {}
};
template <>
struct Work<true> {
  uint32_t tests = 0, nodes = 0;
  uint32_t tests1 = 0, nodes1 = 0;  // of the nearest-hit searches of reflected rays (levels >= 1)
  uint32_t boxes = 0;  // of the node tests, the culling tree's box tests (the rest: frustum planes and
                       // shadow-grid lookups, priced as node tests)
  uint32_t beamt = 0;  // reflected-ray beam tests: one per live lane and beam pass (RTX_S_BEAMT)
  __device__ __forceinline__ void test(int k) { tests += (uint32_t)k; }
  __device__ __forceinline__ void node() { ++nodes; }
  __device__ __forceinline__ void box() { ++boxes; }
  __device__ __forceinline__ void beam() { ++beamt; }
};

// Shadow any-hit: does test j (root t, validity v) come strictly before the shape's own distance
// t_self? An invalid test is FARAWAY, which is before t_self only when t_self > FARAWAY (far_self).
__device__ __forceinline__ bool shadows(bool valid, double t, double tself, bool far_self) {
  return valid ? t < tself : far_self;
}

// ---- culling hierarchy ---------------------------------------------------------------------
// Conservative test: may any sphere inside a node's box produce, through the reference formula
// (shape.py:34-51), a hit with 0 < t <= tlim? If this returns false, every such sphere provably
// yields FARAWAY (or a t > tlim), so skipping it changes neither the nearest hit nor the tie test
// nor the shadow test.
// Error budget: the reference's discriminant carries an absolute error err <= ~64 eps * scale,
// scale = |Cn-O|^2 + (|Cn|+R)^2 + |O|^2 + R^2 for a sphere inside the bounding sphere (Cn, R) of
// the box (cancellation in c = |C|^2 + |O|^2 - 2 C.O - r^2). A root it reports is therefore within
// sqrt(err) <= lm = 1e-7 (scale + 1) of a point of the sphere's ball, i.e. of the box expanded by
// lm. With |Cn-O|^2 <= 2 (|Cn|+R)^2 + 2 |O|^2, lm <= 1e-7 (3 (|Cn|+R)^2 + R^2 + 1) + 3e-7 |O|^2; the
// box is expanded by twice that (N_MARGIN + 6e-7 |O|^2), which also absorbs the slab arithmetic's
// own rounding (~1e-15 relative) and |D| = 1 +- 1e-15.
struct RaySlab {
  double ix, iy, iz;  // 1 / direction component, components below 1e-200 in magnitude nudged to it
  double mo;          // 6e-7 |O|^2
};
__device__ __forceinline__ double slab_inv(double d) {
  // the reciprocal only places slab boundaries: rcp + one Newton step (~1e-16 relative) suffices;
  // the nudge keeps 0 * inf out of the slab products (a shift of 1e-200 * t is far below lm)
  const double dd = fabs(d) < 1e-200 ? __builtin_copysign(1e-200, d) : d;
  const double r = __builtin_amdgcn_rcp(dd);
  return __builtin_fma(r, __builtin_fma(-dd, r, 1.0), r);
}
__device__ __forceinline__ RaySlab ray_slab(double dx, double dy, double dz, double oo) {
  return RaySlab{slab_inv(dx), slab_inv(dy), slab_inv(dz), 6e-7 * oo};
}
__device__ __forceinline__ bool node_may_hit(const cdouble* nd, double ox, double oy, double oz, const RaySlab& r,
                                             double tlim) {
  const double m = nd[RTX_N_MARGIN] + r.mo;
  const double ax = ((nd[RTX_N_LOX] - m) - ox) * r.ix, bx = ((nd[RTX_N_HIX] + m) - ox) * r.ix;
  const double ay = ((nd[RTX_N_LOY] - m) - oy) * r.iy, by = ((nd[RTX_N_HIY] + m) - oy) * r.iy;
  const double az = ((nd[RTX_N_LOZ] - m) - oz) * r.iz, bz = ((nd[RTX_N_HIZ] + m) - oz) * r.iz;
  // a NaN slab (non-finite origin) is dropped by fmin/fmax: unconstrained, hence conservative
  const double tn = __builtin_fmax(__builtin_fmax(__builtin_fmin(ax, bx), __builtin_fmin(ay, by)), __builtin_fmin(az, bz));
  const double tf = __builtin_fmin(__builtin_fmin(__builtin_fmax(ax, bx), __builtin_fmax(ay, by)), __builtin_fmax(az, bz));
  return tn <= tf && tf >= 0.0 && tn <= tlim;
}

// Nearest hit over entries [first, first + cnt) of the culled geometry list (pairs, scalar loads).
template <bool CAM, typename Wk>
__device__ __forceinline__ void nearest_range(const cdouble* cg, int first, int cnt, double ox, double oy, double oz,
                                              double oo, double dx, double dy, double dz, double& tmin, int& hit,
                                              bool& tie, double tame, Wk& wk) {
  wk.test(cnt);
  const int end = first + cnt;
  int k = first;
  for (; k + 1 < end; k += 2) {
    const cdouble* g0 = cg + __builtin_amdgcn_readfirstlane(k) * RTX_GEOM_WORDS;
    const cdouble* g1 = g0 + RTX_GEOM_WORDS;
    const SphTest a0 = CAM ? isect_disc_cam(g0, ox, oy, oz, dx, dy, dz, tame)
                           : isect_disc(g0, ox, oy, oz, oo, dx, dy, dz, tame);
    const SphTest a1 = CAM ? isect_disc_cam(g1, ox, oy, oz, dx, dy, dz, tame)
                           : isect_disc(g1, ox, oy, oz, oo, dx, dy, dz, tame);
    const int s0 = (int)g0[RTX_G_IDX], s1 = (int)g1[RTX_G_IDX];
    isect_pair(a0, a1, [&](double t0, bool v0, double t1, bool v1) {
      nearest_update(v0, t0, s0, tmin, hit, tie);
      nearest_update(v1, t1, s1, tmin, hit, tie);
    });
  }
  if (k < end) {
    const cdouble* g0 = cg + __builtin_amdgcn_readfirstlane(k) * RTX_GEOM_WORDS;
    const SphTest a0 = CAM ? isect_disc_cam(g0, ox, oy, oz, dx, dy, dz, tame)
                           : isect_disc(g0, ox, oy, oz, oo, dx, dy, dz, tame);
    const int s0 = (int)g0[RTX_G_IDX];
    isect_one(a0, [&](double t0, bool v0) { nearest_update(v0, t0, s0, tmin, hit, tie); });
  }
}

// Nearest hit through the culling tree: the always-tested spheres, then a stackless depth-first
// walk that enters a node when any lane of the wave may hit it before its current nearest t.
// Evaluation order differs from scene order, which the result does not depend on: the nearest t
// is a minimum, `hit` is its unique owner unless tied, and a tie is flagged whatever the order.
template <bool CAM, typename Wk>
__device__ __forceinline__ void nearest_bvh(const cdouble* sc, double ox, double oy, double oz, double dx, double dy,
                                            double dz, double& tmin, int& hit, bool& tie, double tame, Wk& wk) {
  const cdouble* cg = sc + (int)sc[RTX_H_CGEO];
  const cdouble* nodes = sc + (int)sc[RTX_H_NODES];
  const int nn = (int)sc[RTX_H_NNODES];
  const double oo = dot3(ox, oy, oz, ox, oy, oz);
  tmin = FARAWAY;
  hit = -1;
  tie = false;
  nearest_range<CAM>(cg, 0, (int)sc[RTX_H_NALWAYS], ox, oy, oz, oo, dx, dy, dz, tmin, hit, tie, tame, wk);
  const RaySlab rs = ray_slab(dx, dy, dz, oo);
  int i = 0;
  while (i < nn) {
    const cdouble* nd = nodes + __builtin_amdgcn_readfirstlane(i) * RTX_NODE_WORDS;
    wk.node();
    wk.box();
    if (__ballot(node_may_hit(nd, ox, oy, oz, rs, tmin)) != 0) {
      const int cnt = (int)nd[RTX_N_COUNT];
      if (cnt > 0)
        nearest_range<CAM>(cg, (int)nd[RTX_N_FIRST], cnt, ox, oy, oz, oo, dx, dy, dz, tmin, hit, tie, tame, wk);
      ++i;
    } else {
      i = (int)nd[RTX_N_SKIP];
    }
  }
}

// The general kernel's nearest pass through the culling tree: the nearest distance, how many
// shapes share it and the first of them in scene order (base.py:97-103). Traversal order does not
// matter: the minimum is order-free, equal distances are all counted, and the smallest scene index
// among them is kept. A sphere at exactly the current nearest distance is never culled (its box is
// reached at t <= tlim).
__device__ __forceinline__ void count_update(bool valid, double t, int s, double& tmin, int& nh, int& first) {
  if (valid && t < tmin) {
    tmin = t;
    nh = 1;
    first = s;
  } else if (valid && t == tmin) {
    ++nh;
    first = s < first ? s : first;
  }
}
__device__ __forceinline__ void nearest_count_bvh(const cdouble* sc, double ox, double oy, double oz, double oo,
                                                  double dx, double dy, double dz, double& tmin, int& nh,
                                                  int& first) {
  const cdouble* cg = sc + (int)sc[RTX_H_CGEO];
  const cdouble* nodes = sc + (int)sc[RTX_H_NODES];
  const int nn = (int)sc[RTX_H_NNODES];
  auto range = [&](int k, int end) {
    for (; k < end; ++k) {
      const cdouble* g0 = cg + __builtin_amdgcn_readfirstlane(k) * RTX_GEOM_WORDS;
      const int s0 = (int)g0[RTX_G_IDX];
      isect_one(isect_disc(g0, ox, oy, oz, oo, dx, dy, dz, __builtin_nan("")),
                [&](double t0, bool v0) { count_update(v0, t0, s0, tmin, nh, first); });
    }
  };
  range(0, (int)sc[RTX_H_NALWAYS]);
  const RaySlab rs = ray_slab(dx, dy, dz, oo);
  int i = 0;
  while (i < nn) {
    const cdouble* nd = nodes + __builtin_amdgcn_readfirstlane(i) * RTX_NODE_WORDS;
    if (__ballot(node_may_hit(nd, ox, oy, oz, rs, tmin)) != 0) {
      const int cnt = (int)nd[RTX_N_COUNT];
      if (cnt > 0) range((int)nd[RTX_N_FIRST], (int)nd[RTX_N_FIRST] + cnt);
      ++i;
    } else {
      i = (int)nd[RTX_N_SKIP];
    }
  }
}

// Shadow any-hit through the culling tree (shader.py:126-128 in its any-hit form): lit stays true
// unless some sphere is strictly nearer than the shape itself along the light direction. hs: the
// wave-uniform shape of every lane (nsph when the lanes differ), whose own test cannot shadow it.
// Callers guarantee t_self <= FARAWAY in every lane (an invalid test then never shadows).
template <typename Wk>
__device__ __forceinline__ bool lit_bvh(const cdouble* sc, double qx, double qy, double qz, double qq, double lx,
                                        double ly, double lz, double tself, int hs, double tame, Wk& wk) {
  const cdouble* cg = sc + (int)sc[RTX_H_CGEO];
  const cdouble* nodes = sc + (int)sc[RTX_H_NODES];
  const int nn = (int)sc[RTX_H_NNODES];
  const int nal = (int)sc[RTX_H_NALWAYS];
  bool lit = true;
  for (int k = 0; k < nal; ++k) {
    const cdouble* g0 = cg + __builtin_amdgcn_readfirstlane(k) * RTX_GEOM_WORDS;
    if ((int)g0[RTX_G_IDX] == hs) continue;
    wk.test(1);
    isect_one(isect_disc(g0, qx, qy, qz, qq, lx, ly, lz, tame), [&](double t0, bool v0) {
      if (v0 && t0 < tself) lit = false;
    });
  }
  const RaySlab rs = ray_slab(lx, ly, lz, qq);
  int i = 0;
  while (i < nn) {
    const cdouble* nd = nodes + __builtin_amdgcn_readfirstlane(i) * RTX_NODE_WORDS;
    wk.node();
    wk.box();
    if (__ballot(lit && node_may_hit(nd, qx, qy, qz, rs, tself)) != 0) {
      const int cnt = (int)nd[RTX_N_COUNT];
      if (cnt > 0) {
        wk.test(cnt);
        const int first = (int)nd[RTX_N_FIRST], end = first + cnt;
        int k = first;
        for (; k + 1 < end; k += 2) {
          const cdouble* g0 = cg + __builtin_amdgcn_readfirstlane(k) * RTX_GEOM_WORDS;
          const cdouble* g1 = g0 + RTX_GEOM_WORDS;
          isect_pair(isect_disc(g0, qx, qy, qz, qq, lx, ly, lz, tame),
                     isect_disc(g1, qx, qy, qz, qq, lx, ly, lz, tame), [&](double t0, bool v0, double t1, bool v1) {
                       if ((v0 && t0 < tself) || (v1 && t1 < tself)) lit = false;
                     });
        }
        if (k < end) {
          const cdouble* g0 = cg + __builtin_amdgcn_readfirstlane(k) * RTX_GEOM_WORDS;
          isect_one(isect_disc(g0, qx, qy, qz, qq, lx, ly, lz, tame), [&](double t0, bool v0) {
            if (v0 && t0 < tself) lit = false;
          });
        }
      }
      if (__ballot(lit) == 0) break;  // every lane of the wave is in shadow
      ++i;
    } else {
      i = (int)nd[RTX_N_SKIP];
    }
  }
  return lit;
}

// Nearest hit of ray (O, D) over all spheres; wave-uniform loop over sphere pairs, geometry through
// the scalar cache. CAM: O is the camera (level 0), using the host-precomputed c.
template <bool CAM, typename P, typename Wk>
__device__ __forceinline__ void nearest_hit(const P* geo, int nsph, double ox, double oy, double oz, double dx,
                                            double dy, double dz, double& tmin, int& hit, bool& tie, double tame,
                                            Wk& wk) {
  wk.test(nsph);
  tmin = FARAWAY;
  hit = -1;
  tie = false;
  const double oo = CAM ? 0.0 : dot3(ox, oy, oz, ox, oy, oz);
  int s = 0;
  for (; s + 1 < nsph; s += 2) {
    const P* g0 = geo + __builtin_amdgcn_readfirstlane(s) * RTX_GEOM_WORDS;
    const P* g1 = g0 + RTX_GEOM_WORDS;
    const SphTest a0 = CAM ? isect_disc_cam(g0, ox, oy, oz, dx, dy, dz, tame)
                           : isect_disc(g0, ox, oy, oz, oo, dx, dy, dz, tame);
    const SphTest a1 = CAM ? isect_disc_cam(g1, ox, oy, oz, dx, dy, dz, tame)
                           : isect_disc(g1, ox, oy, oz, oo, dx, dy, dz, tame);
    isect_pair(a0, a1, [&](double t0, bool v0, double t1, bool v1) {
      nearest_update(v0, t0, s, tmin, hit, tie);
      nearest_update(v1, t1, s + 1, tmin, hit, tie);
    });
  }
  if (s < nsph) {
    const P* g0 = geo + __builtin_amdgcn_readfirstlane(s) * RTX_GEOM_WORDS;
    const SphTest a0 = CAM ? isect_disc_cam(g0, ox, oy, oz, dx, dy, dz, tame)
                           : isect_disc(g0, ox, oy, oz, oo, dx, dy, dz, tame);
    isect_one(a0, [&](double t0, bool v0) { nearest_update(v0, t0, s, tmin, hit, tie); });
  }
}

// (x)^5 and (x)^2.5 for x in [0, 1] (shader.py:291, :310). NumPy evaluates these with its SIMD pow;
// both are ~1 ulp, not correctly rounded, so neither side is "exact" here.
// np.sin (shader.py:211) for |x| <= 2^20. Neither side is correctly rounded (NumPy's SIMD sin is
// ~1 ulp); this one is <= 2 ulp (tests/test_sin.py: 1.9 ulp measured against long-double sin).
// x - n*pi with n = rint(x/pi): the first fma is exact (x and n*P1 are multiples of 2^-52 and
// their difference is below 2), the next two add the rest of pi to ~160 bits. Then
// sin(r) = r + r^3 * p(r^2) on [-pi/2, pi/2] with the Taylor coefficients up to r^21 (truncation
// 1.2e-18 relative), and sin(x) = (-1)^n sin(r).
__device__ __forceinline__ double sin_reduced(double x) {
  const double n = __builtin_rint(x * 0x1.45f306dc9c883p-2);
  double r = __builtin_fma(-n, 0x1.921fb54442d18p+1, x);
  r = __builtin_fma(-n, 0x1.1a62633145c07p-53, r);
  r = __builtin_fma(-n, -0x1.f1976b7ed8fbcp-109, r);
  const double z = r * r;
  double q = 0x1.71b8ef6dcf572p-66;  // 1/21!
  q = __builtin_fma(z, q, -0x1.2f49b46814157p-57);
  q = __builtin_fma(z, q, 0x1.952c77030ad4ap-49);
  q = __builtin_fma(z, q, -0x1.ae7f3e733b81fp-41);
  q = __builtin_fma(z, q, 0x1.6124613a86d09p-33);
  q = __builtin_fma(z, q, -0x1.ae64567f544e4p-26);
  q = __builtin_fma(z, q, 0x1.71de3a556c734p-19);
  q = __builtin_fma(z, q, -0x1.a01a01a01a01ap-13);
  q = __builtin_fma(z, q, 0x1.1111111111111p-7);
  q = __builtin_fma(z, q, -0x1.5555555555555p-3);  // -1/3!
  const double s = __builtin_fma(r * z, q, r);
  return ((int)n & 1) ? -s : s;
}
__device__ __forceinline__ double sin_ref(const cdouble* sc, double x) {
  // the reduction above when the host bounded every material's phase (RTX_H_SINRED), else
  // wave-uniform: unless some active lane is out of its range (or NaN / inf)
  if (sc[RTX_H_SINRED] != 0.0 || __ballot(!(fabs(x) <= 0x1.0p20)) == 0) return sin_reduced(x);
  return sin(x);
}

// Shading-only arithmetic (kShadeMath): operands are non-negative and far from the overflow range
// by construction (denominators >= 1e-8, square-root arguments in [0, 2], |V|^2 and |H|^2 the
// squared lengths of finite vectors; a zero argument is selected around the core). The cores are
// bit-identical to the range-checked paths for operands above ~2^-900; below, only terms that are
// themselves below ~1e-250 can differ.
// rcp: the hardware estimate (~2^-24) and two Newton steps, correctly rounded on 4 M random
// operands (tools/approx_probe); a * rcp(b) is then within ~1 ulp of a / b.
__device__ __forceinline__ double div_shade(double a, double b) {
  if constexpr (kShadeMath == 0) return div_cr(a, b);
  if constexpr (kShadeMath == 1) return div_core(a, b);  // (2, 3, 4: the Newton sequence below)
  double r = __builtin_amdgcn_rcp(b);
  r = __builtin_fma(r, __builtin_fma(-b, r, 1.0), r);
  r = __builtin_fma(r, __builtin_fma(-b, r, 1.0), r);
  return a * r;
}
// sqrt: the library core without its second correction (correctly rounded on the same sample);
// 0 stays 0 (rsq(0) = inf)
__device__ __forceinline__ double sqrt_shade(double x) {
  if constexpr (kShadeMath == 0) return sqrt_cr(x);
  if constexpr (kShadeMath == 1) return x == 0.0 ? 0.0 : sqrt_core(x);
  const double y = __builtin_amdgcn_rsq(x);
  double g = x * y, h = y * 0.5;
  const double r = __builtin_fma(-h, g, 0.5);
  g = __builtin_fma(g, r, g);
  h = __builtin_fma(h, r, h);
  const double d = __builtin_fma(-g, g, x);
  g = __builtin_fma(d, h, g);
  return x == 0.0 ? 0.0 : g;
}
// 1 / where(|v| == 0, 1, |v|) for d = |v|^2: rsq and two Newton steps (~1 ulp)
__device__ __forceinline__ double inv_mag_shade(double d) {
  if constexpr (kShadeMath == 0) return inv_mag(d);
  if constexpr (kShadeMath == 1 || kShadeMath == 3) return d == 0.0 ? 1.0 : div_core(1.0, sqrt_core(d));
  double y = __builtin_amdgcn_rsq(d);
  y = __builtin_fma(y * 0.5, __builtin_fma(-d * y, y, 1.0), y);
  y = __builtin_fma(y * 0.5, __builtin_fma(-d * y, y, 1.0), y);
  return d == 0.0 ? 1.0 : y;
}

// the view vector: N.V near grazing amplifies its rounding (4 N.V + 1e-8 and G1(N.V) divide by
// it), so variants 3 and 4 keep its normalisation correctly rounded
__device__ __forceinline__ double inv_mag_shade_v(double d) {
  if constexpr (kShadeMath == 3 || kShadeMath == 4) return d == 0.0 ? 1.0 : div_core(1.0, sqrt_core(d));
  return inv_mag_shade(d);
}

__device__ __forceinline__ double pow5(double x) {
  const double x2 = x * x;
  return (x2 * x2) * x;
}
__device__ __forceinline__ double pow25(double x) { return (x * x) * sqrt_shade(x); }

// A level's key: the hit sphere (RTX_MAX_SPHERES <= 2^kKeyShift) and its texture key above it.
constexpr int kKeyShift = 11;
__device__ __forceinline__ int level_key(int hit, int tk) { return hit | (tk << kKeyShift); }
__device__ __forceinline__ int key_hit(int key) { return key & ((1 << kKeyShift) - 1); }
__device__ __forceinline__ int key_tex(int key) { return (int)((unsigned)key >> kKeyShift); }
static_assert(RTX_MAX_SPHERES <= (1 << kKeyShift) && RTX_MAX_TEXELS <= (1 << (31 - kKeyShift)), "level key");

// Image texture (HipTexturedSphere / ImageTexture): the texel of hit point P on sphere (centre C)
// at the spherical coordinates of NumpyTexturedSphere.diffusecolor (shape.py:66-79): n = (P - C)
// normalised, u = 0.5 + atan2(n.z, n.x) / (2 pi), v = 0.5 - asin(n.y) / pi, each mod 1, texel
// (int(v (h-1)), int(u (w-1))). atan2/asin are ROCm's (not correctly rounded, like NumPy's), so
// a point within an ulp of a texel edge may take the neighbour texel: parity unpinned (the reference
// class cannot render).
template <typename T, typename G>
__device__ __forceinline__ int image_texel(const T* mh, const G* gh, double px, double py, double pz) {
  double nx = px - gh[RTX_G_CX], ny = py - gh[RTX_G_CY], nz = pz - gh[RTX_G_CZ];
  norm3(nx, ny, nz);
  double u = 0.5 + atan2(nz, nx) / (2.0 * RTX_PI);
  double v = 0.5 - asin(ny) / RTX_PI;
  u = u - floor(u);  // % 1 (Python / NumPy remainder: non-negative)
  v = v - floor(v);
  if (!(u >= 0.0 && u < 1.0)) u = 0.0;  // NaN (a degenerate point): texel 0
  if (!(v >= 0.0 && v < 1.0)) v = 0.0;
  const int w = (int)mh[RTX_M_TG], h = (int)mh[RTX_M_TB];
  const int i = (int)(u * (double)(w - 1)), j = (int)(v * (double)(h - 1));
  return j * w + i;
}

// The inputs of one shaded hit's colour terms (everything else comes from the material record).
struct Hit {
  double dli;    // max(N.L, 0)                                shader.py:138
  double di;     // sum_domes intensity * max(N.(0,1,0), 0)     shader.py:239-242
  double spec;   // physical specular (0 unless lit && g != 0)  shader.py:100-104
  double va;     // clip(N.V, 0, 1) (iridescence input)         shader.py:201
  double g;      // specular_gain
  int h;         // hit sphere
  int tk;        // texture key: the checker cell (shader.py:30) or the image texel (shape.py:66-79)
  bool lit;      //                                              shader.py:79-84
  double qx, qy, qz;  // nudged hit point = reflected ray origin  shader.py:77
  double nx, ny, nz;  // normal
};

// _calculate_physical_specular, shader.py:246-320, for unit-ish L (once normalised) and V.
// Sums of non-negative terms here and in hit_color are fused multiply-adds (one rounding fewer,
// within an ulp of the term; A/B r5e: C2 -1.6%, C2main -1.4%, C3 -1.2%, C4 -0.6%): none of them
// decides anything, and none cancels, so the colour moves by at most a few ulp.
template <typename M>
__device__ __forceinline__ double specular(const M* mh, double g, double nx, double ny, double nz, double lx,
                                           double ly, double lz, double vx, double vy, double vz) {
  double Lx = lx, Ly = ly, Lz = lz;
  norm3_unit(Lx, Ly, Lz);  // :278 (normalised a second time; an ulp of L moves a sharp highlight's
                           // D by ~2500 ulp: skipping it put main.py's 1080p frame 6e-10 off, r4s2)
  double Vx = vx, Vy = vy, Vz = vz;
  norm3_unit(Vx, Vy, Vz);  // :279 (likewise)
  double Hx = Lx + Vx, Hy = Ly + Vy, Hz = Lz + Vz;
  {  // :280
    const double dh = dot3(Hx, Hy, Hz, Hx, Hy, Hz);
    const double rh = kShadeMath == 4 ? inv_mag_shade(dh) : inv_mag_shade_v(dh);
    Hx = Hx * rh;
    Hy = Hy * rh;
    Hz = Hz * rh;
  }
  const double NdotV = clip01(dot3(nx, ny, nz, Vx, Vy, Vz));  // :283
  // :318 (the select at the end, taken early: a wave whose hits all face away from the camera
  // skips the rest; A/B C2 -0.2%, C2main -0.5%, C1 -0.8%)
  if (!(NdotV > 0.0)) return 0.0;
  const double NdotH = clip01(dot3(nx, ny, nz, Hx, Hy, Hz));  // :284
  const double VdotH = clip01(dot3(Vx, Vy, Vz, Hx, Hy, Hz));  // :285
  const double NdotL = clip01(dot3(nx, ny, nz, Lx, Ly, Lz));  // :287
  const double F = __builtin_fma(mh[RTX_M_1MF0], pow5(1.0 - VdotH), mh[RTX_M_F0]);  // :291
  const double a2 = mh[RTX_M_A2];
  const double denom = (NdotH * NdotH) * mh[RTX_M_A2M1] + 1.0;  // :295 (not fused: the sum cancels
  // to ~a^2 near the highlight's peak, and D amplifies the product's rounding by ~1/a^2)
  const double Dd = RTX_PI * __builtin_fma(denom, denom, 1e-8);  // :296
  const double oma2 = mh[RTX_M_1MA2];
  const double dL = (NdotL + sqrt_shade(__builtin_fma(oma2, NdotL * NdotL, a2))) + 1e-8;  // :299-301
  const double dV = (NdotV + sqrt_shade(__builtin_fma(oma2, NdotV * NdotV, a2))) + 1e-8;
  // G = G1L * G1V and spec_base = (F D G) / (4 N.V + 1e-8) with D = a2 / Dd: the four quotients
  // of :296-306 as two reciprocals (a few ulp, like the single quotients' Newton sequences; the
  // 1e-12 parity bar holds on every test and 8,600 random scenes)
  const double spec_base = ((F * a2) * ((2.0 * NdotL) * (2.0 * NdotV))) *
                           div_shade(1.0, (dL * dV) * (Dd * __builtin_fma(4.0, NdotV, 1e-8)));  // :303-306
  // (G = G1L G1V and spec_base = F D G / (4 N.V + 1e-8) with D = a2 / Dd share one reciprocal;
  // A/B r5h: C2 -0.6%, C3 -0.7%, C4 -0.5%)
  const double glint = pow25(1.0 - NdotV) * NdotL;  // :310-312
  const double sf = __builtin_fma(g, glint, spec_base);  // :315
  return (NdotV <= 0.0) ? 0.0 : sf;  // :318
}


// Colour of one shaded hit given the reflected colour R (shader.py:86-110):
//   ((((0.004 + diffuse) + dome) + (spec + R*0.5)*g*lit) + irid)
// `weighted` = lit && g != 0; otherwise the specular/reflection term is x*0 == 0 (R is finite).
// IMG: image textures are handled (the general kernel, and k_render_fast's texturing build for
// RTX_F_IMAGES launches); the other k_render_fast builds defer every pixel that meets an
// image-textured sphere and compile no texture lookup (A/B: carrying it cost C2 +3.4%, C2main +7%).
template <bool IMG = false, typename M>
__device__ __forceinline__ void hit_color(const M* mh, const cdouble* sc, double dli, double di, int tk, bool lit,
                                          bool weighted, double spec, double va, double Rr, double Rg, double Rb,
                                          double& cr, double& cg, double& cb) {
  const double litf = lit ? 1.0 : 0.0;
  double tr, tg, tb;
  const double tex = mh[RTX_M_TEX];
  if (tex == RTX_TEX_CHECKER) {  // TextureChecker.get_color (:29-32): white * checker
    tr = tg = tb = tk ? 1.0 : 0.0;
  } else if (IMG && tex == RTX_TEX_IMAGE) {  // the texel shade() picked (texel table in the blob)
    const cdouble* t = sc + ((int64_t)mh[RTX_M_TR] + 3 * (int64_t)tk);
    tr = t[0];
    tg = t[1];
    tb = t[2];
  } else {  // Texture.get_color (:17-19)
    tr = mh[RTX_M_TR];
    tg = mh[RTX_M_TG];
    tb = mh[RTX_M_TB];
  }
  const double dg = mh[RTX_M_DG];
  // ambient + diffuse (:86-88, :138-141), dome (:98, :244)
  const double ar = __builtin_fma(sc[RTX_H_DOMEC + 0], di, __builtin_fma((tr * dli) * litf, dg, 0.004));
  const double ag = __builtin_fma(sc[RTX_H_DOMEC + 1], di, __builtin_fma((tg * dli) * litf, dg, 0.004));
  const double ab = __builtin_fma(sc[RTX_H_DOMEC + 2], di, __builtin_fma((tb * dli) * litf, dg, 0.004));
  // specular + reflection (:106)
  const double g = mh[RTX_M_G];
  const double xr = weighted ? (spec + Rr * 0.5) * g : 0.0;
  const double xg = weighted ? (spec + Rg * 0.5) * g : 0.0;
  const double xb = weighted ? (spec + Rb * 0.5) * g : 0.0;
  // thin-film iridescence (:186-232); zero when iridescence_gain == 0 (x * 0 == 0)
  double ir = 0.0, ig = 0.0, ib = 0.0;
  const double igain = mh[RTX_M_IG];
  if (igain != 0.0) {
    const double af = fabs(va - 0.5) * 2.0;  // :204
    const double phase = ((af * RTX_PI) * mh[RTX_M_TFT]) * 10.0;  // :208
    const double ip = sin_ref(sc, phase);  // :211
    const double hs = mh[RTX_M_HS], omhs = mh[RTX_M_1MHS];
    const double r = __builtin_fma(ip, hs, omhs * (1.0 - ip));  // :221
    const double gg = __builtin_fma(ip, omhs, hs * (1.0 - ip));  // :222
    const double b = __builtin_fma(0.5, ip, 0.5);  // :223
    const double w = mh[RTX_M_TFW];
    ir = (r * w) * igain;  // :229-232
    ig = (gg * w) * igain;
    ib = (b * w) * igain;
  }
  cr = (ar + xr) + ir;
  cg = (ag + xg) + ig;
  cb = (ab + xb) + ib;
}

// ---- shadow grid (RTX_H_SHGRID, scene_pack._append_shadow_grid) ---------------------------
// The union, over the wave's lanes, of the masks of their shadow rays (origin q, direction L_dir):
// a lane whose q lies in the grid takes its voxel's mask (the spheres that may shadow any point of
// it); a lane outside takes the huge spheres' mask if its ray's line passes the small spheres'
// bounding ball at more than its radius plus the rounding reach (distance^2 from the centre: |w|^2 -
// (w.L_dir)^2, whose rounding, <= 4.4e-16 |w|^2, the 3e-8 (|w|^2 + 1) term covers; the host grows
// the radius by 1e-6 (|Cb| + Rb + 1), the lane adds 1e-6 |q| <= 5e-7 (|q|^2 + 1)). The wave-uniform
// own shape hs is removed. False (use the culling tree or the linear loop) when some lane fails
// both, has |N|^2 > 4 (the voxel masks' nudge bound) or NaNs, or when the lanes span more than
// kGridWaterfall distinct masks.
constexpr int kGridWaterfall = 16;  // (A/B r6ac/r6ad against 8: C4 -0.7/-1.0%, C3 -0.4%, C5 -1.1%; 32: C4 +-0)
__device__ __forceinline__ bool grid_mask(const cdouble* sc, double qx, double qy, double qz, double qq, double lx,
                                          double ly, double lz, double n2, int hs, uint64_t& m0, uint64_t& m1) {
  const cdouble* gr = sc + (int)sc[RTX_H_SHGRID];
  const double fx = (qx - gr[0]) * gr[3], fy = (qy - gr[1]) * gr[4], fz = (qz - gr[2]) * gr[5];
  const bool in = fx >= 0.0 && fx < gr[6] && fy >= 0.0 && fy < gr[7] && fz >= 0.0 && fz < gr[8] && n2 <= 4.0;
  const int nx = (int)gr[6], ny = (int)gr[7];
  int key = ((int)fz * ny + (int)fy) * nx + (int)fx;
  bool ok = in;
  if (!in) {
    const double wx = gr[9] - qx, wy = gr[10] - qy, wz = gr[11] - qz;
    const double ww = (wx * wx + wy * wy) + wz * wz;
    const double hh = (wx * lx + wy * ly) + wz * lz;
    const double R = (gr[12] + 5e-7 * (qq + 1.0)) + 3e-8 * (ww + 1.0);
    ok = ww - hh * hh > R * R;
    key = nx * ny * (int)gr[8];  // the huge spheres' mask
  }
  if (__ballot(!ok) != 0) return false;
  const cdouble* masks = gr + RTX_SHGRID_WORDS;
  m0 = 0;
  m1 = 0;
  bool pend = true;
  for (int it = 0;; ++it) {
    const uint64_t b = __ballot(pend);
    if (b == 0) break;
    if (it == kGridWaterfall) return false;
    const int k0 = __builtin_amdgcn_readlane(key, (int)__builtin_ctzll(b));
    m0 |= (uint64_t)__double_as_longlong(masks[2 * k0]);
    m1 |= (uint64_t)__double_as_longlong(masks[2 * k0 + 1]);
    pend = pend && key != k0;
  }
  if (hs < 64) m0 &= ~(uint64_t(1) << hs);
  else if (hs < 128) m1 &= ~(uint64_t(1) << (hs - 64));
  return true;
}

// The smallest valid root over the candidate spheres of masks m0/m1 (scene order, pairs) and
// whether there is one: the shadow test's candidates before t_self (shade's grid path).
template <typename G, typename Wk>
__device__ __forceinline__ void min_masked(const G* geo, uint64_t m0, uint64_t m1, double qx, double qy, double qz,
                                           double qq, double lx, double ly, double lz, double tame, double& tsh,
                                           bool& anyv, Wk& wk) {
  wk.test(__builtin_popcountll(m0) + __builtin_popcountll(m1));
  tsh = FARAWAY;
  anyv = false;
  for (int half = 0; half < 2; ++half) {
    uint64_t m = half ? m1 : m0;
    const int base = half * 64;
    while (m) {
      const int s0 = base + __builtin_ctzll(m);
      m &= m - 1;
      const SphTest a0 = isect_disc(geo + s0 * RTX_GEOM_WORDS, qx, qy, qz, qq, lx, ly, lz, tame);
      if (m) {
        const int s1 = base + __builtin_ctzll(m);
        m &= m - 1;
        isect_pair(a0, isect_disc(geo + s1 * RTX_GEOM_WORDS, qx, qy, qz, qq, lx, ly, lz, tame),
                   [&](double t0, bool v0, double t1, bool v1) {
                     if (v0) tsh = __builtin_fmin(tsh, t0);
                     if (v1) tsh = __builtin_fmin(tsh, t1);
                     anyv = anyv || v0 || v1;
                   });
      } else {
        isect_one(a0, [&](double t0, bool v0) {
          if (v0) tsh = __builtin_fmin(tsh, t0);
          anyv = anyv || v0;
        });
      }
    }
  }
}

// NumpyShader.create (shader.py:63-112) for a hit of sphere h at distance t, minus the colour
// assembly (hit_color) and the reflection recursion (driven by the caller).
// geo: scalar-cache view of the sphere table (wave-uniform loops); tab: the per-lane view of the
// same table (LDS copy or global).
// mat: a material record replacing sphere h's own (Shader.create on another shape's shader), or null.
// TREE = false: the scene has no culling tree (fewer than kTreeMinSpheres spheres), compiled out.
template <bool IMG = false, bool TREE = true, typename T, typename G, typename Wk>
__device__ __forceinline__ void shade(const cdouble* sc, const G* geo, const T* tab, int nsph, int h, double ox,
                                      double oy, double oz, double dx, double dy, double dz, double t, Hit& s,
                                      double tame, Wk& wk, const T* mat = nullptr) {
  const T* gh = tab + h * RTX_GEOM_WORDS;
  const T* mh = mat ? mat : tab + nsph * RTX_GEOM_WORDS + h * RTX_MAT_WORDS;
  const double px = ox + dx * t, py = oy + dy * t, pz = oz + dz * t;  // :73
  const double inv_r = gh[RTX_G_INVR];
  const double nx = (px - gh[RTX_G_CX]) * inv_r;  // :74 (not renormalised)
  const double ny = (py - gh[RTX_G_CY]) * inv_r;
  const double nz = (pz - gh[RTX_G_CZ]) * inv_r;
  double lx = sc[RTX_H_LIGHT + 0] - px, ly = sc[RTX_H_LIGHT + 1] - py, lz = sc[RTX_H_LIGHT + 2] - pz;
  norm3(lx, ly, lz);  // :75
  const double qx = px + nx * 0.0001, qy = py + ny * 0.0001, qz = pz + nz * 0.0001;  // :77

  // _calculate_shadow (:114-128): lit == (t_self == min_j t_j), no light-distance cutoff.
  // Equivalent any-hit form: lit unless some sphere is strictly nearer than the shape itself.
  const double qq = dot3(qx, qy, qz, qx, qy, qz);
  // The shape's own test is t_self itself (same expression), and t_self < t_self never holds: when
  // every active lane hit the same sphere, the loops skip it (wave-uniform index remap below).
  const int h0 = __builtin_amdgcn_readfirstlane(h);
  const int hs = __ballot(h != h0) == 0 ? h0 : nsph;
  bool lit = true;
  uint64_t m0, m1;
  // The shadow grid (tame scenes: t_self < 2^62 < FARAWAY, so no lane is far_self): only the
  // candidate occluders are tested, and t_self only if there is one (with none, t_self is the
  // minimum whatever it is: lit). Scenes with a culling tree only: below kTreeMinSpheres the linear
  // loop is as cheap as the lookup (A/B: C2 +0.7%, C2main +2.7%, C1 +5% with the grid).
  if (TREE && sc[RTX_H_SHGRID] != 0.0 && sc[RTX_H_TAME] != 0.0 &&
      grid_mask(sc, qx, qy, qz, qq, lx, ly, lz, dot3(nx, ny, nz, nx, ny, nz), hs, m0, m1)) {
    wk.node();  // the voxel lookup, priced as one node test
    if ((m0 | m1) != 0) {
      // the candidates first (each lane's smallest valid root), t_self only where some lane has one:
      // lit <=> no valid candidate root below t_self, and a lane without one is lit whatever t_self is
      // (round 6, as the small-scene loop below; A/B r6z: C4 -2.0%, C3 -0.4%, C5 within noise)
      double tsh;
      bool anyv;
      min_masked(geo, m0, m1, qx, qy, qz, qq, lx, ly, lz, tame, tsh, anyv, wk);
      if (__ballot(anyv) != 0) {
        const double tself = isect_t(gh, qx, qy, qz, qq, lx, ly, lz, tame);
        wk.test(1);
        lit = !(anyv && tsh < tself);
      }
    }
  } else if (!TREE && sc[RTX_H_TAME] != 0.0) {
    // Scenes without a culling tree, tame: the other spheres first, and t_self only when some lane
    // has a valid root (t_self < 2^62 < FARAWAY in a tame scene, so an invalid test never shadows
    // and a lane without a valid root is lit whatever t_self is). lit <=> no valid root strictly
    // below t_self <=> !(smallest valid root < t_self); a lane's own shape, tested when the wave's
    // shapes differ, gives t_self itself, which is not below it.
    const int nshadow = nsph - (hs < nsph);
    double tsh = FARAWAY;
    bool anyv = false;
    int j = 0;
    for (; j + 1 < nshadow; j += 2) {  // sphere pairs (one scalar-load wait, two interleaved chains)
      const G* g0 = geo + __builtin_amdgcn_readfirstlane(j + (j >= hs)) * RTX_GEOM_WORDS;
      const G* g1 = geo + __builtin_amdgcn_readfirstlane(j + 1 + (j + 1 >= hs)) * RTX_GEOM_WORDS;
      wk.test(2);
      isect_pair(isect_disc(g0, qx, qy, qz, qq, lx, ly, lz, tame), isect_disc(g1, qx, qy, qz, qq, lx, ly, lz, tame),
                 [&](double t0, bool v0, double t1, bool v1) {
                   if (v0) tsh = __builtin_fmin(tsh, t0);
                   if (v1) tsh = __builtin_fmin(tsh, t1);
                   anyv = anyv || v0 || v1;
                 });
    }
    if (j < nshadow) {
      const G* g0 = geo + __builtin_amdgcn_readfirstlane(j + (j >= hs)) * RTX_GEOM_WORDS;
      wk.test(1);
      isect_one(isect_disc(g0, qx, qy, qz, qq, lx, ly, lz, tame), [&](double t0, bool v0) {
        if (v0) tsh = __builtin_fmin(tsh, t0);
        anyv = anyv || v0;
      });
    }
    if (__ballot(anyv) != 0) {
      const double tself = isect_t(gh, qx, qy, qz, qq, lx, ly, lz, tame);
      wk.test(1);
      lit = !(anyv && tsh < tself);
    }
  } else {
    const double tself = isect_t(gh, qx, qy, qz, qq, lx, ly, lz, tame);
    wk.test(1);
    // t_self beyond FARAWAY (a hit past the reference's sentinel distance): every missing sphere
    // shadows. The linear loop handles it exactly; the culling tree skips missing spheres, so such
    // a wave takes the linear loop.
    const bool far_self = tself > FARAWAY;
    const bool culled = TREE && sc[RTX_H_NNODES] != 0.0 && __ballot(far_self) == 0;
    if (culled) lit = lit_bvh(sc, qx, qy, qz, qq, lx, ly, lz, tself, hs, tame, wk);
    const int nshadow = culled ? 0 : nsph - (hs < nsph);
    int j = 0;
    for (; j + 1 < nshadow; j += 2) {  // sphere pairs (one scalar-load wait, two interleaved chains)
      const int j0 = __builtin_amdgcn_readfirstlane(j + (j >= hs));
      const int j1 = __builtin_amdgcn_readfirstlane(j + 1 + (j + 1 >= hs));
      const G* g0 = geo + j0 * RTX_GEOM_WORDS;
      const G* g1 = geo + j1 * RTX_GEOM_WORDS;
      wk.test(2);
      bool sh = far_self;  // lanes without a valid root in either test
      isect_pair(isect_disc(g0, qx, qy, qz, qq, lx, ly, lz, tame), isect_disc(g1, qx, qy, qz, qq, lx, ly, lz, tame),
                 [&](double t0, bool v0, double t1, bool v1) {
                   sh = shadows(v0, t0, tself, far_self) || shadows(v1, t1, tself, far_self);
                 });
      if (sh) {
        lit = false;
        break;
      }
    }
    if (lit && j < nshadow) {
      const G* g0 = geo + __builtin_amdgcn_readfirstlane(j + (j >= hs)) * RTX_GEOM_WORDS;
      wk.test(1);
      bool sh = far_self;
      isect_one(isect_disc(g0, qx, qy, qz, qq, lx, ly, lz, tame),
                [&](double t0, bool v0) { sh = shadows(v0, t0, tself, far_self); });
      if (sh) lit = false;
    }
  }

  const double dli = max0(dot3(nx, ny, nz, lx, ly, lz));  // :138
  // dome (:239-242): light_direction (0, 1, 0)
  // N.(0, 1, 0) = ((nx*0) + ny*1) + nz*0 is ny itself for finite N (N is finite: P and C are), up to
  // the sign of a zero, which max0 and the sum below (0.0 + I*(+-0) = +0) erase
  const double up = ny;
  const int ndome = (int)sc[RTX_H_NDOME];
  double di = 0.0;
  for (int j = 0; j < ndome; ++j) di = di + sc[RTX_H_DOMEI + j] * max0(up);

  const double g = mh[RTX_M_G];
  const bool weighted = lit && g != 0.0;
  const bool need_irid = mh[RTX_M_IG] != 0.0;
  double spec = 0.0, va = 0.0;
  if (weighted || need_irid) {
    double vx = sc[RTX_H_CAM + 0] - px, vy = sc[RTX_H_CAM + 1] - py, vz = sc[RTX_H_CAM + 2] - pz;
    {  // :76 (towards the camera on every level); V only feeds the specular and the iridescence
      const double rv = inv_mag_shade_v(dot3(vx, vy, vz, vx, vy, vz));
      vx = vx * rv;
      vy = vy * rv;
      vz = vz * rv;
    }
    if (weighted) spec = specular(mh, g, nx, ny, nz, lx, ly, lz, vx, vy, vz);
    if (need_irid) va = clip01(dot3(nx, ny, nz, vx, vy, vz));  // :201
  }
  s.dli = dli;
  s.di = di;
  s.spec = spec;
  s.va = va;
  s.g = g;
  s.h = h;
  const double tex = mh[RTX_M_TEX];
  s.tk = tex == RTX_TEX_CHECKER ? (trunc_parity(px * 2.0) == trunc_parity(pz * 2.0))  // :30
         : tex != RTX_TEX_IMAGE ? 0
         : IMG ? image_texel(mh, gh, px, py, pz) : -1;  // -1: an untextured k_render_fast build defers the ray
  s.lit = lit;
  s.qx = qx; s.qy = qy; s.qz = qz;
  s.nx = nx; s.ny = ny; s.nz = nz;
}

// Reflected direction (shader.py:151): norm(D - (N*2) * (D.N))
__device__ __forceinline__ void reflect_dir(double& dx, double& dy, double& dz, double nx, double ny, double nz) {
  const double dn = dot3(dx, dy, dz, nx, ny, nz);
  double rx = dx - (nx * 2.0) * dn, ry = dy - (ny * 2.0) * dn, rz = dz - (nz * 2.0) * dn;
  norm3_unit(rx, ry, rz);  // |D| = |N| = 1 up to rounding, so |R| too
  dx = rx;
  dy = ry;
  dz = rz;
}

// ------------------------------------------------------------------------------------------
// ray setup / output
// ------------------------------------------------------------------------------------------

__device__ __forceinline__ int global_row(const Params& p, int lr) {
  if (p.n_parts == 1) return lr;  // a whole frame (uniform branch: no integer divisions)
  // a run of part_run consecutive parts owns part_run * row_block consecutive rows of every cycle of
  // n_parts * row_block rows, from row part * row_block of the cycle (part_run == 1: one row block)
  const int own = p.row_block * p.part_run;
  return (lr / own) * (p.n_parts * p.row_block) + p.part * p.row_block + (lr % own);
}

// get_ray_directions (base.py:123-141) for pixel (col, global row r).
__device__ __forceinline__ void camera_dir(const cdouble* sc, int col, int r, int W, int H, double& dx, double& dy,
                                           double& dz) {
  // np.linspace: i*step + start, last element set to stop exactly
  const double x = (sc[RTX_H_XFIX] != 0.0 && col == W - 1) ? sc[RTX_H_XSTOP]
                                                            : (double)col * sc[RTX_H_XSTEP] + sc[RTX_H_XSTART];
  const double y = (sc[RTX_H_YFIX] != 0.0 && r == H - 1) ? sc[RTX_H_YSTOP]
                                                          : (double)r * sc[RTX_H_YSTEP] + sc[RTX_H_YSTART];
  const double vx = x - sc[RTX_H_CAM + 0];
  const double vy = y - sc[RTX_H_CAM + 1];
  const double vz = sc[RTX_H_VZ];
  const double rr = inv_mag(((vx * vx) + (vy * vy)) + sc[RTX_H_VZ2]);
  dx = vx * rr;
  dy = vy * rr;
  dz = vz * rr;
}

// the camera ray of pixel (col, local row lr) of the launch's tile
__device__ __forceinline__ void camera_ray(const Params& p, int col, int lr, double& ox, double& oy, double& oz,
                                           double& dx, double& dy, double& dz) {
  const cdouble* sc = (const cdouble*)p.scene;
  camera_dir(sc, col, global_row(p, lr), p.width, p.height, dx, dy, dz);
  ox = sc[RTX_H_CAM + 0];
  oy = sc[RTX_H_CAM + 1];
  oz = sc[RTX_H_CAM + 2];
}

// spheres [nb, nsph) are all huge (RTX_H_NBEAM): candidates of every tile and beam without a test
__device__ __forceinline__ int huge_tail(const cdouble* sc, int nsph) {
  const int nb = (int)sc[RTX_H_NBEAM];
  return nb > 0 && nb < nsph ? nb : nsph;
}

// ---- level-0 candidates of a wave tile ------------------------------------------------------
// The camera rays of a wave's pixels leave one origin O through points (x, y, 0) of the image
// plane (camera_dir, base.py:123-141), and x (y) is monotone in the column (row), so the plane
// points of the tile's lanes lie in the rectangle of its extreme columns and rows (a lane's ray
// passes through O + (fl(x - Ox), fl(y - Oy), VZ), within an ulp of (x, y, 0)). The host gives every
// sphere an image-plane box for this camera (RTX_H_SBOX, scene_pack.sphere_plane_boxes): a camera
// ray through a plane point outside it yields FARAWAY for that sphere. The box is built from the
// sphere's radius expanded by the culling margin lm (node_may_hit: a root the reference reports lies
// within lm of the ball), with scale = |C - O|^2 + 2|C|^2 + 3r^2 + |O|^2 (>= node_may_hit's scale for
// a single sphere) and lm = 1e-7 (scale + 1), doubled like the node margin: that also absorbs
// |D| = 1 +- 1e-15 and the plane point's ulp. A sphere whose box misses the tile's rectangle is
// skipped by the tile's level-0 nearest hit: the nearest hit and the tie flag are unchanged.
// Comparisons are written so that NaN keeps the sphere; the huge tail (RTX_H_NBEAM) is kept without
// a test. One lane tests one sphere (two passes for 65..128 spheres); the ballots are the tile's
// candidate masks. Needs the full wave (call before any lane diverges). (Rounds 3-4 tested each
// sphere against the tile's four frustum planes, ~40 VALU a lane; A/B r5q: the boxes take C3 -7.6%,
// C4 -4.9%, C5 -3.8%.)
__device__ __forceinline__ bool wave_frustum(const Params& p, int c0, int lr0, uint64_t& m0, uint64_t& m1) {
  const cdouble* sc = (const cdouble*)p.scene;
  const int W = p.width;
  if (c0 >= W || lr0 >= p.n_rows) return false;  // no pixel of this wave lies in the frame
  const int c1 = c0 + kWaveW - 1 < W - 1 ? c0 + kWaveW - 1 : W - 1;
  const int l1 = lr0 + kWaveH - 1 < p.n_rows - 1 ? lr0 + kWaveH - 1 : p.n_rows - 1;
  const int H = p.height;
  auto xv = [&](int c) {
    return (sc[RTX_H_XFIX] != 0.0 && c == W - 1) ? sc[RTX_H_XSTOP] : (double)c * sc[RTX_H_XSTEP] + sc[RTX_H_XSTART];
  };
  auto yv = [&](int r) {
    return (sc[RTX_H_YFIX] != 0.0 && r == H - 1) ? sc[RTX_H_YSTOP] : (double)r * sc[RTX_H_YSTEP] + sc[RTX_H_YSTART];
  };
  const double xa = xv(c0), xb = xv(c1), ya = yv(global_row(p, lr0)), yb = yv(global_row(p, l1));
  const double xlo = __builtin_fmin(xa, xb), xhi = __builtin_fmax(xa, xb);
  const double ylo = __builtin_fmin(ya, yb), yhi = __builtin_fmax(ya, yb);
  const double* bx = p.scene + (int64_t)sc[RTX_H_SBOX];  // per-lane loads: a generic pointer
  const int lane = (int)__lane_id();
  const int nb = huge_tail(sc, p.nsph);
  auto may = [&](int s) {
    if (s >= p.nsph) return false;
    if (s >= nb) return true;
    const double* e = bx + 4 * s;
    return !(e[1] < xlo || e[0] > xhi || e[3] < ylo || e[2] > yhi);
  };
  m0 = __ballot(may(lane));
  // the second pass only when a sphere above 63 needs its test (C4: 65 spheres, the 65th the ground)
  m1 = p.nsph <= 64 ? 0ull
       : nb > 64    ? __ballot(may(64 + lane))
                    : (p.nsph >= 128 ? ~0ull : (uint64_t(1) << (p.nsph - 64)) - 1);
  return true;
}

// Nearest hit over the candidate spheres of masks m0 (spheres 0..63) and m1 (64..127), in scene
// order, pairs at a time like nearest_hit. CAM: camera rays (level 0, the host's c).
template <bool CAM, typename P, typename Wk>
__device__ __forceinline__ void nearest_masked(const P* geo, uint64_t m0, uint64_t m1, double ox, double oy,
                                               double oz, double dx, double dy, double dz, double& tmin, int& hit,
                                               bool& tie, double tame, Wk& wk) {
  wk.test(__builtin_popcountll(m0) + __builtin_popcountll(m1));
  tmin = FARAWAY;
  hit = -1;
  tie = false;
  const double oo = CAM ? 0.0 : dot3(ox, oy, oz, ox, oy, oz);
  auto disc = [&](const P* g) {
    return CAM ? isect_disc_cam(g, ox, oy, oz, dx, dy, dz, tame) : isect_disc(g, ox, oy, oz, oo, dx, dy, dz, tame);
  };
  auto run = [&](uint64_t m, int base) {
    while (m) {
      const int s0 = base + __builtin_ctzll(m);
      m &= m - 1;
      const P* g0 = geo + s0 * RTX_GEOM_WORDS;
      const SphTest a0 = disc(g0);
      if (m) {
        const int s1 = base + __builtin_ctzll(m);
        m &= m - 1;
        const SphTest a1 = disc(geo + s1 * RTX_GEOM_WORDS);
        isect_pair(a0, a1, [&](double t0, bool v0, double t1, bool v1) {
          nearest_update(v0, t0, s0, tmin, hit, tie);
          nearest_update(v1, t1, s1, tmin, hit, tie);
        });
      } else {
        isect_one(a0, [&](double t0, bool v0) { nearest_update(v0, t0, s0, tmin, hit, tie); });
      }
    }
  };
  run(m0, 0);
  run(m1, 64);
}

// ---- candidates of a wave's reflected rays (levels >= 1 of tree scenes) --------------------------
// The wave's active rays (O, D) leave from a ball around the first active lane's origin Oc, of
// radius rho >= |O - Oc|, in directions within angle theta of that lane's direction A
// (1 - cos theta >= 1 - D.A in every lane). A point X = O + tD (t > 0) within R' of a centre C puts
// Oc + tD within R = R' + rho of it, so D lies within phi = asin(R / |W|) of W = C - Oc and A
// within theta + phi: A.W >= |W| cos(theta + phi) = cos theta sqrt(|W|^2 - R^2) - sin theta R
// (theta, phi <= 90 degrees). With R' = r + lm (the culling margin of wave_frustum, doubled again and
// taken over the whole ball: |C - O|^2 <= 2|W|^2 + 2 rho^2, |O|^2 <= 2|Oc|^2 + 2 rho^2), a sphere
// failing that test (and not reaching the ball itself) yields FARAWAY for every ray of the wave, so
// the nearest hit (and the tie flag) over the others is unchanged. The test is evaluated squared,
// without a square root of |W|^2 - R^2 (round 6): with t1 = A.W + sin theta R (plus an absolute
// slack for its rounding), a sphere is dropped when t1 < 0 (the right side is >= 0) or when
// t1^2 < (|W|^2 - R^2) cos^2 theta, the difference lowered by its rounding bound and the product
// by a relative 1e-12, so every rounding keeps the sphere. rho^2 and 1 - cos theta are bounded by
// powers of two, the wave maxima of the lanes' exponents (wave_max_jump: exact under any exec mask,
// no cross-lane arithmetic). Comparisons keep the sphere on NaN.
// Only the active lanes run here (the bounce loop's lanes leave it one by one), so the spheres are
// dealt out by rank: the active lane of rank k tests spheres k, k + n, k + 2n (n active lanes), and
// pass j's ballot holds sphere j n + rank(lane) at the lane's bit. False (take the culling tree)
// when that needs more than kBeamPasses passes, the beam is wider than 60 degrees, the ball larger
// than 2^6 or the candidates more than kBeamMaxCand.
constexpr int kBeamPasses = 3;
constexpr int kBeamMaxCand = 24;
// The beam kernels stage, in the LDS copy of the sphere table, each sphere's own part of the test's
// radius in geometry word RTX_G_IDX (unused in the main table): r (bounded above) plus the margin's
// per-sphere terms, beam_word below. The per-lane test then needs no square root of its own.
constexpr bool kBeamStaged = true;
static_assert(RTX_GEOM_WORDS == 8 && RTX_G_IDX == 7, "beam word: the last geometry word");
struct Beam {
  uint64_t m[kBeamPasses];  // pass j: candidate bits at the testing lanes' positions
  uint64_t ex;              // the active lanes
  int n;                    // their count
  int passes;
  int nb;                   // spheres [nb, nsph): the huge tail, candidates without a test
};
__device__ __forceinline__ double rfl_d(double x) {
  const int hi = __builtin_amdgcn_readfirstlane(__double2hiint(x));
  const int lo = __builtin_amdgcn_readfirstlane(__double2loint(x));
  return __hiloint2double(hi, lo);
}
// Max over the active lanes of a small int v: start from the last active lane's value and jump to
// a larger value some lane holds until no lane holds one (exact under any exec mask; one or two
// ballots for the nearby origins and directions of a wave tile, where the binary search of rounds
// 3-5 took seven and six).
__device__ __forceinline__ int wave_max_jump(int v) {
  const uint64_t ex = __ballot(1);
  int cur = __builtin_amdgcn_readlane(v, 63 - __builtin_clzll(ex));
  for (;;) {
    const uint64_t b = __ballot(v > cur);
    if (b == 0) return cur;
    cur = __builtin_amdgcn_readlane(v, __builtin_ctzll(b));
  }
}
// e with x < 2^e for x in [0, 2^hi): exponents below lo report lo; NaN and anything larger hi + 1
__device__ __forceinline__ int pow2_above(double x, int lo, int hi) {
  if (!(x < __builtin_ldexp(1.0, hi))) return hi + 1;
  if (x < __builtin_ldexp(1.0, lo - 1)) return lo;
  const int e = __builtin_amdgcn_frexp_exp(x);  // x = m 2^e, m in [0.5, 1)
  return e < lo ? lo : e;
}
// sqrt for the beam's culling test: the hardware reciprocal square root (~2^-24 relative) and one
// Newton step (~1e-15 relative: quadratic in the estimate's error); callers scale by 1 + 1e-11
// towards keeping the sphere. 0 and inf give NaN, which the test's comparisons read as "keep".
__device__ __forceinline__ double sqrt_cull(double x) {
  const double y = __builtin_amdgcn_rsq(x);
  return x * (y * __builtin_fma(-0.5 * x * y, y, 1.5));
}
// r (bounded above) + 4e-7 (2 C.C + 3 r^2) (1 + 1e-12): the sphere's own part of R (the same sum as
// wave_beam's unstaged R, reassociated; the test's outer 1 + 1e-12 covers the reassociation)
__device__ __forceinline__ double beam_word(double cc, double rr) {
  return sqrt_cull(rr) * (1.0 + 1e-11) + 4e-7 * ((2.0 * cc + 3.0 * rr) * (1.0 + 1e-12));
}
// STAGED: tab is the LDS copy whose word RTX_G_IDX holds beam_word (k_render_fast's staging loop)
template <bool STAGED, typename T>
__device__ __forceinline__ bool wave_beam(const T* tab, int nb, double ox, double oy, double oz, double dx,
                                          double dy, double dz, Beam& bm) {
  bm.ex = __ballot(1);
  bm.n = __builtin_popcountll(bm.ex);
  bm.nb = nb;
  bm.passes = (nb + bm.n - 1) / bm.n;  // the huge tail [nb, nsph) is dealt out to nobody
  if (bm.passes > kBeamPasses) return false;
  const double Ox = rfl_d(ox), Oy = rfl_d(oy), Oz = rfl_d(oz);
  const double Ax = rfl_d(dx), Ay = rfl_d(dy), Az = rfl_d(dz);
  const double wox = ox - Ox, woy = oy - Oy, woz = oz - Oz;
  const int er = wave_max_jump(pow2_above((wox * wox + woy * woy) + woz * woz, -60, 12));
  const double omc = 1.0 - ((dx * Ax + dy * Ay) + dz * Az);
  const int ea = wave_max_jump(pow2_above(omc, -60, -1));
  if (er > 12 || ea > -1) return false;
  const double rho2 = __builtin_ldexp(1.0, er);                 // > |O - Oc|^2 in every lane
  const double rho = sqrt_cull(rho2) * (1.0 + 1e-11);            // >= its square root
  const double ct = 1.0 - __builtin_ldexp(1.0, ea);              // <= cos theta (>= 1/2)
  const double ct2 = (ct * ct) * (1.0 - 1e-12);                  // <= cos^2 theta
  const double st = sqrt_cull(__builtin_ldexp(1.0, ea + 1)) * (1.0 + 1e-11);  // >= sin theta
  // the margin's terms common to every sphere: 2 rho^2 of |C - O|^2 and the bound on |O|^2
  const double lmk = ((2.0 * rho2 + 2.0 * ((Ox * Ox + Oy * Oy) + Oz * Oz)) + 2.0 * rho2) + 1.0;
  const int rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(bm.ex >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bm.ex, 0));
  auto may = [&](int s) {
    if (s >= nb) return false;
    const T* e = tab + s * RTX_GEOM_WORDS;
    const double wx = e[RTX_G_CX] - Ox, wy = e[RTX_G_CY] - Oy, wz = e[RTX_G_CZ] - Oz;
    const double ww = (wx * wx + wy * wy) + wz * wz;  // |W|^2
    double R;
    if constexpr (STAGED) {
      R = ((e[RTX_G_IDX] + 4e-7 * ((2.0 * ww + lmk) * (1.0 + 1e-12))) + rho) * (1.0 + 1e-12);
    } else {
      const double rr = e[RTX_G_RR];
      const double lm = 4e-7 * ((((2.0 * ww + 2.0 * e[RTX_G_CC]) + 3.0 * rr) + lmk) * (1.0 + 1e-12));
      R = ((sqrt_cull(rr) * (1.0 + 1e-11) + lm) + rho) * (1.0 + 1e-12);
    }
    const double R2 = R * R;
    if (!(ww > R2 * (1.0 + 1e-12))) return true;  // the ball may reach the sphere
    const double aw = (Ax * wx + Ay * wy) + Az * wz;
    const double t1 = (aw + st * R) + 1e-9 * ((ww + R2) + 2.0);  // (the slack: >= 1e-9 (|W| + R + 1))
    if (t1 < 0.0) return false;
    return !(t1 * t1 < (((ww - R2) - 1e-15 * (ww + R2)) * ct2));
  };
  int cand = 0;
#pragma unroll
  for (int j = 0; j < kBeamPasses; ++j) {
    bm.m[j] = j < bm.passes ? __ballot(may(j * bm.n + rank)) : 0ull;
    cand += __builtin_popcountll(bm.m[j]);
  }
  return cand <= kBeamMaxCand;
}

// Nearest hit over a wave beam's candidates (pass j, bit b: sphere j n + popcount(ex below b)),
// pairs at a time like nearest_hit; in scene order.
template <typename P, typename Wk>
__device__ __forceinline__ void nearest_beam(const P* geo, int nsph, const Beam& bm, double ox, double oy, double oz,
                                             double dx, double dy, double dz, double& tmin, int& hit, bool& tie,
                                             double tame, Wk& wk) {
  tmin = FARAWAY;
  hit = -1;
  tie = false;
  const double oo = dot3(ox, oy, oz, ox, oy, oz);
  auto sph = [&](uint64_t& m, int base) {
    const int b = __builtin_ctzll(m);
    m &= m - 1;
    return base + __builtin_popcountll(bm.ex & ((uint64_t(1) << b) - 1));
  };
#pragma unroll
  for (int j = 0; j < kBeamPasses; ++j) {
    uint64_t m = bm.m[j];
    wk.test(__builtin_popcountll(m));
    const int base = j * bm.n;
    while (m) {
      const int s0 = sph(m, base);
      const SphTest a0 = isect_disc(geo + s0 * RTX_GEOM_WORDS, ox, oy, oz, oo, dx, dy, dz, tame);
      if (m) {
        const int s1 = sph(m, base);
        const SphTest a1 = isect_disc(geo + s1 * RTX_GEOM_WORDS, ox, oy, oz, oo, dx, dy, dz, tame);
        isect_pair(a0, a1, [&](double t0, bool v0, double t1, bool v1) {
          nearest_update(v0, t0, s0, tmin, hit, tie);
          nearest_update(v1, t1, s1, tmin, hit, tie);
        });
      } else {
        isect_one(a0, [&](double t0, bool v0) { nearest_update(v0, t0, s0, tmin, hit, tie); });
      }
    }
  }
  // the huge tail, tested by every ray (wave-uniform bounds)
  wk.test(nsph - bm.nb);
  int s = bm.nb;
  for (; s + 1 < nsph; s += 2) {
    const P* g0 = geo + s * RTX_GEOM_WORDS;
    const SphTest a0 = isect_disc(g0, ox, oy, oz, oo, dx, dy, dz, tame);
    const SphTest a1 = isect_disc(g0 + RTX_GEOM_WORDS, ox, oy, oz, oo, dx, dy, dz, tame);
    isect_pair(a0, a1, [&](double t0, bool v0, double t1, bool v1) {
      nearest_update(v0, t0, s, tmin, hit, tie);
      nearest_update(v1, t1, s + 1, tmin, hit, tie);
    });
  }
  if (s < nsph) {
    const SphTest a0 = isect_disc(geo + s * RTX_GEOM_WORDS, ox, oy, oz, oo, dx, dy, dz, tame);
    isect_one(a0, [&](double t0, bool v0) { nearest_update(v0, t0, s, tmin, hit, tie); });
  }
}

__device__ __forceinline__ void load_ray(const Params& p, int64_t i, double& ox, double& oy, double& oz, double& dx,
                                         double& dy, double& dz) {
  if (p.mode == 0) {
    camera_ray(p, (int)(i % p.width), (int)(i / p.width), ox, oy, oz, dx, dy, dz);
  } else {
    const int64_t n = p.n;
    dx = p.dir[i];
    dy = p.dir[n + i];
    dz = p.dir[2 * n + i];
    const int64_t s = p.org_stride;
    const int64_t j = s ? i : 0;
    ox = p.org[j];
    oy = p.org[s + j + (s ? 0 : 1)];
    oz = p.org[2 * s + j + (s ? 0 : 2)];
  }
}

__device__ __forceinline__ unsigned char quant_u8(double c) {
  // (255 * np.clip(c, 0, 1)).astype(np.uint8)  (base.py:147): truncation (NaN -> 0)
  const double v = 255.0 * clip01(c);
  return v >= 0.0 ? (unsigned char)(int)v : (unsigned char)0;
}

// The lane's index in its wave by two VALU instructions the compiler cannot merge with an earlier
// lane id, so that a value derived from it is recomputed instead of kept live (fast_tile's tail).
__device__ __forceinline__ int lane_id_fresh() {
  int l;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
  return l;
}

__device__ __forceinline__ void write_out(const Params& p, int64_t i, double r, double g, double b) {
  // the frame is written once and never read back by the kernel: streaming (nontemporal) stores
  // (A/B, identical output: C5 -1.5..-1.9%, C3 -0.9%, C2 -0.4..-0.8%)
  if (p.out_kind == RTX_OUT_F32_SOA) {
    float* o = (float*)p.out;
    __builtin_nontemporal_store((float)r, o + i);
    __builtin_nontemporal_store((float)g, o + p.n + i);
    __builtin_nontemporal_store((float)b, o + 2 * p.n + i);
  } else if (p.out_kind == RTX_OUT_F64_SOA) {
    double* o = (double*)p.out;
    __builtin_nontemporal_store(r, o + i);
    __builtin_nontemporal_store(g, o + p.n + i);
    __builtin_nontemporal_store(b, o + 2 * p.n + i);
  } else {
    unsigned char* o = (unsigned char*)p.out + 3 * i;
    o[0] = quant_u8(r);
    o[1] = quant_u8(g);
    o[2] = quant_u8(b);
  }
}

__device__ __forceinline__ void stat_add(unsigned long long* st, int word, unsigned long long v) {
  atomicAdd(st + word, v);
}

// one count per wave (from its first active lane): how many waves execute a stage
__device__ __forceinline__ void stat_wave(unsigned long long* st, int word) {
  const unsigned long long m = __ballot(1);
  if ((int)__lane_id() == __ffsll((long long)m) - 1) atomicAdd(st + word, 1ull);
}

// ------------------------------------------------------------------------------------------
// k_render_fast<B, LDS, DEEP>
// ------------------------------------------------------------------------------------------

// One block tile: (bx, by) in camera mode, block bx of 256 rays in explicit-ray mode, 256 entries
// of in_list in continuation mode. `first`: the block's first tile, whose level-0 nearest-hit test
// overlaps the LDS staging of the scene table. DEEP (caps above 8 or none): chains still alive
// after B levels are deferred with a resume record, and the continuation mode exists; the capped
// instantiations compile none of it.
// IMG: image-textured spheres are shaded here (the texel lookup compiled in, RTX_F_IMAGES launches)
// instead of deferred to the general kernel.
// NSPH > 0: the scene has exactly NSPH spheres, a compile-time count (the timed small-scene kernels,
// rtx_small.hip: their sphere loops unroll; A/B r6b, C2 -2.7%); 0: p.nsph at run time.
template <int B, bool LDS, int DEEP, bool LVL, bool STATS, bool TREE, bool BEAM, bool IMG = false, int NSPH = 0>
__device__ __forceinline__ void fast_tile(const Params& p, int bx, int by, bool first, const double* lds_tab,
                                          bool wave_tile = false) {
  constexpr int FB = fast_block<TREE>();  // threads per block of this instantiation
  const cdouble* sc = (const cdouble*)p.scene;
  const cdouble* geo = sc + RTX_HDR_WORDS;
  const int nsph = NSPH > 0 ? NSPH : p.nsph;
  const int nb = TREE ? huge_tail(sc, nsph) : nsph;  // the beams' tested spheres
  // the half-b sphere test (SphTest): origins the kernel generates itself, in a tame scene
  const double tame = p.mode != 1 && p.mode != 3 && sc[RTX_H_TAME] != 0.0 ? 0x1.0p-350 : __builtin_nan("");

  int64_t i = 0;
  bool active;
  int kb = 0;                  // absolute level of this launch's first ray (mode 2: the resumed level)
  const double* rin = nullptr;  // mode 2: the chain's resume record (levels 0..kb-1)
  int col = 0, lr = 0;         // mode 0: the pixel's column and local row
  // WX x WY waves per block; wave w -> WW x WH sub-tile, lane -> (l % WW, l / WW)
  // (wave_tile: (bx, by) is this wave's own WW x WH tile; TREE only, so WW = kWaveW there)
  constexpr int WW = wave_w<TREE>(), WH = 64 / WW, WX = waves_x<TREE>(), WY = fast_waves<TREE>() / WX;
  const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));  // the wave in the block
  // The pixel index (modes 0, 1, 3) from the block's tile, the wave and a lane id. The culled
  // kernels' write-out recomputes it from a fresh lane id (lane_id_fresh): kept live across the
  // bounce loop, the 64-bit index spilled in the one-tile culled kernels (C3) and cost the persistent
  // one registers (A/B r5v: C4 -1.8%); the small-scene kernels keep it (C2 +1.4% recomputed).
  auto pixel_index = [&](int lane) -> int64_t {
    if (p.mode == 0) {
      const int c = wave_tile ? bx * WW + (lane % WW) : bx * (WX * WW) + (wv % WX) * WW + (lane % WW);
      const int r = wave_tile ? by * WH + (lane / WW) : by * (WY * WH) + (wv / WX) * WH + (lane / WW);
      return (int64_t)r * p.width + c;
    }
    return (int64_t)bx * FB + wv * 64 + lane;
  };
  if (DEEP != 2 && p.mode == 0) {
    const int lane = threadIdx.x & 63, w = TREE ? wv : (int)(threadIdx.x >> 6);
    col = wave_tile ? bx * WW + (lane % WW) : bx * (WX * WW) + (w % WX) * WW + (lane % WW);
    lr = wave_tile ? by * WH + (lane / WW) : by * (WY * WH) + (w / WX) * WH + (lane / WW);
    active = col < p.width && lr < p.n_rows;
    if constexpr (!TREE) i = (int64_t)lr * p.width + col;  // (kept live: A/B r5v C2 +1.4% recomputed)
  } else if (DEEP != 2) {  // (modes 1 and 3)
    i = (int64_t)bx * FB + threadIdx.x;
    active = i < p.n;
  } else {  // continuation: entry `item` of in_list
    const int64_t item = (int64_t)bx * FB + threadIdx.x;
    active = item < (int64_t)*p.in_count;
    if (active) {
      const uint64_t e = p.in_list[item];
      i = (int64_t)(e & ((uint64_t(1) << kFrameShift) - 1));
      const int rt = (int)((e >> kRaysShift) & kLevelMask) - 1, ht = (int)((e >> kHitsShift) & kLevelMask) - 1;
      if (rt == p.in_level && ht == rt && item < p.in_rec_cap) {
        rin = p.in_rec + item * rec_words(p.in_level);
        kb = rt + 1;
      } else {  // a tie, or a chain without a record: on to the general kernel unchanged
        append_deferred(p, e);
        active = false;
      }
    }
  }
  const bool cam0 = DEEP != 2 && p.mode == 0;
  // per-level counters: the stats instantiation only (the timed kernels compile none of it)
  unsigned long long* const st = STATS ? p.stats : nullptr;
  Work<STATS> wk;
  double ox = 0.0, oy = 0.0, oz = 0.0, dx = 0.0, dy = 0.0, dz = 1.0;
  // nearest hit of the current level's ray over all shapes (base.py:97-103): wave-uniform loop,
  // geometry via s_load
  double tmin = FARAWAY;
  int hit = -1;
  bool tie = false;
  // level-0 candidate spheres of the wave tile (wave_frustum) instead of the culling tree: camera
  // rays of a tame scene with a tree and at most 128 spheres
  uint64_t fm0 = 0, fm1 = 0;
  bool fr = false;
  if constexpr (TREE) {
    if (cam0 && nsph <= 128 && sc[RTX_H_NNODES] != 0.0 && sc[RTX_H_SBOX] != 0.0 && sc[RTX_H_TAME] != 0.0 &&
        sc[RTX_H_VZ] != 0.0) {
      const int lane = threadIdx.x & 63;
      fr = wave_frustum(p, __builtin_amdgcn_readfirstlane(col - lane % kWaveW),
                        __builtin_amdgcn_readfirstlane(lr - lane / kWaveW), fm0, fm1);
    }
  }
  if (active) {
    if (rin) {
      ox = rin[0]; oy = rin[1]; oz = rin[2];
      dx = rin[3]; dy = rin[4]; dz = rin[5];
    } else if (cam0) {
      camera_ray(p, col, lr, ox, oy, oz, dx, dy, dz);  // no division of the pixel index
    } else {
      load_ray(p, i, ox, oy, oz, dx, dy, dz);
    }
    if (st) {
      if (!rin) stat_add(st, RTX_S_PIXELS, 1);
      if (kb < RTX_S_LEVELS) {
        stat_add(st, RTX_S_RAYS + kb, 1);
        stat_wave(st, RTX_S_WTRACE + kb);
      }
    }
    if (p.mode == 3) {  // NumpyShader.create: the hit is given (shader.py:63-73)
      tmin = p.hit_t[i];
      hit = p.hit_shape;
      // create on another shape's shader (RTX_H_MAT0): the general kernel shades this level-0 hit
      // with that material, deferred like a tie
      tie = sc[RTX_H_MAT0] != 0.0;
    } else if (TREE && sc[RTX_H_NNODES] != 0.0) {
      if (fr) {  // (the image-plane boxes' comparisons are not priced)
        nearest_masked<true>(geo, fm0, fm1, ox, oy, oz, dx, dy, dz, tmin, hit, tie, tame, wk);
      } else if (cam0) {
        nearest_bvh<true>(sc, ox, oy, oz, dx, dy, dz, tmin, hit, tie, tame, wk);
      } else {
        nearest_bvh<false>(sc, ox, oy, oz, dx, dy, dz, tmin, hit, tie, tame, wk);
      }
    } else if (cam0) {
      nearest_hit<true>(geo, nsph, ox, oy, oz, dx, dy, dz, tmin, hit, tie, tame, wk);
    } else {
      nearest_hit<false>(geo, nsph, ox, oy, oz, dx, dy, dz, tmin, hit, tie, tame, wk);
    }
  }
  if constexpr (LDS) {
    if (first) __syncthreads();
  }
  if (!active) return;
  constexpr bool CL = kForwardFold && !DEEP && LDS && TREE && !BEAM;  // colour in LDS (kColourLdsBytes)
  static_assert(!CL || 3 * sizeof(double) * FB == kColourLdsBytes, "colour LDS");
  double* const cl = CL ? const_cast<double*>(lds_tab) + nsph * kSphWords + threadIdx.x : nullptr;
  if constexpr (CL) {
    cl[0] = 0.0;
    cl[FB] = 0.0;
    cl[2 * FB] = 0.0;
  }

  // shift register of the non-terminal levels' colour inputs (slot 0 = most recent level), or,
  // levels_in_lds, LDS slots indexed by the level (slot j = level kb + j)
  constexpr bool LV = LVL && LDS && B > 0 && !kForwardFold;
  constexpr int NS = B > 0 ? B : 1;
  constexpr int NL = LV ? level_lds_slots<(DEEP != 0)>(B) : 0;  // levels 0..NL-1 in LDS, NL..B-1 in registers
  constexpr int NR = LV ? (B > NL ? B - NL : 1) : NS;
  double sDli[NR], sDi[NR], sSpec[NR], sVa[NR];
  int sKey[NR];  // hit sphere | checker bit << 16
  double* const lvd = LV ? const_cast<double*>(lds_tab) + nsph * kSphWords : nullptr;  // [NL][4][FB]
  int* const lvk = LV ? (int*)(lvd + NL * 4 * FB) : nullptr;                          // [NL][FB]
  const int lt = threadIdx.x;
  int depth = 0;
  double cr = 0.0, cg = 0.0, cb = 0.0;
  // kForwardFold (capped kernels): colour accumulated level by level, thr = T_k
  constexpr bool FWD = kForwardFold;
  double thr = 1.0;
  if constexpr (FWD && DEEP == 2) {  // a continued chain: its colour so far and the next level's weight
    if (rin) {
      cr = rin[6];
      cg = rin[7];
      cb = rin[8];
      thr = rin[9];
    }
  }
  bool deferred = false, appended = false;
  int rays_through = 0, hits_through = -1;  // per-level counts already made for this pixel

  for (int k = 0;; ++k) {
    if (hit < 0) {  // nothing hit: NumpyRGBColor(0, 0, 0) (base.py:100)
      if constexpr (!FWD) cr = cg = cb = 0.0;  // (forwards: a black reflection adds nothing)
      break;
    }
    if (tie) {  // several shapes shaded and summed: the general kernel takes this ray
      deferred = true;
      rays_through = kb + k;
      hits_through = kb + k - 1;
      if (st && !(p.mode == 3 && kb + k == 0)) stat_add(st, RTX_S_TIES, 1);  // (not the RTX_H_MAT0 deferral)
      break;
    }
    Hit s;
    if constexpr (LDS) {
      shade<IMG, TREE>(sc, geo, (const double*)lds_tab, nsph, hit, ox, oy, oz, dx, dy, dz, tmin, s, tame, wk);
    } else {
      shade<IMG, TREE>(sc, geo, p.scene + RTX_HDR_WORDS, nsph, hit, ox, oy, oz, dx, dy, dz, tmin, s, tame, wk);
    }
    if (s.tk < 0) {  // an image-textured sphere: so is this one (the texel lookup stays out of here)
      deferred = true;
      rays_through = kb + k;
      hits_through = kb + k - 1;
      break;
    }
    if (st && kb + k < RTX_S_LEVELS) {
      stat_add(st, RTX_S_HITS + kb + k, 1);
      stat_wave(st, RTX_S_WSHADE + kb + k);
    }
    const bool weighted = s.lit && s.g != 0.0;
    // the cap itself (absolute level; a continuation pass may run into a cap of 9 or 10)
    const bool at_cap = DEEP && p.max_bounces >= 0 && kb + k >= p.max_bounces;
    if (!FWD && DEEP && weighted && k >= B && !at_cap) {  // the chain goes on beyond this kernel's levels
      // k == B: levels kb..kb+B-1 are in the shift register (slot j = level kb+B-1-j), kb+B in s
      deferred = true;
      appended = true;
      rays_through = hits_through = kb + B;
      const int64_t slot =
          append_deferred(p, deferred_entry(DEEP == 2 || !TREE ? i : pixel_index(lane_id_fresh()), p.frame, kb + B, kb + B));
      if (p.drec && slot >= 0 && slot < p.rec_cap && kb + B == p.drec_level) {
        double* rec = p.drec + slot * rec_words(kb + B);
        double rx = dx, ry = dy, rz = dz;
        reflect_dir(rx, ry, rz, s.nx, s.ny, s.nz);
        rec[0] = s.qx; rec[1] = s.qy; rec[2] = s.qz;
        rec[3] = rx; rec[4] = ry; rec[5] = rz;
        for (int w = 0; w < kRecLevelWords * kb; ++w) rec[6 + w] = rin[6 + w];  // levels 0..kb-1
        double* lv = rec + 6 + kRecLevelWords * (kb + B);
        lv[0] = s.dli; lv[1] = s.di; lv[2] = s.spec; lv[3] = s.va; lv[4] = (double)level_key(hit, s.tk);
        if constexpr (LV) {  // LDS slot d = level kb + d (a DEEP kernel keeps all B levels there)
          static_assert(!LV || !DEEP || NL == B, "DEEP level slots");
          for (int d = 0; d < NL; ++d) {
            const double* const l = lvd + (d * 4) * FB + lt;
            double* lj = rec + 6 + kRecLevelWords * (kb + d);
            lj[0] = l[0]; lj[1] = l[FB]; lj[2] = l[2 * FB]; lj[3] = l[3 * FB];
            lj[4] = (double)lvk[d * FB + lt];
          }
        } else if constexpr (B > 0) {
#pragma unroll
          for (int j = 0; j < NS; ++j) {
            double* lj = rec + 6 + kRecLevelWords * (kb + B - 1 - j);
            lj[0] = sDli[j]; lj[1] = sDi[j]; lj[2] = sSpec[j]; lj[3] = sVa[j]; lj[4] = (double)sKey[j];
          }
        }
      }
      break;
    }
    if (FWD) {
      // this level's colour with a black reflection, weighted by the chain's throughput (at level 0
      // cr = 0 + 1 * L_0 = L_0 exactly: a chain of one level is bit-identical to the backward fold)
      const double* tab = LDS ? (const double*)lds_tab : p.scene + RTX_HDR_WORDS;
      double lr_, lg_, lb_;
      hit_color<IMG>(tab + nsph * RTX_GEOM_WORDS + hit * RTX_MAT_WORDS, sc, s.dli, s.di, s.tk, s.lit, weighted, s.spec,
                     s.va, 0.0, 0.0, 0.0, lr_, lg_, lb_);
      if constexpr (CL) {
        cl[0] = __builtin_fma(thr, lr_, cl[0]);
        cl[FB] = __builtin_fma(thr, lg_, cl[FB]);
        cl[2 * FB] = __builtin_fma(thr, lb_, cl[2 * FB]);
      } else {
        cr = __builtin_fma(thr, lr_, cr);
        cg = __builtin_fma(thr, lg_, cg);
        cb = __builtin_fma(thr, lb_, cb);
      }
      // a DEEP launch goes on to its record level (the first pass: level B; the continuation pass:
      // kDeepLevel3, the registers holding nothing per level), then defers the chain with a record
      const int kmax = DEEP ? p.drec_level - kb : B;
      if (DEEP && weighted && k >= kmax && !at_cap) {  // the chain goes on beyond this launch's levels
        deferred = true;
        appended = true;
        rays_through = hits_through = kb + kmax;
        const int64_t slot = append_deferred(p, deferred_entry(DEEP == 2 || !TREE ? i : pixel_index(lane_id_fresh()),
                                                               p.frame, kb + kmax, kb + kmax));
        if (p.drec && slot >= 0 && slot < p.rec_cap) {
          double* rec = p.drec + slot * rec_words(kb + kmax);
          double rx = dx, ry = dy, rz = dz;
          reflect_dir(rx, ry, rz, s.nx, s.ny, s.nz);
          rec[0] = s.qx; rec[1] = s.qy; rec[2] = s.qz;
          rec[3] = rx; rec[4] = ry; rec[5] = rz;
          rec[6] = cr; rec[7] = cg; rec[8] = cb;
          rec[9] = (thr * 0.5) * s.g;  // the next level's weight, as below
        }
        break;
      }
      if (!weighted || k >= kmax || at_cap) break;
      thr = (thr * 0.5) * s.g;  // the reflection's weight, (R * 0.5) * g (shader.py:106)
    } else if (!weighted || k >= B || at_cap) {
      // terminal level: the reflection is black (capped: R = 0) or multiplied by zero
      const double* tab = LDS ? (const double*)lds_tab : p.scene + RTX_HDR_WORDS;
      hit_color<IMG>(tab + nsph * RTX_GEOM_WORDS + hit * RTX_MAT_WORDS, sc, s.dli, s.di, s.tk, s.lit, weighted, s.spec,
                s.va, 0.0, 0.0, 0.0, cr, cg, cb);
      break;
    }
    // push this level's colour inputs; the reflected ray becomes the next level
    if constexpr (FWD) {
      // (nothing to keep: the level's colour is already in cr, cg, cb)
    } else if constexpr (LV) {
      if (NL == B || k < NL) {  // k: wave-uniform, == depth of every active lane
        double* const l = lvd + (depth * 4) * FB + lt;
        l[0] = s.dli; l[FB] = s.di; l[2 * FB] = s.spec; l[3 * FB] = s.va;
        lvk[depth * FB + lt] = level_key(hit, s.tk);
      } else {  // levels beyond the LDS slots: a register shift (slot 0 = the most recent)
#pragma unroll
        for (int j = NR - 1; j > 0; --j) {
          sDli[j] = sDli[j - 1]; sDi[j] = sDi[j - 1]; sSpec[j] = sSpec[j - 1]; sVa[j] = sVa[j - 1];
          sKey[j] = sKey[j - 1];
        }
        sDli[0] = s.dli; sDi[0] = s.di; sSpec[0] = s.spec; sVa[0] = s.va;
        sKey[0] = level_key(hit, s.tk);
      }
    } else {
#pragma unroll
      for (int j = NS - 1; j > 0; --j) {
        sDli[j] = sDli[j - 1]; sDi[j] = sDi[j - 1]; sSpec[j] = sSpec[j - 1]; sVa[j] = sVa[j - 1];
        sKey[j] = sKey[j - 1];
      }
      sDli[0] = s.dli; sDi[0] = s.di; sSpec[0] = s.spec; sVa[0] = s.va;
      sKey[0] = level_key(hit, s.tk);
    }
    if constexpr (!FWD) ++depth;
    reflect_dir(dx, dy, dz, s.nx, s.ny, s.nz);
    ox = s.qx;
    oy = s.qy;
    oz = s.qz;
    if (st && kb + k + 1 < RTX_S_LEVELS) {
      stat_add(st, RTX_S_RAYS + kb + k + 1, 1);
      stat_wave(st, RTX_S_WTRACE + kb + k + 1);
    }
    [[maybe_unused]] uint32_t tests0 = 0, nodes0 = 0;
    if constexpr (STATS) {
      tests0 = wk.tests;
      nodes0 = wk.nodes;
    }
    if (TREE && sc[RTX_H_NNODES] != 0.0) {
      // the wave's beam candidates (tame scenes up to 128 spheres), else the culling tree
      Beam bm;
      const double* btab = LDS ? (const double*)lds_tab : p.scene + RTX_HDR_WORDS;
      if (BEAM && sc[RTX_H_TAME] != 0.0 && wave_beam<kBeamStaged && LDS>(btab, nb, ox, oy, oz, dx, dy, dz, bm)) {
        if (st) stat_wave(st, RTX_S_BEAMW);
        for (int j = 0; j < bm.passes; ++j) wk.beam();  // a lane's cone test of one sphere per pass
        nearest_beam(geo, nsph, bm, ox, oy, oz, dx, dy, dz, tmin, hit, tie, tame, wk);
      } else {
        nearest_bvh<false>(sc, ox, oy, oz, dx, dy, dz, tmin, hit, tie, tame, wk);
      }
    } else if constexpr (LDS) {
      nearest_hit<false>(geo, nsph, ox, oy, oz, dx, dy, dz, tmin, hit, tie, tame, wk);
    } else {
      nearest_hit<false>(geo, nsph, ox, oy, oz, dx, dy, dz, tmin, hit, tie, tame, wk);
    }
    if constexpr (STATS) {
      wk.tests1 += wk.tests - tests0;
      wk.nodes1 += wk.nodes - nodes0;
    }
  }

  if constexpr (STATS) {
    if (st) {
      stat_add(st, RTX_S_TESTS, wk.tests);
      stat_add(st, RTX_S_NODES, wk.nodes);
      stat_add(st, RTX_S_TESTS1, wk.tests1);
      stat_add(st, RTX_S_NODES1, wk.nodes1);
      stat_add(st, RTX_S_BOXES, wk.boxes);
      stat_add(st, RTX_S_BEAMT, wk.beamt);
    }
  }
  const int64_t io = DEEP == 2 || !TREE ? i : pixel_index(lane_id_fresh());
  if constexpr (CL) {
    cr = cl[0];
    cg = cl[FB];
    cb = cl[2 * FB];
  }
  if (deferred) {
    // a tie (deep deferrals were appended with their resume record)
    if (!appended) append_deferred(p, deferred_entry(io, p.frame, rays_through, hits_through));
    if (st && !rin) stat_add(st, RTX_S_DEFERRED, 1);
    return;
  }
  // fold back (shader.py:106-110): col_k = ((A_k + (spec_k + col_{k+1}*0.5) * g_k) + I_k); the
  // stored levels were lit with g != 0
  const double* mtab = (LDS ? (const double*)lds_tab : p.scene + RTX_HDR_WORDS) + nsph * RTX_GEOM_WORDS;
  if constexpr (LV) {
    if constexpr (NL < B) {
      for (int d = depth - 1; d >= NL; --d) {  // the register levels first (the deepest)
        const int key = sKey[0];
        hit_color<IMG>(mtab + key_hit(key) * RTX_MAT_WORDS, sc, sDli[0], sDi[0], key_tex(key), true, true,
                  sSpec[0], sVa[0], cr, cg, cb, cr, cg, cb);
#pragma unroll
        for (int j = 0; j < NR - 1; ++j) {
          sDli[j] = sDli[j + 1]; sDi[j] = sDi[j + 1]; sSpec[j] = sSpec[j + 1]; sVa[j] = sVa[j + 1];
          sKey[j] = sKey[j + 1];
        }
      }
    }
    for (int d = (depth < NL ? depth : NL) - 1; d >= 0; --d) {
      const double* const l = lvd + (d * 4) * FB + lt;
      const int key = lvk[d * FB + lt];
      hit_color<IMG>(mtab + key_hit(key) * RTX_MAT_WORDS, sc, l[0], l[FB], key_tex(key), true, true,
                l[2 * FB], l[3 * FB], cr, cg, cb, cr, cg, cb);
    }
  } else {
    for (int d = 0; d < depth; ++d) {
      const int key = sKey[0];
      hit_color<IMG>(mtab + key_hit(key) * RTX_MAT_WORDS, sc, sDli[0], sDi[0], key_tex(key), true, true, sSpec[0],
                sVa[0], cr, cg, cb, cr, cg, cb);
#pragma unroll
      for (int j = 0; j < NS - 1; ++j) {
        sDli[j] = sDli[j + 1]; sDi[j] = sDi[j + 1]; sSpec[j] = sSpec[j + 1]; sVa[j] = sVa[j + 1];
        sKey[j] = sKey[j + 1];
      }
    }
  }
  if constexpr (DEEP && !FWD) {  // a continued chain: fold on through the levels of its record (same fold)
    for (int l = kb - 1; l >= 0; --l) {
      const double* lv = rin + 6 + kRecLevelWords * l;
      const int key = (int)lv[4];
      hit_color<IMG>(mtab + key_hit(key) * RTX_MAT_WORDS, sc, lv[0], lv[1], key_tex(key), true, true, lv[2], lv[3],
                cr, cg, cb, cr, cg, cb);
    }
  }
  write_out(p, io, cr, cg, cb);
}

// TP: 0 = no culling tree and no persistent launch (scenes below kTreeMinSpheres), 1 = culling tree,
// one tile per block (the launch is not persistent), 2 = both (persistent launches)
// DEEP: 0 capped (the chain ends at level B), 1 the first pass of an uncapped render (chains alive at
// its record level are deferred with a resume record), 2 a continuation pass (mode 2: chains resumed
// from their records; its own instantiation, so that the first pass compiles no resume code)
template <int B, bool LDS, int DEEP, bool LVL, bool STATS, int TP, bool IMG, int NSPH>
__device__ __forceinline__ void k_render_fast_tiles(const Params& p, const double* lds_tab);

// WAVES > 0: that many waves/SIMD instead of the rule below (kFwdWavesLarge)
template <int B, bool LDS, int DEEP, bool LVL = levels_in_lds<B, LDS, (DEEP != 0)>(), bool STATS = false, int TP = 2,
          bool IMG = false, int NSPH = 0, int WAVES = 0>
__global__ __launch_bounds__(fast_block<(TP >= 1)>(),
                             WAVES > 0 ? WAVES
                             : (DEEP  ? (TP >= 2 || DEEP == 2 ? kDeepWaves : kDeepWavesTile)
                              : LVL ? (B >= 5 ? kB5Waves : TP ? kLvWaves : kLvWavesSmall)
                              : kForwardFold ? (TP >= 2 ? kFwdWavesPersist : TP ? kFwdWaves : kFwdWavesSmall)
                                             : kFastWavesPerSimd)) void k_render_fast(Params p0) {
  constexpr bool TREE = TP >= 1;
  // reflected-ray beams (wave_beam): the persistent launches, scenes of kPersistMinSpheres and more
  // (A/B: C4 -5.3%; with 16 spheres the tree walk is cheaper than the beam, C3 +7%, C5 +4%), capped
  // or not (the DEEP first pass since round 6, with kDeepWaves 4: A/B r6ap, unbounded C4 2,101 ->
  // 1,800 us)
  constexpr bool BEAM = TP >= 2;
  extern __shared__ double lds_tab[];
  const Params p = frame_view(p0, blockIdx.z);  // frame of a multi-frame launch (grid z)
  {
    // a blob that is not a packed scene of p.nsph spheres (the LDS table and every sphere loop are
    // sized by p.nsph): render nothing and flag it (block-uniform, so the persistent launch's
    // fetch counters stay untouched)
    const cdouble* sc = (const cdouble*)p.scene;
    if (sc[RTX_H_MAGIC] != RTX_MAGIC || sc[RTX_H_NSPH] != (double)p.nsph || (NSPH > 0 && p.nsph != NSPH)) {
      if (threadIdx.x == 0) atomicOr((uint32_t*)p.ws + RTX_WS_STATUS, (uint32_t)RTX_ST_BAD_SCENE);
      return;
    }
  }
  if constexpr (LDS) {  // per-lane view of the sphere table: one LDS copy per block (the barrier is
                        // in fast_tile, after the first tile's level-0 nearest-hit test)
    const double* src = p.scene + RTX_HDR_WORDS;
    for (int k = threadIdx.x; k < p.nsph * kSphWords; k += fast_block<TREE>()) {
      // (the beam kernels: geometry word RTX_G_IDX of the copy holds beam_word, see wave_beam)
      const bool bw = BEAM && kBeamStaged && k < p.nsph * RTX_GEOM_WORDS && (k & (RTX_GEOM_WORDS - 1)) == RTX_G_IDX;
      lds_tab[k] = bw ? beam_word(src[k - RTX_G_IDX + RTX_G_CC], src[k - RTX_G_IDX + RTX_G_RR]) : src[k];
    }
  }
  if constexpr (DEEP == 2) {  // continuation pass (mode 2): 256 entries of in_list per tile, grid-stride
    const int64_t count = (int64_t)*p.in_count;
    for (int64_t t = blockIdx.x; t * fast_block<TREE>() < count; t += gridDim.x) {
      fast_tile<B, LDS, DEEP, LVL, STATS, TREE, BEAM, IMG, NSPH>(p, (int)t, 0, t == (int64_t)blockIdx.x, lds_tab);
    }
  } else {
    k_render_fast_tiles<B, LDS, DEEP, LVL, STATS, TP, IMG, NSPH>(p, lds_tab);
  }
}

// the camera / explicit-ray launches of k_render_fast (every instantiation but the continuation's)
template <int B, bool LDS, int DEEP, bool LVL, bool STATS, int TP, bool IMG, int NSPH>
__device__ __forceinline__ void k_render_fast_tiles(const Params& p, const double* lds_tab) {
  constexpr bool TREE = TP >= 1;
  constexpr bool BEAM = TP >= 2;
  if (TP >= 2 && p.n_fetch > 0) {  // (persistent launches are for scenes of kPersistMinSpheres and more)
    // Persistent waves fetching kWaveW x kWaveH tiles, bottom-up (longest work first, as below).
    // Counter c (of n_fetch) hands out tiles c, c + n_fetch, ... . Waves are numbered XCD-major
    // (pw; block b runs on XCD b % 8) and wave pw uses counter pw % n_fetch, so every counter's
    // waves are spread over all XCDs. Wave pw renders tile pw first (static, no fetch); the next
    // tile's atomic is always issued before the current tile renders, hiding its latency. Each
    // wave makes exactly one out-of-range fetch, so the wave receiving a counter's last value is
    // its last user and resets it to 0 for the next launch (no per-launch memset).
    if constexpr (LDS) __syncthreads();  // the table staged above
    const int lane = threadIdx.x & 63;
    const int nc = p.n_fetch;
    const int nx = (gridDim.x % 8 == 0) ? 8 : 1;
    const int pw = ((int)(blockIdx.x % nx) * (int)(gridDim.x / nx) + (int)(blockIdx.x / nx)) * kFastWaves +
                   (threadIdx.x >> 6);
    const int waves_c = (int)(gridDim.x * kFastWaves) / nc;  // the host makes nc divide the waves per XCD
    const int c = pw % nc;
    const int nt = p.n_tiles_x * p.n_tiles_y;
    const int tiles_c = (nt - c + nc - 1) / nc;
    uint32_t* const ctr = p.fetch + c * kFetchStride;
    uint32_t nxt = 0;
    if (lane == 0) nxt = atomicAdd(ctr, 1u);
    int k = pw / nc;
    int v = 0;
    // the host's dispatch order (longest tiles first, learnt from an earlier launch's tile_cost), read
    // through the scalar cache: the index is wave-uniform
    const uint32_t __attribute__((address_space(4)))* const order =
        (const uint32_t __attribute__((address_space(4)))*)p.tile_order;
    while (k < tiles_c) {
      const int t = order ? (int)order[c + k * nc] : c + k * nc;
      // (an order entry outside the launch's tiles — a stale or foreign order buffer — renders nothing
      // rather than writing outside the frame)
      if ((unsigned)t < (unsigned)nt) {
        const int row = t / p.n_tiles_x;
        // the tile's time as -start + end in its cost word. Cost records are kept to the STATS
        // instantiations (run_render picks one for a launch that records them): in the timed kernel
        // the record costs C4 six more spilled VGPRs and 2.5% (A/B r4h)
        if (STATS && p.tile_cost && lane == 0) p.tile_cost[t] = 0u - (uint32_t)__builtin_amdgcn_s_memrealtime();
        fast_tile<B, LDS, DEEP, LVL, STATS, TREE, BEAM, IMG, NSPH>(p, t - row * p.n_tiles_x, p.n_tiles_y - 1 - row, false,
                                                              lds_tab, true);
        if (STATS && p.tile_cost && lane == 0) atomicAdd(p.tile_cost + t, (uint32_t)__builtin_amdgcn_s_memrealtime());
      }
      v = __builtin_amdgcn_readfirstlane(nxt);
      k = waves_c + v;
      if (k < tiles_c && lane == 0) nxt = atomicAdd(ctr, 1u);
    }
    if (k == pw / nc) v = __builtin_amdgcn_readfirstlane(nxt);  // no tile rendered: the first fetch
    const int dyn = tiles_c > waves_c ? tiles_c - waves_c : 0;  // in-range fetches on this counter
    if (lane == 0 && v == dyn + waves_c - 1) atomicExch(ctr, 0u);
    return;
  }
  // one tile per block. Bottom tile rows are dispatched first: they hold the ground and the
  // spheres, whose pixels run long bounce chains, while sky rows finish at level 0 and so fill the
  // end of the grid (longest-first order; A/B: C2 -10%, C5 -8%, C4 -2%). Output does not depend on
  // the order. Blocks are dispatched in blockIdx order: a host order (camera launches,
  // rtx_render_camera_sched) maps dispatch slot b to block tile order[b], block tile t being
  // (t % gridDim.x, bottom-up row t / gridDim.x), and a cost record takes each block's time.
  const uint64_t t_entry = STATS && p.tile_cost ? __builtin_amdgcn_s_memrealtime() : 0;  // (learning the order)
  int bx = blockIdx.x, by = gridDim.y - 1 - blockIdx.y, tb = blockIdx.y * gridDim.x + blockIdx.x;
  if (p.tile_order) {
    tb = (int)((const uint32_t __attribute__((address_space(4)))*)p.tile_order)[tb];
    if ((unsigned)tb >= gridDim.x * gridDim.y) return;  // (block-uniform: a stale order renders nothing)
    bx = tb % gridDim.x;
    by = gridDim.y - 1 - tb / gridDim.x;
  }
  fast_tile<B, LDS, DEEP, LVL, STATS, TREE, BEAM, IMG, NSPH>(p, bx, by, true, lds_tab);
  if (STATS && p.tile_cost && (threadIdx.x & 63) == 0)  // the block's time: the slowest of its waves
    atomicMax(p.tile_cost + tb, (uint32_t)(__builtin_amdgcn_s_memrealtime() - t_entry));
}

// ------------------------------------------------------------------------------------------
// k_render_general: explicit depth-first ray tree (ties and any bounce cap)
// ------------------------------------------------------------------------------------------

// frame fields: the ray, its nearest distance, the next shape to examine (-1: new ray), the
// weight of its hits (the product of (0.5 g) along the path to it), the hit whose reflection is
// being traced, and the hits of the ray not yet shaded.
enum { F_OX = 0, F_OY, F_OZ, F_DX, F_DY, F_DZ, F_TMIN, F_NEXT, F_THR, F_KEY, F_LEFT };
static_assert(F_LEFT < kFrameWords, "frame layout");

struct Stack {
  double* base;
  int64_t nw;
  int64_t w;
  __device__ __forceinline__ double& at(int d, int f) const { return base[((int64_t)d * kFrameWords + f) * nw + w]; }
};

// rays_through / hits_through: per-level counts the fast kernel already made for this pixel.
// The walk sums every shaded hit's colour with a black reflection, weighted by the product of
// (0.5 g) along its path (shader.py:106-110 unrolled: the sum over the tree of hits, ties included,
// base.py:100-119), in depth-first order: on a chain without ties these are the fast kernels'
// forward-fold operations in their order, so a pixel's colour does not depend on which kernel
// traced which of its levels. rec: a resume record (deep deferral: the next ray, the colour summed
// through level L and level L + 1's weight), the walk starting at depth L + 1; or null.
template <typename Stk>
__device__ void trace_general(const Params& p, const Stk& S, double ox0, double oy0, double oz0, double dx0,
                              double dy0, double dz0, double& cr, double& cg, double& cb, int rays_through,
                              int hits_through, const double* rec = nullptr, int h_given = -1,
                              double t_given = 0.0) {
  static_assert(kForwardFold, "the general kernel sums forwards, like the fast kernels");
  const cdouble* sc = (const cdouble*)p.scene;
  const cdouble* geo = sc + RTX_HDR_WORDS;
  const double* tab = p.scene + RTX_HDR_WORDS;
  const double* mtab = tab + p.nsph * RTX_GEOM_WORDS;
  const int nsph = p.nsph;
  const int B = p.max_bounces;  // < 0: unbounded (bounded by the stack depth)
  // Shader.create on another shape's shader: level 0 shades with that material (RTX_H_MAT0)
  const double* mat0 = (h_given >= 0 && sc[RTX_H_MAT0] != 0.0) ? p.scene + (int64_t)sc[RTX_H_MAT0] : nullptr;
  unsigned long long* st = p.stats;

  int d = 0;
  double ar = 0.0, ag = 0.0, ab = 0.0, thr0 = 1.0;
  if (rec) {
    d = rays_through + 1;
    ar = rec[6];
    ag = rec[7];
    ab = rec[8];
    thr0 = rec[9];
    ox0 = rec[0]; oy0 = rec[1]; oz0 = rec[2];
    dx0 = rec[3]; dy0 = rec[4]; dz0 = rec[5];
  }
  const int d0 = d;  // the depth whose finished ray ends the walk
  S.at(d, F_OX) = ox0; S.at(d, F_OY) = oy0; S.at(d, F_OZ) = oz0;
  S.at(d, F_DX) = dx0; S.at(d, F_DY) = dy0; S.at(d, F_DZ) = dz0;
  S.at(d, F_NEXT) = -1.0;
  S.at(d, F_THR) = thr0;
  for (;;) {
    const double ox = S.at(d, F_OX), oy = S.at(d, F_OY), oz = S.at(d, F_OZ);
    const double dx = S.at(d, F_DX), dy = S.at(d, F_DY), dz = S.at(d, F_DZ);
    const double oo = dot3(ox, oy, oz, ox, oy, oz);
    const int next = (int)S.at(d, F_NEXT);
    double tmin;
    int left;   // hits of this ray not yet shaded, this one included
    int h = nsph;  // the shape shaded now (nsph: the ray is done)
    if (next < 0) {  // new ray: nearest distance (base.py:97-98) and its first shape in scene order
      if (st && d < RTX_S_LEVELS && d > rays_through) stat_add(st, RTX_S_RAYS + d, 1);
      tmin = FARAWAY;
      int nh = 0, first = nsph;
      if (d == 0 && h_given >= 0) {  // Shader.create's ray: the level-0 hit is given
        tmin = t_given;
        nh = 1;
        first = h_given;
      } else if (sc[RTX_H_NNODES] != 0.0 && nsph >= kGeneralTreeMin) {
        nearest_count_bvh(sc, ox, oy, oz, oo, dx, dy, dz, tmin, nh, first);
      } else {
        for (int s = 0; s < nsph; ++s) {
          const double t = isect(tab + s * RTX_GEOM_WORDS, ox, oy, oz, oo, dx, dy, dz);
          if (t < tmin) {
            tmin = t;
            nh = 1;
            first = s;
          } else if (t == tmin && t != FARAWAY) {
            ++nh;
          }
        }
      }
      if (st && nh > 1 && d > rays_through) stat_add(st, RTX_S_TIES, 1);
      left = (tmin != FARAWAY || (d == 0 && h_given >= 0)) ? nh : 0;  // (nearest != FARAWAY) & (t == nearest), base.py:102-103
      S.at(d, F_TMIN) = tmin;
      S.at(d, F_LEFT) = (double)left;
      if (left > 0) h = first;
    } else {
      tmin = S.at(d, F_TMIN);
      left = (int)S.at(d, F_LEFT);
      if (left > 0) {  // a tie: the next shape (scene order) with t == nearest
        for (int s = next; s < nsph; ++s) {
          if (isect(tab + s * RTX_GEOM_WORDS, ox, oy, oz, oo, dx, dy, dz) == tmin) {
            h = s;
            break;
          }
        }
      }
    }
    if (h == nsph) {  // this ray is done (its hits' colours are in the sum)
      if (d == d0) {
        cr = ar; cg = ag; cb = ab;
        return;
      }
      --d;  // back to the parent ray: on to its next hit
      S.at(d, F_NEXT) = (double)(key_hit((int)S.at(d, F_KEY)) + 1);
      S.at(d, F_LEFT) = S.at(d, F_LEFT) - 1.0;
      continue;
    }
    if (st && d < RTX_S_LEVELS && d > hits_through) stat_add(st, RTX_S_HITS + d, 1);
    Hit s;
    Work<false> nowk;
    shade<true>(sc, geo, tab, nsph, h, ox, oy, oz, dx, dy, dz, tmin, s, __builtin_nan(""), nowk,
                d == 0 ? mat0 : nullptr);
    const bool weighted = s.lit && s.g != 0.0;
    bool descend = weighted && (B < 0 || d < B);
    if (descend && d + 1 >= p.stack_levels) {  // deeper than the stack: RecursionError on the host
      atomicOr((uint32_t*)p.ws + RTX_WS_STATUS, (uint32_t)RTX_ST_STACK_OVERFLOW);
      descend = false;
    }
    // this hit's colour with a black reflection, weighted (the fast kernels' forward fold)
    const double thr = S.at(d, F_THR);
    double xr, xg, xb;
    hit_color<true>((d == 0 && mat0) ? mat0 : mtab + h * RTX_MAT_WORDS, sc, s.dli, s.di, s.tk, s.lit, weighted,
                    s.spec, s.va, 0.0, 0.0, 0.0, xr, xg, xb);
    ar = __builtin_fma(thr, xr, ar);
    ag = __builtin_fma(thr, xg, ag);
    ab = __builtin_fma(thr, xb, ab);
    if (!descend) {
      S.at(d, F_NEXT) = (double)(h + 1);
      S.at(d, F_LEFT) = (double)(left - 1);
      continue;
    }
    S.at(d, F_KEY) = (double)level_key(h, s.tk);
    double rx = dx, ry = dy, rz = dz;
    reflect_dir(rx, ry, rz, s.nx, s.ny, s.nz);
    ++d;
    S.at(d, F_OX) = s.qx; S.at(d, F_OY) = s.qy; S.at(d, F_OZ) = s.qz;
    S.at(d, F_DX) = rx; S.at(d, F_DY) = ry; S.at(d, F_DZ) = rz;
    S.at(d, F_NEXT) = -1.0;
    S.at(d, F_THR) = (thr * 0.5) * s.g;  // the reflection's weight, (R * 0.5) * g (shader.py:106)
  }
}

__global__ __launch_bounds__(64) void k_render_general(Params p0) {
  const int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const Params& p = p0;
  uint32_t* hdr = (uint32_t*)p.ws;
  // Nothing deferred in this launch (the rule for capped renders): every counter is already zero,
  // so there is nothing to render and nothing to reset, and no block touches the done counter
  // (its 64 returning atomics on one address were most of this launch's 5 us).
  if (p.deferred_out && blockIdx.x == 0 && threadIdx.x == 0) *p.deferred_out = hdr[RTX_WS_COUNT];  // before any reset
  if (hdr[RTX_WS_COUNT] == 0u && hdr[RTX_WS_COUNT2] == 0u && hdr[RTX_WS_COUNT3] == 0u) return;
  int64_t count = (int64_t)*p.in_count;
  if (count > p.list_cap) count = p.list_cap;
  const uint64_t* list = p.in_list;
  if (w < p.n_workers) {
    Stack S{p.stack, p.n_workers, w};
    for (int64_t item = w; item < count; item += p.n_workers) {
      const uint64_t e = list[item];
      const int64_t i = (int64_t)(e & ((uint64_t(1) << kFrameShift) - 1));
      const int f = (int)((e >> kFrameShift) & 0xFFFF);
      const int rays_through = (int)((e >> kRaysShift) & kLevelMask) - 1;
      const int hits_through = (int)((e >> kHitsShift) & kLevelMask) - 1;
      // The scene is read through the scalar cache (wave-uniform pointers) while a wave's lanes may
      // hold rays of different frames of a multi-frame launch: lanes sharing the first active
      // lane's frame run together, then the next frame (a waterfall over the wave's frames).
      for (bool todo = true; todo;) {
        const int f0 = __builtin_amdgcn_readfirstlane(f);
        if (f == f0) {
          const Params q = frame_view(p0, f0);
          // a chain deferred for depth (rays and hits counted through the same level) resumes from
          // its record when it has one
          const bool resume = p.in_rec && rays_through == p.in_level && hits_through == rays_through &&
                              item < p.in_rec_cap;
          double ox = 0.0, oy = 0.0, oz = 0.0, dx = 0.0, dy = 0.0, dz = 0.0;
          if (!resume) load_ray(q, i, ox, oy, oz, dx, dy, dz);
          double cr, cg, cb;
          const bool given = q.mode == 3;
          trace_general(q, S, ox, oy, oz, dx, dy, dz, cr, cg, cb, rays_through, hits_through,
                        resume ? p.in_rec + item * rec_words(p.in_level) : nullptr, given ? q.hit_shape : -1,
                        given ? q.hit_t[i] : 0.0);
          write_out(q, i, cr, cg, cb);
          todo = false;
        }
      }
    }
  }
  // leave the workspace clean for the next call: the last block to finish zeroes the counter
  // (every block has read it before arriving; the next kernel on the stream sees the store)
  __syncthreads();
  if (threadIdx.x == 0) {
    if (gridDim.x == 1) {  // one block: no other reader of the counters
      hdr[RTX_WS_COUNT] = 0u;
      hdr[RTX_WS_COUNT2] = 0u;
      hdr[RTX_WS_COUNT3] = 0u;
    } else if (atomicAdd(hdr + RTX_WS_DONE, 1u) == gridDim.x - 1) {
      hdr[RTX_WS_COUNT] = 0u;
      hdr[RTX_WS_COUNT2] = 0u;
      hdr[RTX_WS_COUNT3] = 0u;
      hdr[RTX_WS_DONE] = 0u;
    }
  }
}

// ------------------------------------------------------------------------------------------
// boundary helpers
// ------------------------------------------------------------------------------------------

__global__ __launch_bounds__(kBlock) void k_ray_dirs(Params p, double* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= p.n) return;
  const int lr = (int)(i / p.width), col = (int)(i % p.width);
  double dx, dy, dz;
  camera_dir((const cdouble*)p.scene, col, global_row(p, lr), p.width, p.height, dx, dy, dz);
  out[i] = dx;
  out[p.n + i] = dy;
  out[2 * p.n + i] = dz;
}

__global__ __launch_bounds__(kBlock) void k_intersect(const double* __restrict__ g, const double* __restrict__ org,
                                                      int64_t s, const double* __restrict__ dir, int64_t n,
                                                      double* __restrict__ t) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const int64_t j = s ? i : 0;
  const double ox = org[j], oy = org[s + j + (s ? 0 : 1)], oz = org[2 * s + j + (s ? 0 : 2)];
  const double dx = dir[i], dy = dir[n + i], dz = dir[2 * n + i];
  t[i] = isect(g, ox, oy, oz, dot3(ox, oy, oz, ox, oy, oz), dx, dy, dz);
}

// bit-exactness check of the sqrt / division fast paths against the compiler's full expansions
__global__ __launch_bounds__(kBlock) void k_selftest_math(const double* __restrict__ a, const double* __restrict__ b,
                                                          int64_t n, double* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const double x = a[i], y = b[i];
  out[i] = sqrt_cr(x);
  out[n + i] = __builtin_sqrt(x);
  out[2 * n + i] = div_cr(x, y);
  out[3 * n + i] = x / y;
  out[4 * n + i] = inv_mag_unit(x);  // the closed form where every lane of the wave is near 1
  out[5 * n + i] = 1.0 / (x == 0.0 ? 1.0 : __builtin_sqrt(x));
}

template <typename T>
__global__ __launch_bounds__(kBlock) void k_quantize(const T* __restrict__ c, int64_t n, uint8_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  out[3 * i + 0] = quant_u8((double)c[i]);
  out[3 * i + 1] = quant_u8((double)c[n + i]);
  out[3 * i + 2] = quant_u8((double)c[2 * n + i]);
}

// Rows of the run of `run` parts from part p of the interleaved row tiling (python_ray_tracer_amd/
// tiling.py n_local_rows): run * row_block rows of every cycle, the last cycle's prefix.
__host__ __device__ __forceinline__ int tile_local_rows(int height, int row_block, int n_parts, int p, int run = 1) {
  const int cycle = row_block * n_parts, own = row_block * run;
  const int q = height / cycle, rem = height % cycle - p * row_block;
  return q * own + (rem < 0 ? 0 : rem > own ? own : rem);
}
// The rank that owns block-in-cycle b when rank 0 runs parts [0, root_run) and rank i >= 1 parts
// [root_run + (i - 1) run, root_run + i run): its index, first part and run length.
__host__ __device__ __forceinline__ void run_owner(int b, int root_run, int run, int& rank, int& first, int& len) {
  if (b < root_run) {
    rank = 0, first = 0, len = root_run;
  } else {
    rank = 1 + (b - root_run) / run, first = root_run + (rank - 1) * run, len = run;
  }
}

// Un-permute of gathered row tiles (the multi-GPU frame, application.render_frame_distributed):
// rank r's buffer (at tiles + r * part_stride) holds the rows of its run of parts in local order, as
// rtx_render_camera_sched wrote them, [planes][rows_r][row_bytes]; the frame is
// [planes][height][row_bytes]. One block per (frame row, plane): a contiguous row copy, 16 B per
// lane when the row and buffers allow it.
__global__ __launch_bounds__(kBlock) void k_assemble_rows(const uint8_t* __restrict__ tiles, int64_t part_stride,
                                                          int n_parts, int root_run, int run, int height,
                                                          int row_block, int64_t row_bytes, bool vec16,
                                                          uint8_t* __restrict__ out) {
  const int g = blockIdx.x;  // frame row
  const int c = blockIdx.y;  // plane
  const int cyc = n_parts * row_block;
  const int pos = g % cyc;
  int r, first, len;
  run_owner(pos / row_block, root_run, run, r, first, len);
  const int lr = (g / cyc) * len * row_block + pos - first * row_block;
  const int rows_r = tile_local_rows(height, row_block, n_parts, first, len);
  const uint8_t* src = tiles + r * part_stride + ((int64_t)c * rows_r + lr) * row_bytes;
  uint8_t* dst = out + ((int64_t)c * height + g) * row_bytes;
  if (vec16) {
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    const u32x4* s4 = (const u32x4*)src;
    u32x4* d4 = (u32x4*)dst;
    for (int64_t k = threadIdx.x; k < row_bytes / 16; k += kBlock) __builtin_nontemporal_store(s4[k], d4 + k);
  } else {
    for (int64_t k = threadIdx.x; k < row_bytes; k += kBlock) dst[k] = src[k];
  }
}

}  // namespace

// The TREE = false instantiations of k_render_fast (scenes below kTreeMinSpheres) are compiled and
// launched by their own translation unit, csrc/rtx_small.hip: it includes the device code above and
// stops here. It builds with the max-ilp machine scheduler (_build.SMALL_FLAGS), a per-unit flag: it
// gains the small-scene kernels C2 -0.5..-0.9%, C1 -2.4% and costs the culled kernels C4 +1.4%
// (profiles/r3_ab_variants.txt r3x-r3z).
#ifndef RTX_DEVICE_CODE_ONLY
// Launches k_render_fast<B, true, deep, lvl, stats, 0>(*params) on s (events e0/e1 as
// hipExtLaunchKernelGGL's); hipErrorInvalidValue, nothing launched, for an instantiation the unit
// does not carry.
__attribute__((visibility("hidden"))) hipError_t rtx_launch_small(int B, int deep, bool lvl, bool stats, bool img,
                                                                  const void* params, dim3 grid, uint32_t lds,
                                                                  hipStream_t s, hipEvent_t e0, hipEvent_t e1);
namespace {

// ------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------

thread_local char g_err[512] = "";

int fail(int code, const char* fmt, const char* a = "", long long b = 0) {
  snprintf(g_err, sizeof(g_err), fmt, a, b);
  return code;
}

thread_local hipError_t g_small_err = hipSuccess;  // a launch rtx_launch_small refused

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e == hipSuccess) e = g_small_err;
  g_small_err = hipSuccess;
  if (e != hipSuccess) {
    snprintf(g_err, sizeof(g_err), "%s: %s", what, hipGetErrorString(e));
    return RTX_E_LAUNCH;
  }
  return RTX_OK;
}

// Optional live timing of the dominant kernel (bench.py's roofline): a pool of event pairs handed to
// the k_render_fast launch itself (hipExtLaunchKernelGGL), so they time the dispatch from its start
// to its end, as rocprofv3's kernel trace does, without the gap an event recorded before it adds.
// The state belongs to the calling thread: render calls from other threads are never timed by it
// and never touch it (the entry points stay re-entrant).
struct Prof {
  int cap = 0;
  int used = 0;
  hipEvent_t* ev = nullptr;  // 2 * cap
  int every = 1;             // record one launch in `every` (rtx_profile_sample)
  long long seen = 0;        // launches since rtx_profile_enable
  bool on = false;           // the current launch is recorded
};
thread_local Prof g_prof;

void prof_free() {
  for (int i = 0; i < 2 * g_prof.cap; ++i) (void)hipEventDestroy(g_prof.ev[i]);
  delete[] g_prof.ev;
  const int every = g_prof.every;
  g_prof = Prof{};
  g_prof.every = every;
}

inline void prof_mark(int which, hipStream_t) {
  // launches every-1, 2*every-1, ...: not the first one after rtx_profile_enable, which follows an
  // idle GPU in bench.py (barrier + synchronize) and runs a few µs slow
  if (which == 0)
    g_prof.on = g_prof.cap && g_prof.used < g_prof.cap && g_prof.seen++ % g_prof.every == g_prof.every - 1;
}
// the start / stop event of the launch being timed (null: not timed)
inline hipEvent_t prof_event(int which) { return g_prof.on ? g_prof.ev[2 * g_prof.used + which] : nullptr; }
inline void prof_next() {
  if (g_prof.on) ++g_prof.used;
  g_prof.on = false;
}


int device_cus() {  // compute units of the current device (cached per device)
  static int cus[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (cus[dev] == 0) {
    int v = 0;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0) v = 256;
    cus[dev] = v;
  }
  return cus[dev];
}

int stack_levels_for(int max_bounces) {
  return max_bounces < 0 ? RTX_UNBOUNDED_LEVELS : max_bounces + 1;
}

constexpr size_t kStackBudget = size_t(512) << 20;  // general-kernel frame stacks: <= 512 MiB
constexpr int64_t kMaxWorkers = 65536;

int64_t workers_for(int64_t n, int max_bounces) {
  const size_t per = (size_t)stack_levels_for(max_bounces) * kFrameWords * sizeof(double);
  int64_t w = (int64_t)(kStackBudget / per);
  if (w > kMaxWorkers) w = kMaxWorkers;
  const bool capped = max_bounces >= 0 && max_bounces <= kCappedMax;
  const int64_t cap = capped ? kDeferredWorkers : kDeepWorkers;
  if (w > cap) w = cap;
  const int64_t need = ((n + 63) / 64) * 64;
  if (w > need) w = need;
  w = (w / 64) * 64;
  return w < 64 ? 64 : w;
}

size_t list_bytes(int64_t n) { return (size_t)n * sizeof(int64_t); }

// resume records of deferral pass `pass`: only when chains are deferred for depth
int64_t records_for(int64_t n, int max_bounces, int pass = 0) {
  const bool capped = max_bounces >= 0 && max_bounces <= kCappedMax;
  return capped ? 0 : records_cap(n, pass);
}

size_t round256(size_t b) { return (b + 255) / 256 * 256; }

// Workspace: header | tile counters | list 1 | (deep chains:) lists 2 and 3 | records of level
// kDeepLevels, kDeepLevel2 and kDeepLevel3 | general-kernel stacks
struct WsLayout {
  size_t fetch, list1, list2, list3, rec1, rec2, rec3, stack, total;
};
WsLayout ws_layout(int64_t n, int max_bounces) {
  WsLayout w{};
  const int64_t nrec = records_for(n, max_bounces);
  const int64_t nrec2 = records_for(n, max_bounces, 1);
  const int64_t nrec3 = records_for(n, max_bounces, 2);
  w.fetch = RTX_WS_HDR_BYTES;
  w.list1 = w.fetch + (size_t)kMaxFetch * kFetchStride * sizeof(uint32_t);
  // (forward fold: the first continuation pass, list 2 and its records, is never launched — run_render
  // starts at the second — so they take no bytes; ADVICE r5: 275 MB of the unbounded C4 workspace)
  w.list2 = w.list1 + round256(list_bytes(n));
  w.list3 = w.list2 + (nrec && !kForwardFold ? round256(list_bytes(n)) : 0);
  w.rec1 = w.list3 + (nrec ? round256(list_bytes(n)) : 0);
  w.rec2 = w.rec1 + round256((size_t)nrec * rec_words(kDeepLevels) * sizeof(double));
  w.rec3 = w.rec2 + (kForwardFold ? 0 : round256((size_t)nrec2 * rec_words(kDeepLevel2) * sizeof(double)));
  w.stack = w.rec3 + round256((size_t)nrec3 * rec_words(kDeepLevel3) * sizeof(double));
  w.total = w.stack + (size_t)workers_for(n, max_bounces) * stack_levels_for(max_bounces) * kFrameWords * 8;
  return w;
}

size_t ws_bytes(int64_t n, int max_bounces) { return ws_layout(n, max_bounces).total; }

// The block-tile grid of a camera launch that is not persistent: the TREE = false kernels (scenes below
// kTreeMinSpheres, launch_fast_lds_s) use wave_w<false>() pixels per wave row.
void block_grid(int nsph, int width, int n_rows, int64_t& gx, int64_t& gy) {
  const bool small = nsph < kTreeMinSpheres;
  const int wx = small ? waves_x<false>() : waves_x<true>();
  const int tw = wx * (small ? wave_w<false>() : wave_w<true>());
  const int th = ((small ? fast_waves<false>() : fast_waves<true>()) / wx) * (64 / (small ? wave_w<false>() : wave_w<true>()));
  gx = (width + tw - 1) / tw;
  gy = (n_rows + th - 1) / th;
}

// Persistent launch (p.n_fetch > 0 on entry): as many blocks as the device holds at once, at most one
// wave per tile; sets n_fetch to the counters in use (every counter needs at least one wave).
template <typename K>
dim3 persistent_grid(K kernel, size_t lds, Params& p) {
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, kFastBlock, lds) != hipSuccess || per_cu < 1)
    per_cu = 1;
  const int64_t nt = (int64_t)p.n_tiles_x * p.n_tiles_y;
  int64_t blocks = (int64_t)per_cu * device_cus() - p.reserve;  // (room for a concurrent collective)
  if (blocks < 8) blocks = 8;
  const int64_t need = (nt + kFastWaves - 1) / kFastWaves;
  if (blocks > need) blocks = need;
  if (blocks >= 8) blocks -= blocks % 8;  // whole XCD groups (the kernel numbers waves XCD-major)
  const int64_t per_xcd = blocks * kFastWaves / (blocks % 8 == 0 ? 8 : 1);
  int nc = kMaxFetch;  // a power of two dividing the waves per XCD
  while (nc > 1 && per_xcd % nc != 0) nc /= 2;
  p.n_fetch = nc;
  if (getenv("RTX_DEBUG_GRID"))
    fprintf(stderr, "persistent grid: %d blocks/CU x %d CUs -> %lld blocks, %d counters, %lld tiles\n", per_cu,
            device_cus(), (long long)blocks, p.n_fetch, (long long)nt);
  return dim3((unsigned)blocks);
}

// STATS: the instantiation with the per-level and executed-work counters (stats buffer given) and
// the per-unit cost records (tile_cost given; counters only where p.stats is set).
// Launches that are not persistent run instantiations without the persistent tile loop (TP 1), and
// scenes below kTreeMinSpheres, which carry no culling tree (scene_pack.BVH_MIN_SPHERES), ones
// without the tree walks either (TP 0) (A/B in DESIGN.md §4).
template <int B, int DEEP, bool LVL, bool STATS, bool IMG = false>
void launch_fast_lds_s(Params& p, dim3 grid, hipStream_t s) {
  const bool small = p.nsph < kTreeMinSpheres;  // the TREE = false kernels: fast_block<false>() threads
  const size_t lds = (size_t)p.nsph * kSphWords * sizeof(double) +
                     (LVL ? (small ? level_lds_bytes<(DEEP != 0), false>(B) : level_lds_bytes<(DEEP != 0)>(B)) : 0) +
                     (kForwardFold && !DEEP && !small && p.n_fetch == 0 ? kColourLdsBytes : 0);  // TP 1
  if (p.n_fetch == 0) {  // one tile per block: the instantiations without the persistent loop
    if (p.nsph < kTreeMinSpheres) {  // TP 0: the rtx_small.hip unit
      const hipError_t e =
          rtx_launch_small(B, DEEP, LVL, STATS, IMG, &p, grid, (uint32_t)lds, s, prof_event(0), prof_event(1));
      if (e != hipSuccess) g_small_err = e;
    } else {
      if constexpr (!DEEP && !STATS && !IMG && kForwardFold) {
        if ((int64_t)p.n * p.n_frames >= kWavesLargeMinPixels) {  // a large launch: more waves (kFwdWavesLarge)
          hipExtLaunchKernelGGL((k_render_fast<B, true, DEEP, LVL, STATS, 1, IMG, 0, kFwdWavesLarge>), grid,
                                dim3(kFastBlock), (uint32_t)lds, s, prof_event(0), prof_event(1), 0u, p);
          return;
        }
      }
      hipExtLaunchKernelGGL((k_render_fast<B, true, DEEP, LVL, STATS, 1, IMG>), grid, dim3(kFastBlock), (uint32_t)lds,
                            s, prof_event(0), prof_event(1), 0u, p);
    }
    return;
  }
  if (p.n_fetch > 0) grid = persistent_grid(k_render_fast<B, true, DEEP, LVL, STATS, 2, IMG>, lds, p);
  hipExtLaunchKernelGGL((k_render_fast<B, true, DEEP, LVL, STATS, 2, IMG>), grid, dim3(kFastBlock), (uint32_t)lds, s,
                        prof_event(0), prof_event(1), 0u, p);
}
template <int B, int DEEP, bool LVL>
void launch_fast_lds(Params& p, dim3 grid, hipStream_t s) {
  if (p.stats || p.tile_cost) {  // (the cost records of a learning launch live in the STATS kernels)
    launch_fast_lds_s<B, DEEP, LVL, true>(p, grid, s);
  } else if (!DEEP && p.images) {  // image textures shaded in place (capped renders only)
    launch_fast_lds_s<B, DEEP, LVL, false, !DEEP>(p, grid, s);
  } else {
    launch_fast_lds_s<B, DEEP, LVL, false>(p, grid, s);
  }
}

template <int B, int DEEP = 0>
void launch_fast_b(const Params& p0, dim3 grid, hipStream_t s) {
  Params p = p0;
  if (p.nsph <= kLdsMaxSpheres) {
    if constexpr (DEEP) {
      // (forward fold: no level slots, so no LDS for them and the occupancy the registers allow)
      if (!kForwardFold && kLevelsInLds && p.nsph <= kDeepLvMaxSpheres) {
        launch_fast_lds<B, DEEP, true>(p, grid, s);
      } else {
        launch_fast_lds<B, DEEP, false>(p, grid, s);
      }
    } else {
      // caps 3-4 in big scenes: three LDS level slots beside a large scene table leave room for
      // fewer than 4 blocks per CU; the register-level kernel (128 VGPRs, 4 waves/SIMD) then runs
      // more waves than the LDS-slot kernel can
      constexpr bool kTry = B == 3 || B == 4;
      if (kTry && (size_t)p.nsph * kSphWords * sizeof(double) + level_lds_bytes(B) > kLdsBytesPerCu / 4) {
        if constexpr (kTry) launch_fast_lds<B, false, false>(p, grid, s);
      } else {
        launch_fast_lds<B, false, levels_in_lds<B, true, false>()>(p, grid, s);
      }
    }
  } else {
    if (p.stats || p.tile_cost) {
      if (p.n_fetch > 0) grid = persistent_grid(k_render_fast<B, false, DEEP, false, true>, 0, p);
      hipExtLaunchKernelGGL((k_render_fast<B, false, DEEP, false, true>), grid, dim3(kFastBlock), 0u, s,
                            prof_event(0), prof_event(1), 0u, p);
    } else {
      if (p.n_fetch > 0) grid = persistent_grid(k_render_fast<B, false, DEEP>, 0, p);
      hipExtLaunchKernelGGL((k_render_fast<B, false, DEEP>), grid, dim3(kFastBlock), 0u, s, prof_event(0),
                            prof_event(1), 0u, p);
    }
  }
}

// caps above kCappedMax or none: kDeepLevels levels, longer chains deferred with a record
void launch_fast_deep(const Params& p, dim3 grid, hipStream_t s) { launch_fast_b<kDeepLevels, 1>(p, grid, s); }
// ... and their continuation passes (mode 2)
void launch_fast_cont(const Params& p, dim3 grid, hipStream_t s) { launch_fast_b<kDeepLevels, 2>(p, grid, s); }

void launch_fast(int B, const Params& p, dim3 grid, hipStream_t s) {
  switch (B) {
    case 0: launch_fast_b<0>(p, grid, s); break;
    case 1: launch_fast_b<1>(p, grid, s); break;
    case 2: launch_fast_b<2>(p, grid, s); break;
    case 3: launch_fast_b<3>(p, grid, s); break;
    case 4: launch_fast_b<4>(p, grid, s); break;
    case 5: launch_fast_b<5>(p, grid, s); break;
    default: launch_fast_b<6>(p, grid, s); break;
  }
}
static_assert(RTX_FAST_MAX_BOUNCES == 6, "launch_fast switch covers 0..6");

// no_general: the caller knows this exact render defers no ray (rtx_render_camera_ex): no general
// kernel, and for an uncapped render no continuation pass either
int run_render(Params& p, void* workspace, size_t workspace_bytes, hipStream_t s, bool no_general = false) {
  if (p.nsph <= 0 || p.nsph > RTX_MAX_SPHERES) return fail(RTX_E_ARG, "n_spheres out of range%s (%lld)", "", p.nsph);
  if (!p.scene || !workspace) return fail(RTX_E_ARG, "null pointer argument%s", "");
  if (p.out_kind < 0 || p.out_kind > 2) return fail(RTX_E_ARG, "bad out_kind%s %lld", "", p.out_kind);
  if (p.max_bounces < RTX_UNBOUNDED) return fail(RTX_E_ARG, "bad max_bounces%s %lld", "", p.max_bounces);
  if (p.n_frames <= 0) p.n_frames = 1;
  if (p.n_frames > 65535) return fail(RTX_E_ARG, "at most 65535 frames per launch%s (%lld)", "", p.n_frames);
  if (p.n <= 0) return RTX_OK;  // (an empty tile, e.g. a rank's share of a small frame: out may be null)
  if (!p.out) return fail(RTX_E_ARG, "null pointer argument%s", "");
  if (p.n >= (int64_t(1) << kFrameShift)) return fail(RTX_E_ARG, "too many pixels per frame%s (%lld)", "", p.n);
  const int64_t n_all = p.n * p.n_frames;  // pixels of the whole launch
  const size_t need = ws_bytes(n_all, p.max_bounces);
  if (workspace_bytes < need) return fail(RTX_E_WORKSPACE, "workspace too small%s (need %lld bytes)", "", (long long)need);
  p.ws = (uint8_t*)workspace;
  p.list_cap = n_all;
  const WsLayout lay = ws_layout(n_all, p.max_bounces);
  uint32_t* const hdr = (uint32_t*)p.ws;
  uint64_t* const list1 = (uint64_t*)(p.ws + lay.list1);
  uint64_t* const list2 = (uint64_t*)(p.ws + lay.list2);
  double* const rec1 = (double*)(p.ws + lay.rec1);
  double* const rec2 = (double*)(p.ws + lay.rec2);
  p.rec_cap = records_for(n_all, p.max_bounces);
  p.in_rec_cap = p.rec_cap;
  p.stack = (double*)(p.ws + lay.stack);
  // The fast kernel renders every ray up to min(cap, RTX_FAST_MAX_BOUNCES) levels; a pixel whose
  // chain outlives that (a larger or no cap) is deferred, like a tie, to the general kernel.
  const bool capped = p.max_bounces >= 0 && p.max_bounces <= kCappedMax;
  p.no_general = no_general ? 1 : 0;
  p.n_workers = workers_for(n_all, p.max_bounces);
  p.stack_levels = stack_levels_for(p.max_bounces);
  {
    dim3 grid;
    const int64_t fb = p.nsph < kTreeMinSpheres ? fast_block<false>() : fast_block<true>();
    int64_t tx = (p.n + fb - 1) / fb, ty = 1;
    if (p.mode == 0) block_grid(p.nsph, p.width, p.n_rows, tx, ty);
    p.n_fetch = 0;
    if (p.nsph >= kPersistMinSpheres && p.mode == 0 && p.n_frames == 1) {
      p.n_tiles_x = (p.width + kWaveW - 1) / kWaveW;  // wave tiles
      p.n_tiles_y = (p.n_rows + kWaveH - 1) / kWaveH;
      p.fetch = (uint32_t*)(p.ws + lay.fetch);
      p.n_fetch = kMaxFetch;  // launch_fast_b sizes the grid and the counters in use
      grid = dim3(1);
    } else {
      p.n_tiles_x = p.n_tiles_y = 0;
      grid = dim3((unsigned)tx, (unsigned)ty, (unsigned)p.n_frames);
    }
    p.dlist = list1;
    p.dcount = hdr + RTX_WS_COUNT;
    p.drec = capped ? nullptr : rec1;
    p.drec_level = kForwardFold ? kFirstPassLevels : kDeepLevels;
    prof_mark(0, s);
    if (capped) {
      launch_fast(p.max_bounces, p, grid, s);
    } else {
      launch_fast_deep(p, grid, s);
    }
    prof_mark(1, s);
    prof_next();
    if (int e = check_launch("k_render_fast")) return e;
  }
  p.in_list = list1;
  p.in_count = hdr + RTX_WS_COUNT;
  p.in_rec = capped ? nullptr : rec1;
  p.in_level = kForwardFold ? kFirstPassLevels : kDeepLevels;
  if (!capped && p.n_frames == 1 && !no_general) {
    // continuation passes: chains deferred for depth go on for kDeepLevels + 1 more levels in
    // the register-resident kernel, twice; ties and what is still alive after them go to the
    // general kernel
    uint64_t* const lists[2] = {list2, (uint64_t*)(p.ws + lay.list3)};
    uint32_t* const counts[2] = {hdr + RTX_WS_COUNT2, hdr + RTX_WS_COUNT3};
    double* const recs[2] = {rec2, (double*)(p.ws + lay.rec3)};
    const int levels[2] = {kDeepLevel2, kDeepLevel3};
    const int64_t caps[2] = {records_for(n_all, p.max_bounces, 1), records_for(n_all, p.max_bounces, 2)};
    // (forward fold: one continuation pass goes on from level kDeepLevels + 1 to kDeepLevel3)
    for (int pass = kForwardFold ? 1 : 0; pass < 2; ++pass) {
      Params q = p;
      q.mode = 2;
      q.n_tiles_x = q.n_tiles_y = 0;
      q.n_fetch = 0;
      q.dlist = lists[pass];
      q.dcount = counts[pass];
      q.drec = recs[pass];
      q.drec_level = levels[pass];
      q.rec_cap = caps[pass];
      q.in_rec_cap = p.in_rec_cap;
      const int64_t fb = p.nsph < kTreeMinSpheres ? fast_block<false>() : fast_block<true>();
      const int64_t tiles = (n_all + fb - 1) / fb;
      const int64_t cap = 4 * (int64_t)device_cus();
      launch_fast_cont(q, dim3((unsigned)(tiles < cap ? tiles : cap)), s);
      if (int e = check_launch("k_render_fast (continuation)")) return e;
      p.in_list = lists[pass];
      p.in_count = counts[pass];
      p.in_rec = recs[pass];
      p.in_level = levels[pass];
      p.in_rec_cap = caps[pass];
    }
  }
  // deferred rays: ties, and chains longer than the fast kernel's levels
  if (no_general) return RTX_OK;  // (an uncapped render: nor the continuation pass)
  hipLaunchKernelGGL(k_render_general, dim3((unsigned)(p.n_workers / 64)), dim3(64), 0, s, p);
  return check_launch("k_render_general");
}

}  // namespace

// ------------------------------------------------------------------------------------------
// C ABI
// ------------------------------------------------------------------------------------------

extern "C" {

int rtx_abi_version(int* layout, int n) {
  const int v[] = {RTX_HDR_WORDS, RTX_GEOM_WORDS, RTX_MAT_WORDS, RTX_MAX_DOMES, RTX_S_WORDS, RTX_WS_HDR_BYTES,
                   RTX_FAST_MAX_BOUNCES, RTX_UNBOUNDED_LEVELS};
  for (int i = 0; layout && i < n && i < (int)(sizeof(v) / sizeof(v[0])); ++i) layout[i] = v[i];
  return RTX_ABI_VERSION;
}

const char* rtx_last_error(void) { return g_err; }

int rtx_profile_enable(int max_launches) {
  prof_free();
  if (max_launches <= 0) return RTX_OK;
  g_prof.ev = new hipEvent_t[2 * (size_t)max_launches];
  // timing-only events: no system-scope fence when they are recorded (the default fence writes back
  // and invalidates the caches around the timed dispatch, which lengthened the timed launches by
  // ~0.6 us and read ~0.8 us more on C2, session r6s; the HIP header recommends the flag for
  // events used only to measure time)
  for (int i = 0; i < 2 * max_launches; ++i) {
    if (hipEventCreateWithFlags(&g_prof.ev[i], hipEventDisableSystemFence) != hipSuccess) {
      g_prof.cap = i / 2;
      prof_free();
      return fail(RTX_E_LAUNCH, "hipEventCreate failed%s", "");
    }
  }
  g_prof.cap = max_launches;
  return RTX_OK;
}

int rtx_profile_sample(int every) {
  if (every < 1) return fail(RTX_E_ARG, "profile sampling stride must be >= 1%s (%lld)", "", every);
  g_prof.every = every;
  return RTX_OK;
}

int rtx_profile_collect(double* total_ms, int* n_launches) {
  double tot = 0.0;
  for (int i = 0; i < g_prof.used; ++i) {
    if (hipEventSynchronize(g_prof.ev[2 * i + 1]) != hipSuccess) return check_launch("hipEventSynchronize");
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, g_prof.ev[2 * i], g_prof.ev[2 * i + 1]) != hipSuccess)
      return check_launch("hipEventElapsedTime");
    tot += ms;
  }
  if (total_ms) *total_ms = tot;
  if (n_launches) *n_launches = g_prof.used;
  g_prof.used = 0;
  return RTX_OK;
}

size_t rtx_workspace_bytes(int64_t n_rays, int max_bounces) {
  if (n_rays < 1) n_rays = 1;
  if (max_bounces < RTX_UNBOUNDED) max_bounces = RTX_UNBOUNDED;
  return ws_bytes(n_rays, max_bounces);
}

int rtx_sched_tiles(int width, int n_local_rows, int n_spheres, int64_t* n_tiles) {
  if (!n_tiles) return fail(RTX_E_ARG, "null pointer argument%s", "");
  *n_tiles = 0;
  if (width <= 0 || n_local_rows <= 0 || n_spheres <= 0) return RTX_OK;
  if (n_spheres >= kPersistMinSpheres) {  // persistent launch: wave tiles
    *n_tiles = (int64_t)((width + kWaveW - 1) / kWaveW) * ((n_local_rows + kWaveH - 1) / kWaveH);
    return RTX_OK;
  }
  int64_t gx, gy;  // one block tile per block (run_render's grid)
  block_grid(n_spheres, width, n_local_rows, gx, gy);
  *n_tiles = gx * gy;
  return RTX_OK;
}

int rtx_render_camera_ex(const double* scene, int n_spheres, int width, int height, int row_block, int n_parts,
                         int part, int n_local_rows, int max_bounces, void* out, int out_kind, void* workspace,
                         size_t workspace_bytes, uint64_t* stats, void* stream, unsigned flags,
                         uint32_t* deferred_out) {
  return rtx_render_camera_sched(scene, n_spheres, width, height, row_block, n_parts, part, 1, n_local_rows,
                                 max_bounces, out, out_kind, workspace, workspace_bytes, stats, stream, flags,
                                 deferred_out, nullptr, nullptr);
}

int rtx_render_camera_sched(const double* scene, int n_spheres, int width, int height, int row_block, int n_parts,
                            int part, int part_run, int n_local_rows, int max_bounces, void* out, int out_kind,
                            void* workspace,
                            size_t workspace_bytes, uint64_t* stats, void* stream, unsigned flags,
                            uint32_t* deferred_out, const uint32_t* tile_order, uint32_t* tile_cost) {
  if (width <= 0 || height <= 0 || row_block <= 0 || n_parts <= 0 || part < 0 || part_run < 1 ||
      part_run > n_parts - part || n_local_rows < 0 ||
      n_local_rows > tile_local_rows(height, row_block, n_parts, part, part_run))
    return fail(RTX_E_ARG, "bad frame/tile geometry%s", "");
  if (flags & ~(unsigned)(RTX_F_NO_GENERAL | RTX_F_IMAGES | RTX_F_RESERVE(0xFFF)))
    return fail(RTX_E_ARG, "unknown flags%s (%lld)", "", (long long)flags);
  Params p{};
  p.images = (flags & RTX_F_IMAGES) ? 1 : 0;
  p.scene = scene;
  p.nsph = n_spheres;
  p.mode = 0;
  p.width = width;
  p.height = height;
  p.row_block = row_block;
  p.n_parts = n_parts;
  p.part = part;
  p.part_run = part_run;
  p.n_rows = n_local_rows;
  p.n = (int64_t)width * n_local_rows;
  p.max_bounces = max_bounces;
  p.out = out;
  p.out_kind = out_kind;
  p.stats = (unsigned long long*)stats;
  p.deferred_out = deferred_out;
  p.tile_order = tile_order;  // rtx_sched_tiles units of this launch (the first pass: mode 0, one frame)
  p.tile_cost = tile_cost;
  p.reserve = (int)((flags >> RTX_F_RESERVE_SHIFT) & 0xFFFu);
  // a launch with counters or cost records runs the STATS kernels, which have no texturing build:
  // they defer image-textured hits, so the general kernel must follow whatever the caller learnt
  // from the texturing build's deferral count
  const bool no_general = (flags & RTX_F_NO_GENERAL) && !(p.images && (stats || tile_cost));
  return run_render(p, workspace, workspace_bytes, (hipStream_t)stream, no_general);
}

int rtx_render_camera(const double* scene, int n_spheres, int width, int height, int row_block, int n_parts,
                      int part, int n_local_rows, int max_bounces, void* out, int out_kind, void* workspace,
                      size_t workspace_bytes, uint64_t* stats, void* stream) {
  return rtx_render_camera_ex(scene, n_spheres, width, height, row_block, n_parts, part, n_local_rows, max_bounces,
                              out, out_kind, workspace, workspace_bytes, stats, stream, 0u, nullptr);
}

int rtx_render_frames(const double* scenes, int64_t scene_stride, int n_frames, int n_spheres, int width, int height,
                      int max_bounces, void* out, int out_kind, void* workspace, size_t workspace_bytes,
                      uint64_t* stats, void* stream) {
  if (width <= 0 || height <= 0) return fail(RTX_E_ARG, "bad frame geometry%s", "");
  if (n_frames < 0) return fail(RTX_E_ARG, "bad n_frames%s (%lld)", "", n_frames);
  if (n_frames > 1 && scene_stride < RTX_HDR_WORDS) return fail(RTX_E_ARG, "bad scene_stride%s (%lld)", "", scene_stride);
  if (n_frames == 0) return RTX_OK;
  Params p{};
  p.scene = scenes;
  p.scene_stride = scene_stride;
  p.n_frames = n_frames;
  p.nsph = n_spheres;
  p.mode = 0;
  p.width = width;
  p.height = height;
  p.row_block = 1;
  p.n_parts = 1;
  p.part = 0;
  p.n_rows = height;
  p.n = (int64_t)width * height;
  p.max_bounces = max_bounces;
  p.out = out;
  p.out_kind = out_kind;
  p.stats = (unsigned long long*)stats;
  return run_render(p, workspace, workspace_bytes, (hipStream_t)stream);
}

int rtx_trace_rays(const double* scene, int n_spheres, const double* origins, int64_t origin_stride,
                   const double* dirs, int64_t n, int max_bounces, void* out, int out_kind, void* workspace,
                   size_t workspace_bytes, uint64_t* stats, void* stream) {
  if (!origins || !dirs) return fail(RTX_E_ARG, "null ray pointer%s", "");
  if (origin_stride != 0 && origin_stride != n) return fail(RTX_E_ARG, "origin_stride must be 0 or n%s", "");
  Params p{};
  p.scene = scene;
  p.nsph = n_spheres;
  p.mode = 1;
  p.org = origins;
  p.org_stride = origin_stride;
  p.dir = dirs;
  p.n = n;
  p.max_bounces = max_bounces;
  p.out = out;
  p.out_kind = out_kind;
  p.stats = (unsigned long long*)stats;
  return run_render(p, workspace, workspace_bytes, (hipStream_t)stream);
}

int rtx_shade_hits(const double* scene, int n_spheres, int shape, const double* origins, int64_t origin_stride,
                   const double* dirs, const double* t, int64_t n, int max_bounces, void* out, int out_kind,
                   void* workspace, size_t workspace_bytes, uint64_t* stats, void* stream) {
  if (!origins || !dirs || !t) return fail(RTX_E_ARG, "null ray pointer%s", "");
  if (origin_stride != 0 && origin_stride != n) return fail(RTX_E_ARG, "origin_stride must be 0 or n%s", "");
  if (shape < 0 || shape >= n_spheres) return fail(RTX_E_ARG, "shape index out of range%s (%lld)", "", shape);
  Params p{};
  p.scene = scene;
  p.nsph = n_spheres;
  p.mode = 3;
  p.org = origins;
  p.org_stride = origin_stride;
  p.dir = dirs;
  p.hit_t = t;
  p.hit_shape = shape;
  p.n = n;
  p.max_bounces = max_bounces;
  p.out = out;
  p.out_kind = out_kind;
  p.stats = (unsigned long long*)stats;
  return run_render(p, workspace, workspace_bytes, (hipStream_t)stream);
}

int rtx_ray_directions(const double* scene, int width, int height, int row_block, int n_parts, int part,
                       int n_local_rows, double* dirs_out, void* stream) {
  if (!scene || !dirs_out) return fail(RTX_E_ARG, "null pointer argument%s", "");
  if (width <= 0 || height <= 0 || row_block <= 0 || n_parts <= 0 || part < 0 || part >= n_parts ||
      n_local_rows < 0 || n_local_rows > tile_local_rows(height, row_block, n_parts, part))
    return fail(RTX_E_ARG, "bad frame/tile geometry%s", "");
  Params p{};
  p.scene = scene;
  p.width = width;
  p.height = height;
  p.row_block = row_block;
  p.n_parts = n_parts;
  p.part = part;
  p.n_rows = n_local_rows;
  p.n = (int64_t)width * n_local_rows;
  if (p.n == 0) return RTX_OK;
  hipLaunchKernelGGL(k_ray_dirs, dim3((unsigned)((p.n + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                     (hipStream_t)stream, p, dirs_out);
  return check_launch("k_ray_dirs");
}

int rtx_sphere_intersect(const double* sphere, const double* origins, int64_t origin_stride, const double* dirs,
                         int64_t n, double* t_out, void* stream) {
  if (!sphere || !origins || !dirs || !t_out) return fail(RTX_E_ARG, "null pointer argument%s", "");
  if (origin_stride != 0 && origin_stride != n) return fail(RTX_E_ARG, "origin_stride must be 0 or n%s", "");
  if (n <= 0) return RTX_OK;
  hipLaunchKernelGGL(k_intersect, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, (hipStream_t)stream,
                     sphere, origins, origin_stride, dirs, n, t_out);
  return check_launch("k_intersect");
}

int rtx_selftest_math(const double* a, const double* b, int64_t n, double* out, void* stream) {
  if (!a || !b || !out) return fail(RTX_E_ARG, "null pointer argument%s", "");
  if (n <= 0) return RTX_OK;
  hipLaunchKernelGGL(k_selftest_math, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                     (hipStream_t)stream, a, b, n, out);
  return check_launch("k_selftest_math");
}

int rtx_quantize_u8(const void* color, int color_kind, int64_t n, uint8_t* out, void* stream) {
  if (!color || !out) return fail(RTX_E_ARG, "null pointer argument%s", "");
  if (n <= 0) return RTX_OK;
  const dim3 grid((unsigned)((n + kBlock - 1) / kBlock));
  if (color_kind == RTX_OUT_F32_SOA) {
    hipLaunchKernelGGL(k_quantize<float>, grid, dim3(kBlock), 0, (hipStream_t)stream, (const float*)color, n, out);
  } else if (color_kind == RTX_OUT_F64_SOA) {
    hipLaunchKernelGGL(k_quantize<double>, grid, dim3(kBlock), 0, (hipStream_t)stream, (const double*)color, n, out);
  } else {
    return fail(RTX_E_ARG, "bad color_kind%s %lld", "", color_kind);
  }
  return check_launch("k_quantize");
}

int rtx_assemble_rows(const void* tiles, int64_t part_stride_bytes, int n_parts, int width, int height,
                      int row_block, int kind, void* out, void* stream) {
  return rtx_assemble_runs(tiles, part_stride_bytes, n_parts, 1, 1, width, height, row_block, kind, out, stream);
}

int rtx_assemble_runs(const void* tiles, int64_t part_stride_bytes, int n_ranks, int root_run, int run, int width,
                      int height, int row_block, int kind, void* out, void* stream) {
  if (!tiles || !out) return fail(RTX_E_ARG, "null pointer argument%s", "");
  if (width <= 0 || height <= 0 || row_block <= 0 || n_ranks <= 0 || root_run <= 0 || run <= 0)
    return fail(RTX_E_ARG, "bad frame/tile geometry%s", "");
  const int n_parts = root_run + (n_ranks - 1) * run;
  int planes = 3;
  int64_t row_bytes;
  if (kind == RTX_OUT_F32_SOA) {
    row_bytes = 4 * (int64_t)width;
  } else if (kind == RTX_OUT_F64_SOA) {
    row_bytes = 8 * (int64_t)width;
  } else if (kind == RTX_OUT_U8_HWC) {
    row_bytes = 3 * (int64_t)width;
    planes = 1;
  } else {
    return fail(RTX_E_ARG, "bad kind%s %lld", "", kind);
  }
  int rmax = 0;  // the longest run's rows
  for (int r = 0; r < n_ranks; ++r) {
    const int len = r == 0 ? root_run : run, first = r == 0 ? 0 : root_run + (r - 1) * run;
    const int rows = tile_local_rows(height, row_block, n_parts, first, len);
    rmax = rows > rmax ? rows : rmax;
  }
  if (part_stride_bytes < planes * rmax * row_bytes)
    return fail(RTX_E_ARG, "part_stride too small%s (need %lld bytes)", "", (long long)(planes * rmax * row_bytes));
  const bool vec16 = row_bytes % 16 == 0 && part_stride_bytes % 16 == 0 && (uintptr_t)tiles % 16 == 0 &&
                     (uintptr_t)out % 16 == 0;
  hipLaunchKernelGGL(k_assemble_rows, dim3((unsigned)height, (unsigned)planes), dim3(kBlock), 0, (hipStream_t)stream,
                     (const uint8_t*)tiles, part_stride_bytes, n_parts, root_run, run, height, row_block, row_bytes,
                     vec16, (uint8_t*)out);
  return check_launch("k_assemble_rows");
}

}  // extern "C"

// the error message of the other host units (csrc/rtx_tiles.hip), read through rtx_last_error
__attribute__((visibility("hidden"))) int rtx_set_error(int code, const char* msg) {
  snprintf(g_err, sizeof(g_err), "%s", msg);
  return code;
}

#endif  // RTX_DEVICE_CODE_ONLY
