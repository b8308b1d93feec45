// rtx_small.hip — the k_render_fast instantiations of scenes below kTreeMinSpheres (TP 0: no culling
// tree, no persistent loop; the README and main.py scenes, BASELINE configs C1/C2), in a translation
// unit of their own so that they build with the max-ilp machine scheduler (_build.SMALL_FLAGS) while
// the culled kernels keep the default one (profiles/r3_ab_variants.txt r3x-r3z). The device code is
// rtx_kernels.hip's, included up to its host section; the launch sites there call rtx_launch_small.
#define RTX_DEVICE_CODE_ONLY
#include "rtx_kernels.hip"

namespace {

template <int B, int DEEP, bool LVL, bool STATS, bool IMG = false, int NSPH = 0>
hipError_t go(const void* params, dim3 grid, uint32_t lds, hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
  const Params& p = *static_cast<const Params*>(params);
  hipExtLaunchKernelGGL((k_render_fast<B, true, DEEP, LVL, STATS, 0, IMG, NSPH>), grid, dim3(fast_block<false>()), lds,
                        s, e0, e1, 0u, p);
  return hipSuccess;  // launch errors reach the caller's check_launch through hipGetLastError
}

// The kernels without counters or image textures (the timed capped ones and the DEEP ones of
// unbounded renders) of each sphere count below kTreeMinSpheres, with the count a compile-time
// constant (fast_tile's NSPH: the sphere loops unroll; A/B r6b, C2 -2.7%); the counter and
// texturing kernels keep the run-time count.
template <int B, int DEEP, bool LVL>
hipError_t go_ns(const void* params, dim3 grid, uint32_t lds, hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
  static_assert(kTreeMinSpheres == 8, "one instantiation per sphere count 1..7");
  switch (static_cast<const Params*>(params)->nsph) {
    case 1: return go<B, DEEP, LVL, false, false, 1>(params, grid, lds, s, e0, e1);
    case 2: return go<B, DEEP, LVL, false, false, 2>(params, grid, lds, s, e0, e1);
    case 3: return go<B, DEEP, LVL, false, false, 3>(params, grid, lds, s, e0, e1);
    case 4: return go<B, DEEP, LVL, false, false, 4>(params, grid, lds, s, e0, e1);
    case 5: return go<B, DEEP, LVL, false, false, 5>(params, grid, lds, s, e0, e1);
    case 6: return go<B, DEEP, LVL, false, false, 6>(params, grid, lds, s, e0, e1);
    case 7: return go<B, DEEP, LVL, false, false, 7>(params, grid, lds, s, e0, e1);
    default: return go<B, DEEP, LVL, false>(params, grid, lds, s, e0, e1);
  }
}

// the (lvl, stats) instantiations launch_fast_b can request for a scene below kTreeMinSpheres: its
// table always fits the LDS beside the level slots (levels_in_lds); a DEEP kernel kept every level in
// LDS (S <= kDeepLvMaxSpheres) before the forward fold
template <int B, int DEEP>
hipError_t go_b(bool lvl, bool stats, bool img, const void* params, dim3 grid, uint32_t lds, hipStream_t s,
                hipEvent_t e0, hipEvent_t e1) {
  // (the forward fold keeps no levels: DEEP kernels too run without level slots)
  constexpr bool kLvl = DEEP ? (kLevelsInLds && !kForwardFold) : levels_in_lds<B, true, false>();
  static_assert(!DEEP || kForwardFold || kDeepLvMaxSpheres >= kTreeMinSpheres,
                "small DEEP scenes keep their levels in LDS");
  if (lvl != kLvl) return hipErrorInvalidValue;
  if (img) {  // image textures shaded in place: capped, counter-free launches only
    if constexpr (DEEP) return hipErrorInvalidValue;
    else return stats ? hipErrorInvalidValue : go<B, DEEP, kLvl, false, true>(params, grid, lds, s, e0, e1);
  }
  return stats ? go<B, DEEP, kLvl, true>(params, grid, lds, s, e0, e1)
               : go_ns<B, DEEP, kLvl>(params, grid, lds, s, e0, e1);
}

}  // namespace

__attribute__((visibility("hidden"))) hipError_t rtx_launch_small(int B, int deep, bool lvl, bool stats, bool img,
                                                                  const void* params, dim3 grid, uint32_t lds,
                                                                  hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
  if (deep) {  // 1: an uncapped render's first pass, 2: its continuation passes
    if (B != kDeepLevels) return hipErrorInvalidValue;
    return deep == 2 ? go_b<kDeepLevels, 2>(lvl, stats, img, params, grid, lds, s, e0, e1)
                     : go_b<kDeepLevels, 1>(lvl, stats, img, params, grid, lds, s, e0, e1);
  }
  switch (B) {
    case 0: return go_b<0, false>(lvl, stats, img, params, grid, lds, s, e0, e1);
    case 1: return go_b<1, false>(lvl, stats, img, params, grid, lds, s, e0, e1);
    case 2: return go_b<2, false>(lvl, stats, img, params, grid, lds, s, e0, e1);
    case 3: return go_b<3, false>(lvl, stats, img, params, grid, lds, s, e0, e1);
    case 4: return go_b<4, false>(lvl, stats, img, params, grid, lds, s, e0, e1);
    case 5: return go_b<5, false>(lvl, stats, img, params, grid, lds, s, e0, e1);
    case 6: return go_b<6, false>(lvl, stats, img, params, grid, lds, s, e0, e1);
    default: return hipErrorInvalidValue;
  }
}
