"""A/B patch (timing only, wrong when a frame has ties): the tie launch replaced by a trivial kernel
of the same grid that only reads the deferred-list counters, to separate the cost of a second
launch from the cost of k_render_general's own properties (code size, 144 VGPRs)."""


def patch(src):
    a = '''  hipLaunchKernelGGL(k_render_general, dim3((unsigned)(p.n_workers / 64)), dim3(64), 0, s, p);'''
    assert a in src
    src = src.replace(a, '''  if (capped) {
    hipLaunchKernelGGL(k_noop_general, dim3((unsigned)(p.n_workers / 64)), dim3(64), 0, s, p);
  } else {
    hipLaunchKernelGGL(k_render_general, dim3((unsigned)(p.n_workers / 64)), dim3(64), 0, s, p);
  }''')
    b = '''// ------------------------------------------------------------------------------------------
// boundary helpers'''
    assert b in src
    return src.replace(b, '''__global__ __launch_bounds__(64) void k_noop_general(Params p) {
  uint32_t* hdr = (uint32_t*)p.ws;
  if (hdr[RTX_WS_COUNT] != 0u && threadIdx.x == 0) hdr[RTX_WS_STATUS] |= 8u;
}

''' + b)
