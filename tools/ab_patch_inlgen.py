"""A/B patch (timing only): k_render_fast carries the general kernel's depth-first path behind a
branch that is never taken (mode 7), to measure what its registers / scratch cost the fast path
(the question behind rendering ties inside the fast kernel's launch)."""


def patch(src):
    a = '''  fast_tile<B, LDS, DEEP, LVL, STATS>(p, blockIdx.x, gridDim.y - 1 - blockIdx.y, true, lds_tab);
}'''
    assert a in src
    src = src.replace(a, '''  fast_tile<B, LDS, DEEP, LVL, STATS>(p, blockIdx.x, gridDim.y - 1 - blockIdx.y, true, lds_tab);
  if (p.mode == 7) general_tail(p);
}''')
    b = '''template <int B, bool LDS, bool DEEP, bool LVL = levels_in_lds<B, LDS, DEEP>(), bool STATS = false>'''
    assert b in src
    src = src.replace(b, '''__device__ void general_tail(const Params& p);
''' + b)
    c = '''__global__ __launch_bounds__(64) void k_render_general(Params p0) {'''
    assert c in src
    src = src.replace(c, '''__device__ void general_tail(const Params& p) {
  Stack S{p.stack, p.n_workers, (int64_t)blockIdx.x * kFastBlock + threadIdx.x};
  double cr, cg, cb;
  trace_general(p, S, 0.0, 0.0, 0.0, 0.0, 0.0, 1.0, cr, cg, cb, -1, -1);
  write_out(p, 0, cr, cg, cb);
}

''' + c)
    return src
