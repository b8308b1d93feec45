def patch(src):
    a = '''  hipLaunchKernelGGL(k_render_general, dim3((unsigned)(p.n_workers / 64)), dim3(64), 0, s, p);'''
    assert a in src
    return src.replace(a, '''  if (!capped) hipLaunchKernelGGL(k_render_general, dim3((unsigned)(p.n_workers / 64)), dim3(64), 0, s, p);''')
