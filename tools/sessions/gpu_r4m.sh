#!/bin/bash
# Round-4 session m: GPU tests with the fast kernel's texturing build (RTX_F_IMAGES); textured-scene
# timing, texturing build against deferral; C2 bench line (the untextured kernels unchanged).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r4m; mkdir -p $O
run() { local name=$1 t=$2; shift 2; echo "[$(date +%T)] $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "[$(date +%T)] $name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread
run smoke 300 python __graft_entry__.py smoke
run tex_ab 200 python tools/texture_ab.py --json-out $O/tex_ab.json
run bench_C2 200 python bench.py --config C2 --steps 200 --warmup 20 --cpu-seconds 0 --json-out $O/bench_C2.json
