#!/bin/bash
# Round-4 session b: GPU tests (learnt tile order, octant tree layouts, native tiles), C4 part
# emulation A/B (tile order, octant layouts), the C4 bench line with the reflected-ray counters, the
# unperturbed tile trace.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r4b; mkdir -p $O
run() { local name=$1 t=$2; shift 2; echo "[$(date +%T)] $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "[$(date +%T)] $name rc=$rc"; [ $rc -le 1 ] || exit $rc; }
run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread
run emul_order 300 python bench.py --config C4 --emulate-parts 8 --steps 20 --json-out $O/emul_C4_order.json
run emul_plain 300 python bench.py --config C4 --emulate-parts 8 --steps 20 --no-tile-order --json-out $O/emul_C4_plain.json
run emul_nooct 300 python bench.py --config C4 --emulate-parts 8 --steps 20 --no-octant-tree --json-out $O/emul_C4_nooct.json
run bench_C4 300 python bench.py --config C4 --steps 30 --warmup 3 --cpu-seconds 0 --json-out $O/bench_C4.json
run bench_C4_nooct 300 python bench.py --config C4 --steps 30 --warmup 3 --cpu-seconds 0 --no-secondary --no-octant-tree --json-out $O/bench_C4_nooct.json
bash tools/sessions/gpu_trace_session.sh r4b_trace "C4,8,0 C4,1,0 C2,1,0"
