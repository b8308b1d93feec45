#!/bin/bash
# Round-4 session n: GPU tests after the box-test counter (RTX_S_BOXES); C3 / C4 bench lines with it.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r4n; mkdir -p $O
run() { local name=$1 t=$2; shift 2; echo "[$(date +%T)] $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "[$(date +%T)] $name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread
run smoke 300 python __graft_entry__.py smoke
run bench_C4 300 python bench.py --config C4 --steps 30 --warmup 3 --cpu-seconds 10 --json-out $O/bench_C4.json
run bench_C3 300 python bench.py --config C3 --steps 100 --warmup 10 --cpu-seconds 10 --json-out $O/bench_C3.json
run bench_default 300 python bench.py --json-out $O/bench_default.json
