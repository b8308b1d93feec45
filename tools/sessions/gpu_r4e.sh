#!/bin/bash
# Round-4 session e: GPU tests; the gather beside the render (C4 loopback plan) by capped RCCL CTAs
# and reserved slots; the round-4 bench lines and rocprof timed regions of C2 and C4.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r4e; mkdir -p $O
run() { local name=$1 t=$2; shift 2; echo "[$(date +%T)] $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "[$(date +%T)] $name rc=$rc"; [ $rc -le 1 ] || exit $rc; }
run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread
T="--config C4 --mode tiles --steps 20 --warmup 3 --cpu-seconds 0"
run direct 200 python bench.py $T --json-out $O/direct.json
for c in 2 4 8; do
  for r in 0 64; do
    RTX_COMM_MAX_CTAS=$c run loop_cta${c}_r$r 200 python bench.py $T --loopback --comm-reserve $r --json-out $O/loop_cta${c}_r$r.json
  done
done
run loop_r0 200 python bench.py $T --loopback --comm-reserve 0 --json-out $O/loop_r0.json
run bench_C2 300 python bench.py --config C2 --steps 200 --warmup 20 --cpu-seconds 10 --json-out $O/bench_C2.json
run rocprof_C2 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_C2 -o run -- python3 bench.py --config C2 --steps 200 --warmup 20 --cpu-seconds 0 --no-secondary
run bench_C4 300 python bench.py --config C4 --steps 30 --warmup 3 --cpu-seconds 10 --json-out $O/bench_C4.json
run rocprof_C4 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_C4 -o run -- python3 bench.py --config C4 --steps 30 --warmup 3 --cpu-seconds 0 --no-secondary
