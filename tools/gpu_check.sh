#!/bin/bash
# One GPU-box session: smoke, GPU parity tests, the C2 bench, a 2-rank tiles-mode bench (ranks
# sharing the GPU over gloo: the N>1 code path), optionally a rocprofv3 kernel-trace profile.
# Usage (from the repo root, on the GPU box):  bash tools/gpu_check.sh <tag> [pytest-args...]
#   env: GC_TESTS=0 skips pytest, GC_PROF=1 adds the rocprofv3 run, GC_BENCH=0 skips the benches
# Every GPU step runs under its own time limit; a Python-level failure (rc 1) lets the next step run,
# anything else (fault, abort, timeout) ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-check}; shift || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
: > "$OUT/status.txt"
step() {
  local name=$1 t=$2; shift 2
  echo "[$(date +%T)] start $name" >> "$OUT/status.txt"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" >> "$OUT/status.txt"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "stopping after $name (rc=$rc)" >> "$OUT/status.txt"
    cat "$OUT/status.txt"; tail -30 "$OUT/$name.log"
    exit $rc
  fi
  return 0
}
step smoke 420 python __graft_entry__.py smoke
if [ "${GC_TESTS:-1}" = 1 ]; then
  step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread "$@"
fi
if [ "${GC_BENCH:-1}" = 1 ]; then
  step bench 300 python bench.py --steps 200 --warmup 20 --cpu-seconds 10 --json-out "$OUT/bench.json"
  step bench_2rank 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --gpus 2 --backend gloo --steps 20 --warmup 3 --json-out "$OUT/bench_2rank.json"
fi
if [ "${GC_PROF:-0}" = 1 ]; then
  step rocprof 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
    python3 bench.py --steps 100 --warmup 10 --cpu-seconds 0
fi
cat "$OUT/status.txt"
grep -E "passed|failed|error" "$OUT/pytest_gpu.log" | tail -3
cat "$OUT/bench.json" "$OUT/bench_2rank.json" 2>/dev/null || true
