#!/bin/bash
# One GPU-box session: smoke, GPU parity tests, a short bench, a rocprofv3 kernel-trace profile.
# Usage (from the repo root, on the GPU box):  bash tools/gpu_check.sh <tag> [pytest-args...]
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
step pytest_gpu 600 python -m pytest tests -m gpu -x -q "$@"
step bench 300 python bench.py --steps 100 --warmup 20 --cpu-seconds 10 --json-out "$OUT/bench.json"
step rocprof 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
  python3 bench.py --steps 100 --warmup 10 --cpu-seconds 0
cat "$OUT/status.txt"
tail -5 "$OUT/pytest_gpu.log"
cat "$OUT/bench.json" 2>/dev/null
