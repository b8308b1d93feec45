#!/bin/bash
# Per-config measurement session on the GPU box: GPU tests, then for each BASELINE config a
# bench.py line (roofline + CPU baselines) and a rocprofv3 kernel-trace of the same command.
# Usage: bash tools/gpu_profile.sh <tag> "<configs>"      (env GP_TESTS=0 skips pytest)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-prof}; CFGS=${2:-"C1 C2 C2main C3 C4 C5"}
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
    echo "stopping after $name (rc=$rc)" >> "$OUT/status.txt"; cat "$OUT/status.txt"; tail -30 "$OUT/$name.log"; exit $rc
  fi
  return 0
}
bargs() {  # bench arguments of a config: C5 renders one rank's 32 orbit frames per step (one launch)
  case $1 in
    C5) echo "--config C5 --frames-per-step 32 --steps 20 --warmup 3" ;;
    C4) echo "--config C4 --steps 30 --warmup 3" ;;
    C3) echo "--config C3 --steps 100 --warmup 10" ;;
    *) echo "--config $1 --steps 200 --warmup 20" ;;
  esac
}
if [ "${GP_TESTS:-1}" = 1 ]; then
  step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread
fi
for c in $CFGS; do
  step "bench_$c" 300 python bench.py $(bargs $c) --cpu-seconds 10 --json-out "$OUT/bench_$c.json"
  step "rocprof_$c" 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$c" -o run -- \
    python3 bench.py $(bargs $c) --cpu-seconds 0
done
cat "$OUT/status.txt"
for c in $CFGS; do cat "$OUT/bench_$c.json" 2>/dev/null | cut -c1-400; done
