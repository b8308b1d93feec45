#!/bin/bash
# Generic GPU-box session: run named steps in order, each under its own time limit, logs under
# gpurun_out/<tag>/<name>.log. A Python-level failure (rc 1) lets the next step run; a fault, abort,
# timeout or hang (any other rc) ends the session there.
# Usage (repo root, on the GPU box):  bash tools/gpu_steps.sh <tag> "<name>|<seconds>|<command>" ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
: > "$OUT/status.txt"
for spec in "$@"; do
  name=${spec%%|*}; rest=${spec#*|}; t=${rest%%|*}; cmd=${rest#*|}
  cmd=${cmd//@OUT@/$OUT}
  echo "[$(date +%T)] start $name" >> "$OUT/status.txt"
  timeout -k 10 "$t" bash -c "$cmd" > "$OUT/$name.log" 2>&1
  rc=$?
  echo "[$(date +%T)] $name rc=$rc" >> "$OUT/status.txt"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "stopping after $name (rc=$rc)" >> "$OUT/status.txt"
    cat "$OUT/status.txt"; tail -30 "$OUT/$name.log"
    exit $rc
  fi
done
cat "$OUT/status.txt"
