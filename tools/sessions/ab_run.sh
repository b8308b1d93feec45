#!/bin/bash
# A/B session on the GPU box: GPU tests on the default build, then tools/ab.py over configs.
# Usage: bash tools/sessions/ab_run.sh <tag> <configs (comma list)> <lib.so>...   (env: AB_ROUNDS, AB_ITERS, AB_BOUNCES)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1; CFGS=$2; shift 2
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
if [ "${AB_TESTS:-1}" = 1 ]; then
  step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
fi
for c in ${CFGS//,/ }; do
  B=()
  if [ -n "${AB_BOUNCES:-}" ]; then B=(--bounces "$AB_BOUNCES"); fi
  step "ab_$c" 300 python -u tools/ab.py --config "$c" --rounds "${AB_ROUNDS:-7}" --iters "${AB_ITERS:-30}" "${B[@]}" "$@"
done
cat "$OUT/status.txt"
tail -3 "$OUT/pytest_gpu.log" 2>/dev/null
for c in ${CFGS//,/ }; do echo "== $c"; cat "$OUT/ab_$c.log"; done
