#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, no tracing domains combined with --pmc) over the
# bench command, plus the FP64 peak microbenchmark and the counter list.
# Usage on the GPU box: bash tools/pmc.sh <tag> [bench args...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-pmc}; shift || true
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
BENCH=(python3 bench.py --steps 20 --warmup 3 --cpu-seconds 0 "$@")
if [ -x tools/fp64_peak ]; then step fp64_peak 120 tools/fp64_peak; fi
step list 120 rocprofv3 -L
step pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- "${BENCH[@]}"
step pmc_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- "${BENCH[@]}"
step pmc_sq 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --output-format csv -d "$OUT/sq" -o run -- "${BENCH[@]}"
step pmc_valu 300 rocprofv3 --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_THREAD_CYCLES_VALU --output-format csv -d "$OUT/valu" -o run -- "${BENCH[@]}"
cat "$OUT/status.txt"
cat "$OUT/fp64_peak.log" 2>/dev/null
