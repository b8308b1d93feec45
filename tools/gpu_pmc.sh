#!/bin/bash
# PMC session on the GPU box (each counter group in its own rocprofv3 run, nothing else combined
# with --pmc): the traffic calibration kernels, FETCH_SIZE/WRITE_SIZE per config, the SQ/VALU groups
# for C2 and C4, and optionally extra library builds on C2.
# Usage: bash tools/gpu_pmc.sh <tag> [lib.so ...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-pmc}; shift || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
: > "$OUT/status.txt"
run() {  # run <name> <counters...> -- <cmd...>
  local name=$1; shift
  local ctr=()
  while [ "$1" != "--" ]; do ctr+=("$1"); shift; done; shift
  echo "[$(date +%T)] start $name" >> "$OUT/status.txt"
  timeout -k 10 240 rocprofv3 --pmc "${ctr[@]}" --output-format csv -d "$OUT/$name" -o run -- "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" >> "$OUT/status.txt"
  if [ $rc -ne 0 ]; then cat "$OUT/status.txt"; tail -20 "$OUT/$name.log"; exit $rc; fi
}
bargs() {
  case $1 in
    C5) echo "--config C5 --frames-per-step 32 --steps 4 --warmup 1" ;;
    C4) echo "--config C4 --steps 6 --warmup 1" ;;
    *) echo "--config $1 --steps 10 --warmup 2" ;;
  esac
}
run calib_write WRITE_SIZE -- tools/traffic_calib
run calib_fetch FETCH_SIZE -- tools/traffic_calib
for c in C1 C2 C2main C3 C4 C5; do
  run "${c}_fetch" FETCH_SIZE -- python3 bench.py $(bargs $c) --cpu-seconds 0 --no-secondary
  run "${c}_write" WRITE_SIZE -- python3 bench.py $(bargs $c) --cpu-seconds 0 --no-secondary
done
for c in C2 C4; do
  run "${c}_sq" SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY -- python3 bench.py $(bargs $c) --cpu-seconds 0
  run "${c}_valu" SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_THREAD_CYCLES_VALU -- python3 bench.py $(bargs $c) --cpu-seconds 0
done
for lib in "$@"; do
  n=$(basename "$lib" .so)
  RTX_HIP_LIB="$lib" run "lib_${n}_C2_fetch" FETCH_SIZE -- python3 bench.py $(bargs C2) --cpu-seconds 0
  RTX_HIP_LIB="$lib" run "lib_${n}_C2_write" WRITE_SIZE -- python3 bench.py $(bargs C2) --cpu-seconds 0
done
cat "$OUT/status.txt"
