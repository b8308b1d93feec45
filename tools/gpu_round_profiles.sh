#!/bin/bash
# End-of-round measurement session on the GPU box: per BASELINE config a bench.py line (CPU
# baselines included) and a rocprofv3 kernel-trace of the same command, then the PMC passes
# (FETCH_SIZE, WRITE_SIZE, SQ instruction mix, each its own run) for the configs given in PMC_CFGS.
# Usage: bash tools/gpu_round_profiles.sh <tag> "<configs>"   (env PMC_CFGS="C2 C3"; "-" = none)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; CFGS=${2:-"C1 C2 C2main C3 C4 C5"}; PMC=${PMC_CFGS:-"C2 C3"}
bargs() {
  case $1 in
    C5) echo "--config C5 --frames-per-step 32 --steps 20 --warmup 3" ;;
    C4) echo "--config C4 --steps 30 --warmup 3" ;;
    C3) echo "--config C3 --steps 100 --warmup 10" ;;
    *) echo "--config $1 --steps 200 --warmup 20" ;;
  esac
}
steps=()
[ "$CFGS" = "-" ] && CFGS=""
[ "$PMC" = "-" ] && PMC=""
for c in $CFGS; do
  steps+=("bench_$c|300|python bench.py $(bargs $c) --cpu-seconds 10 --json-out @OUT@/bench_$c.json")
  steps+=("rocprof_$c|300|rocprofv3 --kernel-trace --stats --output-format csv -d @OUT@/prof_$c -o run -- python3 bench.py $(bargs $c) --cpu-seconds 0 --no-secondary")
done
for c in $PMC; do
  steps+=("pmc_fetch_$c|120|rocprofv3 --pmc FETCH_SIZE --output-format csv -d @OUT@/pmc_$c/fetch -o run -- python3 bench.py --config $c --steps 10 --warmup 2 --cpu-seconds 0 --no-secondary --ramp-ms 50")
  steps+=("pmc_write_$c|120|rocprofv3 --pmc WRITE_SIZE --output-format csv -d @OUT@/pmc_$c/write -o run -- python3 bench.py --config $c --steps 10 --warmup 2 --cpu-seconds 0 --no-secondary --ramp-ms 50")
  steps+=("pmc_sq_$c|120|rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --output-format csv -d @OUT@/pmc_$c/sq -o run -- python3 bench.py --config $c --steps 10 --warmup 2 --cpu-seconds 0 --no-secondary --ramp-ms 50")
  steps+=("pmc_valu_$c|120|rocprofv3 --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_THREAD_CYCLES_VALU --output-format csv -d @OUT@/pmc_$c/valu -o run -- python3 bench.py --config $c --steps 10 --warmup 2 --cpu-seconds 0 --no-secondary --ramp-ms 50")
done
exec_steps() { bash tools/gpu_steps.sh "$TAG" "${steps[@]}"; }
exec_steps
