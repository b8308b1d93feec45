#!/bin/bash
# Dynamic instruction counts of several library builds (one rocprofv3 --pmc run per build and
# counter group). Usage on the GPU box:
#   bash tools/sessions/pmc_ab.sh <tag> <config> <lib.so>...
# Summaries: python tools/pmc_summary.py gpurun_out/<tag>/<lib-name>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1; CFG=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for lib in "$@"; do
  name=$(basename "$lib" .so)
  for grp in ${PMC_GROUPS:-sq valu}; do
    if [ $grp = sq ]; then
      ctr="SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_ACTIVE_INST_ANY"
    elif [ $grp = lat ]; then
      ctr="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INST_LEVEL_SMEM SQ_INSTS_SMEM SQ_INST_LEVEL_LDS SQ_INSTS_LDS SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM"
    else
      ctr="SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_VALU_INT32"
    fi
    d="$OUT/$name/$grp"; mkdir -p "$OUT/$name"
    RTX_HIP_LIB="$lib" timeout -k 10 240 rocprofv3 --pmc $ctr --output-format csv -d "$d" -o run -- \
      python3 bench.py --config "$CFG" --steps 10 --warmup 2 --cpu-seconds 0 --no-secondary > "$d.log" 2>&1
    rc=$?; echo "$name $grp rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
