#!/bin/bash
# HBM traffic (FETCH_SIZE and WRITE_SIZE, separate rocprofv3 passes) of bench.py for several library
# builds and configs. Usage on the GPU box:
#   bash tools/pmc_traffic.sh <tag> "<configs>" <lib.so>...      (configs: space-separated, e.g. "C2 C3")
# Output: gpurun_out/<tag>/<lib>_<config>_{fetch,write}/ ; summarise with tools/pmc_summary.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1; CFGS=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for lib in "$@"; do
  name=$(basename "$lib" .so)
  for c in $CFGS; do
    for ctr in FETCH_SIZE WRITE_SIZE; do
      d="$OUT/${name}_${c}_${ctr}"
      RTX_HIP_LIB="$lib" timeout -k 10 300 rocprofv3 --pmc "$ctr" --output-format csv -d "$d" -o run -- \
        python3 bench.py --config "$c" --steps 10 --warmup 2 --cpu-seconds 0 > "$d.log" 2>&1
      rc=$?; echo "$name $c $ctr rc=$rc"; [ $rc -eq 0 ] || exit $rc
    done
  done
done
