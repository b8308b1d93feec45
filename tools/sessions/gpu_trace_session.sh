#!/bin/bash
# Tile-trace session on the GPU box (tools/tile_trace.py over a library built with the tile_trace
# instrument: python tools/ab_build.py ab/trace.so --patch tile_trace --only-b 3,4,5).
# Usage: bash tools/sessions/gpu_trace_session.sh <tag> "<config parts part> ..."
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${1:-trace}; mkdir -p $O
CASES=${2:-"C4,8,0 C4,1,0 C2,1,0"}
for c in $CASES; do
  IFS=, read -r cfg parts part <<< "$c"
  echo "[$(date +%T)] $cfg $parts $part"
  timeout -k 10 150 python tools/tile_trace.py ab/trace.so --config $cfg --parts $parts --part $part \
    --dump $O/rec_${cfg}_${parts}_${part}.npy > $O/trace_${cfg}_${parts}_${part}.json 2> $O/trace_${cfg}_${parts}_${part}.err \
    || { echo "rc=$? on $c"; tail -20 $O/trace_${cfg}_${parts}_${part}.err; exit 1; }
done
echo done
