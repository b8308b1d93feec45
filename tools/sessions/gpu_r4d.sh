#!/bin/bash
# Round-4 session d: the gather beside the next render (C4 loopback plan) by reserved block slots.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r4d; mkdir -p $O
run() { local name=$1 t=$2; shift 2; echo "[$(date +%T)] $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "[$(date +%T)] $name rc=$rc"; [ $rc -le 1 ] || exit $rc; }
T="--config C4 --mode tiles --steps 20 --warmup 3 --cpu-seconds 0"
run direct 200 python bench.py $T --json-out $O/direct.json
for r in 0 16 64 128 256; do
  run loop_$r 200 python bench.py $T --loopback --comm-reserve $r --json-out $O/loop_$r.json
done
run direct2 200 python bench.py $T --json-out $O/direct2.json
run loop_C2 200 python bench.py --config C2 --mode tiles --steps 200 --warmup 20 --cpu-seconds 0 --loopback --json-out $O/loop_C2.json
# C4 kernel variants (tools/ab_build.py --only-b 5; bench through RTX_HIP_LIB, learnt order on)
for v in base5 nopersist nobeam base5; do
  RTX_HIP_LIB=ab/$v.so run C4_$v 200 python bench.py --config C4 --steps 30 --warmup 3 --cpu-seconds 0 --no-secondary --json-out $O/C4_$v.json
done
for i in 1 2; do
  run C2main_order_$i 120 python bench.py --config C2main --steps 400 --warmup 20 --cpu-seconds 0 --no-secondary --json-out $O/C2main_order_$i.json
  run C2main_plain_$i 120 python bench.py --config C2main --steps 400 --warmup 20 --cpu-seconds 0 --no-secondary --no-tile-order --json-out $O/C2main_plain_$i.json
done
