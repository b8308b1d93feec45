#!/bin/bash
# Round-4 session f: C2 block size (waves per block) with and without the learnt order; variants
# built by tools/ab_build.py --only-b 3 (ab/c2_*.so), benched through RTX_HIP_LIB, alternating.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r4f; mkdir -p $O
run() { local name=$1 t=$2; shift 2; echo "[$(date +%T)] $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "[$(date +%T)] $name rc=$rc"; [ $rc -le 1 ] || exit $rc; }
B="--config C2 --steps 400 --warmup 20 --cpu-seconds 0 --no-secondary"
for i in 1 2; do
  for v in c2_base c2_w1 c2_w2; do
    RTX_HIP_LIB=ab/$v.so run ${v}_order_$i 120 python bench.py $B --json-out $O/${v}_order_$i.json
    RTX_HIP_LIB=ab/$v.so run ${v}_plain_$i 120 python bench.py $B --no-tile-order --json-out $O/${v}_plain_$i.json
  done
done
for v in c2_base c2_w1 c2_w2; do
  RTX_HIP_LIB=ab/$v.so run ${v}_C1 120 python bench.py --config C1 --steps 400 --warmup 20 --cpu-seconds 0 --no-secondary --json-out $O/${v}_C1.json
  RTX_HIP_LIB=ab/$v.so run ${v}_C2main 120 python bench.py --config C2main --steps 400 --warmup 20 --cpu-seconds 0 --no-secondary --json-out $O/${v}_C2main.json
done
run bench_default 300 python bench.py --steps 200 --warmup 20 --cpu-seconds 0 --json-out $O/bench_default.json
