#!/bin/bash
# Round-4 session c: GPU tests, then the learnt dispatch order A/B (bench lines with and without it,
# alternating, one box) on C2 / C2main / C3 / C5, and the C4 8-part emulation.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r4c; mkdir -p $O
run() { local name=$1 t=$2; shift 2; echo "[$(date +%T)] $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "[$(date +%T)] $name rc=$rc"; [ $rc -le 1 ] || exit $rc; }
run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread
B="--cpu-seconds 0 --no-secondary"
for i in 1 2 3; do
  run C2_order_$i 120 python bench.py --config C2 --steps 400 --warmup 20 $B --json-out $O/C2_order_$i.json
  run C2_plain_$i 120 python bench.py --config C2 --steps 400 --warmup 20 $B --no-tile-order --json-out $O/C2_plain_$i.json
done
for c in C2main C1; do
  run ${c}_order 120 python bench.py --config $c --steps 400 --warmup 20 $B --json-out $O/${c}_order.json
  run ${c}_plain 120 python bench.py --config $c --steps 400 --warmup 20 $B --no-tile-order --json-out $O/${c}_plain.json
done
run C3_order 200 python bench.py --config C3 --steps 100 --warmup 10 $B --json-out $O/C3_order.json
run C3_plain 200 python bench.py --config C3 --steps 100 --warmup 10 $B --no-tile-order --json-out $O/C3_plain.json
run C5_order 200 python bench.py --config C5 --frames-per-step 32 --steps 20 --warmup 3 $B --json-out $O/C5_order.json
run C4_order 200 python bench.py --config C4 --steps 30 --warmup 3 $B --json-out $O/C4_order.json
run C4_plain 200 python bench.py --config C4 --steps 30 --warmup 3 $B --no-tile-order --json-out $O/C4_plain.json
run emul_C4 300 python bench.py --config C4 --emulate-parts 2,4,8 --steps 20 --json-out $O/emul_C4.json
run emul_C2 300 python bench.py --config C2 --emulate-parts 2,4,8 --steps 50 --json-out $O/emul_C2.json
run C4_tiles_direct 200 python bench.py --config C4 --mode tiles --steps 10 --warmup 2 --cpu-seconds 0 --json-out $O/C4_tiles_direct.json
run C4_tiles_loop 200 python bench.py --config C4 --mode tiles --loopback --steps 10 --warmup 2 --cpu-seconds 0 --json-out $O/C4_tiles_loop.json
run C2_tiles_loop 200 python bench.py --config C2 --mode tiles --loopback --steps 200 --warmup 20 --cpu-seconds 0 --json-out $O/C2_tiles_loop.json
