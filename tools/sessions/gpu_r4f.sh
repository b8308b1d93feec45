#!/bin/bash
# Round-4 session f: GPU tests; the row-block gather (RTX_TILES_ROWS) against gather + assembly on
# the C4 loopback plan (row blocks of 8 and 32); C2 block size (waves per block) with and without
# the learnt order (ab/c2_*.so through RTX_HIP_LIB); the default bench line.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r4f; mkdir -p $O
run() { local name=$1 t=$2; shift 2; echo "[$(date +%T)] $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "[$(date +%T)] $name rc=$rc"; [ $rc -le 1 ] || exit $rc; }
run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread
T="--config C4 --mode tiles --steps 20 --warmup 3 --cpu-seconds 0"
run direct 200 python bench.py $T --json-out $O/direct.json
for rb in 8 32; do
  run loop_rows_rb$rb 200 python bench.py $T --loopback --row-block $rb --json-out $O/loop_rows_rb$rb.json
  run loop_asm_rb$rb 200 python bench.py $T --loopback --assemble --row-block $rb --json-out $O/loop_asm_rb$rb.json
done
run emul_rb32 300 python bench.py --config C4 --emulate-parts 8 --row-block 32 --steps 20 --json-out $O/emul_C4_rb32.json
B="--config C2 --steps 400 --warmup 20 --cpu-seconds 0 --no-secondary"
for v in c2_base c2_w1 c2_w2; do
  RTX_HIP_LIB=ab/$v.so run ${v}_order 120 python bench.py $B --json-out $O/${v}_order.json
  RTX_HIP_LIB=ab/$v.so run ${v}_plain 120 python bench.py $B --no-tile-order --json-out $O/${v}_plain.json
done
run bench_default 300 python bench.py --steps 200 --warmup 20 --cpu-seconds 0 --json-out $O/bench_default.json
# C3: 5 waves with spills (base) against 4 waves without (kLvWaves=4); C4: B=5 at 4 waves with two LDS
# level slots (base, 47 spilled VGPRs) against 3 waves with three (no spills)
for v in c3_base c3_lv4 c3_base; do
  RTX_HIP_LIB=ab/$v.so run ${v}_C3 200 python bench.py --config C3 --steps 100 --warmup 10 --cpu-seconds 0 --no-secondary --json-out $O/${v}_C3.json
done
for v in c4_base c4_b5s3 c4_base; do
  RTX_HIP_LIB=ab/$v.so run ${v}_C4 200 python bench.py --config C4 --steps 30 --warmup 3 --cpu-seconds 0 --no-secondary --json-out $O/${v}_C4.json
done
