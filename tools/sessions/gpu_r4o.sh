#!/bin/bash
# Round-4 session o: randomised parity sweep including the timed kernels (learnt order, probe,
# weighted row shares) against the counting render and the oracle.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r4o; mkdir -p $O
run() { local name=$1 t=$2; shift 2; echo "[$(date +%T)] $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "[$(date +%T)] $name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
run fuzz_s1 500 python -u tools/fuzz_parity.py --n 400 --seed0 40000 --out $O/fuzz_s1.json
run fuzz_s4 400 python -u tools/fuzz_parity.py --n 80 --seed0 41000 --scale 4 --out $O/fuzz_s4.json
