#!/bin/bash
# Round-4 session j: (1) HBM traffic of the round-3 build (git worktree _r3 at the round-3 commit,
# built in place) against this build, same box, same bench command, C3 and C4 (the round-4 PMC
# passes read more WRITE_SIZE per launch than round 3's for kernels whose code is unchanged);
# (2) C4 part emulation over root shares at N = 2 and 4.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=$PWD/gpurun_out/r4j; mkdir -p $O
run() { local name=$1 t=$2; shift 2; echo "[$(date +%T)] $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "[$(date +%T)] $name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
for c in C3 C4; do
  P="--config $c --steps 10 --warmup 2 --cpu-seconds 0 --no-secondary"
  for v in r3 r4 r3 r4; do
    if [ $v = r3 ]; then D=_r3; else D=.; fi
    k=$((k+1))
    ( cd $D && run pmc_write_${c}_${v}_$k 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_${c}_${v}_$k/write -o run -- python3 bench.py $P ) || exit 1
    ( cd $D && run pmc_fetch_${c}_${v}_$k 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_${c}_${v}_$k/fetch -o run -- python3 bench.py $P ) || exit 1
  done
done
for sh in 1,1 5,6 8,9 12,13; do
  run emul_C4_n2_s${sh/,/_} 300 python bench.py --config C4 --emulate-parts 2 --shares $sh --steps 20 --json-out $O/emul_C4_n2_s${sh/,/_}.json
done
for sh in 1,1 3,4 4,5 5,6; do
  run emul_C4_n4_s${sh/,/_} 300 python bench.py --config C4 --emulate-parts 4 --shares $sh --steps 20 --json-out $O/emul_C4_n4_s${sh/,/_}.json
done
