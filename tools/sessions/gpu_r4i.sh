#!/bin/bash
# Round-4 session i: GPU tests (part_run fix, weighted-share parity); C4 / C2 part emulation with the
# default shares, equal shares and candidate root shares at N = 8; C3 / C4 bench lines and C4 HBM
# traffic with the cost records moved to the STATS kernels.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r4i; mkdir -p $O
run() { local name=$1 t=$2; shift 2; echo "[$(date +%T)] $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "[$(date +%T)] $name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread
run emul_C4 300 python bench.py --config C4 --emulate-parts 2,4,8 --steps 20 --json-out $O/emul_C4.json
for sh in 1,1 3,4 5,6 2,3; do
  run emul_C4_s${sh/,/_} 300 python bench.py --config C4 --emulate-parts 8 --shares $sh --steps 20 --json-out $O/emul_C4_s${sh/,/_}.json
done
run emul_C2 300 python bench.py --config C2 --emulate-parts 2,4,8 --steps 50 --json-out $O/emul_C2.json
run t_C4 200 python bench.py --config C4 --steps 30 --warmup 3 --cpu-seconds 0 --no-secondary --json-out $O/t_C4.json
run t_C3 200 python bench.py --config C3 --steps 100 --warmup 10 --cpu-seconds 0 --no-secondary --json-out $O/t_C3.json
P="--config C4 --steps 10 --warmup 2 --cpu-seconds 0 --no-secondary --ramp-ms 50"
run pmc_fetch_C4 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_C4/fetch -o run -- python3 bench.py $P
run pmc_write_C4 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_C4/write -o run -- python3 bench.py $P
