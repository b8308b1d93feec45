#!/bin/bash
# Round-4 session h: GPU tests (weighted-share parity); C4 / C2 part emulation with the default shares
# and with equal shares; HBM traffic (FETCH_SIZE, WRITE_SIZE) and kernel time of C3 / C4 with and
# without the learnt order and its cost records (ab/h_*.so through RTX_HIP_LIB).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r4h; mkdir -p $O
run() { local name=$1 t=$2; shift 2; echo "[$(date +%T)] $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "[$(date +%T)] $name rc=$rc"; [ $rc -le 1 ] || exit $rc; }
run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread
run emul_C4 300 python bench.py --config C4 --emulate-parts 2,4,8 --steps 20 --json-out $O/emul_C4.json
run emul_C4_eq 300 python bench.py --config C4 --emulate-parts 4,8 --shares 1,1 --steps 20 --json-out $O/emul_C4_eq.json
run emul_C2 300 python bench.py --config C2 --emulate-parts 2,4,8 --steps 50 --json-out $O/emul_C2.json
for c in C3 C4; do
  P="--config $c --steps 10 --warmup 2 --cpu-seconds 0 --no-secondary --ramp-ms 50"
  for v in h_base h_plain h_pplain; do
    for o in order plain; do
      [ $o = plain ] && X=--no-tile-order || X=
      [ $v != h_base ] && [ $o = order ] && continue
      RTX_HIP_LIB=ab/$v.so run pmc_fetch_${c}_${v}_$o 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_${c}_${v}_$o/fetch -o run -- python3 bench.py $P $X
      RTX_HIP_LIB=ab/$v.so run pmc_write_${c}_${v}_$o 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_${c}_${v}_$o/write -o run -- python3 bench.py $P $X
    done
  done
done
for c in C3 C4; do
  [ $c = C4 ] && S="--steps 30 --warmup 3" || S="--steps 100 --warmup 10"
  for v in h_base h_plain h_pplain h_base; do
    RTX_HIP_LIB=ab/$v.so run t_${c}_$v 200 python bench.py --config $c $S --cpu-seconds 0 --no-secondary --json-out $O/t_${c}_$v.json
  done
  RTX_HIP_LIB=ab/h_base.so run t_${c}_h_base_plain 200 python bench.py --config $c $S --cpu-seconds 0 --no-secondary --no-tile-order --json-out $O/t_${c}_h_base_plain.json
done
