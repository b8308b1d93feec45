#!/bin/bash
# Round-4 session k (final build, weighted shares, cost records in the STATS kernels): GPU tests; per BASELINE config the bench line (CPU baselines
# included) and a rocprofv3 kernel trace of the same command; PMC passes (traffic, SQ instruction
# mix) for C2, C3, C4; the C4 / C2 part emulation.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r4k; mkdir -p $O
run() { local name=$1 t=$2; shift 2; echo "[$(date +%T)] $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "[$(date +%T)] $name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
bargs() {
  case $1 in
    C5) echo "--config C5 --frames-per-step 32 --steps 20 --warmup 3" ;;
    C4) echo "--config C4 --steps 30 --warmup 3" ;;
    C3) echo "--config C3 --steps 100 --warmup 10" ;;
    *) echo "--config $1 --steps 200 --warmup 20" ;;
  esac
}
run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread
run smoke 300 python __graft_entry__.py smoke
run bench_default 300 python bench.py --json-out $O/bench_default.json
for c in C2 C1 C2main C3 C4 C5; do
  run bench_$c 300 python bench.py $(bargs $c) --cpu-seconds 10 --json-out $O/bench_$c.json
  run rocprof_$c 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$c -o run -- python3 bench.py $(bargs $c) --cpu-seconds 0 --no-secondary
done
for c in C2 C3 C4; do
  P="--config $c --steps 10 --warmup 2 --cpu-seconds 0 --no-secondary --ramp-ms 50"
  run pmc_fetch_$c 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_$c/fetch -o run -- python3 bench.py $P
  run pmc_write_$c 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_$c/write -o run -- python3 bench.py $P
  run pmc_sq_$c 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $O/pmc_$c/sq -o run -- python3 bench.py $P
  run pmc_valu_$c 120 rocprofv3 --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_THREAD_CYCLES_VALU --output-format csv -d $O/pmc_$c/valu -o run -- python3 bench.py $P
done
run emul_C4 300 python bench.py --config C4 --emulate-parts 2,4,8 --steps 20 --json-out $O/emul_C4.json
run emul_C2 300 python bench.py --config C2 --emulate-parts 2,4,8 --steps 50 --json-out $O/emul_C2.json
