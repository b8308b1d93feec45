#!/bin/bash
# Round-4 session l: instruction-cache counters of the render kernels (the C4 kernel is ~28 k
# instructions, C3 ~12 k, C2 ~5 k): list the box's counters, then one SQC pass and one SQ pass per
# config, each under a hard time limit.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r4l; mkdir -p $O
timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1; echo "list rc=$?"
grep -iE "icache|ifetch|SQC_" $O/counters.txt | head -60 > $O/icache_counters.txt
cat $O/icache_counters.txt | head -40
for c in C2 C3 C4; do
  P="--config $c --steps 10 --warmup 2 --cpu-seconds 0 --no-secondary --ramp-ms 50"
  timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES --output-format csv -d $O/pmc_$c/sqc -o run -- python3 bench.py $P > $O/sqc_$c.log 2>&1
  rc=$?; echo "sqc $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
  timeout -s KILL 90 rocprofv3 --pmc SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU --output-format csv -d $O/pmc_$c/sq -o run -- python3 bench.py $P > $O/sq_$c.log 2>&1
  rc=$?; echo "sq $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
