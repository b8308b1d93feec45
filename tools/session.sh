#!/bin/bash
# One parameterised GPU-box measurement session (replaces the one-off tools/sessions/gpu_r4*.sh
# scripts, which stay in git history). Usage, from the repo root on the box:
#
#   bash tools/session.sh TAG STEP [STEP ...]
#
# Every step runs under its own time limit; the session stops at the first failing step (a fault,
# an abort or a time limit ends the GPU work of the call). Output: gpurun_out/TAG/<step>.log (+ the
# step's JSON / rocprof directories). Steps:
#   tests            pytest -m gpu (one process, per-test time limit)
#   tests:EXPR       pytest -m gpu -k EXPR
#   smoke            __graft_entry__.smoke()
#   bench            the default bench line (bench.py with no flags: what the driver runs)
#   bench2[:C]       bench.py at N = 2 over gloo, both ranks on the one GPU (the N > 1 code path)
#   unbounded:C      config C's line with the reference's unbounded recursion (HipRenderer's default)
#   bench:C          bench line of config C (C1 C2 C2main C3 C4 C5), CPU baselines included
#   rocprof:C        rocprofv3 --kernel-trace --stats of config C's timed bench (no secondary legs)
#   pmc:C            the PMC passes of config C: FETCH_SIZE, WRITE_SIZE, SQ cycles, VALU mix (one pass each)
#   emul:C           bench.py --emulate-parts 2,4,8 for config C
#   tiles:C          bench.py --mode tiles --loopback for config C (the RCCL gather path on one GPU)
#   fuzz:N:SEED[:SCALE]  tools/fuzz_parity.py over N random scenes from SEED (frames SCALE times larger)
#   repro:VARIANT[:BYTES]  tools/capture_repro VARIANT (RCCL under graph capture; memcpy|plain|fork|stale)
#   capture:VARIANT  tools/capture_tiles.py VARIANT (a gathering tiles plan under graph capture)
#   ab:ARGS          tools/ab.py with ARGS (comma-separated, e.g. ab:--config,C2,--variants,base,x)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:?usage: tools/session.sh TAG STEP...}
shift
O=gpurun_out/$TAG
mkdir -p "$O"
run() {
  local name=$1 t=$2
  shift 2
  echo "[$(date +%T)] $name"
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc"
  [ $rc -eq 0 ] || { tail -25 "$O/$name.log"; exit $rc; }
}
bargs() {
  case $1 in
    C5) echo "--config C5 --frames-per-step 32 --steps 20 --warmup 3" ;;
    C4) echo "--config C4 --steps 30 --warmup 3" ;;
    C3) echo "--config C3 --steps 100 --warmup 10" ;;
    *) echo "--config $1 --steps 200 --warmup 20" ;;
  esac
}
for step in "$@"; do
  kind=${step%%:*}
  arg=${step#*:}
  [ "$arg" = "$step" ] && arg=""
  case $kind in
    tests)
      if [ -n "$arg" ]; then
        run "pytest_gpu_$(echo "$arg" | tr -c 'a-zA-Z0-9_' '_')" 900 python -u -m pytest tests -m gpu -x -v -rP \
          -p no:cacheprovider --timeout 120 --timeout-method thread -k "$arg"
      else
        run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v -rP -p no:cacheprovider --timeout 120 \
          --timeout-method thread
      fi ;;
    smoke) run smoke 300 python __graft_entry__.py smoke ;;
    unbounded)
      # the drop-in default: HipRenderer() with the reference's unbounded recursion
      run "unbounded_$arg" 300 python bench.py $(bargs "$arg") --bounces -1 --cpu-seconds 0 --no-secondary \
        --json-out "$O/unbounded_$arg.json" ;;
    bench)
      if [ -n "$arg" ]; then
        run "bench_$arg" 300 python bench.py $(bargs "$arg") --cpu-seconds 10 --json-out "$O/bench_$arg.json"
      else
        run bench_default 300 python bench.py --json-out "$O/bench_default.json"
      fi ;;
    bench2)
      # two ranks sharing the box's one GPU over gloo (bench.py --backend gloo): the N > 1 frames line
      # (distinct frames per rank), strong_scaling and the tiles legs through the gloo path
      run bench2_gloo 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
        --master-port 29517 bench.py --gpus 2 --backend gloo --config "${arg:-C2}" --steps 50 --warmup 5 \
        --cpu-seconds 0 --json-out "$O/bench2_gloo.json" ;;
    rocprof)
      run "rocprof_$arg" 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_$arg" -o run -- \
        python3 bench.py $(bargs "$arg") --cpu-seconds 0 --no-secondary ;;
    pmc)
      P="--config $arg --steps 10 --warmup 2 --cpu-seconds 0 --no-secondary --ramp-ms 50"
      [ "$arg" = C5 ] && P="$P --frames-per-step 32"  # the C5 bench line's launch: 32 frames
      run "pmc_fetch_$arg" 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/pmc_$arg/fetch" -o run -- \
        python3 bench.py $P
      run "pmc_write_$arg" 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/pmc_$arg/write" -o run -- \
        python3 bench.py $P
      run "pmc_sq_$arg" 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
        SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --output-format csv -d "$O/pmc_$arg/sq" -o run -- \
        python3 bench.py $P
      run "pmc_valu_$arg" 120 rocprofv3 --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 \
        SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_THREAD_CYCLES_VALU --output-format csv \
        -d "$O/pmc_$arg/valu" -o run -- python3 bench.py $P ;;
    emul)
      run "emul_$arg" 300 python bench.py --config "$arg" --emulate-parts 2,4,8 --steps 20 --json-out "$O/emul_$arg.json" ;;
    tiles)
      run "tiles_$arg" 300 python bench.py --config "$arg" --mode tiles --loopback --steps 20 --warmup 3 --cpu-seconds 0 \
        --json-out "$O/tiles_$arg.json" ;;
    fuzz)
      n=${arg%%:*}
      rest=${arg#*:}
      seed=${rest%%:*}
      scale=${rest#*:}
      [ "$scale" = "$rest" ] && scale=1
      run "fuzz_${seed}_x$scale" 500 python -u tools/fuzz_parity.py --n "$n" --seed0 "$seed" --scale "$scale" \
        --out "$O/fuzz_${seed}_x$scale.json" ;;
    repro)
      # tools/capture_repro.cpp variant ARG over torch's librccl and HIP runtime (the crash's setting)
      TL=$(python -c "import torch, os; print(os.path.dirname(torch.__file__) + '/lib')")
      v=${arg%%:*}
      bytes=${arg#*:}
      [ "$bytes" = "$arg" ] && bytes=""
      LD_LIBRARY_PATH=$TL run "repro_${v}_${bytes:-1MiB}" 60 tools/capture_repro "$v" "$TL/librccl.so" $bytes ;;
    capture)
      # tools/capture_tiles.py ARG: a gathering tiles plan captured into a HIP graph (native backtrace on a crash)
      run "capture_$arg" 120 python -u tools/capture_tiles.py "$arg" ;;
    ab)
      run "ab_$(echo "$arg" | tr -c 'a-zA-Z0-9_' '_' | cut -c1-90)" 900 python -u tools/ab.py $(echo "$arg" | tr ',' ' ') ;;
    *)
      echo "unknown step $step"
      exit 2 ;;
  esac
done
echo "[$(date +%T)] session $TAG done"
