set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r4a; mkdir -p $O
for c in "C4 8 0" "C4 1 0" "C4 8 3" "C2 1 0" "C2 8 0" "C3 1 0" "C5 1 0"; do
  set -- $c
  echo "[$(date +%T)] $1 $2 $3"
  timeout -k 10 150 python tools/tile_trace.py ab/trace.so --config $1 --parts $2 --part $3 --dump $O/rec_$1_$2_$3.npy > $O/trace_$1_$2_$3.json 2> $O/trace_$1_$2_$3.err || { echo "rc=$? on $c"; tail -20 $O/trace_$1_$2_$3.err; exit 1; }
done
echo done
