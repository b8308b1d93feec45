set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r2i; mkdir -p $OUT
RTX_HIP_LIB=ab/core.so timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/pytest_core.log 2>&1; echo "core rc=$?"
tail -4 $OUT/pytest_core.log
AB_TESTS=0 bash tools/ab_run.sh r2i_ab C2,C2main,C5,C3,C4 ab/cur.so ab/core.so ab/approx.so ab/inlgen.so 2>&1 | grep -E "median|=="
