set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r2h; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/pytest_default.log 2>&1; echo "default rc=$?"
tail -3 $OUT/pytest_default.log
RTX_HIP_LIB=ab/approx.so timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/pytest_approx.log 2>&1; echo "approx rc=$?"
tail -15 $OUT/pytest_approx.log
AB_TESTS=0 bash tools/ab_run.sh r2h_ab C2,C2main,C5,C3 ab/cur.so ab/approx.so 2>&1 | grep -E "median|=="
