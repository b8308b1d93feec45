set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r2j; mkdir -p $OUT
for v in sm3 sm4; do
  RTX_HIP_LIB=ab/$v.so timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/pytest_$v.log 2>&1; echo "$v rc=$?"
  grep -E "passed|failed|AssertionError: \(" $OUT/pytest_$v.log | tail -6
done
AB_TESTS=0 bash tools/ab_run.sh r2j_ab C2,C2main,C5,C3 ab/cur.so ab/sm3.so ab/sm4.so ab/approx.so 2>&1 | grep -E "median|=="
