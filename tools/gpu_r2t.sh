set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r2t; mkdir -p $OUT
timeout -k 10 120 python tools/debug_diff.py 96 54 3 > $OUT/debug.txt 2>&1; cat $OUT/debug.txt | grep -v amdgpu.ids; timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; echo "tests rc=$?"
grep -E "passed|failed|Error" $OUT/pytest.log | tail -5
AB_TESTS=0 bash tools/ab_run.sh r2t_ab C2,C2main,C5,C3,C4 ab/halfb.so ab/inties.so 2>&1 | grep -E "median|=="
