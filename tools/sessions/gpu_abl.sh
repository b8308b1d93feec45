# A/B of ablation builds (timing only; outputs differ by construction)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
AB_TESTS=0 bash tools/sessions/ab_run.sh ${ABL_TAG:-abl} ${ABL_CFGS:-C2,C2main,C3} "$@" 2>&1 | grep -E "median|=="
