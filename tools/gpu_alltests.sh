cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/all
timeout -k 10 500 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread "$@" > gpurun_out/all/t.log 2>&1; rc=$?
grep -E "FAILED|passed|failed" gpurun_out/all/t.log | tail -30; exit $rc
