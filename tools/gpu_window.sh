cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/win
timeout -k 10 300 python tools/window_rates.py "$@" > gpurun_out/win/w.log 2>&1; rc=$?
cat gpurun_out/win/w.log | grep -v "^$" | tail -30; exit $rc
