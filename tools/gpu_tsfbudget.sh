cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/tsfb
timeout -k 10 300 python tools/tsf_error_budget.py > gpurun_out/tsfb/b.log 2>&1; rc=$?
grep -v "^$\|amdgpu.ids" gpurun_out/tsfb/b.log | tail -60; exit $rc
