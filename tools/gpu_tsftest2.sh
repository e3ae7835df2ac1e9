cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/tsft2
timeout -k 10 300 python -u -m pytest tests/test_gpu_phi.py -v --timeout 120 --timeout-method thread > gpurun_out/tsft2/t.log 2>&1; rc=$?
grep -E "PASSED|FAILED|Error|^E " gpurun_out/tsft2/t.log | head -60; exit $rc
