cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/tsft
timeout -k 10 300 python -u -m pytest tests/test_gpu_tsf.py -v -s --timeout 120 --timeout-method thread > gpurun_out/tsft/t.log 2>&1; rc=$?
grep -E "PASSED|FAILED|Mismatch|Max abs|Max rel|assert " gpurun_out/tsft/t.log | head -60; exit $rc
