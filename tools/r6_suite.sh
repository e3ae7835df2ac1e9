# full GPU suite, then the drop-in phase profile and the headline's early windows
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/su
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/su/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/su/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/dropin_phases.py > gpurun_out/su/phases.txt 2>&1 && head -3 gpurun_out/su/phases.txt && \
timeout -k 10 200 python3 tools/first_windows.py > gpurun_out/su/windows.txt 2>&1 && cat gpurun_out/su/windows.txt
