cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/hb
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/hb/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/hb/pytest.log; [ $rc -eq 0 ] || exit $rc
BUFFER=host timeout -k 10 200 python3 tools/dropin_phases.py > gpurun_out/hb/out.txt 2>&1 && head -3 gpurun_out/hb/out.txt
