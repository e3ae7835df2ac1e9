# The -m gpu suite as the driver runs it (one process, per-test time limit), plus the drop-in host-ring
# profile.  Used to look for flaky tests before the round ends.
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/hb
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/hb/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/hb/pytest.log; exit $rc
