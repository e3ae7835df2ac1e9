cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
timeout -k 10 120 python tools/dbg_shard2.py none > gpurun_out/r02h_dbg0.log 2>&1
timeout -k 10 120 python tools/dbg_shard2.py first > gpurun_out/r02h_dbg1.log 2>&1
tail -2 gpurun_out/r02h_dbg0.log gpurun_out/r02h_dbg1.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_dropin.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r02h_tests.log 2>&1
rc=$?
tail -14 gpurun_out/r02h_tests.log
exit $rc
