cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_native_shard.py tests/test_gpu_runner.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r02c_tests.log 2>&1
rc=$?
tail -25 gpurun_out/r02c_tests.log
exit $rc
