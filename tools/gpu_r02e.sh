cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_native_shard.py tests/test_gpu_shard.py tests/test_gpu_runner.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r02e_tests.log 2>&1
rc=$?
tail -40 gpurun_out/r02e_tests.log
[ $rc -eq 0 ] && timeout -k 10 300 python bench.py --no-other --no-cpu-baseline --repeats 1 > gpurun_out/r02e_bench.log 2>&1
rc=$?
tail -c 1500 gpurun_out/r02e_bench.log
exit $rc
