#!/bin/bash
# TSF GPU tests, then A/B of this build vs libsfx_prev.so on Hopper TSF-NF (K = 100)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_tsf.py tests/test_gpu_tsf_test.py tests/test_gpu_shard.py > gpurun_out/tsf_tests.log 2>&1
rc=$?; tail -1 gpurun_out/tsf_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_libs.sh "libsfx_prev.so libsfx.so" --workload hopper-tsf-nf
