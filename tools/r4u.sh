#!/bin/bash
# The bounds-check build (libsfx_check.so) over the GPU suite with the round-4 defaults (tail tile,
# 2 column tiles), then the runner + engine suites with the tail on every plain launch.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-r4u}
mkdir -p $O
L=$PWD/deep-successor-features-for-transfer_amd/sfx/libsfx_check.so
SFX_LIB=$L SFX_CHECK_RUN=1 timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $O/check_suite.log 2>&1; rc=$?; tail -2 $O/check_suite.log; [ $rc -eq 0 ] || exit $rc
SFX_FWD_TAIL=2 SFX_LIB=$L SFX_CHECK_RUN=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_runner.py tests/test_gpu_engine.py -q --timeout 200 --timeout-method thread > $O/check_tail2.log 2>&1; rc=$?; tail -2 $O/check_tail2.log; exit $rc
