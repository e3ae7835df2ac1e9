#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_phi.py tests/test_gpu_engine.py > gpurun_out/phi_tests.log 2>&1 && tail -2 gpurun_out/phi_tests.log && bash tools/ab_head.sh
