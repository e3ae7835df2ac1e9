#!/bin/bash
# Lockstep test phase on the box: its GPU tests, the GPI / runner tests the shared row kernel
# touches, and the test-phase rates both ways.
set -o pipefail
mkdir -p gpurun_out/lockstep
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_lockstep.py ${LOCKSTEP_TESTS:-tests/test_gpu_engine.py tests/test_gpu_runner.py} > gpurun_out/lockstep/pytest.log 2>&1 &&
timeout -k 10 240 python -u tools/test_phase.py > gpurun_out/lockstep/rates.json 2> gpurun_out/lockstep/rates.err
