#!/bin/bash
# drop-in loop: GPU test + the two timings (tools/dropin_loop.py)
set -o pipefail
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_dropin_loop.py > gpurun_out/dropin_test.log 2>&1 &&
timeout -k 10 300 python -u tools/dropin_loop.py > gpurun_out/dropin_bench.log 2>&1
rc=$?
tail -5 gpurun_out/dropin_test.log; cat gpurun_out/dropin_bench.log | tail -5
exit $rc
