#!/bin/bash
# the gate-timeout stress test, 10 times under each environment setting (assertion flakes, not faults)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/gate
for E in "$@"; do
  f=0
  n=$(echo "$E" | tr -c 'A-Za-z0-9_\n' '_')
  for i in 1 2 3 4 5 6 7 8 9 10; do
    env $E timeout -k 10 120 python -u -m pytest -q --timeout 100 --timeout-method thread "tests/test_gpu_runner.py::test_runner_gate_timeouts_cancel_and_retry" > gpurun_out/gate/$n.$i.log 2>&1
    rc=$?
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "$E run $i rc=$rc"; exit $rc; fi
    [ $rc -eq 1 ] && f=$((f+1))
  done
  echo "$E: $f of 10 runs failed"
done
