#!/bin/bash
# the gate-timeout stress test, 10 times with each library (assertion flakes, not faults)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/gate
L=deep-successor-features-for-transfer_amd/sfx
for lib in libsfx.so libsfx_nowt.so; do
  f=0
  for i in 1 2 3 4 5 6 7 8 9 10; do
    SFX_LIB=$L/$lib timeout -k 10 120 python -u -m pytest -q --timeout 100 --timeout-method thread "tests/test_gpu_runner.py::test_runner_gate_timeouts_cancel_and_retry" > gpurun_out/gate/$lib.$i.log 2>&1
    rc=$?
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "$lib run $i rc=$rc"; exit $rc; fi
    [ $rc -eq 1 ] && f=$((f+1)) && grep FAILED gpurun_out/gate/$lib.$i.log
  done
  echo "$lib: $f of 10 runs failed"
done
