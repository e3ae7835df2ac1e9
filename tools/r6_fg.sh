cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/fg && timeout -k 10 400 python -u -m pytest tests/test_gpu_dropin_fused_gpi.py tests/test_gpu_dropin_loop.py tests/test_gpu_dropin_buffer.py tests/test_gpu_dropin.py -x -v --timeout 120 --timeout-method thread > gpurun_out/fg/pytest.log 2>&1; rc=$?; tail -5 gpurun_out/fg/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/dropin_phases.py > gpurun_out/fg/phases.txt 2>&1 && head -16 gpurun_out/fg/phases.txt
CALL_COSTS=1 timeout -k 10 200 python3 tools/dropin_phases.py > gpurun_out/fg/calls.txt 2>&1 && cat gpurun_out/fg/calls.txt
timeout -k 10 200 python3 -c "
import sys, json; sys.path.insert(0, 'deep-successor-features-for-transfer_amd'); sys.path.insert(0, 'tools')
import dropin_loop
for b in ('reference', 'reference', 'host'):
    print(json.dumps({b: dropin_loop.measure(b)}), flush=True)
" > gpurun_out/fg/measure.txt 2>&1 && cat gpurun_out/fg/measure.txt
