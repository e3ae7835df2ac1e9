#!/bin/bash
# The drop-in's device ring (sfx_replay_put / sfx_replay_gather): its GPU tests and the drop-in
# loop's rates (the agents.buffer alias leg against >= 2,500 env-steps/s).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-r4n}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_dropin_buffer.py tests/test_gpu_dropin_loop.py tests/test_gpu_dropin.py -x -q \
  --timeout 200 --timeout-method thread > $O/t1.log 2>&1; rc=$?; tail -3 $O/t1.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python tools/dropin_loop.py > $O/dropin$i.json 2> $O/dropin$i.err || { tail -5 $O/dropin$i.err; exit 1; }
  cat $O/dropin$i.json
done
