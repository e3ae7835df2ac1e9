#!/bin/bash
# sharded-path GPU tests, then the headline vs one-rank sharded rate in the same window
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_native_shard.py tests/test_gpu_shard.py tests/test_gpu_runner.py > gpurun_out/shard_tests.log 2>&1
rc=$?; tail -2 gpurun_out/shard_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 2000 --warmup 200 --no-cpu-baseline --no-other --repeats 0 > gpurun_out/shard_cmp$i.log 2>&1 || exit 1
  python -c "
import json; d=json.loads(open('gpurun_out/shard_cmp$i.log').read().strip().splitlines()[-1]); print(d['value'], d['sharded']['value'], round(d['sharded']['value']/d['value'],3), d['sharded']['rounds']['host_round_steps'])"
done
