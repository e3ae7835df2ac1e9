#!/bin/bash
# quick GPU check: chosen tests (TESTS, -k KEXPR) then the T = 64 legs (all-task one GPU; the sharded C4 layout at world 1, RCCL)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r6q}; mkdir -p $O
T="${TESTS:-tests/test_gpu_runner.py tests/test_gpu_native_shard.py}"
timeout -k 10 900 python -u -m pytest $T -x -q -m gpu --timeout 200 --timeout-method thread ${KEXPR:+-k "$KEXPR"} > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 tools/shard_leg.py --heads 64 > $O/c4.log 2>&1 || exit 1
grep -ho '"value": [0-9.]*, "unit": "env steps/s", "ms_per_step": [0-9.]*' $O/c4.log
timeout -k 10 300 python3 bench.py --heads 64 --steps 2000 --warmup 200 --prof-steps 10 --repeats 0 --no-cpu-baseline --no-other --shard-steps 0 > $O/t64.log 2>&1 || exit 1
python3 -c "
import json
l=[x for x in open('$O/t64.log') if x.startswith('{')][-1];d=json.loads(l)
print('all-task T64', d['value'], d['ms_per_step'], d['roofline']['per_kind_avg_us'])"
