#!/bin/bash
# quick GPU check: chosen tests (TESTS, -k KEXPR) then the sharded legs (C4 64 heads, C5 TSF-NF 8 heads, world 1, RCCL)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r6q}; mkdir -p $O
T="${TESTS:-tests/test_gpu_shard.py}"
timeout -k 10 900 python -u -m pytest $T -x -q -m gpu --timeout 200 --timeout-method thread ${KEXPR:+-k "$KEXPR"} > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 tools/shard_leg.py --heads 64 > $O/c4.log 2>&1 || exit 1
timeout -k 10 200 python3 tools/shard_leg.py --workload hopper-tsf-nf --heads 8 --steps 1000 --warmup 100 > $O/c5.log 2>&1 || exit 1
timeout -k 10 200 python3 tools/shard_leg.py --workload hopper-tsf-nf --heads 8 --steps 1000 --warmup 100 --no-rccl > $O/c5n.log 2>&1 || exit 1
grep -ho '"value": [0-9.]*, "unit": "env steps/s", "ms_per_step": [0-9.]*' $O/c4.log $O/c5.log $O/c5n.log
