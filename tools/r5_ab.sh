#!/bin/bash
# A/B of a kernel change on one box: stepbench of the committed build (tools/stepbench_base) and of
# the working tree, alternating, then the runner / engine GPU tests of the working tree and a short
# bench line.  Each GPU step has its own limit; the chain stops at the first failure.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r5ab}
mkdir -p $O
for i in 1 2; do
  timeout -k 10 120 tools/stepbench_base 300 0 > $O/base_$i.txt 2>&1 || exit 1
  timeout -k 10 120 tools/stepbench 300 0 > $O/new_$i.txt 2>&1 || exit 1
done
grep -h 'K_BWD\|launches per step' $O/base_1.txt $O/new_1.txt $O/base_2.txt $O/new_2.txt | head -20
timeout -k 10 900 python -u -m pytest tests/test_gpu_runner.py tests/test_gpu_engine.py tests/test_gpu_step.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
[ -n "$2" ] || exit 0
timeout -k 10 400 python bench.py --no-other --no-cpu-baseline --shard-steps 0 > $O/bench.log 2>&1; rc=$?; python3 -c "
import json,sys
l=[x for x in open('$O/bench.log') if x.startswith('{')][-1]; d=json.loads(l); r=d['roofline']
print('value', d['value'], 'repeats', d['repeats']['values'], 'k_bwd', r['avg_launch_us'], 'frac', r['frac'], 'frac_unskipped', r.get('frac_unskipped'), r['per_kind_avg_us'])"; exit $rc
