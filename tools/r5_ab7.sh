#!/bin/bash
# GPU suite, drop-in phase timings, drop-in loop (each step time-limited; stop at the first failure)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r5ab7}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/dropin_phases.py > $O/phases.txt 2>&1 || exit 1
cat $O/phases.txt
timeout -k 10 300 python tools/dropin_loop.py > $O/dropin.txt 2>&1; rc=$?; cat $O/dropin.txt; exit $rc
