#!/bin/bash
# Round-5 GPU pass: the GPU suite, the host-sanitizer runner (UBSan every check, ASan) over every
# scenario once, and the default bench line.  Each GPU step has its own time limit; the chain stops
# at the first failure.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r5}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
UBSAN_OPTIONS=print_stacktrace=1 timeout -k 10 300 tools/hostsan/runner_ubsan_full > $O/hostsan_ubsan_full.txt 2>&1; rc=$?; tail -2 $O/hostsan_ubsan_full.txt; [ $rc -eq 0 ] || exit $rc
ASAN_OPTIONS=detect_leaks=0:verify_asan_link_order=0 timeout -k 10 300 tools/hostsan/runner_asan_full > $O/hostsan_asan_full.txt 2>&1; rc=$?; tail -2 $O/hostsan_asan_full.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > $O/bench.log 2>&1; rc=$?; tail -c 600 $O/bench.log; exit $rc
