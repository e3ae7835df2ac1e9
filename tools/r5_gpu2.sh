#!/bin/bash
# ASan runner (every scenario, once), the default bench line, and the 8-rank C4 bench path rehearsed
# on one GPU (gloo host transport).  Each GPU step has its own limit; the chain stops at a failure.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r5g}
mkdir -p $O
timeout -k 10 120 tools/stepbench 300 1 > $O/stepbench_skip.txt 2>&1 && timeout -k 10 120 tools/stepbench 300 0 > $O/stepbench_noskip.txt 2>&1 || exit 1
ASAN_OPTIONS=detect_leaks=0:verify_asan_link_order=0 timeout -k 10 300 tools/hostsan/runner_asan_full > $O/hostsan_asan_full.txt 2>&1; rc=$?; tail -2 $O/hostsan_asan_full.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench.py > $O/bench.log 2>&1; rc=$?; tail -c 400 $O/bench.log; [ $rc -eq 0 ] || exit $rc
SFX_BENCH_BACKEND=gloo timeout -k 20 600 python bench.py --gpus 8 --steps 200 --warmup 50 --repeats 0 > $O/gloo8.log 2>&1; rc=$?; tail -c 1500 $O/gloo8.log; exit $rc
