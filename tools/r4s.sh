#!/bin/bash
# 33-row groups in one 48-row tile (FwdArgs::tail): fwdbench, the runner's look-ahead tests (tail on
# row-split launches), runner + engine suites with the tail on every plain launch, then A/B
# (2000-step windows, alternating): TP3+tail (default), TP3 without tail, TP2+tail.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-r4s}
mkdir -p $O
timeout -k 10 120 tools/fwdbench > $O/fwdbench.txt 2>&1; rc=$?; cat $O/fwdbench.txt; [ $rc -eq 0 ] || exit 1
SFX_FWD_TAIL=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_runner.py -x -q -k lookahead --timeout 150 --timeout-method thread > $O/t1.log 2>&1; rc=$?; tail -2 $O/t1.log; [ $rc -eq 0 ] || exit $rc
SFX_FWD_TAIL=2 timeout -k 10 400 python -u -m pytest tests/test_gpu_runner.py tests/test_gpu_engine.py -x -q --timeout 150 --timeout-method thread > $O/t2.log 2>&1; rc=$?; tail -2 $O/t2.log; [ $rc -eq 0 ] || exit $rc
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 2000 --warmup 200 --no-other --no-cpu-baseline --shard-steps 0 \
    --repeats 2 > $O/bench_$tag.json 2>/dev/null || return 1
  python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().splitlines()[-1]);print(sys.argv[2], d['value'], d['repeats']['values'])" $O/bench_$tag.json $tag
}
run tail_a SFX_FWD_TAIL=1 && run notail_a SFX_FWD_TAIL=0 && run tp2tail_a SFX_FWD_TAIL=1 SFX_AHEAD_TP=2 && \
  run tail_b SFX_FWD_TAIL=1 && run notail_b SFX_FWD_TAIL=0 && run tp2tail_b SFX_FWD_TAIL=1 SFX_AHEAD_TP=2 || exit 1
