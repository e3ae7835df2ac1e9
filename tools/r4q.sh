#!/bin/bash
# 3 column tiles per workgroup in the look-ahead's row-split forwards (one workgroup per CU):
# fwdbench, the runner tests, A/B against 4 (2000-step windows, alternating).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-r4q}
mkdir -p $O
timeout -k 10 120 tools/fwdbench > $O/fwdbench.txt 2>&1; rc=$?; cat $O/fwdbench.txt; [ $rc -eq 0 ] || exit 1
SFX_AHEAD_TP=3 timeout -k 10 300 python -u -m pytest tests/test_gpu_runner.py -x -q -k lookahead --timeout 150 --timeout-method thread > $O/t1.log 2>&1; rc=$?; tail -2 $O/t1.log; [ $rc -eq 0 ] || exit $rc
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 2000 --warmup 200 --no-other --no-cpu-baseline --shard-steps 0 \
    --repeats 2 > $O/bench_$tag.json 2>/dev/null || return 1
  python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().splitlines()[-1]);print(sys.argv[2], d['value'], d['repeats']['values'])" $O/bench_$tag.json $tag
}
run tp3_a SFX_AHEAD_TP=3 && run tp4_a SFX_AHEAD_TP=4 && run tp3_b SFX_AHEAD_TP=3 && run tp4_b SFX_AHEAD_TP=4 && \
  run tp3_c SFX_AHEAD_TP=3 && run tp4_c SFX_AHEAD_TP=4 || exit 1
