#!/bin/bash
# Fused layer-0 tiles two at a time (SFX_V0_PAIR=1): runner + engine suites with it on, then A/B
# against the default (2000-step windows, alternating).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-r4v}
mkdir -p $O
SFX_V0_PAIR=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_runner.py tests/test_gpu_engine.py tests/test_gpu_shard.py -x -q --timeout 150 --timeout-method thread > $O/t1.log 2>&1; rc=$?; tail -2 $O/t1.log; [ $rc -eq 0 ] || exit $rc
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 2000 --warmup 200 --no-other --no-cpu-baseline --shard-steps 0 \
    --repeats 2 > $O/bench_$tag.json 2>/dev/null || return 1
  python -c "import json,sys;d=json.loads([l for l in open(sys.argv[1]).read().splitlines() if l.startswith('{')][-1]);print(sys.argv[2], d['value'], d['repeats']['values'], d['roofline']['per_kind_avg_us'])" $O/bench_$tag.json $tag
}
run pair_a SFX_V0_PAIR=1 && run base_a SFX_V0_PAIR=0 && run pair_b SFX_V0_PAIR=1 && run base_b SFX_V0_PAIR=0 && \
  run pair_c SFX_V0_PAIR=1 && run base_c SFX_V0_PAIR=0 || exit 1
