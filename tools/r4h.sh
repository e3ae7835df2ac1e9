#!/bin/bash
# Round-4 checks on one box: the runner / TSF / engine GPU tests, A/B of the all-task look-ahead
# placements (final round vs after the publication; 2000-step windows), the probe timeline of the
# post-publish placement, then the UBSan function-check bisection.  Every GPU step time-limited; stops at a time-out or crash.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-r4h}
mkdir -p $O
ok() { local rc=$1; [ $rc -le 1 ] || { echo "rc=$rc: stopping"; exit $rc; }; }
timeout -k 10 500 python -u -m pytest tests/test_gpu_runner.py tests/test_gpu_tsf.py tests/test_gpu_engine.py -x -q \
  --timeout 150 --timeout-method thread > $O/t1.log 2>&1; rc=$?; tail -3 $O/t1.log; [ $rc -eq 0 ] || exit $rc
run() {  # tag, env VAR=value..., then bench flags
  local tag=$1; shift
  local ev=()
  while [ $# -gt 0 ] && [[ $1 == *=* ]]; do ev+=("$1"); shift; done
  env "${ev[@]}" timeout -k 10 200 python bench.py --steps 2000 --warmup 200 --no-other --no-cpu-baseline --shard-steps 0 \
    --repeats 2 "$@" > $O/bench_$tag.json 2>/dev/null || return 1
  python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().splitlines()[-1]);print(sys.argv[2], d['value'], d['repeats']['values'], d['speculation'].get('ahead_pre_steps'))" $O/bench_$tag.json $tag
}
run post_a SFX_AHEAD_POST=1 && run round_a SFX_AHEAD_POST=0 && run post_b SFX_AHEAD_POST=1 && \
  run round_b SFX_AHEAD_POST=0 && run off_a SFX_AHEAD=0 || exit 1
P=$PWD/deep-successor-features-for-transfer_amd/sfx/libsfx_probe.so
SFX_AHEAD_POST=1 SFX_LIB=$P timeout -k 10 150 python tools/probe_run.py 30 > $O/probe_post.txt 2>&1 || { tail -5 $O/probe_post.txt; exit 1; }
grep -E "sum" $O/probe_post.txt
HOSTSAN_BISECT=1 UBSAN_OPTIONS=print_stacktrace=1 timeout -k 10 300 tools/hostsan/runner_ubsan_fn > $O/hostsan_ubsan_fn_bisect.txt 2>&1
rc=$?; echo "ubsan_fn bisect rc=$rc"; cat $O/hostsan_ubsan_fn_bisect.txt | head -30; ok $rc
