#!/bin/bash
# Look-ahead A/B on one box: runner parity tests, probe timelines (look-ahead in round 0 / in the final round)
# and alternating 2000-step bench windows (early, late, TP 2, look-ahead off).  Every GPU step time-limited.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-r4e}
mkdir -p $O
P=$PWD/deep-successor-features-for-transfer_amd/sfx/libsfx_probe.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_runner.py tests/test_gpu_tsf.py tests/test_gpu_engine.py -x -q --timeout 120 \
  --timeout-method thread > $O/t1.log 2>&1 || { tail -20 $O/t1.log; exit 1; }
tail -1 $O/t1.log
SFX_LIB=$P timeout -k 10 120 python tools/probe_run.py 30 > $O/probe_early.txt 2>&1 || exit 1
SFX_AHEAD_EARLY=0 SFX_LIB=$P timeout -k 10 120 python tools/probe_run.py 30 > $O/probe_late.txt 2>&1 || exit 1
run() {  # tag, env VAR=value..., then bench flags
  local tag=$1; shift
  local ev=()
  while [ $# -gt 0 ] && [[ $1 == *=* ]]; do ev+=("$1"); shift; done
  env "${ev[@]}" timeout -k 10 200 python bench.py --steps 2000 --warmup 200 --no-other --no-cpu-baseline --shard-steps 0 \
    --repeats 2 "$@" > $O/bench_$tag.json 2>/dev/null || return 1
  python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().splitlines()[-1]);print(sys.argv[2], d['value'], d['repeats']['values'])" $O/bench_$tag.json $tag
}
run early_a SFX_AHEAD_EARLY=1 && run late_a SFX_AHEAD_EARLY=0 && run tp2_a SFX_AHEAD_TP=2 && run off_a SFX_AHEAD=0 && \
  run early_b SFX_AHEAD_EARLY=1 && run late_b SFX_AHEAD_EARLY=0 && run tp2_b SFX_AHEAD_TP=2 && run off_b SFX_AHEAD=0 || exit 1
grep -E "sum" $O/probe_early.txt $O/probe_late.txt | cut -c1-150
# the one-state selection (k_sel1 with the publication folded in vs k_gpi + k_publish): Hopper TSF-NF
# and the Reacher active-task step
run tsf_sel1 SFX_SEL1=1 --workload hopper-tsf-nf && run tsf_gpi SFX_SEL1=0 --workload hopper-tsf-nf && \
  run act_sel1 SFX_SEL1=1 --schedule active && run act_gpi SFX_SEL1=0 --schedule active || exit 1
# the whole GPU suite on the device bounds-check build (no check may fire)
SFX_LIB=$PWD/deep-successor-features-for-transfer_amd/sfx/libsfx_check.so SFX_CHECK_RUN=1 timeout -k 10 600 \
  python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $O/check_suite.log 2>&1
rc=$?; tail -3 $O/check_suite.log
[ $rc -le 1 ] || { echo "check suite rc=$rc: stopping"; exit $rc; }
# the host-sanitizer drivers with every flag (the round-3 hang: ASan's default use-after-return
# mode, UBSan's function / vptr checks); each bounded
ASAN_OPTIONS=detect_leaks=0:verify_asan_link_order=0 timeout -k 10 300 tools/hostsan/runner_asan_full > $O/hostsan_asan_full.txt 2>&1
rc=$?; echo "asan_full rc=$rc"; tail -3 $O/hostsan_asan_full.txt
[ $rc -le 1 ] || exit $rc
UBSAN_OPTIONS=print_stacktrace=1 timeout -k 10 300 tools/hostsan/runner_ubsan_full > $O/hostsan_ubsan_full.txt 2>&1
echo "ubsan_full rc=$?"; tail -3 $O/hostsan_ubsan_full.txt
