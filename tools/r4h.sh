#!/bin/bash
# Round-4 checks on one box: the runner / TSF / engine GPU tests (look-ahead of the active and TSF
# schedules), A/B of that look-ahead (2000-step windows), the TSF-NF probe timeline, then the
# diagnostics of tools/r4g.sh.  Every GPU step time-limited; stops at a time-out or crash.
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
run nf_on SFX_AHEAD=1 --workload hopper-tsf-nf && run nf_off SFX_AHEAD=0 --workload hopper-tsf-nf && \
  run tsf_on SFX_AHEAD=1 --workload hopper-tsf && run tsf_off SFX_AHEAD=0 --workload hopper-tsf && \
  run act_on SFX_AHEAD=1 --schedule active && run act_off SFX_AHEAD=0 --schedule active && \
  run nf_on2 SFX_AHEAD=1 --workload hopper-tsf-nf && run nf_off2 SFX_AHEAD=0 --workload hopper-tsf-nf && \
  run c2 || exit 1
P=$PWD/deep-successor-features-for-transfer_amd/sfx/libsfx_probe.so
SFX_LIB=$P timeout -k 10 150 python tools/probe_run.py 30 tsf-nf > $O/probe_tsfnf_ahead.txt 2>&1 || { tail -5 $O/probe_tsfnf_ahead.txt; exit 1; }
SFX_AHEAD=0 SFX_LIB=$P timeout -k 10 150 python tools/probe_run.py 30 tsf-nf > $O/probe_tsfnf_noahead.txt 2>&1 || exit 1
grep -E "sum" $O/probe_tsfnf_ahead.txt $O/probe_tsfnf_noahead.txt
timeout -k 10 120 tools/fwdbench > $O/fwdbench.txt 2>&1; rc=$?; echo "fwdbench rc=$rc"; cat $O/fwdbench.txt; ok $rc
timeout -k 10 60 tools/hostsan/fnptr_plain > $O/fnptr_plain.txt 2>&1; rc=$?; echo "fnptr_plain rc=$rc"; cat $O/fnptr_plain.txt; ok $rc
timeout -k 10 60 tools/hostsan/fnptr_function > $O/fnptr_function.txt 2>&1; rc=$?; echo "fnptr_function rc=$rc"; cat $O/fnptr_function.txt; ok $rc
UBSAN_OPTIONS=print_stacktrace=1 timeout -k 10 300 tools/hostsan/runner_ubsan_fn > $O/hostsan_ubsan_fn.txt 2>&1
rc=$?; echo "ubsan_fn rc=$rc"; tail -3 $O/hostsan_ubsan_fn.txt; ok $rc
UBSAN_OPTIONS=print_stacktrace=1 timeout -k 10 300 tools/hostsan/runner_ubsan_vptr > $O/hostsan_ubsan_vptr.txt 2>&1
rc=$?; echo "ubsan_vptr rc=$rc"; tail -3 $O/hostsan_ubsan_vptr.txt; ok $rc
