#!/bin/bash
# the one-state selection over one workgroup per head (k_sel1m): selection / runner / TSF GPU tests, the TSF-NF
# and active-task rates with k_sel1 and with k_gpi + k_publish, the TSF-NF probe timeline.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-r4j}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_runner.py tests/test_gpu_tsf.py -x -q \
  --timeout 150 --timeout-method thread > $O/t1.log 2>&1; rc=$?; tail -3 $O/t1.log; [ $rc -eq 0 ] || exit $rc
run() {  # tag, env VAR=value..., then bench flags
  local tag=$1; shift
  local ev=()
  while [ $# -gt 0 ] && [[ $1 == *=* ]]; do ev+=("$1"); shift; done
  env "${ev[@]}" timeout -k 10 200 python bench.py --steps 2000 --warmup 200 --no-other --no-cpu-baseline --shard-steps 0 \
    --repeats 2 "$@" > $O/bench_$tag.json 2>/dev/null || return 1
  python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().splitlines()[-1]);print(sys.argv[2], d['value'], d['repeats']['values'])" $O/bench_$tag.json $tag
}
run nf_m SFX_SEL1=2 --workload hopper-tsf-nf && run nf_one SFX_SEL1=1 --workload hopper-tsf-nf && \
  run nf_gpi SFX_SEL1=0 --workload hopper-tsf-nf && run tsf_m SFX_SEL1=2 --workload hopper-tsf && \
  run tsf_gpi SFX_SEL1=0 --workload hopper-tsf && run act_m SFX_SEL1=2 --schedule active && \
  run act_gpi SFX_SEL1=0 --schedule active && run nf_m2 SFX_SEL1=2 --workload hopper-tsf-nf || exit 1
P=$PWD/deep-successor-features-for-transfer_amd/sfx/libsfx_probe.so
SFX_LIB=$P timeout -k 10 150 python tools/probe_run.py 30 tsf-nf > $O/probe_tsfnf.txt 2>&1 || { tail -5 $O/probe_tsfnf.txt; exit 1; }
grep -E " gpi | tdg |fwd_gemv|sum" $O/probe_tsfnf.txt | cut -c1-120
# the drop-in's rates under the reference user's Python loop (the agents.buffer alias leg: >= 2,500?)
timeout -k 10 300 python tools/dropin_loop.py > $O/dropin.json 2> $O/dropin.err || { tail -5 $O/dropin.err; exit 1; }
cat $O/dropin.json
