#!/bin/bash
# Round-4 diagnostics on one box: (1) the sanitizer hang -- kernel launches through a function
# pointer with and without -fsanitize=function, then the runner driver with UBSan's function check
# alone and its vptr check alone; (2) kernel time of the one-state selection (k_sel1 vs k_gpi +
# k_publish) in the Hopper TSF-NF step.  Every GPU step time-limited; stops at a time-out or crash.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-r4g}
mkdir -p $O
ok() { local rc=$1; [ $rc -le 1 ] || { echo "rc=$rc: stopping"; exit $rc; }; }
timeout -k 10 120 tools/fwdbench > $O/fwdbench.txt 2>&1; rc=$?; echo "fwdbench rc=$rc"; cat $O/fwdbench.txt; ok $rc
timeout -k 10 60 tools/hostsan/fnptr_plain > $O/fnptr_plain.txt 2>&1; rc=$?; echo "fnptr_plain rc=$rc"; cat $O/fnptr_plain.txt; ok $rc
timeout -k 10 60 tools/hostsan/fnptr_function > $O/fnptr_function.txt 2>&1; rc=$?; echo "fnptr_function rc=$rc"; cat $O/fnptr_function.txt; ok $rc
UBSAN_OPTIONS=print_stacktrace=1 timeout -k 10 300 tools/hostsan/runner_ubsan_fn > $O/hostsan_ubsan_fn.txt 2>&1
rc=$?; echo "ubsan_fn rc=$rc"; tail -3 $O/hostsan_ubsan_fn.txt; ok $rc
UBSAN_OPTIONS=print_stacktrace=1 timeout -k 10 300 tools/hostsan/runner_ubsan_vptr > $O/hostsan_ubsan_vptr.txt 2>&1
rc=$?; echo "ubsan_vptr rc=$rc"; tail -3 $O/hostsan_ubsan_vptr.txt; ok $rc
P=$PWD/deep-successor-features-for-transfer_amd/sfx/libsfx_probe.so
SFX_LIB=$P timeout -k 10 150 python tools/probe_run.py 30 tsf-nf > $O/probe_tsfnf_sel1.txt 2>&1 || { tail -5 $O/probe_tsfnf_sel1.txt; exit 1; }
SFX_SEL1=0 SFX_LIB=$P timeout -k 10 150 python tools/probe_run.py 30 tsf-nf > $O/probe_tsfnf_gpi.txt 2>&1 || { tail -5 $O/probe_tsfnf_gpi.txt; exit 1; }
grep -E "gpi|publish|sum" $O/probe_tsfnf_sel1.txt $O/probe_tsfnf_gpi.txt | cut -c1-150
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for v in 1 0; do
  SFX_SEL1=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_sel$v -o run -- \
    python bench.py --workload hopper-tsf-nf --steps 400 --warmup 100 --no-other --no-cpu-baseline --shard-steps 0 \
    --repeats 1 > $O/bench_sel$v.json 2> $O/bench_sel$v.err || { echo "rocprof sel$v failed"; tail -5 $O/bench_sel$v.err; exit 1; }
  f=$(find $O/prof_sel$v -name "*kernel_stats.csv" | head -1)
  echo "== SFX_SEL1=$v"; cut -d, -f1-5 "$f" | head -14
done
