#!/bin/bash
# A/B/C of stepbench builds on one box, alternating: tools/stepbench_base (committed),
# tools/stepbench_reorder, tools/stepbench (working tree); then the GPU tests of the step paths
# and the probe timelines of the working tree (C2 all-task, TSF-NF).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r5ab4}
mkdir -p $O
for i in 1 2; do
  timeout -k 10 120 tools/stepbench_base 300 0 > $O/base_$i.txt 2>&1 || exit 1
  timeout -k 10 120 tools/stepbench_reorder 300 0 > $O/reorder_$i.txt 2>&1 || exit 1
  timeout -k 10 120 tools/stepbench 300 0 > $O/new_$i.txt 2>&1 || exit 1
done
for f in $O/base_1.txt $O/reorder_1.txt $O/new_1.txt $O/base_2.txt $O/reorder_2.txt $O/new_2.txt; do echo "$f: $(grep -E 'K_BWD|launches per step' $f | tr '\n' ' ')"; done
timeout -k 10 900 python -u -m pytest tests/test_gpu_runner.py tests/test_gpu_engine.py tests/test_gpu_step.py tests/test_gpu_shard.py tests/test_gpu_tsf.py tests/test_gpu_dropin.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
SFX_LIB=$PWD/deep-successor-features-for-transfer_amd/sfx/libsfx_probe.so timeout -k 10 150 python tools/probe_run.py 30 > $O/probe_new.txt 2>&1 || exit 1
SFX_LIB=$PWD/deep-successor-features-for-transfer_amd/sfx/libsfx_probe.so timeout -k 10 150 python tools/probe_run.py 30 tsf-nf > $O/probe_tsfnf.txt 2>&1 || exit 1
timeout -k 10 200 python tools/prof_dropin.py reference > $O/prof_dropin_reference.txt 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 400 --warmup 50 > $O/bench.json 2> $O/bench.err || exit 1
tail -c 600 $O/bench.json
