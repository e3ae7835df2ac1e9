#!/bin/bash
# A/B of stepbench builds on one box (tools/stepbench_base = committed, tools/stepbench = working
# tree), alternating; then the backward-path GPU tests and the probe timeline of the working tree.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r5ab3}
mkdir -p $O
for i in 1 2; do
  timeout -k 10 120 tools/stepbench_base 300 0 > $O/base_$i.txt 2>&1 || exit 1
  timeout -k 10 120 tools/stepbench 300 0 > $O/new_$i.txt 2>&1 || exit 1
done
for f in $O/base_1.txt $O/new_1.txt $O/base_2.txt $O/new_2.txt; do echo "$f: $(grep -A19 '== 18 launches' $f | grep -E 'K_BWD|launches per step' | tr '\n' ' ')"; done
timeout -k 10 900 python -u -m pytest tests/test_gpu_runner.py tests/test_gpu_engine.py tests/test_gpu_step.py tests/test_gpu_shard.py tests/test_gpu_tsf.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
SFX_LIB=$PWD/deep-successor-features-for-transfer_amd/sfx/libsfx_probe.so timeout -k 10 150 python tools/probe_run.py 30 > $O/probe_new.txt 2>&1 || exit 1
SFX_LIB=$PWD/deep-successor-features-for-transfer_amd/sfx/libsfx_probe.so timeout -k 10 150 python tools/probe_run.py 30 tsf-nf > $O/probe_tsfnf.txt 2>&1 || exit 1
timeout -k 10 200 python tools/prof_dropin.py reference > gpurun_out/${1:-r5ab3}/prof_dropin_reference.txt 2>&1
