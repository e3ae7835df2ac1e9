#!/bin/bash
# A/B/C of stepbench builds on one box (tools/stepbench_base = committed, tools/stepbench = working
# tree, tools/stepbench_plain = working tree with default-policy dW stores), alternating, then the
# probe timeline of the working tree's probe build.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r5ab2}
mkdir -p $O
for i in 1 2; do
  for v in base new plain; do
    b=tools/stepbench; [ $v = base ] && b=tools/stepbench_base; [ $v = plain ] && b=tools/stepbench_plain
    timeout -k 10 120 $b 300 0 > $O/${v}_$i.txt 2>&1 || exit 1
  done
done
for f in $O/base_1.txt $O/new_1.txt $O/plain_1.txt $O/base_2.txt $O/new_2.txt $O/plain_2.txt; do echo "$f: $(grep -A19 '== 18 launches' $f | grep -E 'K_BWD|launches per step' | tr '\n' ' ')"; done
SFX_LIB=$PWD/deep-successor-features-for-transfer_amd/sfx/libsfx_probe.so timeout -k 10 150 python tools/probe_run.py 30 > $O/probe_new.txt 2>&1; exit $?
