#!/bin/bash
# GPU suite, TSF-NF probe timeline, default bench line (each step time-limited; stop at the first failure)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r5ab6}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
SFX_LIB=$PWD/deep-successor-features-for-transfer_amd/sfx/libsfx_probe.so timeout -k 10 150 python tools/probe_run.py 30 tsf-nf > $O/probe_tsfnf.txt 2>&1 || exit 1
timeout -k 10 400 python bench.py > $O/bench.log 2>&1; rc=$?; tail -c 600 $O/bench.log; exit $rc
