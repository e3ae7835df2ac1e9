#!/bin/bash
# GPU pass on one box: the whole -m gpu suite, optional probe timelines (PROBE="fp32 bf16"), and the
# bench line as the driver runs it (--gpus 1 --steps 20 --warmup 5).  Each GPU step has its own time
# limit; the chain stops at the first failure.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${1:-pass}; mkdir -p $O
timeout -k 10 1000 python -u -m pytest ${TESTS:-tests} -x -q -m gpu --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for p in $PROBE; do
  SFX_PROBE_PREC=$p SFX_LIB=$PWD/deep-successor-features-for-transfer_amd/sfx/libsfx_probe.so timeout -k 10 150 python3 tools/probe_run.py 30 > $O/probe_$p.txt 2>&1 || exit 1
done
timeout -k 10 500 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2>&1; rc=$?; tail -c 400 $O/bench.log; exit $rc
