cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r02c2; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_runner.py -x -v --timeout 120 --timeout-method thread > $O/t.log 2>&1
rc=$?; tail -5 $O/t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/dbg_shard2.py first > $O/dbg1.log 2>&1 && tail -1 $O/dbg1.log && \
bash tools/ab_tsf2.sh
