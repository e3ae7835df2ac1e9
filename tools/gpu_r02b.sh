cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r02b
timeout -k 10 120 python tools/dbg_shard2.py first > gpurun_out/r02b/dbg1.log 2>&1 && \
timeout -k 10 400 python bench.py > gpurun_out/r02b/bench.log 2>&1
rc=$?
tail -2 gpurun_out/r02b/dbg1.log
tail -c 600 gpurun_out/r02b/bench.log
exit $rc
