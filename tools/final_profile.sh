#!/bin/bash
# Round-end evidence on one MI355X box: GPU tests, smoke, the default bench line, a rocprofv3
# kernel-trace summary of the default bench (and of its prof window: tools/rocprof_window.py) and of the TSF-NF workload, and the HBM traffic
# (FETCH_SIZE / WRITE_SIZE passes, MI355X_MICROARCH.md corrections) of the default workload.
# Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=${1:-final}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 && \
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 400 python bench.py > $O/bench.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --no-cpu-baseline --no-other --shard-steps 0 > $O/prof.log 2>&1 && \
python3 tools/rocprof_window.py $O/prof/run_kernel_trace.csv $O/prof.log $O/rocprof_window.json > $O/window.log 2>&1 && \
rm -f $O/prof/run_kernel_trace.csv && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_tsfnf -o run -- python3 bench.py --workload hopper-tsf-nf --steps 500 --warmup 50 --no-cpu-baseline --shard-steps 0 > $O/prof_tsfnf.log 2>&1 && \
SFX_RUNNER_PIPELINE=0 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 bench.py --steps 100 --warmup 10 --prof-steps 20 --no-cpu-baseline --no-other --shard-steps 0 > $O/fetch.log 2>&1 && \
SFX_RUNNER_PIPELINE=0 timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 bench.py --steps 100 --warmup 10 --prof-steps 20 --no-cpu-baseline --no-other --shard-steps 0 > $O/write.log 2>&1
rc=$?
tail -2 $O/pytest.log; tail -1 $O/smoke.log
exit $rc
