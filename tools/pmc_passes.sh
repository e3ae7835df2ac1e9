#!/bin/bash
# HBM traffic per kernel (MI355X_MICROARCH.md §HBM): FETCH_SIZE and WRITE_SIZE in separate
# rocprofv3 --pmc passes (they do not fit one pass), kernel trace only, over a short bench.
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-pmc}
export SFX_RUNNER_PIPELINE=0  # the profiler serialises dispatches: a pre-launched gate would wait on the blocked host
ARGS="--steps 100 --warmup 10 --prof-steps 20 --no-cpu-baseline --shard-steps 0"
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${TAG}_fetch -o run -- python3 bench.py $ARGS > gpurun_out/${TAG}_fetch.log 2>&1 && \
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${TAG}_write -o run -- python3 bench.py $ARGS > gpurun_out/${TAG}_write.log 2>&1
rc=$?
ls gpurun_out/${TAG}_fetch gpurun_out/${TAG}_write
exit $rc
