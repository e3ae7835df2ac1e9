#!/bin/bash
# GPU-box routine: parity tests, then the default bench, then a rocprofv3 kernel-trace summary
# of a short bench.  Each GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-check}
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/${TAG}_pytest.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python3 bench.py --steps 500 --warmup 50 --no-cpu-baseline > gpurun_out/${TAG}_prof.log 2>&1
rc=$?
tail -3 gpurun_out/${TAG}_pytest.log; cat gpurun_out/${TAG}_bench.log 2>/dev/null | tail -1
exit $rc
