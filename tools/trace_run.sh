#!/bin/bash
# rocprofv3 kernel trace of a short bench per env config; prints the per-(kernel, grid) table.
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-tr}; shift
i=0
for cfg in "$@"; do
  i=$((i+1))
  env $cfg timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${TAG}_$i -o run -- python3 bench.py --steps 300 --warmup 30 --no-cpu-baseline --shard-steps 0 > gpurun_out/${TAG}_$i.log 2>&1 || exit 1
  echo "== $cfg"
  python3 tools/trace_breakdown.py gpurun_out/${TAG}_$i/run_kernel_trace.csv | head -12
done
