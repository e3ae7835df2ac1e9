#!/bin/bash
# rocprofv3 kernel-trace summaries of the sharded legs (C4 at 64 heads, C5 TSF-NF at 8 heads), world 1, RCCL.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r6p}
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c4 -o run -- python3 tools/shard_leg.py --heads 64 --steps 500 --warmup 100 > $O/c4.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c5 -o run -- python3 tools/shard_leg.py --workload hopper-tsf-nf --heads 8 --steps 500 --warmup 100 > $O/c5.log 2>&1 || exit 1
rm -f $O/c4/run_kernel_trace.csv $O/c5/run_kernel_trace.csv
tail -1 $O/c4.log; tail -1 $O/c5.log
