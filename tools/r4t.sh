#!/bin/bash
# The roofline kernel's live average (HIP events, bench.py's prof window) against rocprofv3's
# kernel trace of the same command over the same window (tools/rocprof_window.py).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r4t}
mkdir -p $O
timeout -k 10 200 python bench.py --no-cpu-baseline --no-other --shard-steps 0 > $O/bench.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --no-cpu-baseline --no-other --shard-steps 0 > $O/prof.log 2>&1 && \
python3 tools/rocprof_window.py $O/prof/run_kernel_trace.csv $O/prof.log $O/rocprof_window.json > $O/window.log 2>&1; rc=$?
rm -f $O/prof/run_kernel_trace.csv
cat $O/window.log
python3 -c "import json,sys;d=json.loads([l for l in open(sys.argv[1]).read().splitlines() if l.startswith('{')][-1]);r=d['roofline'];print('plain run:', d['value'], r['avg_launch_us'], r['prof_window']['launches'])" $O/bench.log
exit $rc
