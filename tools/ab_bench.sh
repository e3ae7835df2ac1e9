#!/bin/bash
# A/B of library knobs on the default bench (no CPU baseline, short sharded leg).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${1:-ab}; shift
i=0
for cfg in "$@"; do
  i=$((i+1))
  env $cfg timeout -k 10 200 python bench.py --no-cpu-baseline --shard-steps 0 --steps 6000 --warmup 300 > gpurun_out/${TAG}_$i.log 2>&1 || exit 1
  echo "$cfg: $(tail -1 gpurun_out/${TAG}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["per_kind_avg_us"])')"
done
