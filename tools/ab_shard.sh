#!/bin/bash
# A/B of an environment setting on the one-rank sharded rate (bench's sharded side measurement)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/abshard
for i in 1 2 3; do
  for E in "$1" "$2"; do
    n=$(echo "$E" | tr -c 'A-Za-z0-9_\n' '_')
    env $E timeout -k 10 300 python bench.py --steps 3000 --warmup 300 --no-cpu-baseline --no-other --repeats 0 > gpurun_out/abshard/$n.$i.log 2>&1 || exit 1
    python -c "
import json; d=json.loads(open('gpurun_out/abshard/$n.$i.log').read().strip().splitlines()[-1]); print('$E', d['value'], d['sharded']['value'])"
  done
done
