#!/bin/bash
# The driver's early window (--steps 20 --warmup 5) under switches: where do its host rounds come from?
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r6w}
mkdir -p $O
A="--steps 20 --warmup 5 --no-cpu-baseline --no-other --shard-steps 0"
for v in base "SFX_AHEAD=0" "SFX_SKIP=0" "SFX_RUNNER_PIPELINE=0" "LOOP=python"; do
  n=$(echo $v | tr '=' '_')
  if [ "$v" = base ]; then timeout -k 10 120 python3 bench.py $A > $O/$n.log 2>&1 || exit 1
  elif [ "$v" = "LOOP=python" ]; then timeout -k 10 120 python3 bench.py $A --loop python > $O/$n.log 2>&1 || exit 1
  else env $v timeout -k 10 120 python3 bench.py $A > $O/$n.log 2>&1 || exit 1; fi
  python3 -c "
import json,sys
l=[x for x in open('$O/$n.log') if x.startswith('{')][-1];d=json.loads(l);s=d['speculation']
print('$v', d['value'], {k:s.get(k) for k in ('steps','host_round_steps','policies_checked','policies_skipped','rounds')}, {k:d['roofline'].get(k) for k in ('mfma_util','compute_frac','mfma_executed_frac')})"
done
