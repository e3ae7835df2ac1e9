#!/bin/bash
# A/B of environment settings on the headline workload, alternated on one box.
# usage: ab_env.sh "VAR=a" "VAR=b" [bench args]   (use "-" for no setting)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/abenv; mkdir -p $O
E1="$1"; E2="$2"; shift 2
A="--steps 3000 --warmup 300 --no-cpu-baseline --no-other --shard-steps 0 --repeats 0 $*"
v() { python - "$1" <<'PY'
import json,sys
l=[x for x in open(sys.argv[1]) if x.startswith("{")]
d=json.loads(l[-1]); r=d["roofline"]; print(sys.argv[1], d["value"], r["per_kind_avg_us"])
PY
}
for i in 1 2; do
  for E in "$E1" "$E2"; do
    n=$(echo "$E" | tr -c 'A-Za-z0-9_\n' '_')
    if [ "$E" = "-" ]; then timeout -k 10 200 python bench.py $A > $O/$n.$i.log 2>&1
    else env $E timeout -k 10 200 python bench.py $A > $O/$n.$i.log 2>&1; fi && v $O/$n.$i.log || exit 1
  done
done
