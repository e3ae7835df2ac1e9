#!/bin/bash
# A/B of the headline workload on one box: abtree/old (an older build) vs this tree, alternated.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/abhead; mkdir -p $O
A="--steps 3000 --warmup 300 --no-cpu-baseline --no-other --shard-steps 0 --repeats 0 $*"
v() { python - "$1" <<'PY'
import json,sys
l=[x for x in open(sys.argv[1]) if x.startswith("{")]
d=json.loads(l[-1]); r=d["roofline"]; print(sys.argv[1], d["value"], r["per_kind_avg_us"])
PY
}
for i in 1 2; do
  (cd abtree/old && timeout -k 10 200 python bench.py $A > ../../$O/old$i.log 2>&1) && v $O/old$i.log && \
  timeout -k 10 200 python bench.py $A > $O/cur$i.log 2>&1 && v $O/cur$i.log || exit 1
done
