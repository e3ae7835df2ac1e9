#!/bin/bash
# A/B/C of library variants (SFX_LIB) on the headline workload, alternated on one box.
# usage: ab_libs.sh "lib1 lib2 ..." [bench args]
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/ablibs; mkdir -p $O
LIBS="$1"; shift
A="--steps 3000 --warmup 300 --no-cpu-baseline --no-other --shard-steps 0 --repeats 0 $*"
v() { python - "$1" <<'PY'
import json,sys
l=[x for x in open(sys.argv[1]) if x.startswith("{")]
d=json.loads(l[-1]); r=d["roofline"]; print(sys.argv[1], d["value"], r["per_kind_avg_us"])
PY
}
for i in 1 2; do
  for L in $LIBS; do
    SFX_LIB=deep-successor-features-for-transfer_amd/sfx/$L timeout -k 10 200 python bench.py $A > $O/$L.$i.log 2>&1 && v $O/$L.$i.log || exit 1
  done
done
