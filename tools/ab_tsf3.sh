#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/abtsf3; mkdir -p $O
A="--workload hopper-tsf --steps 3000 --warmup 300 --no-cpu-baseline --no-other --shard-steps 0 --repeats 0"
v() { python - "$1" <<'PY'
import json,sys
l=[x for x in open(sys.argv[1]) if x.startswith("{")]
d=json.loads(l[-1]); r=d["roofline"]; print(sys.argv[1], d["value"], r["per_kind_avg_us"])
PY
}
L=deep-successor-features-for-transfer_amd/sfx
for i in 1 2; do
  SFX_LIB=$L/libsfx_prev.so timeout -k 10 200 python bench.py $A > $O/prev.$i.log 2>&1 && v $O/prev.$i.log && \
  timeout -k 10 200 python bench.py $A > $O/cur.$i.log 2>&1 && v $O/cur.$i.log && \
  SFX_FWD_TPW=1 timeout -k 10 200 python bench.py $A > $O/tpw1.$i.log 2>&1 && v $O/tpw1.$i.log || exit 1
done
