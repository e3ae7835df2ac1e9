# A/B of the TSF-NF workload: round-1 tree (abtree/r1) vs the current tree, fork on/off
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/abtsf; mkdir -p $O
A="--workload hopper-tsf-nf --steps 2000 --warmup 200 --no-cpu-baseline --shard-steps 0"
v() { python - "$1" <<'PY'
import json,sys
l=[x for x in open(sys.argv[1]) if x.startswith("{")]
d=json.loads(l[-1]); print(sys.argv[1], d["value"], d["repeats"]["values"] if d.get("repeats") else "")
PY
}
(cd abtree/r1 && timeout -k 10 200 python bench.py $A > ../../$O/r1.log 2>&1) && v $O/r1.log && \
timeout -k 10 200 python bench.py $A > $O/cur.log 2>&1 && v $O/cur.log && \
SFX_TSF_FORK=0 timeout -k 10 200 python bench.py $A > $O/cur_nofork.log 2>&1 && v $O/cur_nofork.log && \
(cd abtree/r1 && timeout -k 10 200 python bench.py $A > ../../$O/r1b.log 2>&1) && v $O/r1b.log
