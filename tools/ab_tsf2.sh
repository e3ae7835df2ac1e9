cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/abtsf2; mkdir -p $O
A="--workload hopper-tsf-nf --steps 2000 --warmup 200 --no-cpu-baseline --shard-steps 0 --repeats 0"
v() { python - "$1" <<'PY'
import json,sys
l=[x for x in open(sys.argv[1]) if x.startswith("{")]
d=json.loads(l[-1]); print(sys.argv[1], d["value"])
PY
}
(cd abtree/hd && timeout -k 10 200 python bench.py $A > ../../$O/hd.log 2>&1) && v $O/hd.log && \
timeout -k 10 200 python bench.py $A > $O/cur.log 2>&1 && v $O/cur.log
