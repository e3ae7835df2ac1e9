cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r02e2; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1
rc=$?; tail -15 $O/t.log; [ $rc -eq 0 ] || exit $rc
for sk in 1 0 1 0; do
SFX_SKIP=$sk timeout -k 10 200 python bench.py --no-other --no-cpu-baseline --shard-steps 0 > $O/b$sk.log 2>&1 || exit 1
python - $O/b$sk.log $sk <<'PY'
import json,sys
l=[x for x in open(sys.argv[1]) if x.startswith("{")]
d=json.loads(l[-1]); print("skip", sys.argv[2], d["value"], d["repeats"]["values"], d["roofline"]["per_kind_avg_us"], d["speculation"].get("rounds"))
PY
done
