# quick bench line: headline workload only, prints the key numbers
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/quick; mkdir -p $O
timeout -k 10 300 python bench.py --no-other --no-cpu-baseline --shard-steps 0 "$@" > $O/b.log 2>&1 || { tail -20 $O/b.log; exit 1; }
python - $O/b.log <<'PY'
import json,sys
l=[x for x in open(sys.argv[1]) if x.startswith("{")]
d=json.loads(l[-1]); r=d["roofline"]
print("value", d["value"], "repeats", d["repeats"]["values"])
print("kinds", r["per_kind_avg_us"], "frac", r["frac"])
print("per_step", {k: v for k, v in r["per_step"].items() if k not in ("formula",)})
print("spec", d["speculation"])
PY
