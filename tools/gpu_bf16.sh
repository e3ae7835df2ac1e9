cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/bf16; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_bf16.py -x -v -s --timeout 120 --timeout-method thread > $O/t.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|bf16 vs|assert" $O/t.log | head -30; [ $rc -eq 0 ] || { tail -40 $O/t.log; exit $rc; }
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/all.log 2>&1
rc=$?; tail -3 $O/all.log; [ $rc -eq 0 ] || { grep -B5 -A30 "FAILED\|Error" $O/all.log | head -80; exit $rc; }
for p in fp32 bf16; do
timeout -k 10 200 python bench.py --no-other --no-cpu-baseline --shard-steps 0 --precision $p > $O/b_$p.log 2>&1 || { tail $O/b_$p.log; exit 1; }
python - $O/b_$p.log <<'PY'
import json,sys
l=[x for x in open(sys.argv[1]) if x.startswith("{")]
d=json.loads(l[-1]); print(d["dtype"], d["value"], d["repeats"]["values"], d["roofline"]["per_kind_avg_us"])
PY
done
