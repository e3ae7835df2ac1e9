cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_native_shard.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r02f_tests.log 2>&1
rc=$?
tail -12 gpurun_out/r02f_tests.log
[ $rc -eq 0 ] && timeout -k 10 300 python bench.py --no-other --no-cpu-baseline --repeats 1 > gpurun_out/r02f_bench.log 2>&1
rc=$?
python - <<'PY'
import json
l = [x for x in open("gpurun_out/r02f_bench.log") if x.startswith("{")]
d = json.loads(l[-1]); print("value", d["value"], "sharded", d["sharded"]["value"], d["sharded"]["rounds"])
PY
exit $rc
