cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_dropin.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r02g_tests.log 2>&1
rc1=$?
tail -14 gpurun_out/r02g_tests.log
timeout -k 10 120 python tools/dbg_shard.py warm 400 1000 > gpurun_out/r02g_dbg.log 2>&1 && \
timeout -k 10 300 python bench.py --no-other --no-cpu-baseline --repeats 1 > gpurun_out/r02g_bench.log 2>&1
rc=$?
tail -2 gpurun_out/r02g_dbg.log
python - <<'PY'
import json
l = [x for x in open("gpurun_out/r02g_bench.log") if x.startswith("{")]
d = json.loads(l[-1]); print("value", d["value"], "sharded", d["sharded"]["value"], d["sharded"]["rounds"])
PY
exit $((rc1 + rc))
