#!/bin/bash
# Round-6 GPU pass: chosen GPU tests (or the whole suite: TESTS=all), then the bench at T = 64 (the
# all-task step on one GPU and the sharded C4 layout at world 1 over RCCL).  Each GPU step has its
# own time limit; the chain stops at the first failure.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r6g}
mkdir -p $O
T="${TESTS:-tests/test_gpu_runner.py tests/test_gpu_native_shard.py tests/test_gpu_shard.py tests/test_gpu_dropin_buffer.py}"
[ "$T" = all ] && T=tests
timeout -k 10 900 python -u -m pytest $T -x -q -m gpu --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -5 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
[ -n "$NOBENCH" ] && exit 0
timeout -k 10 300 python3 bench.py --heads 64 --steps 2000 --warmup 200 --prof-steps 10 --repeats 0 --no-cpu-baseline --no-other --shard-steps 2000 > $O/t64.log 2>&1
rc=$?; [ $rc -eq 0 ] || { tail -20 $O/t64.log; exit $rc; }
python3 - <<PY
import json
l=[x for x in open('$O/t64.log') if x.startswith('{')][-1];d=json.loads(l)
print('all-task T64', d['value'], d['ms_per_step'], {k:d['speculation'].get(k) for k in ('steps','host_round_steps','rounds','policies_checked','policies_skipped')}, d['roofline']['per_kind_avg_us'])
for k in ('sharded','sharded_rccl_world1'):
    s=d[k]; print(k, s['value'], s['ms_per_step'], {x:s['rounds'].get(x) for x in ('steps','host_round_steps','rounds')})
PY
timeout -k 10 300 python3 bench.py --workload hopper-tsf-nf --heads 8 --steps 1000 --warmup 100 --prof-steps 10 --repeats 0 --no-cpu-baseline --no-other --shard-steps 1000 > $O/tsfnf8.log 2>&1
rc=$?; [ $rc -eq 0 ] || { tail -20 $O/tsfnf8.log; exit $rc; }
python3 - <<PY
import json
l=[x for x in open('$O/tsfnf8.log') if x.startswith('{')][-1];d=json.loads(l)
print('tsf-nf T8 single', d['value'], d['ms_per_step'])
for k in ('sharded','sharded_rccl_world1'):
    s=d[k]; print(k, s.get('value'), s.get('ms_per_step'), s.get('prelaunched'), s.get('error'))
PY
