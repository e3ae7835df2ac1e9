#!/bin/bash
# bf16 operand mode vs fp32 on one box (alternating pairs of the C2 bench), the bf16 GPU test, and
# the C2 probe timelines of both modes.  Each GPU step has its own limit; the first failure ends it.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r6bf}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_bf16.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  for p in fp32 bf16; do
    timeout -k 10 200 python3 bench.py --steps 2000 --warmup 200 --repeats 1 --precision $p --no-other --no-cpu-baseline --shard-steps 0 > $O/$p$i.json 2>/dev/null || exit 1
    python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().splitlines()[-1]);r=d['roofline'];print(sys.argv[2], d['value'], d['repeats']['values'], r['per_kind_avg_us'])" $O/$p$i.json $p$i
  done
done
for p in fp32 bf16; do
  SFX_PROBE_PREC=$p SFX_LIB=$PWD/deep-successor-features-for-transfer_amd/sfx/libsfx_probe.so timeout -k 10 150 python3 tools/probe_run.py 30 > $O/probe_$p.txt 2>&1 || exit 1
done
