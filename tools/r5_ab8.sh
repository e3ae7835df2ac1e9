#!/bin/bash
# A/B on one box: a libsfx variant (sfx/libsfx_<V>.so, sfx/libsfx_probe_<V>.so; V = $2, default b)
# against another (sfx/libsfx<A>.so; A = $3, default: the tree's build) -- runner parity tests on the
# variant, C2 probe timelines of both, alternating bench pairs.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r5ab8}
mkdir -p $O
S=$PWD/deep-successor-features-for-transfer_amd/sfx
V=${2:-b}
A=${3:-}
SFX_LIB=$S/libsfx_$V.so timeout -k 10 400 python -u -m pytest tests/test_gpu_runner.py tests/test_gpu_engine.py -x -q \
  --timeout 120 --timeout-method thread > $O/t_b.log 2>&1 || { tail -20 $O/t_b.log; exit 1; }
tail -1 $O/t_b.log
SFX_LIB=$S/libsfx_probe$A.so timeout -k 10 120 python tools/probe_run.py 30 > $O/probe_a.txt 2>&1 || exit 1
SFX_LIB=$S/libsfx_probe_$V.so timeout -k 10 120 python tools/probe_run.py 30 > $O/probe_b.txt 2>&1 || exit 1
run() {  # tag, lib
  SFX_LIB=$2 timeout -k 10 200 python bench.py --steps 2000 --warmup 200 --no-other --no-cpu-baseline --shard-steps 0 \
    --repeats 2 > $O/bench_$1.json 2>/dev/null || return 1
  python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().splitlines()[-1]);print(sys.argv[2], d['value'], d['repeats']['values'], d['roofline']['avg_launch_us'])" $O/bench_$1.json $1
}
run a1 $S/libsfx$A.so && run b1 $S/libsfx_$V.so && run a2 $S/libsfx$A.so && run b2 $S/libsfx_$V.so && \
  run a3 $S/libsfx$A.so && run b3 $S/libsfx_$V.so || exit 1
grep -E "sum" $O/probe_a.txt $O/probe_b.txt | cut -c1-150
