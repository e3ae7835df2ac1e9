#!/bin/bash
# TSF A/B on one box: a libsfx variant (sfx/libsfx_<V>.so, probe sfx/libsfx_probe_<V>.so) against the
# tree's build -- TSF / runner parity tests on the variant, TSF-NF probe timelines of both,
# alternating Hopper TSF and TSF-NF bench pairs.  Every GPU step time-limited.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r5ab9}
mkdir -p $O
S=$PWD/deep-successor-features-for-transfer_amd/sfx
V=${2:-g}
SFX_LIB=$S/libsfx_$V.so timeout -k 10 500 python -u -m pytest tests/test_gpu_tsf.py tests/test_gpu_tsf_test.py tests/test_gpu_runner.py tests/test_gpu_shard.py tests/test_gpu_native_shard.py tests/test_gpu_dropin.py -x -q \
  --timeout 200 --timeout-method thread > $O/t_b.log 2>&1 || { tail -20 $O/t_b.log; exit 1; }
tail -1 $O/t_b.log
SFX_LIB=$S/libsfx_probe.so timeout -k 10 150 python tools/probe_run.py 30 tsf-nf > $O/probe_a.txt 2>&1 || exit 1
SFX_LIB=$S/libsfx_probe_$V.so timeout -k 10 150 python tools/probe_run.py 30 tsf-nf > $O/probe_b.txt 2>&1 || exit 1
SFX_LIB=$S/libsfx_probe.so timeout -k 10 150 python tools/probe_run.py 30 tsf > $O/probe_tsf_a.txt 2>&1 || exit 1
SFX_LIB=$S/libsfx_probe_$V.so timeout -k 10 150 python tools/probe_run.py 30 tsf > $O/probe_tsf_b.txt 2>&1 || exit 1
run() {  # tag, lib, workload
  SFX_LIB=$2 timeout -k 10 200 python bench.py --workload $3 --steps 2000 --warmup 200 --no-other --no-cpu-baseline \
    --shard-steps 0 > $O/bench_$1.json 2>/dev/null || return 1
  python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().splitlines()[-1]);print(sys.argv[2], d['value'])" $O/bench_$1.json $1
}
for w in hopper-tsf hopper-tsf-nf; do
  run ${w}_a1 $S/libsfx.so $w && run ${w}_b1 $S/libsfx_$V.so $w && run ${w}_a2 $S/libsfx.so $w && \
    run ${w}_b2 $S/libsfx_$V.so $w && run ${w}_a3 $S/libsfx.so $w && run ${w}_b3 $S/libsfx_$V.so $w || exit 1
done
grep -E "sum" $O/probe_a.txt $O/probe_b.txt $O/probe_tsf_a.txt $O/probe_tsf_b.txt | cut -c1-150
