#!/bin/bash
# A/B of a HIP runtime environment setting on the C2 bench (alternating pairs, one box)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r5env}
mkdir -p $O
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 2000 --warmup 200 --no-other --no-cpu-baseline --shard-steps 0 \
    --repeats 2 > $O/bench_$tag.json 2>/dev/null || return 1
  python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().splitlines()[-1]);print(sys.argv[2], d['value'], d['repeats']['values'], d['roofline']['avg_launch_us'])" $O/bench_$tag.json $tag
}
run a1 X=0 && run b1 HIP_FORCE_DEV_KERNARG=1 && run a2 X=0 && run b2 HIP_FORCE_DEV_KERNARG=1 && run a3 X=0 && run b3 HIP_FORCE_DEV_KERNARG=1
