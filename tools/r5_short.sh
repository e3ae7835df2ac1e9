#!/bin/bash
# The driver's short bench window (--steps 20 --warmup 5) against longer ones, one box.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r5short}
mkdir -p $O
run() {  # tag, flags
  local tag=$1; shift
  timeout -k 10 200 python bench.py --no-other --no-cpu-baseline --shard-steps 0 "$@" > $O/bench_$tag.json 2>/dev/null || return 1
  python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().splitlines()[-1]);print(sys.argv[2], d['value'], d['ms_per_step'], d['repeats']['values'] if d['repeats'] else None, d['speculation'])" $O/bench_$tag.json $tag
}
run s20w5a --steps 20 --warmup 5 && run s20w5b --steps 20 --warmup 5 && run s20w200 --steps 20 --warmup 200 && \
  run s200w5 --steps 200 --warmup 5
