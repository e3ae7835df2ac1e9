#!/bin/bash
# the driver's short window with 2 / 3 device rounds per step, one box
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r5short2}
mkdir -p $O
run() {  # tag, flags
  local tag=$1; shift
  timeout -k 10 200 python bench.py --no-other --no-cpu-baseline --shard-steps 0 "$@" > $O/bench_$tag.json 2>/dev/null || return 1
  python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().splitlines()[-1]);s=d['speculation'];print(sys.argv[2], d['value'], d['ms_per_step'], d['repeats']['values'] if d['repeats'] else None, s['steps'], s['host_round_steps'], s['prelaunched'])" $O/bench_$tag.json $tag
}
run r2a --steps 20 --warmup 5 && run r3a --steps 20 --warmup 5 --spec-rounds 3 && run r2b --steps 20 --warmup 5 && \
  run r3b --steps 20 --warmup 5 --spec-rounds 3 && run r2long --steps 2000 --warmup 200 --repeats 1 && \
  run r3long --steps 2000 --warmup 200 --spec-rounds 3 --repeats 1
