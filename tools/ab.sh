#!/bin/bash
# Alternating A/B of two arms on ONE box (the only comparison this pool's box-to-box spread allows):
#   tools/ab.sh TAG PAIRS 'ARM_A' 'ARM_B' [bench.py args ...]
# An arm is a space-separated list of VAR=value settings for the bench process ('' = as is), e.g.
#   tools/ab.sh skip 3 'SFX_SKIP=1' 'SFX_SKIP=0' --steps 2000 --warmup 200
#   tools/ab.sh lib 3 '' "SFX_LIB=$PWD/deep-successor-features-for-transfer_amd/sfx/libsfx_probe.so"
# Default bench args: the C2 headline without the side legs.  Prints tag, value, repeats and the
# dominant kernel's live average per run; each run has its own time limit, the first failure ends it.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=$1; PAIRS=$2; A=$3; B=$4; shift 4
ARGS="$*"; [ -n "$ARGS" ] || ARGS="--steps 2000 --warmup 200 --repeats 2"
O=gpurun_out/ab_$TAG; mkdir -p $O
run() {  # name, settings
  env $2 timeout -k 10 300 python3 bench.py $ARGS --no-other --no-cpu-baseline --shard-steps 0 > $O/$1.json 2>$O/$1.err || return 1
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().splitlines()[-1]);r=d['roofline'];print(sys.argv[2], d['value'], (d.get('repeats') or {}).get('values'), r['kernel'], r['avg_launch_us'])" $O/$1.json $1
}
for i in $(seq 1 $PAIRS); do
  run a$i "$A" && run b$i "$B" || exit 1
done
