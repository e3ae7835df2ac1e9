#!/bin/bash
# UBSan function-check bisection of the runner's stalled first update step: its result published
# by a separate k_publish instead of k_ver's last workgroup; its inputs pulled instead of pushed.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-r4o}
mkdir -p $O
for m in 2 3; do
  HOSTSAN_BISECT=$m UBSAN_OPTIONS=print_stacktrace=1 timeout -k 10 120 tools/hostsan/runner_ubsan_fn > $O/bisect$m.txt 2>&1
  rc=$?; echo "bisect $m rc=$rc"; tail -3 $O/bisect$m.txt
  [ $rc -le 1 ] || exit $rc
done
