#!/bin/bash
# the whole GPU suite twice in a row (flake check; assertion failures are reported, faults stop it)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/x2
for i in 1 2; do
  timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/x2/t$i.log 2>&1
  rc=$?; echo "run $i rc=$rc: $(tail -1 gpurun_out/x2/t$i.log)"; grep FAILED gpurun_out/x2/t$i.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
