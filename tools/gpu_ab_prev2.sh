#!/bin/bash
# GPU tests, then A/B of this build vs libsfx_prev.so on the headline and on Hopper TSF
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/gpu_alltests.sh && bash tools/ab_libs.sh "libsfx_prev.so libsfx.so" && \
  O2=1 bash tools/ab_libs.sh "libsfx_prev.so libsfx.so" --workload hopper-tsf
