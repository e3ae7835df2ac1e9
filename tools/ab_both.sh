#!/bin/bash
# A/B of this build vs libsfx_prev.so on the headline and on Hopper TSF
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/ab_libs.sh "libsfx_prev.so libsfx.so" && bash tools/ab_libs.sh "libsfx_prev.so libsfx.so" --workload hopper-tsf
