#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/gpu_alltests.sh && bash tools/ab_libs.sh "libsfx_prev.so libsfx.so" && bash tools/ab_env.sh "-" "SFX_FUSE_V0=0"
