#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/gpu_alltests.sh && bash tools/ab_env.sh "SFX_FWD_TPW=1" "SFX_FWD_TPW=2"
