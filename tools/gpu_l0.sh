#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
SFX_LIB=deep-successor-features-for-transfer_amd/sfx/libsfx_probe.so timeout -k 10 200 python tools/probe_run.py 15 all > gpurun_out/probe_l0b.txt 2>&1 || exit 1
grep "fwdL0\|pos" gpurun_out/probe_l0b.txt | head -3
bash tools/gpu_alltests.sh && bash tools/ab_libs.sh "libsfx_prev.so libsfx.so"
