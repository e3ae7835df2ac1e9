#!/bin/bash
# In-kernel probe timeline of the C2 step with the current defaults (look-ahead, 3 column tiles).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-r4r}
mkdir -p $O
P=deep-successor-features-for-transfer_amd/sfx/libsfx_probe.so
SFX_LIB=$P timeout -k 10 150 python tools/probe_run.py 30 > $O/probe_c2.txt 2>&1 || { tail -5 $O/probe_c2.txt; exit 1; }
cat $O/probe_c2.txt
