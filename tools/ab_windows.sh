#!/bin/bash
# A/B of the headline's early windows (tools/first_windows.py) on ONE box, alternating: A = the
# library as built, B = SFX_LIB=.../libsfx_ab.so (build it from the other revision first).
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/abw
for i in 1 2 3; do
  TRIALS=2 timeout -k 10 120 python3 tools/first_windows.py > gpurun_out/abw/a$i.txt 2>&1 || exit 1
  SFX_LIB=deep-successor-features-for-transfer_amd/sfx/libsfx_ab.so TRIALS=2 timeout -k 10 120 python3 tools/first_windows.py > gpurun_out/abw/b$i.txt 2>&1 || exit 1
done
grep -h trial gpurun_out/abw/a*.txt | sed 's/^/A /'; grep -h trial gpurun_out/abw/b*.txt | sed 's/^/B /'
