#!/bin/bash
# The folded publication's setup, printed per k_ver launch (SFX_DEBUG_VER=1), in the plain driver
# build and in the UBSan-function build (which stalls at the first folded publication).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-r4p}
mkdir -p $O
SFX_GRAPHS=0 SFX_DEBUG_VER=1 HOSTSAN_BISECT=4 timeout -k 10 120 tools/hostsan/runner_plain > $O/plain.txt 2>&1
rc=$?; echo "plain rc=$rc"; grep -m3 "k_ver" $O/plain.txt; [ $rc -le 1 ] || exit $rc
SFX_GRAPHS=0 SFX_DEBUG_VER=1 HOSTSAN_BISECT=4 UBSAN_OPTIONS=print_stacktrace=1 timeout -k 10 120 tools/hostsan/runner_ubsan_fn > $O/ubsan_fn.txt 2>&1
rc=$?; echo "ubsan_fn rc=$rc"; grep -m3 "k_ver" $O/ubsan_fn.txt; tail -2 $O/ubsan_fn.txt
