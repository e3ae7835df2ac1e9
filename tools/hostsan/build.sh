#!/bin/bash
# Host-side AddressSanitizer + UndefinedBehaviorSanitizer build of the runner driver with libsfx's
# sources compiled in.  Every -fsanitize= follows -Xarch_host: only host code is instrumented (the
# GPU kernels are built as in csrc/Makefile).  Output: tools/hostsan/runner_hostsan (git-ignored).
# Run on the GPU box:  ASAN_OPTIONS=detect_leaks=0:verify_asan_link_order=0 tools/hostsan/runner_hostsan
set -e
cd "$(dirname "$0")"
CSRC=../../deep-successor-features-for-transfer_amd/csrc
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -g -std=c++17 -ffp-contract=off -fno-omit-frame-pointer \
  -Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-sanitize-recover=undefined \
  -I"$CSRC" -o runner_hostsan runner_hostsan.cpp "$CSRC/sfx.hip" -ldl
echo built tools/hostsan/runner_hostsan
