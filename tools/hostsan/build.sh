#!/bin/bash
# Host-side sanitizer builds of the runner driver with libsfx's sources compiled in.  Every
# -fsanitize= follows -Xarch_host: only host code is instrumented (the GPU kernels are built as in
# csrc/Makefile).  Outputs (git-ignored) in tools/hostsan/:
#   runner_asan   AddressSanitizer                       (default)
#   runner_ubsan  UndefinedBehaviorSanitizer, no recover ("ubsan")
#   runner_asan_full / runner_ubsan_full: the same with every flag ("asan_full": ASan's default
#   use-after-return mode; "ubsan_full": UBSan's function and vptr checks too)
#   runner_ubsan_fn / runner_ubsan_vptr: UBSan's function check alone / its vptr check alone
#   fnptr_plain / fnptr_function: fnptr_launch.hip (kernels launched through a function pointer,
#   eagerly and from a captured graph) without and with -fsanitize=function
# Run on the GPU box:
#   ASAN_OPTIONS=detect_leaks=0:verify_asan_link_order=0 tools/hostsan/runner_asan
#   UBSAN_OPTIONS=print_stacktrace=1 tools/hostsan/runner_ubsan
set -e
cd "$(dirname "$0")"
CSRC=../../deep-successor-features-for-transfer_amd/csrc
F="--offload-arch=gfx950 -O3 -g -std=c++17 -ffp-contract=off -fno-omit-frame-pointer -I$CSRC"
if [ "${1:-asan}" = plain ]; then  # no sanitizer (the reference run for a diff)
  /opt/rocm/bin/hipcc $F -o runner_plain runner_hostsan.cpp "$CSRC/sfx.hip" -ldl
  echo built tools/hostsan/runner_plain
elif [ "${1:-asan}" = ubsan_fn ] || [ "${1:-asan}" = ubsan_vptr ]; then  # one of the two suspects alone
  chk=${1#ubsan_}; [ $chk = fn ] && chk=function
  /opt/rocm/bin/hipcc $F -Xarch_host -fsanitize=$chk -Xarch_host -fno-sanitize-recover=$chk \
    -o runner_$1 runner_hostsan.cpp "$CSRC/sfx.hip" -ldl
  echo built tools/hostsan/runner_$1
elif [ "${1:-asan}" = fnptr ]; then  # kernel launches through a function pointer, plain and -fsanitize=function
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O2 -std=c++17 -o fnptr_plain fnptr_launch.hip
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O2 -std=c++17 -Xarch_host -fsanitize=function \
    -Xarch_host -fno-sanitize-recover=function -o fnptr_function fnptr_launch.hip
  echo built tools/hostsan/fnptr_plain tools/hostsan/fnptr_function
elif [ "${1:-asan}" = ubsan_full ]; then  # every UBSan check, function / vptr included (round-3 hang)
  /opt/rocm/bin/hipcc $F -Xarch_host -fsanitize=undefined -Xarch_host -fno-sanitize-recover=undefined \
    -o runner_ubsan_full runner_hostsan.cpp "$CSRC/sfx.hip" -ldl
  echo built tools/hostsan/runner_ubsan_full
elif [ "${1:-asan}" = asan_full ]; then  # ASan's default use-after-return mode (round-3 hang)
  /opt/rocm/bin/hipcc $F -Xarch_host -fsanitize=address -o runner_asan_full runner_hostsan.cpp "$CSRC/sfx.hip" -ldl
  echo built tools/hostsan/runner_asan_full
elif [ "${1:-asan}" = ubsan ]; then
  /opt/rocm/bin/hipcc $F -Xarch_host -fsanitize=undefined -Xarch_host -fno-sanitize=function,vptr \
    -Xarch_host -fno-sanitize-recover=undefined -o runner_ubsan runner_hostsan.cpp "$CSRC/sfx.hip" -ldl
  echo built tools/hostsan/runner_ubsan
else
  /opt/rocm/bin/hipcc $F -Xarch_host -fsanitize=address -Xarch_host -fsanitize-address-use-after-return=never \
    -o runner_asan runner_hostsan.cpp "$CSRC/sfx.hip" -ldl
  echo built tools/hostsan/runner_asan
fi
