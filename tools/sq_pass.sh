#!/bin/bash
# Wave-level counters per dispatch (one --pmc pass; SQ block has 8 slots, GRBM 2).
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-sq}
export SFX_RUNNER_PIPELINE=0
timeout -k 10 400 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
  --output-format csv -d gpurun_out/${TAG} -o run -- python3 bench.py --steps 60 --warmup 10 --prof-steps 10 --no-cpu-baseline --shard-steps 0 > gpurun_out/${TAG}.log 2>&1
