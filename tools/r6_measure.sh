#!/bin/bash
# Round-6 measurement pass: MFMA counters of the headline kernels (fp32 and bf16 operand modes) and
# the speculation at T_glob = 64 on one GPU (all-task schedule and the sharded schedule, RCCL at
# world 1).  Each GPU step has its own time limit; the chain stops at the first failure.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r6m}
mkdir -p $O
export SFX_RUNNER_PIPELINE=0  # the profiler serialises dispatches (see tools/pmc_passes.sh)
timeout -s KILL 60 rocprofv3 --list-avail > $O/list_avail.txt 2>&1 || true
grep -o "SQ_[A-Z_]*MFMA[A-Z_0-9]*\|SQ_BUSY_CU_CYCLES\|GRBM_GUI_ACTIVE" $O/list_avail.txt | sort -u > $O/mfma_counters.txt || true
ARGS="--steps 100 --warmup 10 --prof-steps 20 --no-cpu-baseline --no-other --shard-steps 0 --repeats 0"
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE \
  --kernel-trace --output-format csv -d $O/mfma_fp32 -o run -- python3 bench.py $ARGS > $O/mfma_fp32.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE \
  --kernel-trace --output-format csv -d $O/mfma_bf16 -o run -- python3 bench.py $ARGS --precision bf16 > $O/mfma_bf16.log 2>&1
rc=$?; [ $rc -eq 0 ] || { tail -5 $O/mfma_fp32.log $O/mfma_bf16.log; exit $rc; }
unset SFX_RUNNER_PIPELINE
timeout -k 10 300 python3 bench.py --heads 64 --steps 2000 --warmup 200 --prof-steps 10 --repeats 0 --no-cpu-baseline --no-other --shard-steps 2000 > $O/t64.log 2>&1
rc=$?; tail -c 3000 $O/t64.log; exit $rc
