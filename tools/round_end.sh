#!/bin/bash
# Round-end evidence on one MI355X box, in one call: GPU tests, smoke, the default bench line, a
# rocprofv3 kernel-trace summary of the default bench (and its prof window: tools/rocprof_window.py)
# and of TSF-NF, the HBM traffic (FETCH_SIZE / WRITE_SIZE passes, MI355X_MICROARCH.md corrections)
# and the MFMA counters (fp32 and bf16 operand modes) of the default workload, the drop-in's
# phases.  Every GPU step has its own time limit; the chain stops at the first failure.  The
# summaries are then copied into profiles/ by hand.
#   tools/round_end.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${1:-final}
mkdir -p $O
PMC="--steps 100 --warmup 10 --prof-steps 20 --no-cpu-baseline --no-other --shard-steps 0 --repeats 0"
MF="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 && \
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 500 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --no-cpu-baseline --no-other --shard-steps 0 > $O/prof.log 2>&1 && \
python3 tools/rocprof_window.py $O/prof/run_kernel_trace.csv $O/prof.log $O/rocprof_window.json > $O/window.log 2>&1 && \
rm -f $O/prof/run_kernel_trace.csv && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_tsfnf -o run -- python3 bench.py --workload hopper-tsf-nf --steps 500 --warmup 50 --no-cpu-baseline --no-other --shard-steps 0 > $O/prof_tsfnf.log 2>&1 && \
rm -f $O/prof_tsfnf/run_kernel_trace.csv && \
SFX_RUNNER_PIPELINE=0 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 bench.py $PMC > $O/fetch.log 2>&1 && \
SFX_RUNNER_PIPELINE=0 timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 bench.py $PMC > $O/write.log 2>&1 && \
python3 tools/pmc_traffic.py $O/fetch $O/write reacher17-all-T8-B32 $O/pmc_traffic.json > $O/traffic.log 2>&1 && \
SFX_RUNNER_PIPELINE=0 timeout -s KILL 120 rocprofv3 --pmc $MF --kernel-trace --output-format csv -d $O/mfma_fp32 -o run -- python3 bench.py $PMC > $O/mfma_fp32.log 2>&1 && \
SFX_RUNNER_PIPELINE=0 timeout -s KILL 120 rocprofv3 --pmc $MF --kernel-trace --output-format csv -d $O/mfma_bf16 -o run -- python3 bench.py $PMC --precision bf16 > $O/mfma_bf16.log 2>&1 && \
timeout -k 10 300 python3 tools/dropin_phases.py > $O/dropin_phases.txt 2>&1 && \
SFX_LIB=$PWD/deep-successor-features-for-transfer_amd/sfx/libsfx_probe.so timeout -k 10 150 python3 tools/probe_run.py 30 > $O/probe_c2.txt 2>&1 && \
SFX_CHECK_RUN=1 SFX_LIB=$PWD/deep-successor-features-for-transfer_amd/sfx/libsfx_check.so timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/check_suite.log 2>&1
rc=$?
tail -2 $O/pytest.log; tail -1 $O/smoke.log; tail -c 300 $O/bench.log
exit $rc
