# TSF lockstep test phase: its GPU tests, its rate, then the whole GPU suite and a quick bench
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/tsflock; mkdir -p $O
timeout -k 10 300 python -u tools/tsf_test_phase.py > $O/rate.log 2>&1 || { tail -20 $O/rate.log; exit 1; }
cat $O/rate.log
bash tools/gpu_alltests.sh && bash tools/gpu_quick_bench.sh
