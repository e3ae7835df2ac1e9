# rocprofv3 kernel + memory-copy trace of the drop-in loop (reference buffer), then the per-step timeline
cd "${GRAFT_REPO_ROOT:-/root/repo}" && export TMPDIR=/tmp && mkdir -p gpurun_out/dtl
cat > gpurun_out/dtl/run.py <<'PY'
import os, sys
sys.path.insert(0, 'deep-successor-features-for-transfer_amd'); sys.path.insert(0, 'tools')
import dropin_loop
print(dropin_loop.measure('reference', steps=300, warmup=60))
PY
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/dtl/prof -o dl -- python3 gpurun_out/dtl/run.py > gpurun_out/dtl/run.log 2>&1 || exit 1
K=$(find gpurun_out/dtl/prof -name '*kernel_trace.csv' | head -1); M=$(find gpurun_out/dtl/prof -name '*memory_copy_trace.csv' | head -1)
python3 tools/dropin_timeline.py $K $M > gpurun_out/dtl/timeline.txt 2>&1; cat gpurun_out/dtl/timeline.txt
