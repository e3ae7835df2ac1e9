"""The headline's early windows (bench.py's default C2 run: 5 warm-up steps, then 20-step windows):
each window's env-steps/s beside the host-round steps it took -- how much of the first window's
deficit is the speculation of early training and how much is one-time cost.  Diagnostic only."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "deep-successor-features-for-transfer_amd")]
import torch  # noqa: E402

from sfx.engine import SFEngine  # noqa: E402
from sfx.init import reference_heads  # noqa: E402
from sfx.runner import NativeEnvLoop  # noqa: E402

T, B, n_s, H, A, d = 8, 32, 17, 256, 7, 8
W, N = int(os.environ.get("W", "20")), int(os.environ.get("N", "12"))
for trial in range(int(os.environ.get("TRIALS", "3"))):
    eng = SFEngine(T, n_s, H, A, d, ("relu", "relu"), max_batch=B)
    online, w = reference_heads(T, n_s, H, A, d, ("relu", "relu"), seed=0)
    for t in range(T):
        eng.load_head(t, online[t], 0)
        eng.load_head(t, online[t], 1)
        eng.load_w(t, w[t])
    eng.set_adam(1e-3, 0.0, 1e-3, 0.0)
    eng.set_target_update_ev(1000)
    loop = NativeEnvLoop(eng, batch=B, seed=1, schedule="all", p_end=0.0)
    loop.prefill(1000)
    loop.set_task(0)
    loop.warm()
    loop.run(5)
    torch.cuda.synchronize()
    out = []
    for k in range(N):
        h0 = loop.stats()["host_round_steps"]
        t0 = time.perf_counter()
        loop.run(W)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        out.append(f"{W / dt:7.0f}/{loop.stats()['host_round_steps'] - h0}")
    print(f"trial {trial}: windows of {W} (env-steps/s / host-round steps):", " ".join(out), flush=True)
    loop.close()
    eng.close()
