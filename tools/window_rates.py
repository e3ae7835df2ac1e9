"""Env-steps/s, skip rate and host-round steps per window of the headline workload (C2 all-task,
the bench's setup) from the first step on: where the speculative step's cost comes from over
training.  Usage: python tools/window_rates.py [windows] [steps_per_window]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "deep-successor-features-for-transfer_amd")]
import torch  # noqa: E402

from sfx.engine import SFEngine  # noqa: E402
from sfx.init import reference_heads  # noqa: E402
from sfx.runner import NativeEnvLoop  # noqa: E402

nw = int(sys.argv[1]) if len(sys.argv) > 1 else 12
per = int(sys.argv[2]) if len(sys.argv) > 2 else 500
T = 8
eng = SFEngine(T, 17, 256, 7, 8, ("relu", "relu"), max_batch=32, device="cuda:0")
online, w = reference_heads(T, 17, 256, 7, 8, ("relu", "relu"), seed=0)
for t in range(T):
    eng.load_head(t, online[t], 0)
    eng.load_head(t, online[t], 1)
    eng.load_w(t, w[t])
eng.set_adam(1e-3, 0.0, 1e-3, 0.0)
eng.set_target_update_ev(1000)
loop = NativeEnvLoop(eng, batch=32, seed=1)
loop.prefill(1000)
loop.set_task(0)
loop.warm()
done = 0
for k in range(nw):
    s0, k0, l0 = eng.step_stats(), eng.skip_stats(), loop.stats()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    loop.run(per)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    s1, k1, l1 = eng.step_stats(), eng.skip_stats(), loop.stats()
    chk = k1["policies_checked"] - k0["policies_checked"]
    sk = k1["policies_skipped"] - k0["policies_skipped"]
    print(f"steps {done:6d}-{done + per:6d}: {per / dt:8.1f} env-steps/s  skipped {sk / max(chk, 1):.3f} of "
          f"{chk / per:.2f} policy-rounds/step  host-round steps {l1['host_round_steps'] - l0['host_round_steps']:4d}  "
          f"host wait {(l1['host_wait_us'] - l0['host_wait_us']) / per:6.1f} us/step", flush=True)
    done += per
loop.close()
eng.close()
