"""Debug: the sharded runner at one rank without collectives (8-step graphs)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "deep-successor-features-for-transfer_amd")]
import torch  # noqa: E402

from sfx.engine import SFEngine  # noqa: E402
from sfx.init import reference_heads  # noqa: E402
from sfx.runner import NativeEnvLoop  # noqa: E402
from sfx.shard import init_comm  # noqa: E402

warm = sys.argv[1] == "warm"
n = int(sys.argv[2])
ev = int(sys.argv[3])
eng = SFEngine(8, 17, 256, 7, 8, ("relu", "relu"), max_batch=32, device="cuda:0")
online, w = reference_heads(8, 17, 256, 7, 8, ("relu", "relu"), seed=0)
eng.set_adam(1e-3, 0.0, 1e-3, 0.0)
eng.set_target_update_ev(ev)
eng.shard_setup(8, 0)
for t in range(8):
    eng.load_head(t, online[t], 0)
    eng.load_head(t, online[t], 1)
    eng.load_w(t, w[t])
init_comm(eng, 0, 1)
loop = NativeEnvLoop(eng, batch=32, seed=1, schedule="sharded")
loop.prefill(1000)
loop.set_task(0)
if warm:
    loop.warm()
try:
    for k in range(n // 10):
        loop.run(10)
    print("ok", loop.stats(), eng.step_stats())
except Exception as e:
    print("FAIL after", loop.stats(), eng.step_stats(), e)
