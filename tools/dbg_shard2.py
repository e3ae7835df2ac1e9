"""Debug: bench's sequence -- an all-task runner first, then the sharded runner at one rank."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "deep-successor-features-for-transfer_amd")]
import torch  # noqa: E402

from sfx.engine import SFEngine  # noqa: E402
from sfx.init import reference_heads  # noqa: E402
from sfx.runner import NativeEnvLoop  # noqa: E402
from sfx.shard import init_comm  # noqa: E402

first = sys.argv[1] == "first"


def engine(shard):
    eng = SFEngine(8, 17, 256, 7, 8, ("relu", "relu"), max_batch=32, device="cuda:0")
    online, w = reference_heads(8, 17, 256, 7, 8, ("relu", "relu"), seed=0)
    eng.set_adam(1e-3, 0.0, 1e-3, 0.0)
    eng.set_target_update_ev(1000)
    if shard:
        eng.shard_setup(8, 0)
    for t in range(8):
        eng.load_head(t, online[t], 0)
        eng.load_head(t, online[t], 1)
        eng.load_w(t, w[t])
    return eng


if first:
    e0 = engine(False)
    l0 = NativeEnvLoop(e0, batch=32, seed=1)
    l0.prefill(1000)
    l0.set_task(0)
    l0.warm()
    l0.run(200)
    e0.prof_reset()
    e0.prof_enable(True)
    l0.run(50)
    e0.prof_enable(False)
    e0.prof_reset()
    print("first runner done", l0.stats(), flush=True)
eng = engine(True)
init_comm(eng, 0, 1)
loop = NativeEnvLoop(eng, batch=32, seed=1, schedule="sharded")
loop.prefill(1000)
loop.set_task(0)
loop.warm()
t0 = time.perf_counter()
try:
    loop.run(40)
    loop.run(400)
    print("ok", loop.stats(), eng.step_stats(), time.perf_counter() - t0)
except Exception as e:
    print("FAIL", loop.stats(), eng.step_stats(), e, time.perf_counter() - t0)
