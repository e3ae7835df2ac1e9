"""Host-side cost of the drop-in's per-step library calls (C2 shape): the time each call takes on
the host alone, with the device idle when it starts (synchronised before, settled after, outside
the timed region) -- what a Python agent loop pays per call beside the GPU work."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "deep-successor-features-for-transfer_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from sfx.dropin.agents.buffer import ReplayBuffer  # noqa: E402
from sfx.engine import SFEngine  # noqa: E402

T, n_s, H, A, d, B = 8, 17, 256, 7, 8, 32
eng = SFEngine(T, n_s, H, A, d, ("relu", "relu"), max_batch=B)
torch.manual_seed(0)
for t in range(T):
    flat = torch.randn(eng.P) * 0.05
    eng.load_head(t, flat, 0)
    eng.load_head(t, flat, 1)
    eng.load_w(t, torch.rand(d) * 0.01)
dev = "cuda"
s, s1 = torch.randn(B, n_s, device=dev), torch.randn(B, n_s, device=dev)
a = torch.randint(0, A, (B,), device=dev)
phi = torch.rand(B, d, device=dev)
gamma = torch.full((B,), 0.9, device=dev)
s_one, phi1 = torch.randn(1, n_s, device=dev), torch.rand(d, device=dev)
losses = torch.empty(T, 3, device=dev)
buf = ReplayBuffer({}, n_batch=B)
buf.device = torch.device("cuda", 0)
for _ in range(200):
    buf.append(s_one.reshape(1, -1), torch.tensor(3, device=dev), phi1, s_one.reshape(1, -1), 0.9)


def host(name, fn, after=None, n=300):
    ts = []
    for i in range(n + 20):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        t1 = time.perf_counter()
        if after:
            after()
        if i >= 20:
            ts.append(t1 - t0)
    ts = np.array(ts) * 1e6
    print(f"{name:40s} median {np.median(ts):8.1f} us   p10 {np.percentile(ts, 10):8.1f}", flush=True)


settle = lambda: eng.step_stats()  # noqa: E731  (any entry point settles a pending update_all)
for graphs in (True, False):
    eng.set_graphs(graphs)
    print("graphs", graphs, flush=True)
    host("update_all (launch only)", lambda: eng.update_all(s, a, phi, s1, gamma, losses=losses), settle)

    def busy_then_update():
        torch.cuda._sleep(20000)  # the stream still busy when the update is launched (the agent loop's case)
        t0 = time.perf_counter()
        eng.update_all(s, a, phi, s1, gamma, losses=losses)
        busy_then_update.dt.append(time.perf_counter() - t0)

    busy_then_update.dt = []
    host("  (sleep kernel + update_all)", busy_then_update, settle)
    print(f"{'update_all behind a busy stream':40s} median {np.median(busy_then_update.dt[20:]) * 1e6:8.1f} us", flush=True)
    host("gpi B=1 (idle device)", lambda: eng.gpi(s_one, w_index=0))
    host("lms (device phi, float r)", lambda: eng.lms(0, phi1, 0.5, 0.05))
    host("replay buffer append", lambda: buf.append(s_one.reshape(1, -1), a[:1].reshape(()), phi1, s_one.reshape(1, -1), 0.9))
    host("replay buffer replay", lambda: buf.replay())
    host("torch.empty x1 (reference)", lambda: torch.empty(4, device=dev))
