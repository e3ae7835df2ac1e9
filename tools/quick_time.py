"""Quick GPU timing probe of the engine entry points at the BASELINE C2 shape."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "deep-successor-features-for-transfer_amd")]
import torch
from sfx.engine import SFEngine

T, n_s, H, A, d, B = 8, 17, 256, 7, 8, 32
eng = SFEngine(T, n_s, H, A, d, ("relu", "relu"), max_batch=B)
torch.manual_seed(0)
P = eng.P
for t in range(T):
    flat = torch.randn(P) * 0.05
    eng.load_head(t, flat, 0); eng.load_head(t, flat, 1); eng.load_w(t, torch.rand(d) * 0.01)
dev = "cuda"
s, s1 = torch.randn(B, n_s, device=dev), torch.randn(B, n_s, device=dev)
a = torch.randint(0, A, (B,), device=dev); phi = torch.rand(B, d, device=dev); r = torch.rand(B, device=dev)
gamma = torch.full((B,), 0.9, device=dev); s_one = torch.randn(1, n_s, device=dev)
losses = torch.empty(T, 3, device=dev); l3 = torch.empty(3, device=dev)

def timeit(name, fn, n=200):
    for _ in range(10): fn()
    torch.cuda.synchronize(); t0 = time.perf_counter()
    for _ in range(n): fn()
    torch.cuda.synchronize(); dt = (time.perf_counter() - t0) / n
    print(f"{name:32s} {dt*1e6:9.1f} us")

for graphs in (False, True):
  eng.set_graphs(graphs)
  print("graphs", graphs)
  timeit("select_action (B=1, T=8)", lambda: eng.select_action(s_one, 0, True))
  timeit("select_action + D2H", lambda: eng.select_action(s_one, 0, True).cpu())
  timeit("update active (gpi)", lambda: eng.update(0, s, a, r, phi, s1, gamma, True, losses=l3))
  timeit("update_all (T=8)", lambda: eng.update_all(s, a, phi, s1, gamma, losses=losses))
  timeit("gpi B=32", lambda: eng.gpi(s, w_index=0))
