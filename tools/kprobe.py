"""Drive one engine entry point repeatedly (for rocprofv3 counter passes)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "deep-successor-features-for-transfer_amd")]
import torch
from sfx.engine import SFEngine
what = sys.argv[1] if len(sys.argv) > 1 else "update_all"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 50
T, n_s, H, A, d, B = 8, 17, 256, 7, 8, 32
eng = SFEngine(T, n_s, H, A, d, ("relu", "relu"), max_batch=B)
torch.manual_seed(0)
for t in range(T):
    flat = torch.randn(eng.P) * 0.05
    eng.load_head(t, flat, 0); eng.load_head(t, flat, 1); eng.load_w(t, torch.rand(d) * 0.01)
dev = "cuda"
s, s1 = torch.randn(B, n_s, device=dev), torch.randn(B, n_s, device=dev)
a = torch.randint(0, A, (B,), device=dev); phi = torch.rand(B, d, device=dev)
gamma = torch.full((B,), 0.9, device=dev); losses = torch.empty(T, 3, device=dev)
s_one = torch.randn(1, n_s, device=dev)
for _ in range(n):
    if what == "update_all":
        eng.update_all(s, a, phi, s1, gamma, losses=losses)
    else:
        eng.select_action(s_one, 0, True)
torch.cuda.synchronize()
print("done", what, n)
