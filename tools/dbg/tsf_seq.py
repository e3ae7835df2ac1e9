"""Diagnostic: the ragged-shape TSF test's update sequence, per-update losses and parameter
differences vs the oracle."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "deep-successor-features-for-transfer_amd")]
import torch
from oracle import ref_cpu as R
from sfx.engine import SFEngine
from sfx.init import reference_heads

n_s, B, K, G, d = [int(x) for x in sys.argv[1:6]]
os.environ["SFX_TSF_FORK"] = sys.argv[6] if len(sys.argv) > 6 else "1"
T = 3
spec = R.Spec(n_s, 24, 5, d, ("relu", "relu"))
gs = R.GSpec(n_s, G, K)
online, w = reference_heads(T, spec.n_s, spec.H, spec.A, spec.d, spec.acts, seed=2)
gen = torch.Generator().manual_seed(8)
g = torch.empty(T, gs.P).uniform_(-0.3, 0.3, generator=gen)
h = torch.empty(d * G + d).uniform_(-0.2, 0.2, generator=gen)
st = R.TSFState(spec, online.clone(), online.clone(), w.clone(), gspec=gs, g=g.clone(), h=h.clone())
eng = SFEngine(T, spec.n_s, spec.H, spec.A, spec.d, spec.acts, max_batch=64)
eng.set_adam(1e-3, 0.0, 1e-3, 0.0)
eng.set_target_update_ev(3)
eng.tsf_setup(G, K, 0.5, 1e-3, 0.0, 1e-3, 0.0)
for t in range(T):
    eng.load_head(t, online[t], 0); eng.load_head(t, online[t], 1); eng.load_w(t, w[t]); eng.tsf_load_g(t, g[t])
eng.tsf_load_h(h)
for j, i in enumerate((1, 0, 2, 1, 1)):
    s, s1 = torch.randn(B, n_s, generator=gen), torch.randn(B, n_s, generator=gen)
    a = torch.randint(0, spec.A, (B,), generator=gen)
    phi, r = torch.rand(B, d, generator=gen), torch.rand(B, 1, generator=gen)
    gamma = torch.where(torch.rand(B, generator=gen) < 0.2, 0.0, 0.9)
    loss, l1, l2, na = R.tsf_update(st, (s, a, r, phi, s1, gamma), i, use_gpi=j != 2, beta=0.5, target_update_ev=3)
    lo = eng.tsf_update(i, s, a, r, phi, s1, gamma, use_gpi=j != 2).cpu()
    ref = torch.tensor([float(loss), float(l1), float(l2)])
    dpsi = max((eng.get_head(t, 0) - st.online[t]).abs().max().item() for t in range(T))
    dg = max((torch.as_tensor(eng.tsf_get_g(t)[0]) - st.g[t]).abs().max().item() for t in range(T))
    dh = (torch.as_tensor(eng.tsf_get_h()) - st.h).abs().max().item()
    dw = max((eng.get_w(t)[0].cpu() - st.w[t]).abs().max().item() for t in range(T))
    print(f"j={j} i={i}: loss rel {((lo - ref).abs() / ref.abs()).max().item():.2e}  max|d| psi {dpsi:.2e} g {dg:.2e} "
          f"h {dh:.2e} w {dw:.2e}")

# which g entries differ after the first update (rerun from scratch)
st2 = R.TSFState(spec, online.clone(), online.clone(), w.clone(), gspec=gs, g=g.clone(), h=h.clone())
eng.close()
eng = SFEngine(T, spec.n_s, spec.H, spec.A, spec.d, spec.acts, max_batch=64)
eng.set_adam(1e-3, 0.0, 1e-3, 0.0)
eng.tsf_setup(G, K, 0.5, 1e-3, 0.0, 1e-3, 0.0)
for t in range(T):
    eng.load_head(t, online[t], 0); eng.load_head(t, online[t], 1); eng.load_w(t, w[t]); eng.tsf_load_g(t, g[t])
eng.tsf_load_h(h)
gen = torch.Generator().manual_seed(8)
_ = torch.empty(T, gs.P).uniform_(-0.3, 0.3, generator=gen); _ = torch.empty(d * G + d).uniform_(-0.2, 0.2, generator=gen)
s, s1 = torch.randn(B, n_s, generator=gen), torch.randn(B, n_s, generator=gen)
a = torch.randint(0, spec.A, (B,), generator=gen)
phi, r = torch.rand(B, d, generator=gen), torch.rand(B, 1, generator=gen)
gamma = torch.where(torch.rand(B, generator=gen) < 0.2, 0.0, 0.9)
R.tsf_update(st2, (s, a, r, phi, s1, gamma), 1, beta=0.5)
eng.tsf_update(1, s, a, r, phi, s1, gamma)
ge, gm, gv = (torch.as_tensor(x) for x in eng.tsf_get_g(1))
diff = (ge - st2.g[1]).abs()
fs = 2 * n_s + 1
for j in torch.nonzero(diff > 1e-5).flatten().tolist():
    where = f"flow {j // fs} e {j % fs}" if j < K * fs else f"linear {j - K * fs}"
    print(f"g[{j}] ({where}): before {g[1, j].item():.6e} oracle {st2.g[1, j].item():.6e} gpu {ge[j].item():.6e} "
          f"oracle m {st2.gm[1, j].item():.3e} gpu m {gm[j].item():.3e} oracle v {st2.gv[1, j].item():.3e} gpu v {gv[j].item():.3e}")
