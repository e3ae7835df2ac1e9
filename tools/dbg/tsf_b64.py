"""Diagnostic: first-update losses of the TSF path (and the plain SF update) at several batch
sizes / shapes vs the oracle."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "deep-successor-features-for-transfer_amd")]
import torch
from oracle import ref_cpu as R
from sfx.engine import SFEngine
from sfx.init import reference_heads


def run(n_s, B, K, G, d, tsf=True, use_gpi=True):
    T = 3
    spec = R.Spec(n_s, 24, 5, d, ("relu", "relu"))
    gs = R.GSpec(n_s, G, K)
    online, w = reference_heads(T, n_s, 24, 5, d, spec.acts, seed=2)
    gen = torch.Generator().manual_seed(8)
    g = torch.empty(T, gs.P).uniform_(-0.3, 0.3, generator=gen)
    h = torch.empty(d * G + d).uniform_(-0.2, 0.2, generator=gen)
    st = R.TSFState(spec, online.clone(), online.clone(), w.clone(), gspec=gs, g=g.clone(), h=h.clone())
    eng = SFEngine(T, n_s, 24, 5, d, spec.acts, max_batch=64)
    eng.set_adam(1e-3, 0.0, 1e-3, 0.0)
    if tsf:
        eng.tsf_setup(G, K, 0.5, 1e-3, 0.0, 1e-3, 0.0)
    for t in range(T):
        eng.load_head(t, online[t], 0); eng.load_head(t, online[t], 1); eng.load_w(t, w[t])
        if tsf:
            eng.tsf_load_g(t, g[t])
    if tsf:
        eng.tsf_load_h(h)
    s, s1 = torch.randn(B, n_s, generator=gen), torch.randn(B, n_s, generator=gen)
    a = torch.randint(0, 5, (B,), generator=gen)
    phi, r = torch.rand(B, d, generator=gen), torch.rand(B, 1, generator=gen)
    gamma = torch.where(torch.rand(B, generator=gen) < 0.2, 0.0, 0.9)
    if tsf:
        ref = R.tsf_update(st, (s, a, r, phi, s1, gamma), 1, use_gpi=use_gpi, beta=0.5)
        lo = eng.tsf_update(1, s, a, r, phi, s1, gamma, use_gpi=use_gpi).cpu()
    else:
        ref = R.sf_update(st, (s, a, r, phi, s1, gamma), 1, use_gpi=use_gpi)
        lo = eng.update(1, s, a, r, phi, s1, gamma, use_gpi=use_gpi).cpu()
    refl = torch.tensor([float(x) for x in ref[:3]])
    print(f"tsf={tsf} n_s={n_s} B={B} K={K} G={G} d={d}: gpu {lo.tolist()} ref {refl.tolist()} "
          f"rel {((lo - refl).abs() / refl.abs().clamp_min(1e-12)).max().item():.2e}")
    eng.close()


for B in (16, 32, 33, 48, 63, 64):
    run(30, B, 2, 16, 12)
for B in (32, 64):
    run(30, B, 2, 16, 12, tsf=False)
    run(11, B, 2, 16, 12)
    run(11, B, 2, 16, 8)
    run(30, B, 0, 16, 12)
