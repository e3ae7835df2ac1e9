"""GPU parity of the learned-φ update (sfx_phi_*): features/deep_phi.py
DeepSF_PHI.update_successor against

  * golden vectors from the real reference (tests/golden/upd_phi_{gpi,nogpi}.npz, tools/gen_golden.py
    gen_phi) -- losses, λ, ψ online / target, w and its bias, the φ net;
  * the oracle (oracle/ref_cpu.py phi_update, pinned by those vectors) at the full C2 shape
    (8 heads of 256, n_s = 17, A = 7, d = 8; φ net 35 -> 70 x4 -> 8).

Tolerances: losses, λ and the next actions as elsewhere (1e-4 relative, exact).  Parameters: the
reference's update is a freshly built Adam's first step, lr·g/(|g| + ε) -- ±lr for any gradient
well above ε -- so a parameter whose gradient is at rounding level in either computation may move
the other way: params_close with lr_steps = lr·k bounds those by 2·lr per step, and only a small
fraction of entries may be among them.
"""
import numpy as np
import pytest
import torch

from oracle import ref_cpu as R
from tests.conftest import gpu_available
from tests.test_gpu_engine import params_close, rel_close
from tests.test_oracle_golden import phi_batches, phi_problem

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _need_gpu():
    if not gpu_available():
        pytest.skip("no HIP device")


def engine_of(st: R.PhiState, ev: int, max_batch=32):
    from sfx.engine import SFEngine

    spec, T = st.spec, st.online.shape[0]
    eng = SFEngine(T, spec.n_s, spec.H, spec.A, spec.d, spec.acts, max_batch=max_batch)
    eng.set_adam(1e-3, 0.0, 1e-3, 0.0)
    eng.set_target_update_ev(ev)
    for t in range(T):
        eng.load_head(t, st.online[t], 0)
        eng.load_head(t, st.target[t], 1)
        eng.load_w(t, st.w[t])
    eng.phi_setup(st.pspec.width_mul, st.pspec.n_mid, 1e-3)
    eng.phi_load(st.phi)
    for t in range(T):
        eng.phi_task(t, bias=float(st.wb[t]), lam=float(st.lam[t]))
    return eng


def check_params(eng, st, T, k, frac=2e-3):
    params_close(torch.stack([eng.get_head(t, 0) for t in range(T)]), st.online, 1e-3 * k, max_bad_frac=frac)
    params_close(torch.stack([eng.get_head(t, 1) for t in range(T)]), st.target, 1e-3 * k, max_bad_frac=frac)
    params_close(torch.stack([eng.get_w(t)[0] for t in range(T)]), st.w, 1e-3 * k, max_bad_frac=frac)
    params_close(eng.phi_get(), st.phi, 1e-3 * k, max_bad_frac=frac)
    bl = [eng.phi_task(t) for t in range(T)]
    params_close(torch.tensor([b for b, _ in bl]), st.wb, 1e-3 * k)
    rel_close(torch.tensor([l for _, l in bl]), st.lam, rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize("case", ["phi_gpi", "phi_nogpi"])
def test_phi_update_vs_golden(golden, case):
    g = golden("upd_" + case)
    st0 = phi_problem(g)
    T = int(g["T"])
    eng = engine_of(st0, int(g["target_update_ev"]))
    for j, (s, a, r, _, s1, gamma) in enumerate(phi_batches(g)):
        lo = eng.phi_update(int(g["policies"][j]), s, a, r, s1, gamma, use_gpi=bool(g["use_gpi"]))
        rel_close(lo.cpu(), g["losses"][j], rtol=1e-4, atol=1e-7)
    ref = R.PhiState(st0.spec, st0.pspec, torch.from_numpy(g["online"]), torch.from_numpy(g["target"]),
                     torch.from_numpy(g["w"]), torch.from_numpy(g["wb"]), torch.from_numpy(g["phi"]),
                     torch.from_numpy(g["lam"]).float())
    check_params(eng, ref, T, int(g["k"]))
    eng.close()


@pytest.mark.parametrize("use_gpi", [True, False])
def test_phi_update_full_c2_vs_oracle(use_gpi):
    from sfx.init import reference_heads

    spec = R.Spec(17, 256, 7, 8, ("relu", "relu"))
    T, B, k = 8, 32, 5
    online, w = reference_heads(T, spec.n_s, spec.H, spec.A, spec.d, spec.acts, seed=4)
    ps = R.PhiSpec(spec.n_s, spec.d)
    gen = torch.Generator().manual_seed(5)
    phi0 = torch.empty(ps.P).uniform_(-0.15, 0.15, generator=gen)
    st = R.PhiState(spec, ps, online.clone(), online.clone(), w.clone(), torch.empty(T).uniform_(-0.3, 0.3, generator=gen),
                    phi0, torch.ones(T))
    eng = engine_of(st, 3)
    nxt = torch.empty(B, dtype=torch.int64, device="cuda")
    for j in range(k):
        i = (5 * j) % T
        s, s1 = torch.randn(B, spec.n_s, generator=gen), torch.randn(B, spec.n_s, generator=gen)
        a = torch.randint(0, spec.A, (B,), generator=gen)
        r = torch.rand(B, 1, generator=gen)
        gamma = torch.where(torch.rand(B, generator=gen) < 0.1, 0.0, 0.9)
        loss, psi_loss, phi_loss, lam, na = R.phi_update(st, (s, a, r, None, s1, gamma), i, use_gpi=use_gpi,
                                                         target_update_ev=3)
        lo = eng.phi_update(i, s, a, r, s1, gamma, use_gpi=use_gpi, next_actions=nxt)
        assert torch.equal(nxt.cpu(), na), f"update {j}: next actions"
        rel_close(lo.cpu(), [loss, psi_loss, phi_loss, lam], rtol=1e-4, atol=1e-7)
    check_params(eng, st, T, k)
    eng.close()
    np.testing.assert_equal(k, 5)
