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
    # the reward-model biases and loss coefficients: caller-owned device scalars (the agent's tensors)
    eng.test_wb = st.wb.clone().float().to(eng.device)
    eng.test_lam = st.lam.clone().float().to(eng.device)
    return eng


def update(eng, i, s, a, r, s1, gamma, use_gpi, next_actions=None):
    return eng.phi_update(i, s, a, r, s1, gamma, eng.test_wb[i:i + 1], eng.test_lam[i:i + 1], use_gpi=use_gpi,
                          next_actions=next_actions)


def check_params(eng, st, T, k, frac=2e-3):
    params_close(torch.stack([eng.get_head(t, 0) for t in range(T)]), st.online, 1e-3 * k, max_bad_frac=frac)
    params_close(torch.stack([eng.get_head(t, 1) for t in range(T)]), st.target, 1e-3 * k, max_bad_frac=frac)
    params_close(torch.stack([eng.get_w(t)[0] for t in range(T)]), st.w, 1e-3 * k, max_bad_frac=frac)
    params_close(eng.phi_get(), st.phi, 1e-3 * k, max_bad_frac=frac)
    params_close(eng.test_wb.cpu(), st.wb, 1e-3 * k)
    rel_close(eng.test_lam.cpu(), st.lam, rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize("case", ["phi_gpi", "phi_nogpi"])
def test_phi_update_vs_golden(golden, case):
    g = golden("upd_" + case)
    st0 = phi_problem(g)
    T = int(g["T"])
    eng = engine_of(st0, int(g["target_update_ev"]))
    for j, (s, a, r, _, s1, gamma) in enumerate(phi_batches(g)):
        lo = update(eng, int(g["policies"][j]), s, a, r, s1, gamma, bool(g["use_gpi"]))
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
        lo = update(eng, i, s, a, r, s1, gamma, use_gpi, next_actions=nxt)
        assert torch.equal(nxt.cpu(), na), f"update {j}: next actions"
        rel_close(lo.cpu(), [loss, psi_loss, phi_loss, lam], rtol=1e-4, atol=1e-7)
    check_params(eng, st, T, k)
    eng.close()
    np.testing.assert_equal(k, 5)


def test_phi_error_budget_vs_float64():
    """what the learned-φ parameters are worth.  Five full-C2 updates on the GPU,
    in the fp32 oracle (the reference's ATen arithmetic) and in a float64 oracle following the
    same next actions.  The fresh Adam's first step moves an entry by ±lr whatever the size of
    its gradient, so an entry whose gradient is at rounding level may go either way: measured
    against float64, the GPU must flip no more entries than 2x the fp32 reference does (plus a
    floor of 2e-4 of the entries), every group; the losses within 1e-5 of float64."""
    from sfx.init import reference_heads

    spec = R.Spec(17, 256, 7, 8, ("relu", "relu"))
    T, B, k = 8, 32, 5
    online, w = reference_heads(T, spec.n_s, spec.H, spec.A, spec.d, spec.acts, seed=4)
    ps = R.PhiSpec(spec.n_s, spec.d)
    gen = torch.Generator().manual_seed(5)
    phi0 = torch.empty(ps.P).uniform_(-0.15, 0.15, generator=gen)
    wb0 = torch.empty(T).uniform_(-0.3, 0.3, generator=gen)
    st = R.PhiState(spec, ps, online.clone(), online.clone(), w.clone(), wb0.clone(), phi0.clone(), torch.ones(T))
    s64 = R.PhiState(spec, ps, online.double(), online.double(), w.double(), wb0.double(), phi0.double(),
                     torch.ones(T, dtype=torch.float64))
    eng = engine_of(st, 3)
    rows = []
    for j in range(k):
        i = (5 * j) % T
        s, s1 = torch.randn(B, spec.n_s, generator=gen), torch.randn(B, spec.n_s, generator=gen)
        a = torch.randint(0, spec.A, (B,), generator=gen)
        r = torch.rand(B, 1, generator=gen)
        gamma = torch.where(torch.rand(B, generator=gen) < 0.1, 0.0, 0.9)
        l32 = R.phi_update(st, (s, a, r, None, s1, gamma), i, use_gpi=True, target_update_ev=3)
        l64 = R.phi_update(s64, (s.double(), a, r.double(), None, s1.double(), gamma.double()), i, use_gpi=True,
                           target_update_ev=3, next_actions=l32[4])
        lo = update(eng, i, s, a, r, s1, gamma, True).cpu().double()
        for q in range(4):
            ref = float(l64[q])
            assert abs(float(lo[q]) - ref) <= 1e-5 * abs(ref) + 1e-9, (j, q, float(lo[q]), ref)

    def flips(x, ref64):
        x = torch.as_tensor(x).double().cpu().reshape(-1)
        ref64 = ref64.reshape(-1)
        bad = (x - ref64).abs() > 1e-5 + 1e-4 * ref64.abs()
        return float(bad.double().mean()), float((x - ref64).abs().max())

    groups = [("psi online", torch.stack([eng.get_head(t, 0) for t in range(T)]), st.online, s64.online),
              ("psi target", torch.stack([eng.get_head(t, 1) for t in range(T)]), st.target, s64.target),
              ("w", torch.stack([eng.get_w(t)[0] for t in range(T)]), st.w, s64.w),
              ("phi net", eng.phi_get(), st.phi, s64.phi),
              ("w bias", eng.test_wb, st.wb, s64.wb)]
    for name, gpu, ref32, ref64 in groups:
        (fg, mg), (fr, mr) = flips(gpu, ref64), flips(ref32, ref64)
        rows.append((name, fg, fr, mg, mr))
        print(f"{name:10s} flipped vs float64: GPU {fg:.2e}  reference fp32 {fr:.2e}   max |diff| {mg:.2e} / {mr:.2e}")
        assert fg <= max(2.0 * fr, 2e-4), (name, fg, fr)
        assert mg <= 2.0 * 1e-3 * k + 1e-5, (name, mg)
    eng.close()


class _Task:
    """tasks/task.py interface, enough for add_training_task."""

    def __init__(self, n_s, A, d, idx):
        self.n_s, self.A, self.d, self.idx = n_s, A, d, idx

    def action_count(self):
        return self.A

    def feature_dim(self):
        return self.d

    def encode_dim(self):
        return self.n_s

    def get_w(self):
        w = torch.zeros(self.d, 1)
        w[self.idx % self.d, 0] = 1.0
        return w


def test_dropin_deepsf_phi_vs_golden(golden, monkeypatch):
    """sfx.dropin's features.deep_phi.DeepSF_PHI with the reference's call convention
    (update_successor(transitions, phis_model, i, loss_coefficient, use_gpi), agents/sfdqn_phi.py):
    the golden run's losses, the agent's loss coefficients and reward-model biases updated in place,
    and -- after sync_phi_module -- the agent's φ net, ψ modules and fit_w as the reference left them."""
    from sfx.dropin import _host
    from sfx.dropin.features.deep import _flat, _unflat_into
    from sfx.dropin.features.deep_phi import DeepSF_PHI
    from tests.golden.recipe import agent_psi_lambda

    dev = torch.device("cuda", 0)
    monkeypatch.setattr(_host, "torch_device", lambda: dev)
    monkeypatch.setattr("sfx.dropin.features.deep.get_torch_device", lambda: dev)
    g = golden("upd_phi_gpi")
    spec = R.Spec(int(g["n_s"]), int(g["H"]), int(g["A"]), int(g["d"]), tuple(str(a) for a in g["acts"]))
    T = int(g["T"])
    sf = DeepSF_PHI(pytorch_model_handle=agent_psi_lambda(spec.H, spec.acts, 1e-3, dev), use_true_reward=False,
                    target_update_ev=int(g["target_update_ev"]))
    sf.reset()
    for t in range(T):
        sf.add_training_task(_Task(spec.n_s, spec.A, spec.d, t))
    with torch.no_grad():
        for t in range(T):
            _unflat_into(sf.psi[t][0][0], torch.from_numpy(g["online0"][t]))
            _unflat_into(sf.psi[t][1][0], torch.from_numpy(g["online0"][t]))
            lin = list.__getitem__(sf.fit_w, t)
            lin.weight.copy_(torch.from_numpy(g["w0"][t]).view(1, -1))
            lin.bias.copy_(torch.from_numpy(g["wb0"][t:t + 1]))
    n_in = 2 * spec.n_s + 1
    layers = [torch.nn.Linear(n_in, 2 * n_in), torch.nn.ReLU()]
    for _ in range(3):
        layers += [torch.nn.Linear(2 * n_in, 2 * n_in), torch.nn.ReLU()]
    pm = torch.nn.Sequential(*layers, torch.nn.Linear(2 * n_in, spec.d)).to(dev)
    _unflat_into(pm, torch.from_numpy(g["phi0"]))
    phis_model = ((pm, torch.nn.MSELoss(), None), (None, None, None))
    lams = [torch.ones(1, requires_grad=True, device=dev) for _ in range(T)]
    lam_ptrs = [x.data_ptr() for x in lams]
    for j, b in enumerate(phi_batches(g)):
        b = tuple(x.to(dev) for x in b)
        i = int(g["policies"][j])
        loss, psi_loss, phi_loss, lam = sf.update_successor(b, phis_model, i, lams[i], True)
        assert lam is lams[i]
        rel_close(torch.cat([loss, psi_loss, phi_loss, lam.detach()]).cpu(), g["losses"][j], rtol=1e-4, atol=1e-7)
    assert [x.data_ptr() for x in lams] == lam_ptrs
    rel_close(torch.cat([x.detach() for x in lams]).cpu(), g["lam"], rtol=1e-6, atol=1e-7)
    sf.sync_phi_module()
    k = int(g["k"])
    params_close(_flat(pm), g["phi"], 1e-3 * k, max_bad_frac=2e-3)
    params_close(torch.stack([_flat(sf.psi[t][0][0]) for t in range(T)]), g["online"], 1e-3 * k, max_bad_frac=2e-3)
    params_close(torch.stack([sf.fit_w[t].weight.detach().reshape(-1).cpu() for t in range(T)]), g["w"], 1e-3 * k)
    params_close(torch.stack([sf.fit_w[t].bias.detach().reshape(-1).cpu() for t in range(T)]).reshape(-1), g["wb"],
                 1e-3 * k)
    q, task = sf.GPI(torch.from_numpy(g["b_s"][0][:4]).to(dev), 0)
    assert q.shape == (4, T, spec.A) and task.shape == (4,)
