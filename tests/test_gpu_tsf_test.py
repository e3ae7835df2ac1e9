"""GPU parity of the TSF test-task path: TSFDQN.get_test_action's greedy branch
and update_test_reward_mapper (tsfdqn.py:859-997) as libsfx calls (sfx_tsf_test_action /
sfx_tsf_test_update), against

  * golden vectors from the real reference (tests/golden/test_tsf*.npz, tools/gen_golden.py
    gen_tsf_test: 10 steps with ω's learning rate decaying, tsfdqn.py and tsfdqn_nf.py with 3
    planar layers) -- greedy actions exact, losses / w / ω within 1e-4 relative;
  * the oracle (oracle/ref_cpu.py tsf_test_*, pinned by those vectors) at the full C3 / C5 shape
    (16 heads, H = 256, A = 27, d = 50, G = 100, K = 0 and 100);
  * the drop-in binding: sfx.dropin.bind's get_test_action / update_test_reward_mapper on an agent
    whose tensors live on the GPU, updating w_approx and ω in place.
"""
import types

import numpy as np
import pytest
import torch

from oracle import ref_cpu as R
from tests.conftest import gpu_available
from tests.test_gpu_engine import rel_close
from tests.test_oracle_golden import tsf_test_hyper, tsf_test_problem

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


@pytest.fixture(autouse=True)
def _need_gpu():
    if not gpu_available():
        pytest.skip("no HIP device")


def engine_of(st, max_batch=32):
    from sfx.engine import SFEngine

    spec, gs = st.spec, st.gspec
    eng = SFEngine(st.T, spec.n_s, spec.H, spec.A, spec.d, spec.acts, max_batch=max_batch)
    eng.set_adam(1e-3, 0.0, 1e-3, 0.0)
    eng.tsf_setup(gs.G, gs.K, 1.0, 1e-3, 0.0, 1e-3, 0.0)
    for t in range(st.T):
        eng.load_head(t, st.online[t], 0)
        eng.load_head(t, st.target[t], 1)
        eng.tsf_load_g(t, st.g[t])
    eng.tsf_load_h(st.h)
    return eng


def run_steps(eng, st, tm, steps, check):
    """steps: (s, a, r, phi, s1, a1, hyper) tuples; check(j, greedy_dev, greedy_ref, losses_dev, ref)."""
    d, T = st.spec.d, st.T
    w = tm.w.clone().to(DEV)
    om = tm.omega.clone().to(DEV)
    state = torch.zeros(2 * (d + T), device=DEV)
    for j, (s, a, r, phi, s1, a1, hy) in enumerate(steps):
        greedy = int(eng.tsf_test_action(s.to(DEV), w, om))
        greedy_ref = R.tsf_test_action(st, s, tm.w, tm.omega)
        a_dev = torch.tensor(a, device=DEV)
        a1_dev = torch.tensor(a1, device=DEV)
        lo = eng.tsf_test_update(s.to(DEV), s1.to(DEV), a_dev, a1_dev, r, phi.to(DEV), w, om, state, j + 1,
                                 hy["gamma"], hy["beta"], hy["lasso"], hy["lr_w"], hy["wd_w"], hy["lr_o"], hy["wd_o"])
        ref = R.tsf_test_update(st, tm, s, a, r, phi, s1, a1, **hy)
        check(j, greedy, greedy_ref, lo.cpu(), ref)
        rel_close(w.cpu(), tm.w, rtol=1e-4, atol=1e-7)
        rel_close(om.cpu(), tm.omega, rtol=1e-4, atol=1e-7)
    return w, om


@pytest.mark.parametrize("case", ["tsf", "tsf_nf"])
def test_tsf_test_path_vs_golden(golden, case):
    g = golden("test_" + case)
    st, tm = tsf_test_problem(g)
    eng = engine_of(st)
    steps = [(torch.from_numpy(g["s"][j]), int(g["a"][j]), float(g["r"][j]), torch.from_numpy(g["phi"][j]),
              torch.from_numpy(g["s1"][j]), int(g["a1"][j]), tsf_test_hyper(g, j)) for j in range(int(g["k"]))]

    def check(j, greedy, greedy_ref, lo, ref):
        assert greedy == int(g["greedy"][j]) == greedy_ref, f"step {j}: greedy test action"
        rel_close(lo, [g["loss"][j], g["l2"][j], g["l1"][j]], rtol=1e-4, atol=1e-7)

    w, om = run_steps(eng, st, tm, steps, check)
    rel_close(w.cpu(), g["w"][-1], rtol=1e-4, atol=1e-7)
    rel_close(om.cpu(), g["omega"][-1], rtol=1e-4, atol=1e-7)
    eng.close()


@pytest.mark.parametrize("K", [0, 100])
def test_tsf_test_path_full_c3_vs_oracle(K):
    from tests.test_gpu_tsf import tsf_c3_problem

    T = 16
    spec, gs, st = tsf_c3_problem(T, K)
    gen = torch.Generator().manual_seed(21)
    st.target.add_(torch.randn(st.target.shape, generator=gen) * 1e-3)
    om0 = torch.rand(T, generator=gen)
    tm = R.TestMapper(torch.empty(spec.d).uniform_(-0.01, 0.01, generator=gen), om0 / om0.sum())
    eng = engine_of(st)
    hy = dict(gamma=0.9, beta=0.5, lasso=0.05, lr_w=1e-3, wd_w=1e-3, lr_o=5e-3, wd_o=1e-4)
    steps = []
    for j in range(6):
        s, s1 = torch.randn(1, spec.n_s, generator=gen), torch.randn(1, spec.n_s, generator=gen)
        a, a1 = int(torch.randint(0, spec.A, (1,), generator=gen)), int(torch.randint(0, spec.A, (1,), generator=gen))
        steps.append((s, a, float(torch.rand(1, generator=gen)), torch.rand(1, spec.d, generator=gen), s1, a1,
                      dict(hy, lr_o=hy["lr_o"] * 0.99 ** j)))

    def check(j, greedy, greedy_ref, lo, ref):
        assert greedy == greedy_ref, f"step {j}: greedy test action"
        rel_close(lo, list(ref), rtol=1e-4, atol=1e-7)

    run_steps(eng, st, tm, steps, check)
    eng.close()


def test_dropin_binding_updates_agent_tensors_in_place(golden):
    """bind.tsf_get_test_action / tsf_update_test_reward_mapper on an agent stand-in (the attributes
    the reference's methods use) with its w_approx and ω on the GPU: greedy actions and every step
    as the golden run, the agent's own tensors updated in place, the optimizer untouched."""
    from sfx.dropin import bind

    g = golden("test_tsf")
    st, tm = tsf_test_problem(g)
    eng = engine_of(st)

    class SF:  # the drop-in DeepTSF's test-task methods over this engine
        from sfx.dropin.features.deep_sequential_tsf import DeepTSF as _D
        tsf_test_action = _D.tsf_test_action
        tsf_test_update = _D.tsf_test_update
        _on_engine = _D._on_engine

        def __init__(self):
            self._eng, self._test_state = eng, {}
            self.n_features, self.n_tasks = st.spec.d, st.T

        def _engine(self, batch=1):
            return self._eng

        def _flush(self):
            pass

        def _out_device(self):
            return DEV

    hyper = dict(beta_loss_coefficient=float(g["beta"]), omegas_l1_coefficient=float(g["lasso"]))
    agent = types.SimpleNamespace(sf=SF(), test_epsilon=-1.0, n_actions=st.spec.A, device=DEV, h_function=object(),
                                  hyperparameters=hyper, gamma=float(g["gamma"]), total_training_steps=1)
    w_approx = torch.nn.Linear(st.spec.d, 1, bias=False).to(DEV)
    with torch.no_grad():
        w_approx.weight.copy_(tm.w.view(1, -1))
    omegas = tm.omega.view(1, -1, 1, 1).clone().to(DEV).requires_grad_(True)
    w_ptr, om_ptr = w_approx.weight.data_ptr(), omegas.data_ptr()
    optim = torch.optim.Adam([{"params": w_approx.parameters(), "lr": float(g["lr_w"]), "weight_decay": float(g["wd_w"])},
                              {"params": omegas, "lr": 5e-3, "weight_decay": float(g["wd_o"])}])
    task = types.SimpleNamespace(features=lambda s, a, s1: task.phi, phi=None)
    for j in range(int(g["k"])):
        optim.param_groups[1]["lr"] = float(g["lr_o"][j])
        s, s1 = torch.from_numpy(g["s"][j]).to(DEV), torch.from_numpy(g["s1"][j]).to(DEV)
        a = bind.tsf_get_test_action(agent, s, w_approx, omegas)
        assert int(a) == int(g["greedy"][j])
        task.phi = torch.from_numpy(g["phi"][j]).to(DEV)
        loss, l2, l1 = bind.tsf_update_test_reward_mapper(agent, w_approx, omegas, optim, task, float(g["r"][j]), s,
                                                          torch.tensor(int(g["a"][j]), device=DEV), s1,
                                                          torch.tensor(int(g["a1"][j]), device=DEV))
        rel_close(torch.stack([loss, l2, l1]).cpu(), [g["loss"][j], g["l2"][j], g["l1"][j]], rtol=1e-4, atol=1e-7)
        rel_close(w_approx.weight.detach().reshape(-1).cpu(), g["w"][j], rtol=1e-4, atol=1e-7)
        rel_close(omegas.detach().reshape(-1).cpu(), g["omega"][j], rtol=1e-4, atol=1e-7)
    assert w_approx.weight.data_ptr() == w_ptr and omegas.data_ptr() == om_ptr
    assert not optim.state  # the moments live in the library, the torch optimizer never stepped
    eng.close()
    np.testing.assert_equal(int(g["k"]), 10)
