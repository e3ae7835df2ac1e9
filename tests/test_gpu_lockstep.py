"""Lockstep test-task rollouts on the GPU (sfx/lockstep.py).

* ``sfx_test_actions`` (E test tasks, row e under its own w, agents/sfdqn.py:125-137): q within
  1e-5 relative of ψ·w in float64 from the library's own ψ, (c, a) the first-index argmaxes of
  that q, across launch chunks (E > max_batch).
* A whole test phase over the drop-in DeepSF, sequential as the reference runs it
  (tools/test_phase.py restates agents/sfdqn.py:139-184) vs in lockstep: the same returns, the
  same fitted reward models (bit for bit with the user's torch mapper; within 1e-5 with the
  device mapper), the same log lines and the same random-stream state.
* ``sfx_test_reward_updates`` (agents/sfdqn.py:168-184 for E rows) vs the oracle at 1e-4.
* Episodes that end early: the lockstep entry point runs the sequential loop (decided up front).
"""
import random

import numpy as np
import pytest
import torch

from tests.conftest import gpu_available
from tests.test_gpu_engine import rel_close

pytestmark = pytest.mark.gpu


def _need_gpu():
    if not gpu_available():
        pytest.skip("no HIP device")


@pytest.mark.parametrize("E,d", [(5, 8), (40, 8), (7, 20)])
def test_test_actions_vs_psi_dot_w(E, d):
    _need_gpu()
    from sfx.engine import SFEngine

    torch.manual_seed(E + d)
    T, n_s, H, A = 6, 6, 64, 9
    eng = SFEngine(T, n_s, H, A, d, ("relu", "relu"), max_batch=16)
    try:
        for t in range(T):
            eng.load_head(t, 0.2 * torch.randn(eng.P), 0)
        S = torch.randn(E, n_s, device=eng.device)
        W = torch.randn(E, d, device=eng.device)
        q = torch.empty(E, T, A, device=eng.device)
        out = eng.test_actions(S, W, q_out=q).cpu()
        psi = eng.successors(S).double()
        q_ref = torch.einsum("etad,ed->eta", psi, W.double())
        torch.testing.assert_close(q.double(), q_ref, rtol=1e-5, atol=1e-6)
        qc = q.cpu()
        c = torch.argmax(torch.max(qc, dim=2).values, dim=1)
        a = torch.argmax(qc[torch.arange(E), c], dim=1)
        assert torch.equal(out[:, 0], c) and torch.equal(out[:, 1], a)
    finally:
        eng.close()


@pytest.mark.parametrize("E,eps", [(8, 0.03), (3, 0.5)])
def test_lockstep_phase_matches_sequential(E, eps):
    _need_gpu()
    from tools import test_phase

    ep_len, phases = 25, 2
    sf0, ref, tasks0 = test_phase.make(E=E, ep_len=ep_len, test_epsilon=eps, H=64)
    R0 = [test_phase.run_phase(ref, tasks0, False) for _ in range(phases)]
    st0 = random.getstate()
    w0 = [w.weight.detach().cpu() for w in ref.test_tasks_weights]
    sf0._close()
    sf1, agent, tasks1 = test_phase.make(E=E, ep_len=ep_len, test_epsilon=eps, H=64)
    R1 = [test_phase.run_phase(agent, tasks1, True) for _ in range(phases)]
    assert random.getstate() == st0
    assert R1 == R0
    for wa, wb in zip(agent.test_tasks_weights, w0):
        assert torch.equal(wa.weight.detach().cpu(), wb)
    assert agent.logger.lines == ref.logger.lines
    sf1._close()


@pytest.mark.parametrize("E,d", [(8, 8), (33, 12)])
def test_sf_test_reward_rows_vs_oracle(E, d):
    """sfx_test_reward_updates: E test tasks' SGD steps (agents/sfdqn.py:168-184) in one launch vs the
    oracle's per-task autograd + torch.optim.SGD, 4 steps: losses and w within 1e-4 relative."""
    _need_gpu()
    from oracle import ref_cpu as R
    from sfx.engine import SFEngine

    eng = SFEngine(2, 6, 32, 3, d, ("relu", "relu"), max_batch=16)
    try:
        gen = torch.Generator().manual_seed(E + d)
        w_ref = [torch.empty(1, d).uniform_(-0.01, 0.01, generator=gen) for _ in range(E)]
        W = torch.cat(w_ref).to(eng.device)
        for j in range(4):
            PHI = 2 * torch.rand(E, d, generator=gen) - 0.5
            r = torch.randn(E, generator=gen)
            lo = eng.test_reward_updates(PHI.to(eng.device), r.to(eng.device), W).cpu()
            want = [R.sf_test_reward_update(w_ref[e], PHI[e], float(r[e])) for e in range(E)]
            rel_close(lo, want, rtol=1e-4, atol=1e-7)
            rel_close(W.cpu(), torch.cat(w_ref), rtol=1e-4, atol=1e-7)
    finally:
        eng.close()


def test_lockstep_device_mapper_phase_vs_sequential():
    """The lockstep test phase with agents/sfdqn.py's reward mapper on the device (one
    sfx_test_reward_updates launch per step, losses read once per phase) vs the reference's sequential
    loop with its torch SGD per task and step: the same returns and random state; reward models
    and logged loss sums within 1e-5."""
    _need_gpu()
    from tools import test_phase

    E, ep_len, phases = 8, 25, 2
    sf0, ref, tasks0 = test_phase.make(E=E, ep_len=ep_len, test_epsilon=0.1, H=64)
    R0 = [test_phase.run_phase(ref, tasks0, False) for _ in range(phases)]
    st0 = random.getstate()
    w0 = [w.weight.detach().cpu() for w in ref.test_tasks_weights]
    sf0._close()
    sf1, agent, tasks1 = test_phase.make(E=E, ep_len=ep_len, test_epsilon=0.1, H=64, device_mapper=True)
    R1 = [test_phase.run_phase(agent, tasks1, True) for _ in range(phases)]
    assert random.getstate() == st0
    assert R1 == R0
    for wa, wb in zip(agent.test_tasks_weights, w0):
        torch.testing.assert_close(wa.weight.detach().cpu(), wb, rtol=1e-5, atol=1e-8)
    assert len(agent.logger.lines) == len(ref.logger.lines)
    for xa, xb in zip(agent.logger.lines, ref.logger.lines):
        assert xa["reward"] == xb["reward"] and xa["steps"] == xb["steps"] and xa["task"] == xb["task"]
        assert abs(xa["w_error"] - xb["w_error"]) <= 1e-5 * abs(xb["w_error"]) + 1e-7
    sf1._close()


def test_lockstep_episodes_that_end_run_sequentially():
    """Test tasks whose episodes end early: sfx.lockstep decides before the first step and runs the
    sequential loop -- returns, reward models (bit for bit), log lines and random state as the
    reference's."""
    _need_gpu()
    from tests.test_lockstep import _ending
    from tools import test_phase

    at = [None, 7, None, 3]
    sf0, ref, tasks0 = test_phase.make(E=4, ep_len=15, test_epsilon=0.2, H=64)
    _ending(tasks0, at)
    R0 = [test_phase.run_phase(ref, tasks0, False) for _ in range(2)]
    st0 = random.getstate()
    w0 = [w.weight.detach().cpu() for w in ref.test_tasks_weights]
    sf0._close()
    sf1, agent, tasks1 = test_phase.make(E=4, ep_len=15, test_epsilon=0.2, H=64, device_mapper=True)
    _ending(tasks1, at)
    R1 = [test_phase.run_phase(agent, tasks1, True) for _ in range(2)]
    assert R1 == R0 and random.getstate() == st0
    for wa, wb in zip(agent.test_tasks_weights, w0):
        assert torch.equal(wa.weight.detach().cpu(), wb)
    assert agent.logger.lines == ref.logger.lines
    sf1._close()


@pytest.mark.parametrize("E,K", [(5, 0), (12, 3)])
def test_tsf_test_rows_vs_oracle(E, K):
    """sfx_tsf_test_actions / sfx_tsf_test_updates (E test tasks per launch set, each row its own
    w, ω, moments, r, LR and Adam step) against the oracle's per-task get_test_action /
    update_test_reward_mapper (tsfdqn.py:859-997): actions exact, losses / w / ω / moments within
    1e-4 relative, over 3 steps."""
    _need_gpu()
    from oracle import ref_cpu as R
    from tools.tsf_test_phase import make_engine

    T, n_s, H, A, d, G = 6, 7, 64, 9, 12, 20
    eng = make_engine(T, n_s, H, A, d, G, K, max_batch=16, seed=E)
    try:
        spec, gs = R.Spec(n_s, H, A, d), R.GSpec(n_s, G, K)
        st = R.TSFState(spec, torch.stack([eng.get_head(t, 0) for t in range(T)]),
                        torch.stack([eng.get_head(t, 1) for t in range(T)]), torch.zeros(T, d), gspec=gs,
                        g=torch.stack([eng.tsf_get_g(t)[0] for t in range(T)]), h=eng.tsf_get_h())
        gen = torch.Generator().manual_seed(7 + E)
        om0 = torch.rand(E, T, generator=gen) + 0.1
        tms = [R.TestMapper(0.1 * torch.randn(d, generator=gen), om0[e] / om0[e].sum()) for e in range(E)]
        dev = eng.device
        W = torch.stack([tm.w for tm in tms]).to(dev)
        Om = torch.stack([tm.omega for tm in tms]).to(dev)
        M = torch.zeros(E, 2 * (d + T), device=dev)
        hy = dict(gamma=0.9, beta=0.5, lasso=0.05)
        for j in range(3):
            S, S1 = torch.randn(E, n_s, generator=gen), torch.randn(E, n_s, generator=gen)
            PHI = torch.rand(E, d, generator=gen)
            r = torch.rand(E, generator=gen)
            lrs = [(1e-3 * (1 + e % 3), 1e-4, 5e-3 * 0.99 ** (j + e), 1e-5) for e in range(E)]
            acts = eng.tsf_test_actions(S.to(dev), W, Om).cpu()
            a = torch.tensor([R.tsf_test_action(st, S[e], tms[e].w, tms[e].omega) for e in range(E)])
            assert torch.equal(acts, a), f"step {j}: greedy test actions"
            a1 = torch.randint(0, A, (E,), generator=gen)
            rowp = torch.tensor([[float(r[e]), *lrs[e][:2], *lrs[e][2:], float(j + 1)] for e in range(E)],
                                dtype=torch.float32).to(dev)
            lo = eng.tsf_test_updates(S.to(dev), S1.to(dev), a.to(dev), a1.to(dev), PHI.to(dev), W, Om, M, rowp,
                                      **hy).cpu()
            for e in range(E):
                f = lambda x: float(np.float32(x))  # noqa: E731
                ref = R.tsf_test_update(st, tms[e], S[e], int(a[e]), f(r[e]), PHI[e], S1[e], int(a1[e]), **hy,
                                        lr_w=f(lrs[e][0]), wd_w=f(lrs[e][1]), lr_o=f(lrs[e][2]), wd_o=f(lrs[e][3]))
                rel_close(lo[e], list(ref), rtol=1e-4, atol=1e-7)
                rel_close(W[e].cpu(), tms[e].w, rtol=1e-4, atol=1e-7)
                rel_close(Om[e].cpu(), tms[e].omega, rtol=1e-4, atol=1e-7)
                rel_close(M[e].cpu(), torch.cat([tms[e].wm, tms[e].wv, tms[e].om, tms[e].ov]), rtol=1e-4, atol=1e-9)
    finally:
        eng.close()


@pytest.mark.parametrize("E,eps,total", [(8, 0.03, 0), (3, 0.5, 1000)])
def test_tsf_lockstep_phase_matches_sequential(E, eps, total):
    """A TSF test phase over the library (tools/tsf_test_phase.py), sequential through the drop-in's
    per-call binding vs sfx.lockstep.test_tasks_lockstep_tsf: the same returns, log lines and random
    state; w, ω and the Adam moments within 1e-5 relative (the lockstep forward runs E rows per
    launch, the per-call one a single row)."""
    _need_gpu()
    from tools import tsf_test_phase as P

    ep_len, phases = 20, 2
    sf0, ref, tasks0 = P.make(E=E, ep_len=ep_len, test_epsilon=eps, total_training_steps=total)
    R0 = [P.run_phase(ref, tasks0, False) for _ in range(phases)]
    st0 = random.getstate()
    w0 = [w.weight.detach().cpu() for w, _, _ in ref.test_tasks_weights]
    o0 = [o.detach().cpu() for o in ref.omegas]
    m0 = [v[0].cpu() for v in sf0._test_state.values()]
    sf0._eng.close()
    sf1, agent, tasks1 = P.make(E=E, ep_len=ep_len, test_epsilon=eps, total_training_steps=total)
    R1 = [P.run_phase(agent, tasks1, True) for _ in range(phases)]
    assert random.getstate() == st0
    assert R1 == R0
    for (w, _, _), wb in zip(agent.test_tasks_weights, w0):
        torch.testing.assert_close(w.weight.detach().cpu(), wb, rtol=1e-5, atol=1e-8)
    for o, ob in zip(agent.omegas, o0):
        torch.testing.assert_close(o.detach().cpu(), ob, rtol=1e-5, atol=1e-8)
    for v, mb in zip(sf1._test_state.values(), m0):
        torch.testing.assert_close(v[0].cpu(), mb, rtol=1e-5, atol=1e-10)
    la = [x for x in agent.logger.lines if x[0] == "lr"]
    assert la == [x for x in ref.logger.lines if x[0] == "lr"]
    assert len(agent.logger.lines) == len(ref.logger.lines)
    for xa, xb in zip(agent.logger.lines, ref.logger.lines):
        if xa[0] == "err":
            assert xa[1]["reward"] == xb[1]["reward"]
            for k in ("w_error", "psi_loss", "phi_loss"):
                assert abs(xa[1][k] - xb[1][k]) <= 1e-5 * abs(xb[1][k]) + 1e-7
    sf1._eng.close()
