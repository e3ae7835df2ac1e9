"""Lockstep test-task rollouts on the GPU (sfx/lockstep.py).

* ``sfx_test_actions`` (E test tasks, row e under its own w, agents/sfdqn.py:125-137): q within
  1e-5 relative of ψ·w in float64 from the library's own ψ, (c, a) the first-index argmaxes of
  that q, across launch chunks (E > max_batch).
* A whole test phase over the drop-in DeepSF, sequential as the reference runs it
  (tools/test_phase.py restates agents/sfdqn.py:139-184) vs in lockstep: the same returns, the
  same fitted reward models (bit for bit), the same log lines and the same random-stream state.
"""
import random

import pytest
import torch

from tests.conftest import gpu_available

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
