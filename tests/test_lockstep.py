"""Host logic of the lockstep test phase (sfx/lockstep.py) on the CPU: the reference's sequential
test loop (agents/sfdqn.py:111-115 over test_agent :139-166, restated in tools/test_phase.py) and
the lockstep rollout must draw the same random numbers, take the same actions, fit the same
reward models and log the same lines in the same order.  The GPU's part (sfx_test_actions) is
stood in for here by a torch ψ MLP behind the engine interface; tests/test_gpu_lockstep.py runs
the real one."""
import random

import pytest
import torch

from tools.test_phase import ActionEnv, EvalAgent


class _Psi:
    """ψ of T random heads (torch, CPU) behind the two calls the test phase makes."""

    def __init__(self, T, n_s, A, d, seed=0):
        g = torch.Generator().manual_seed(seed)
        self.W1 = torch.randn(T, 32, n_s, generator=g) / n_s ** 0.5
        self.W2 = torch.randn(T, A * d, 32, generator=g) / 32 ** 0.5
        self.T, self.A, self.d = T, A, d

    def __call__(self, S):
        h = torch.relu(torch.einsum("tkn,bn->btk", self.W1, S))
        return torch.einsum("tok,btk->bto", self.W2, h).reshape(S.shape[0], self.T, self.A, self.d)


class _Engine:
    device = torch.device("cpu")

    def __init__(self, psi):
        self.psi, self.calls = psi, 0

    def test_actions(self, S, W):
        self.calls += 1
        out = []
        for e in range(S.shape[0]):  # row e under its own w, as w(psi) computes it
            q = torch.nn.functional.linear(self.psi(S[e:e + 1]), W[e:e + 1])[:, :, :, 0]
            c = torch.squeeze(torch.argmax(torch.max(q, axis=2).values, axis=1))
            out.append([int(c), int(torch.argmax(q[:, c, :]))])
        return torch.tensor(out)


class _SF:
    def __init__(self, psi):
        self.psi, self.eng, self.flushed = psi, _Engine(psi), 0

    def _engine(self, batch=1):
        return self.eng

    def _flush(self):
        self.flushed += 1

    def get_successors(self, s):
        return self.psi(torch.as_tensor(s).reshape(1, -1))


def _setup(E, ep_len, eps, seed=7):
    T, n_s, A, d = 4, 6, 9, 8
    random.seed(seed)
    torch.manual_seed(seed)
    sf = _SF(_Psi(T, n_s, A, d))
    tasks = [ActionEnv(n_s, A, d, 50 + e, torch.device("cpu")) for e in range(E)]
    return sf, EvalAgent(sf, A, ep_len, tasks, eps, torch.device("cpu")), tasks


@pytest.mark.parametrize("E,eps", [(1, 0.03), (5, 0.3), (6, 0.0), (3, 1.0)])
def test_lockstep_matches_sequential_test_phase(E, eps):
    from sfx.lockstep import test_tasks_lockstep

    ep_len, phases = 12, 2
    sf0, ref, tasks0 = _setup(E, ep_len, eps)
    R0 = [[ref.test_agent(t, i) for i, t in enumerate(tasks0)] for _ in range(phases)]
    st0 = random.getstate()
    sf1, agent, tasks1 = _setup(E, ep_len, eps)
    R1 = [test_tasks_lockstep(agent, tasks1) for _ in range(phases)]
    assert random.getstate() == st0  # the same draws, no more, no fewer
    assert R1 == R0
    assert agent.logger.lines == ref.logger.lines
    for wa, wb in zip(agent.test_tasks_weights, ref.test_tasks_weights):
        assert torch.equal(wa.weight, wb.weight)
    assert sf1.eng.calls == phases * ep_len and sf1.flushed == phases


def test_enable_binds_into_the_reference_train_loop():
    """sfx.lockstep.enable: the reference loop's per-task test_agent calls (sfdqn.py:113-115)
    return the lockstep returns in order; one lockstep rollout per test phase."""
    from sfx import lockstep

    E, ep_len = 4, 10

    def train(agent, test_tasks, phases):  # the shape of agents/sfdqn.py:78-123's test phase
        out = []
        for _ in range(phases):
            out.append([agent.test_agent(t, i) for i, t in enumerate(test_tasks)])
        return out

    _, ref, tasks0 = _setup(E, ep_len, 0.2)
    want = train(ref, tasks0, 3)
    sf, agent, tasks1 = _setup(E, ep_len, 0.2)
    agent.train = lambda train_tasks, n, viewers=None, n_view_ev=None, test_tasks=[], **kw: train(agent, test_tasks, 3)
    lockstep.enable(agent)
    assert agent.train([], 0, test_tasks=tasks1) == want
    assert sf.eng.calls == 3 * ep_len  # E tasks per call
    assert agent.logger.lines == ref.logger.lines


def test_lockstep_refuses_episodes_that_end_early():
    from sfx.lockstep import test_tasks_lockstep

    sf, agent, tasks = _setup(2, 8, 0.0)
    real = tasks[0].transition
    tasks[0].transition = lambda a: real(a)[:2] + (True,)
    with pytest.raises(RuntimeError, match="full-length episodes"):
        test_tasks_lockstep(agent, tasks)


class _SingleFileAgent(EvalAgent):
    """The single-file sfdqn.py's test members (:640-652, :695-738): (w_approx, Adam) per test
    task, the optimizer passed to update_test_reward_mapper, the module-level device."""

    def __init__(self, *a, **k):
        super().__init__(*a, **k)
        self.test_tasks_weights = [(w, torch.optim.Adam([{"params": w.parameters(), "lr": 1e-2,
                                                           "weight_decay": 1e-2}]))
                                   for w in self.test_tasks_weights]
        del self.device

    def get_test_action(self, s_enc, w):
        if random.random() <= self.test_epsilon:
            return torch.tensor(random.randrange(self.n_actions))
        q = w(self.sf.get_successors(s_enc))[:, :, :, 0]
        c = torch.squeeze(torch.argmax(torch.max(q, axis=2).values, axis=1))
        return torch.argmax(q[:, c, :])

    def test_agent(self, task, test_index):
        R, (w, optim) = 0.0, self.test_tasks_weights[test_index]
        s_enc, acc = self.encoding(task.initialize()), 0
        for _ in range(self.T):
            a = self.get_test_action(s_enc, w)
            s1, r, done = task.transition(a)
            acc += self.update_test_reward_mapper(w, optim, task, r, s_enc, a, s1).item()
            s_enc = s1
            R += r
        self.logger.log_target_error_progress(self.get_target_reward_mapper_error(R, acc, test_index, self.T))
        return R

    def update_test_reward_mapper(self, w_approx, optim, task, r, s, a, s1):
        phi = task.features(s, a, s1)
        r_t = torch.tensor(r).float().unsqueeze(0)
        optim.zero_grad()
        loss = torch.nn.MSELoss()(w_approx(phi), r_t)
        loss.backward()
        optim.step()
        return loss


def test_lockstep_single_file_sfdqn_shape():
    from sfx.lockstep import test_tasks_lockstep

    def setup():
        random.seed(11)
        torch.manual_seed(11)
        sf = _SF(_Psi(4, 6, 9, 8))
        sf._out_device = lambda: torch.device("cpu")
        tasks = [ActionEnv(6, 9, 8, 70 + e, torch.device("cpu")) for e in range(4)]
        return sf, _SingleFileAgent(sf, 9, 10, tasks, 0.25, torch.device("cpu")), tasks

    _, ref, tasks0 = setup()
    want = [[ref.test_agent(t, i) for i, t in enumerate(tasks0)] for _ in range(2)]
    st = random.getstate()
    _, agent, tasks1 = setup()
    assert [test_tasks_lockstep(agent, tasks1) for _ in range(2)] == want
    assert random.getstate() == st and agent.logger.lines == ref.logger.lines
    for (wa, _), (wb, _) in zip(agent.test_tasks_weights, ref.test_tasks_weights):
        assert torch.equal(wa.weight, wb.weight)
