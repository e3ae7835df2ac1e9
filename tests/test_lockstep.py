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

    def test_reward_updates(self, phi, r, W, lr=0.005, wd=0.01, losses=None):
        """sfx_test_reward_updates over the oracle (agents/sfdqn.py:168-184 by autograd + SGD), row
        by row: bit-identical to the user's own mapper on the CPU."""
        from oracle import ref_cpu as R
        self.mapper_calls = getattr(self, "mapper_calls", 0) + 1
        out = torch.tensor([R.sf_test_reward_update(W[e], phi[e], float(r[e])) for e in range(W.shape[0])])
        if losses is not None:
            losses.copy_(out)
            return losses
        return out


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

    def train(agent, test_tasks, phases):  # noqa: F811  # the shape of agents/sfdqn.py:78-123's test phase
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


def _ending(tasks, at):
    """Make task e's episodes end after at[e] steps (None: never), as gym's Hopper / CartPole do."""
    for t, n in zip(tasks, at):
        real, t._n = t.transition, 0

        def tr(a, t=t, real=real, n=n):
            s1, r, _ = real(a)
            t._n += 1
            return s1, r, n is not None and t._n % n == 0
        t.transition = tr
        t.episodes_never_end = n is None


@pytest.mark.parametrize("device_mapper", [False, True])
def test_lockstep_decides_up_front_for_episodes_that_end(device_mapper):
    """Test tasks whose episodes end early: the lockstep entry point sees that before the first step
    and runs the reference's sequential loop -- the same returns, reward models, log lines and
    random state, and no lockstep launch."""
    from sfx.lockstep import test_tasks_lockstep

    ep_len, at = 12, [None, 5, None]
    sf0, ref, tasks0 = _setup(3, ep_len, 0.2)
    _ending(tasks0, at)
    R0 = [[ref.test_agent(t, i) for i, t in enumerate(tasks0)] for _ in range(2)]
    st0 = random.getstate()
    sf1, agent, tasks1 = _setup(3, ep_len, 0.2)
    _ending(tasks1, at)
    if device_mapper:
        type(agent).update_test_reward_mapper.__sfx_mapper__ = "sgd"
    try:
        R1 = [test_tasks_lockstep(agent, tasks1) for _ in range(2)]
    finally:
        type(agent).update_test_reward_mapper.__dict__.pop("__sfx_mapper__", None)
    assert R1 == R0 and random.getstate() == st0
    assert agent.logger.lines == ref.logger.lines
    for wa, wb in zip(agent.test_tasks_weights, ref.test_tasks_weights):
        assert torch.equal(wa.weight, wb.weight)
    assert sf1.eng.calls == 0 and sf1.flushed == 0  # never started a lockstep step


def test_lockstep_declared_endless_task_that_ends_warns_and_finishes():
    """A task declared endless that ends anyway: no exception mid-phase; it stops (the reference's
    break), the phase finishes, and the tasks before it match the sequential loop exactly."""
    from sfx.lockstep import test_tasks_lockstep

    sf0, ref, tasks0 = _setup(3, 10, 0.0)
    _ending(tasks0, [None, None, 4])
    want = [ref.test_agent(t, i) for i, t in enumerate(tasks0)]
    sf1, agent, tasks1 = _setup(3, 10, 0.0)
    _ending(tasks1, [None, None, 4])
    with pytest.warns(RuntimeWarning, match="declared never to end"):
        got = test_tasks_lockstep(agent, tasks1, episodes_end=False)
    assert got == want  # ε = 0: no draws depend on where task 2 ended
    assert tasks1[2]._n == 4


@pytest.mark.parametrize("E,eps", [(1, 0.03), (5, 0.3), (4, 1.0)])
def test_lockstep_device_reward_mapper_matches_sequential(E, eps):
    """agents/sfdqn.py's own reward mapper (SGD on w_approx) is recognised and run as one engine
    call per step over all E rows (sfx_test_reward_updates, here over the oracle): returns, reward
    models, log lines (the losses' python sums, read once per phase) and random state as the
    sequential loop with the user's torch SGD."""
    from sfx import lockstep

    ep_len, phases = 9, 2
    sf0, ref, tasks0 = _setup(E, ep_len, eps)
    R0 = [[ref.test_agent(t, i) for i, t in enumerate(tasks0)] for _ in range(phases)]
    st0 = random.getstate()
    sf1, agent, tasks1 = _setup(E, ep_len, eps)
    assert not lockstep.device_reward_mapper(agent)
    type(agent).update_test_reward_mapper.__sfx_mapper__ = "sgd"
    try:
        assert lockstep.device_reward_mapper(agent)
        R1 = [lockstep.test_tasks_lockstep(agent, tasks1) for _ in range(phases)]
    finally:
        del type(agent).update_test_reward_mapper.__sfx_mapper__
    assert random.getstate() == st0 and R1 == R0
    assert agent.logger.lines == ref.logger.lines
    for wa, wb in zip(agent.test_tasks_weights, ref.test_tasks_weights):
        assert torch.equal(wa.weight, wb.weight)
    assert sf1.eng.mapper_calls == phases * ep_len


def test_device_reward_mapper_recognises_only_the_reference_method():
    from sfx.lockstep import device_reward_mapper

    class SFDQN:
        def update_test_reward_mapper(self, w_approx, task, r, s, a, s1):
            pass
    SFDQN.__module__ = "agents.sfdqn"
    SFDQN.update_test_reward_mapper.__module__ = "agents.sfdqn"
    SFDQN.update_test_reward_mapper.__qualname__ = "SFDQN.update_test_reward_mapper"
    assert device_reward_mapper(SFDQN())

    class Mine(SFDQN):
        def update_test_reward_mapper(self, w_approx, task, r, s, a, s1):
            pass
    assert not device_reward_mapper(Mine())
    x = SFDQN()
    x.update_test_reward_mapper = lambda *a: None
    assert not device_reward_mapper(x)


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


# ---- TSF agents' test phase (sfx.lockstep.test_tasks_lockstep_tsf; tools/tsf_test_phase.py) ----

class _TsfOracleEngine:
    """The four TSF test-task calls of the engine over the oracle (oracle/ref_cpu.py
    tsf_test_action / tsf_test_update, pinned by tests/golden/test_tsf*.npz), row by row, with the
    float32 rounding of the C ABI's scalar arguments: the sequential binding and the lockstep rollout
    then agree exactly when the host logic (draws, schedules, LR, steps, write-back) does."""
    device = torch.device("cpu")
    max_batch = 4

    def __init__(self, st):
        self.st, self.batched = st, 0

    def tsf_test_action(self, s, w, om):
        from oracle import ref_cpu as R
        return torch.tensor(R.tsf_test_action(self.st, torch.as_tensor(s).float(), w, om))

    def tsf_test_update(self, s, s1, a, a1, r, phi, w, om, state, step, gamma, beta, lasso, lr_w, wd_w, lr_o, wd_o):
        import numpy as np
        from oracle import ref_cpu as R
        f = lambda x: float(np.float32(x))  # noqa: E731
        d, T = w.numel(), om.numel()
        tm = R.TestMapper(w.clone(), om.clone(), state[:d].clone(), state[d:2 * d].clone(),
                          state[2 * d:2 * d + T].clone(), state[2 * d + T:].clone(), step - 1)
        out = R.tsf_test_update(self.st, tm, torch.as_tensor(s).float(), int(a), f(r), torch.as_tensor(phi).float(),
                                torch.as_tensor(s1).float(), int(a1), gamma=f(gamma), beta=f(beta), lasso=f(lasso),
                                lr_w=f(lr_w), wd_w=f(wd_w), lr_o=f(lr_o), wd_o=f(wd_o))
        w.copy_(tm.w)
        om.copy_(tm.omega)
        state.copy_(torch.cat([tm.wm, tm.wv, tm.om, tm.ov]))
        return torch.tensor(out)

    def tsf_test_actions(self, S, W, Om):
        assert S.shape[0] <= self.max_batch
        self.batched += 1
        return torch.stack([self.tsf_test_action(S[e], W[e], Om[e]) for e in range(S.shape[0])])

    def tsf_test_updates(self, S, S1, A, A1, PHI, W, Om, M, rowp, gamma, beta, lasso, losses=None):
        self.batched += 1
        losses = torch.empty(S.shape[0], 3) if losses is None else losses
        for e in range(S.shape[0]):
            r, lw, ww, lo, wo, step = rowp[e].tolist()
            losses[e] = self.tsf_test_update(S[e], S1[e], A[e], A1[e], r, PHI[e], W[e], Om[e], M[e], int(step), gamma,
                                             beta, lasso, lw, ww, lo, wo)
        return losses


def _tsf_setup(E, ep_len, eps, total=0, seed=11):
    from oracle import ref_cpu as R
    from tools import tsf_test_phase as P

    T, n_s, A, d, G, K = 4, 6, 9, 8, 10, 2
    spec, gs = R.Spec(n_s, 16, A, d), R.GSpec(n_s, G, K)
    g = torch.Generator().manual_seed(5)
    online = 0.3 * torch.randn(T, spec.P, generator=g)
    st = R.TSFState(spec, online, online + 1e-2 * torch.randn(T, spec.P, generator=g), torch.zeros(T, d), gspec=gs,
                    g=0.3 * torch.randn(T, K * (2 * n_s + 1) + G * n_s + G, generator=g),
                    h=0.3 * torch.randn(d * G + d, generator=g))
    _, agent, tasks = P.make(E=E, T_heads=T, n_s=n_s, A=A, d=d, ep_len=ep_len, test_epsilon=eps, seed=seed,
                             total_training_steps=total, eng=_TsfOracleEngine(st), device=torch.device("cpu"))
    return agent, tasks


def _printed(capsys):
    import re
    return sorted(re.sub(r" at 0x[0-9a-f]+", "", x) for x in capsys.readouterr().out.splitlines())


@pytest.mark.parametrize("E,eps,total", [(3, 0.05, 0), (6, 0.4, 5000), (2, 1.0, 1000), (5, 0.0, 7)])
def test_tsf_lockstep_matches_sequential_test_phase(E, eps, total, capsys):
    """Two phases: returns, fitted w / ω, Adam moments, LR schedules, log lines (only when
    total_training_steps % 5000 == 0), the diagnostic prints (randint draws when % 1000 == 0)
    and the random state as the reference's sequential loop; E = 5, 6 run as two lockstep
    groups (max_batch 4)."""
    from sfx.lockstep import test_tasks_lockstep_tsf

    ep_len, phases = 6, 2
    ref, tasks0 = _tsf_setup(E, ep_len, eps, total)
    R0 = [[ref.test_agent(t, i) for i, t in enumerate(tasks0)] for _ in range(phases)]
    st0 = random.getstate()
    out0 = _printed(capsys)
    agent, tasks1 = _tsf_setup(E, ep_len, eps, total)
    R1 = [test_tasks_lockstep_tsf(agent, tasks1) for _ in range(phases)]
    assert random.getstate() == st0
    assert _printed(capsys) == out0
    assert R1 == R0
    assert agent.logger.lines == ref.logger.lines
    assert bool(agent.logger.lines) == (total % 5000 == 0)
    for (wa, oa, sa), (wb, ob, sb) in zip(agent.test_tasks_weights, ref.test_tasks_weights):
        assert torch.equal(wa.weight.detach(), wb.weight.detach())
        assert oa.param_groups[1]["lr"] == ob.param_groups[1]["lr"]
    for oa, ob in zip(agent.omegas, ref.omegas):
        assert torch.equal(oa.detach(), ob.detach())
    for (ka, va), (kb, vb) in zip(agent.sf._test_state.items(), ref.sf._test_state.items()):
        assert torch.equal(va[0], vb[0]) and va[1] == vb[1] == phases * ep_len
    assert agent.sf._eng.batched == phases * ep_len * 3 * ((E + 3) // 4)


def test_tsf_enable_binds_lockstep_into_train_loop():
    """enable() on a TSF agent (it has ``omegas``): the reference's per-task test_agent calls of
    train (agents/tsfdqn_sequential.py:361-364) return the lockstep returns, in order."""
    from sfx import lockstep

    ref, tasks0 = _tsf_setup(3, 5, 0.1)
    R0 = [ref.test_agent(t, i) for i, t in enumerate(tasks0)]
    agent, tasks1 = _tsf_setup(3, 5, 0.1)
    agent.train = lambda *a, **k: [agent.test_agent(t, i) for i, t in enumerate(k["test_tasks"])]
    lockstep.enable(agent)
    assert agent.train([], 0, test_tasks=tasks1) == R0


def test_tsf_lockstep_decides_up_front_for_episodes_that_end(capsys):
    """TSF test tasks whose episodes end early (Hopper / CartPole return gym's done): the lockstep
    entry point runs the sequential loop instead -- returns, w, ω, Adam state, LR schedules, log
    lines and random state as the reference's, and no lockstep launch."""
    from sfx.lockstep import test_tasks_lockstep_tsf

    at = [None, 3, None]
    ref, tasks0 = _tsf_setup(3, 6, 0.3, 5000)
    _ending(tasks0, at)
    R0 = [[ref.test_agent(t, i) for i, t in enumerate(tasks0)] for _ in range(2)]
    st0, out0 = random.getstate(), _printed(capsys)
    agent, tasks1 = _tsf_setup(3, 6, 0.3, 5000)
    _ending(tasks1, at)
    R1 = [test_tasks_lockstep_tsf(agent, tasks1) for _ in range(2)]
    assert R1 == R0 and random.getstate() == st0 and _printed(capsys) == out0
    assert agent.logger.lines == ref.logger.lines
    for (wa, oa, _), (wb, ob, _) in zip(agent.test_tasks_weights, ref.test_tasks_weights):
        assert torch.equal(wa.weight.detach(), wb.weight.detach())
        assert oa.param_groups[1]["lr"] == ob.param_groups[1]["lr"]
    for oa, ob in zip(agent.omegas, ref.omegas):
        assert torch.equal(oa.detach(), ob.detach())
    assert agent.sf._eng.batched == 0


def test_tsf_lockstep_declared_endless_task_that_ends_stops_there():
    """A TSF test task declared endless that ends anyway stops at its done (the reference's break:
    no further env step, Adam step or scheduler step for it) with a warning; with ε = 0 and no
    diagnostic draws every task still matches the sequential loop."""
    from sfx.lockstep import test_tasks_lockstep_tsf

    at = [2, None, None]
    ref, tasks0 = _tsf_setup(3, 5, 0.0, 7)
    _ending(tasks0, at)
    R0 = [ref.test_agent(t, i) for i, t in enumerate(tasks0)]
    agent, tasks1 = _tsf_setup(3, 5, 0.0, 7)
    _ending(tasks1, at)
    with pytest.warns(RuntimeWarning, match="declared never to end"):
        R1 = test_tasks_lockstep_tsf(agent, tasks1, episodes_end=False)
    assert R1 == R0 and tasks1[0]._n == 2
    for (wa, oa, _), (wb, ob, _) in zip(agent.test_tasks_weights, ref.test_tasks_weights):
        assert torch.equal(wa.weight.detach(), wb.weight.detach())
        assert oa.param_groups[1]["lr"] == ob.param_groups[1]["lr"]
    for oa, ob in zip(agent.omegas, ref.omegas):
        assert torch.equal(oa.detach(), ob.detach())


def test_tsf_test_state_survives_sf_reset():
    """the Adam state of each TSF test task's {w, ω} is keyed by the ω tensor object
    (weakly) and survives DeepTSF.reset() -- agent.reset() of a second trial; the reference keeps
    it in the agent's torch optimizers, which reset() never rebuilds."""
    from torch.utils.weak import WeakIdKeyDictionary

    from sfx.dropin.features.deep_sequential_tsf import DeepTSF
    from sfx.lockstep import test_tasks_lockstep_tsf

    agent, tasks = _tsf_setup(3, 4, 0.1)
    test_tasks_lockstep_tsf(agent, tasks)
    st = agent.sf._test_state
    assert isinstance(st, WeakIdKeyDictionary) and len(st) == 3
    assert all(st[o][1] == 4 for o in agent.omegas)

    def lam(n_in, n_out, shape, axis=1):
        m = torch.nn.Sequential(torch.nn.Linear(n_in, 8), torch.nn.Linear(8, n_out))
        return m, torch.nn.MSELoss(), torch.optim.Adam(m.parameters())

    sf = DeepTSF(lam)
    sf.reset()  # agent.reset() of the first trial
    om = torch.ones(1, 3, 1, 1)
    state = [torch.arange(4.0), 7]
    sf._test_state[om] = state
    sf.reset()
    assert sf._test_state.get(om) is state
    del om
    import gc
    gc.collect()
    assert len(sf._test_state) == 0  # weak: goes with the agent's tensor
