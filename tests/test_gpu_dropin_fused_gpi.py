"""The agent loop's next GPI fused into the all-task update (sfx_update_all_select; the drop-in's
DeepSF uses it when the minibatch came from sfx's agents.buffer, whose last append names the state
the agent asks GPI about next -- agents/agent.py:223-245).

Bar: bit-exact.  The fused selection must return what update_all followed by gpi(s_next) returns
(q, task) and leave the heads exactly as update_all does, with and without host rounds; the
drop-in loop must take the same actions and end with the same heads with the fusion on and off."""
import numpy as np
import pytest
import torch

from tests.conftest import gpu_available

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _need_gpu():
    if not gpu_available():
        pytest.skip("no HIP device")


def _pair(T, n_s, H, A, d, B, seed):
    from sfx.engine import SFEngine

    g = torch.Generator().manual_seed(seed)
    engs = [SFEngine(T, n_s, H, A, d, ("relu", "relu"), max_batch=B) for _ in range(2)]
    P = engs[0].P
    for t in range(T):
        on = torch.randn(P, generator=g) * 0.05
        tg = torch.randn(P, generator=g) * 0.05
        w = torch.randn(d, generator=g)
        for e in engs:
            e.load_head(t, on, 0)
            e.load_head(t, tg, 1)
            e.load_w(t, w)
    return engs, g


@pytest.mark.parametrize("slot", [False, True])
@pytest.mark.parametrize("force", [-1, 3])
@pytest.mark.parametrize("geom", [(8, 17, 256, 7, 8, 32), (4, 11, 64, 5, 6, 16)])
def test_update_all_select_matches_update_all_then_gpi(geom, force, slot):
    """With slot: the state through the engine's persistent selection input and an LMS of w[1]
    fused in (against sfx_lms_value before the update)."""
    T, n_s, H, A, d, B = geom
    (e1, e2), g = _pair(T, n_s, H, A, d, B, seed=7 + T)
    dev = e1.device
    for e in (e1, e2):
        if force >= 0:
            e.debug_force_rerun(force)  # every step takes host rounds from this policy on
    # one minibatch allocation refilled every step (the drop-in's buffer slots): fixed pointers
    s, s1 = torch.empty(B, n_s, device=dev), torch.empty(B, n_s, device=dev)
    a, phi = torch.empty(B, dtype=torch.long, device=dev), torch.empty(B, d, device=dev)
    gam, s_next = torch.full((B,), 0.9, device=dev), torch.empty(n_s, device=dev)
    lb = torch.empty(T, 3, device=dev)
    lphi = torch.empty(d, device=dev)
    for step in range(4):
        s.copy_(torch.randn(B, n_s, generator=g))
        s1.copy_(torch.randn(B, n_s, generator=g))
        a.copy_(torch.randint(0, A, (B,), generator=g))
        phi.copy_(torch.randn(B, d, generator=g))
        s_next.copy_(torch.randn(n_s, generator=g))
        lphi.copy_(torch.rand(d, generator=g))
        r = float(torch.randn((), generator=g))
        task = 1 if slot else step % T  # (the task index is part of the step's graph key)
        if slot:  # the state through the engine's persistent selection input, the LMS fused in
            e1._select_slots()[0].copy_(s_next)
            e1.lms_phi.copy_(lphi)
            rr = torch.tensor(r, device=dev) if step % 2 else r  # odd steps: the reward as a device scalar
            q1, c1 = e1.update_all_select(s, a, phi, s1, gam, task, losses=lb, lms_task=1, lms_r=rr, lms_alpha=0.05)
        else:
            q1, c1 = e1.update_all_select(s, a, phi, s1, gam, task, s_next=s_next, losses=lb)
        q1, c1, ch = e1.settle_select(q1, c1)
        if slot:
            e2.lms(1, lphi, r, 0.05)
        e2.update_all(s, a, phi, s1, gam)
        _, q2, c2, _ = e2.gpi(s_next.reshape(1, -1), w_index=task, task_shape=())
        torch.cuda.synchronize()
        assert q1.shape == q2.shape and c1.shape == c2.shape == ()
        assert torch.equal(q1, q2), (step, (q1 - q2).abs().max().item())
        assert int(c1) == int(c2) == ch  # the host's copy of the selection is the device's
        for t in range(T):
            assert torch.equal(e1.get_head(t, 0), e2.get_head(t, 0)), (step, t)
            assert torch.equal(e1.get_w(t)[0], e2.get_w(t)[0]), (step, t)
    st1, st2 = e1.step_stats(), e2.step_stats()
    assert st1 == st2
    if slot:  # one graph per parameter slot parity, not one per step (fresh outputs every step)
        assert e1.graph_stats()["captures"] <= 2
    if force >= 0:
        assert st1["host_round_steps"] == 4
    e1.close()
    e2.close()


def _run_loop(fuse, steps, monkeypatch, dev_reward=False):
    from sfx.dropin.features.deep import DeepSF
    from sfx.engine import SFEngine
    from tools import dropin_loop

    with monkeypatch.context() as m:
        if not fuse:
            m.setattr(DeepSF, "_next_state", lambda self, s: None)
        calls = {"select": 0, "lms": 0}
        real = SFEngine.update_all_select

        def count(self, *a, **k):
            calls["select"] += 1
            calls["lms"] += k.get("lms_task", -1) >= 0
            return real(self, *a, **k)

        m.setattr(SFEngine, "update_all_select", count)
        loop = dropin_loop.DropinLoop(buffer="reference", T=8, batch=32, seed=3)
        actions = []
        for task in loop.tasks:
            real_tr = task.transition

            def rec(a, on_device=True, _real=real_tr):
                actions.append(int(a))
                s1, phi, r, term = _real(a, on_device)
                if dev_reward:  # tasks/reacher.py:51 returns the reward as a device tensor
                    r = torch.tensor(r, dtype=torch.float32, device=loop.device)
                return s1, phi, r, term

            task.transition = rec
        loop.run(steps)
        loop.sf._flush()
        heads = torch.stack([loop.sf._eng.get_head(t, 0) for t in range(8)])
        w = torch.stack([loop.sf._eng.get_w(t)[0] for t in range(8)])
        counters = [np.asarray(c).tolist() for c in loop.sf.gpi_counters]
        loop.close()
    return actions, heads, w, counters, calls


@pytest.mark.parametrize("dev_reward", [False, True])
def test_dropin_loop_same_run_with_fused_gpi(monkeypatch, dev_reward):
    steps = 90  # 32 to fill the minibatch, then fused steps
    a0, h0, w0, c0, n0 = _run_loop(False, steps, monkeypatch, dev_reward)
    a1, h1, w1, c1, n1 = _run_loop(True, steps, monkeypatch, dev_reward)
    # fused: every step but the first (which names the buffer's copy targets), LMS included
    assert n0["select"] == 0 and n1["select"] >= steps - 33 and n1["lms"] == n1["select"], (n0, n1)
    assert a0 == a1
    assert torch.equal(h0, h1)
    assert torch.equal(w0, w1)
    assert c0 == c1


def test_fused_gpi_not_used_for_another_state_or_after_a_reward_update(monkeypatch):
    """A GPI on any other tensor (or the same one changed in place, or after update_reward changed
    w) takes the ordinary path."""
    from tools import dropin_loop

    loop = dropin_loop.DropinLoop(buffer="reference", T=4, batch=8, seed=5)
    loop.run(12)
    sf = loop.sf
    assert sf._pred is not None
    ns = sf._pred[0]()
    q_pred, c_pred = sf._pred[3], sf._pred[4]
    other = ns.clone()
    q, c = sf.GPI(other, loop.task)  # a different tensor: ordinary GPI (and the prediction dropped)
    assert sf._pred is None and q is not q_pred
    assert torch.equal(q, q_pred) and int(c) == int(c_pred)  # the same values, computed again
    loop.run(1)
    assert sf._pred is not None
    ns = sf._pred[0]()
    ns.mul_(1.0)  # an in-place write bumps the version
    q, _ = sf.GPI(ns, loop.task)
    assert q is not None and sf._pred is None
    loop.run(1)
    ns, q_pred = sf._pred[0](), sf._pred[3]
    sf.update_reward(torch.ones(sf.n_features, device=ns.device), 1.0, loop.task)
    q, _ = sf.GPI(ns, loop.task)
    assert q is not q_pred
    loop.close()


def test_buffer_copies_the_appended_next_state_and_features_with_the_replay():
    """sfx_replay_put_gather: the append's row written by the replay's launch (a minibatch row drawn
    at the new row reads the new transition), and its next state / φ copied to the consumer's
    vectors, with the tensors and versions recorded."""
    from sfx.dropin.agents.buffer import ReplayBuffer

    dev = torch.device("cuda", 0)
    n_s, d, B, cap = 5, 3, 16, 16  # a replay draws the newest row with probability 0.64
    buf = ReplayBuffer({}, n_samples=cap, n_batch=B)
    buf.device = dev
    mx, mr = torch.zeros(n_s, device=dev), torch.zeros(d, device=dev)
    buf.mirror, buf.mirror_reward = mx, mr
    gen = torch.Generator().manual_seed(9)
    rows = []
    for k in range(3 * cap):
        s, s1 = torch.randn(1, n_s, generator=gen).to(dev), torch.randn(1, n_s, generator=gen).to(dev)
        phi, a = torch.rand(d, generator=gen).to(dev), torch.tensor(k % 4, device=dev)
        buf.append(s, a, phi, s1, 0.9)
        rows = (rows + [(s, a, phi, s1)])[-cap:]
        if buf.size < B:
            assert buf.replay() is None
            continue
        state = np.random.get_state()
        got = buf.replay()
        np.random.set_state(state)
        idx = np.random.randint(low=0, high=buf.size, size=(B,))
        order = rows[cap - buf.index:] + rows[:cap - buf.index] if len(rows) == cap else rows
        assert torch.equal(got[0], torch.vstack([order[i][0] for i in idx]))
        assert torch.equal(got[1], torch.stack([order[i][1] for i in idx]))
        assert torch.equal(got[3], torch.vstack([order[i][3] for i in idx]))
        assert torch.equal(mx, s1.reshape(-1)) and torch.equal(mr, phi)
        assert buf.last_next[0]() is s1 and buf.last_reward[0]() is phi


def test_deferred_reward_fit_refuses_a_phi_written_in_place():
    """update_reward of a device φ runs with the next step (or the next call that reads w); a φ
    changed in place before then would be fitted on other values than the reference fits: it
    raises instead."""
    from tools import dropin_loop

    loop = dropin_loop.DropinLoop(buffer="reference", T=4, batch=8, seed=5)
    loop.run(10)
    sf = loop.sf
    phi = torch.rand(sf.n_features, device=loop.device)
    w0 = sf.fit_w[0].clone()
    sf.update_reward(phi, 0.5, 0)
    w1 = sf.fit_w[0]  # reading w runs the deferred fit
    assert not torch.equal(w0, w1)
    sf.update_reward(phi, 0.5, 0)
    phi.mul_(2.0)
    with pytest.raises(RuntimeError, match="modified in place"):
        sf.fit_w[0]
    loop.close()
