"""GPU parity of the native env-step runner (sfx_runner_*, pipelined graphs with gate kernels)
against the oracle replaying the runner's own recorded inputs.

Each recorded step holds what the host handed the device: the minibatch, the LMS transition
(φ, r) and the next state.  The oracle applies them in the reference's order (LMS,
agents/sfdqn.py:51; all-task update, :57-60; GPI action for the next state, :39-45) and must
reproduce the greedy action the runner recorded at the following step, the final heads,
the reward weights and the target nets.  Tolerances as in test_gpu_engine.py.
"""
import numpy as np
import pytest
import torch

from oracle import ref_cpu as R
from tests.conftest import gpu_available
from tests.test_gpu_engine import params_close, rel_close

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _need_gpu():
    if not gpu_available():
        pytest.skip("no HIP device")


def make(spec, T, ev, seed=0, max_batch=16):
    from sfx.engine import SFEngine
    from sfx.init import reference_heads

    online, w = reference_heads(T, spec.n_s, spec.H, spec.A, spec.d, spec.acts, seed=seed)
    eng = SFEngine(T, spec.n_s, spec.H, spec.A, spec.d, spec.acts, max_batch=max_batch)
    eng.set_adam(1e-3, 0.0, 1e-3, 0.0)
    eng.set_target_update_ev(ev)
    for t in range(T):
        eng.load_head(t, online[t], 0)
        eng.load_head(t, online[t], 1)
        eng.load_w(t, w[t])
    return eng, R.SFState(spec, online.clone(), online.clone(), w.clone())


def replay_with_oracle(st, spec, recs, alpha, ev, final_action):
    for k, rec in enumerate(recs):
        task = rec["task"]
        st.w[task] = R.lms_update(st.w[task].view(-1, 1), torch.from_numpy(rec["phi1"]), float(rec["r1"][0]),
                                  alpha).view(-1)
        if rec["have"]:
            batch = (torch.from_numpy(rec["s"]), torch.from_numpy(rec["a"]), torch.from_numpy(rec["phi"]),
                     torch.from_numpy(rec["s1"]), torch.from_numpy(rec["gamma"]))
            R.deep_all_task_step(st, batch, lr=1e-3, target_update_ev=ev)
        q, tk = R.gpi_w(R.psi_all(st.online, spec, torch.from_numpy(rec["snext"]).view(1, -1)), st.w[task])
        want = (int(tk[0]), R.select_action(q, tk[0], task, True))
        got = (recs[k + 1]["c"], recs[k + 1]["a_greedy"]) if k + 1 < len(recs) else final_action
        assert got == want, f"step {k}: runner selected {got}, oracle {want}"


def check_state(eng, st, T, k):
    params_close(torch.stack([eng.get_head(t, 0) for t in range(T)]), st.online, 1e-3 * k)
    params_close(torch.stack([eng.get_head(t, 1) for t in range(T)]), st.target, 1e-3 * k)
    rel_close(torch.stack([eng.get_w(t)[0] for t in range(T)]), st.w, rtol=1e-5, atol=1e-7)


@pytest.mark.parametrize("pipeline", [True, False])
def test_runner_matches_oracle(pipeline, monkeypatch):
    from sfx.runner import NativeEnvLoop

    if not pipeline:
        monkeypatch.setenv("SFX_RUNNER_PIPELINE", "0")
    spec = R.Spec(17, 32, 7, 8, ("relu", "relu"))
    T, ev, alpha, n = 3, 4, 0.05, 24
    eng, st = make(spec, T, ev)
    loop = NativeEnvLoop(eng, batch=16, capacity=200, gamma=0.9, epsilon=0.3, alpha_w=alpha, episode_len=7, seed=5)
    loop.prefill(10)  # first 5 env steps run without a minibatch (replay < batch)
    loop.set_task(1)
    first = loop.action()
    loop.record(n)
    loop.run(n)
    recs = loop.records()
    assert len(recs) == n and (recs[0]["c"], recs[0]["a_greedy"]) == first
    assert [r["have"] for r in recs[:6]] == [0, 0, 0, 0, 0, 1]
    replay_with_oracle(st, spec, recs, alpha, ev, loop.action())
    check_state(eng, st, T, n)
    stats = loop.stats()
    assert stats["env_steps"] == n
    if pipeline:
        assert stats["prelaunched"] > n // 2
    else:
        assert stats["prelaunched"] == 0
    counts = loop.gpi_counters()
    assert counts.sum() == n and counts[1].sum() == n
    loop.close()
    eng.close()


def test_runner_four_heads_wide_backward():
    """4 heads sharing each backward launch at 128-wide hidden layers (the geometry the removed
    64 x 64 dW tiles were built for): the 32 x 64 tiles give the oracle's results."""
    from sfx.runner import NativeEnvLoop

    spec = R.Spec(17, 128, 7, 8, ("relu", "relu"))
    T, ev, alpha, n = 4, 5, 0.05, 16
    eng, st = make(spec, T, ev)
    loop = NativeEnvLoop(eng, batch=16, capacity=100, gamma=0.9, epsilon=0.3, alpha_w=alpha, episode_len=7, seed=8)
    loop.prefill(16)
    loop.set_task(2)
    loop.record(n)
    loop.run(n)
    recs = loop.records()
    replay_with_oracle(st, spec, recs, alpha, ev, loop.action())
    check_state(eng, st, T, n)
    loop.close()
    eng.close()


@pytest.mark.parametrize("T,force", [(40, -1), (64, 1)], ids=["40-heads", "64-heads-host-rounds"])
def test_runner_many_heads_matches_oracle(T, force):
    """The all-task step over many heads (T·A > 256): next actions from k_tdgw, verification by
    k_verw (one workgroup per (row, 8 policies), lane = head),
    3 device rounds by default, host rounds forced in the second case.  Every greedy action of the
    runner bit-exact to the oracle's in-order loop (agents/sfdqn.py:57-60), heads within the Adam
    tolerance."""
    from sfx.runner import NativeEnvLoop

    spec = R.Spec(17, 16, 7, 8, ("relu", "relu"))
    ev, alpha, n = 6, 0.05, 14
    eng, st = make(spec, T, ev)
    if force >= 0:
        eng.debug_force_rerun(force)
    loop = NativeEnvLoop(eng, batch=16, capacity=200, gamma=0.9, epsilon=0.3, alpha_w=alpha, episode_len=7, seed=6)
    loop.prefill(20)
    loop.set_task(T - 3)
    loop.record(n)
    loop.run(n)
    recs = loop.records()
    replay_with_oracle(st, spec, recs, alpha, ev, loop.action())
    check_state(eng, st, T, n)
    sk = eng.skip_stats()
    assert sk["policies_checked"] > 0 and sk["policies_skipped"] > 0, sk
    if force >= 0:
        assert loop.stats()["host_round_steps"] >= n // 2
    loop.close()
    eng.close()


def test_runner_with_python_env_callbacks():
    """A host env passed as callbacks (tasks/task.py interface) drives the same loop."""
    from sfx.runner import NativeEnvLoop

    class CountingEnv:
        def __init__(self, n_s, d):
            self.n_s, self.d, self.t, self.actions = n_s, d, 0, []

        def reset(self, task):
            return np.full(self.n_s, 0.1 * task, np.float32)

        def step(self, task, a):
            self.t += 1
            self.actions.append(a)
            s1 = np.linspace(-1, 1, self.n_s).astype(np.float32) * np.float32(self.t % 5)
            phi = np.full(self.d, 0.01 * (self.t % 7), np.float32)
            return s1, phi, float(phi.sum()), self.t % 9 == 0

    spec = R.Spec(6, 16, 3, 4, ("relu", "relu"))
    T, ev, alpha, n = 2, 1000, 0.02, 14
    eng, st = make(spec, T, ev, max_batch=8)
    env = CountingEnv(spec.n_s, spec.d)
    loop = NativeEnvLoop(eng, batch=8, capacity=64, gamma=0.95, epsilon=0.0, alpha_w=alpha, episode_len=100, seed=3,
                         env=env)
    loop.prefill(8)
    loop.set_task(0)
    env.actions.clear()
    loop.record(n)
    loop.run(n)
    recs = loop.records()
    assert [r["a_taken"] for r in recs] == env.actions  # ε = 0: the greedy actions went to the env
    assert [r["terminal"] for r in recs] == [int((8 + i + 1) % 9 == 0) for i in range(n)]
    for r in recs:
        if r["have"]:
            assert set(np.unique(r["gamma"])) <= {np.float32(0.95), np.float32(0.0)}
    replay_with_oracle(st, spec, recs, alpha, ev, loop.action())
    check_state(eng, st, T, n)
    loop.close()
    eng.close()


@pytest.mark.parametrize("schedule,upd_use_gpi", [("active", True), ("active", False), ("tsf", True)])
def test_runner_active_schedules_match_oracle(schedule, upd_use_gpi):
    """Native runner with the active-task schedules: sfdqn.py / agents/sfdqn_sequential.py (one
    head per env step, l1 + l2 with an Adam-trained w) and TSF-DQN (tsfdqn.py).  The oracle
    replays the recorded minibatches (with their rewards) in order and must reproduce every
    recorded greedy action and the final heads / w / g_i / h.  Episodes end at random
    (p_end) so γ = 0 transitions enter the minibatches."""
    from sfx.runner import NativeEnvLoop

    spec = R.Spec(11, 32, 5, 6, ("relu", "relu"))
    T, ev, n, task = 3, 5, 30, 2
    eng, st = make(spec, T, ev)
    if schedule == "tsf":
        K, G = 2, 12
        gs = R.GSpec(spec.n_s, G, K)
        gen = torch.Generator().manual_seed(4)
        g = torch.empty(T, gs.P).uniform_(-0.3, 0.3, generator=gen)
        h = torch.empty(spec.d * G + spec.d).uniform_(-0.2, 0.2, generator=gen)
        eng.tsf_setup(G, K, 1.0, 1e-3, 0.0, 1e-3, 0.0)
        for t in range(T):
            eng.tsf_load_g(t, g[t])
        eng.tsf_load_h(h)
        st = R.TSFState(spec, st.online, st.target, st.w, gspec=gs, g=g.clone(), h=h.clone())
    loop = NativeEnvLoop(eng, batch=16, capacity=200, gamma=0.9, epsilon=0.3, episode_len=11, seed=9,
                         schedule=schedule, upd_use_gpi=upd_use_gpi, p_end=0.1)
    loop.prefill(10)
    loop.set_task(task)
    first = loop.action()
    loop.record(n)
    loop.run(n)
    recs = loop.records()
    assert len(recs) == n and (recs[0]["c"], recs[0]["a_greedy"]) == first
    assert any(r["terminal"] for r in recs)
    for k, rec in enumerate(recs):
        assert rec["task"] == task
        if rec["have"]:
            batch = (torch.from_numpy(rec["s"]), torch.from_numpy(rec["a"]), torch.from_numpy(rec["rb"]).view(-1, 1),
                     torch.from_numpy(rec["phi"]), torch.from_numpy(rec["s1"]), torch.from_numpy(rec["gamma"]))
            if schedule == "tsf":
                R.tsf_update(st, batch, task, use_gpi=upd_use_gpi, target_update_ev=ev)
            else:
                R.sf_update(st, batch, task, use_gpi=upd_use_gpi, target_update_ev=ev)
        q, tk = R.gpi_w(R.psi_all(st.online, spec, torch.from_numpy(rec["snext"]).view(1, -1)), st.w[task])
        want = (int(tk[0]), R.select_action(q, tk[0], task, True))
        got = (recs[k + 1]["c"], recs[k + 1]["a_greedy"]) if k + 1 < len(recs) else loop.action()
        assert got == want, f"step {k}: runner selected {got}, oracle {want}"
    params_close(torch.stack([eng.get_head(t, 0) for t in range(T)]), st.online, 1e-3 * n)
    params_close(torch.stack([eng.get_head(t, 1) for t in range(T)]), st.target, 1e-3 * n)
    rel_close(torch.stack([eng.get_w(t)[0] for t in range(T)]), st.w, rtol=1e-4, atol=1e-7)
    if schedule == "tsf":
        params_close(torch.stack([eng.tsf_get_g(t)[0] for t in range(T)]), st.g, 1e-3 * n)
        params_close(eng.tsf_get_h(), st.h, 1e-3 * n)
    assert loop.stats()["prelaunched"] > n // 2
    loop.close()
    eng.close()


@pytest.mark.parametrize("schedule,force", [("all", -1), ("all", 1), ("active", -1)])
def test_runner_gate_timeouts_cancel_and_retry(schedule, force):
    """A gate bound of 10 ns: every pre-launched step's gate gives up before the host releases
    it, so the step is cancelled (none of its launches commits -- parameters, moments, step
    counters, w) and re-issued from the same staged inputs.  The results must still be the
    oracle's, step for step.  force = 1: every step also finishes with host rounds on the side
    stream -- after the next step's gate gave up (10 ns) and its cancelled launches ran over the
    transient buffers those rounds read (activations, speculative next actions): the runner
    drains them and recomputes the step's forward and device rounds before its host rounds."""
    from sfx.runner import NativeEnvLoop

    spec = R.Spec(17, 32, 7, 8, ("relu", "relu"))
    T, ev, alpha, n = 3, 1000, 0.05, 20
    eng, st = make(spec, T, ev)
    if force >= 0:
        eng.debug_force_rerun(force)
    loop = NativeEnvLoop(eng, batch=16, capacity=200, gamma=0.9, epsilon=0.3, alpha_w=alpha, episode_len=7, seed=5,
                         schedule=schedule)
    loop.prefill(16)
    loop.set_task(1)
    loop.set_gate_timeout(1e-8)
    # a gate gives up when it starts before the host's release: steps pre-launched inside one graph
    # do, a graph's first step races the host -- run until some step was cancelled (bounded)
    loop.record(4 * n)
    for _ in range(4):
        loop.run(n)
        stats = loop.stats()
        if stats["retried"] > 0 and (force < 0 or stats["recomputed"] > 0):
            break
    assert stats["retried"] > 0 and stats["prelaunched"] > 0, stats
    n = stats["env_steps"]
    if force >= 0:  # every step's host rounds found the next steps cancelled: recomputed first
        assert stats["recomputed"] > 0, stats
    recs = loop.records()
    if schedule == "all":
        replay_with_oracle(st, spec, recs, alpha, ev, loop.action())
        check_state(eng, st, T, n)
    else:
        for rec in recs:
            batch = (torch.from_numpy(rec["s"]), torch.from_numpy(rec["a"]), torch.from_numpy(rec["rb"]).view(-1, 1),
                     torch.from_numpy(rec["phi"]), torch.from_numpy(rec["s1"]), torch.from_numpy(rec["gamma"]))
            R.sf_update(st, batch, 1, use_gpi=True, target_update_ev=ev)
        params_close(torch.stack([eng.get_head(t, 0) for t in range(T)]), st.online, 1e-3 * n)
        rel_close(torch.stack([eng.get_w(t)[0] for t in range(T)]), st.w, rtol=1e-4, atol=1e-7)
    # the default bound again: pre-launched steps run without being re-issued
    loop.set_gate_timeout(5.0)
    before = loop.stats()["retried"]
    loop.run(8)
    assert loop.stats()["retried"] == before
    loop.close()
    eng.close()


def test_runner_env_error_cancels_queue():
    """The env callback raises in the middle of a run while later steps are already queued on
    the device (8-step graphs): the run fails, the queued steps are cancelled at their gates, the
    heads hold the last completed step, and the runner continues afterwards -- the whole recorded
    sequence still replays through the oracle step for step."""
    from sfx._lib import SFXError
    from sfx.runner import NativeEnvLoop

    class FlakyEnv:
        def __init__(self, n_s, d, fail_at):
            self.n_s, self.d, self.t, self.fail_at = n_s, d, 0, fail_at

        def reset(self, task):
            return np.full(self.n_s, 0.2 + 0.1 * task, np.float32)

        def step(self, task, a):
            self.t += 1
            if self.t == self.fail_at:
                raise RuntimeError("env failure")
            s1 = np.cos(np.arange(self.n_s, dtype=np.float32) * 0.3 * (self.t % 11)).astype(np.float32)
            phi = ((np.arange(self.d) + self.t) % 5).astype(np.float32) * 0.1
            return s1, phi, float(phi[task % self.d]), False

    spec = R.Spec(17, 32, 7, 8, ("relu", "relu"))
    T, ev, alpha = 3, 1000, 0.05
    eng, st = make(spec, T, ev)
    env = FlakyEnv(spec.n_s, spec.d, fail_at=14 + 12)  # 14 prefill calls, then the 12th env step fails
    loop = NativeEnvLoop(eng, batch=8, capacity=100, gamma=0.9, epsilon=0.2, alpha_w=alpha, episode_len=50, seed=2,
                         env=env)
    loop.prefill(14)
    loop.set_task(2)
    loop.record(40)
    with pytest.raises(SFXError):
        loop.run(20)
    recs = loop.records()
    assert len(recs) == 11
    st_mid = R.SFState(spec, st.online.clone(), st.target.clone(), st.w.clone())
    for k, rec in enumerate(recs):  # the heads after the failure: exactly the 11 completed steps
        st_mid.w[2] = R.lms_update(st_mid.w[2].view(-1, 1), torch.from_numpy(rec["phi1"]), float(rec["r1"][0]),
                                   alpha).view(-1)
        batch = (torch.from_numpy(rec["s"]), torch.from_numpy(rec["a"]), torch.from_numpy(rec["phi"]),
                 torch.from_numpy(rec["s1"]), torch.from_numpy(rec["gamma"]))
        R.deep_all_task_step(st_mid, batch, lr=1e-3, target_update_ev=ev)
    check_state(eng, st_mid, T, len(recs))
    loop.run(10)
    recs = loop.records()
    assert len(recs) == 21
    replay_with_oracle(st, spec, recs, alpha, ev, loop.action())
    check_state(eng, st, T, len(recs))
    loop.close()
    eng.close()


def test_runner_forced_host_rounds_with_spans():
    """sfx_debug_force_rerun on the native runner: every step's device rounds are treated as
    failed from policy 1 on, so each step finishes with host rounds on the side stream while the
    next 8-step graph waits at its gate -- with target syncs every 3 updates.  Same results."""
    from sfx.runner import NativeEnvLoop

    spec = R.Spec(17, 32, 7, 8, ("relu", "relu"))
    T, ev, alpha, n = 4, 3, 0.05, 24
    eng, st = make(spec, T, ev)
    eng.debug_force_rerun(1)
    loop = NativeEnvLoop(eng, batch=8, capacity=100, gamma=0.9, epsilon=0.3, alpha_w=alpha, episode_len=9, seed=7)
    loop.prefill(8)
    loop.set_task(0)
    loop.record(n)
    loop.run(n)
    stats = loop.stats()
    assert stats["host_round_steps"] == n and stats["prelaunched"] > 0, stats
    replay_with_oracle(st, spec, recs := loop.records(), alpha, ev, loop.action())
    assert len(recs) == n
    check_state(eng, st, T, n)
    loop.close()
    eng.close()


def test_runner_gpi_counters_follow_use_gpi():
    """SF.GPI(update_counters=use_gpi) (agents/sfdqn.py:41): without GPI action selection the
    counters stay at zero."""
    from sfx.runner import NativeEnvLoop

    spec = R.Spec(17, 32, 7, 8, ("relu", "relu"))
    eng, _ = make(spec, 2, 1000)
    loop = NativeEnvLoop(eng, batch=8, capacity=100, use_gpi=False, seed=3)
    loop.prefill(8)
    loop.set_task(1)
    loop.run(6)
    assert loop.gpi_counters().sum() == 0
    loop.close()
    eng.close()


@pytest.mark.parametrize("schedule", ["all", "active"])
def test_runner_c1_cartpole_shape(schedule):
    """BASELINE config C1 at its stated shape: CartPole-v2 SF-DQN, n_s=4, A=2, d=20
    (configs/cartpole_phi.cfg:52), 2 source tasks, 256-wide heads, minibatch 32 -- the all-task
    schedule (main_sfdqn_torch.py) and the active-task one (sfdqn.py), against the oracle."""
    from sfx.runner import NativeEnvLoop

    spec = R.Spec(4, 256, 2, 20, ("relu", "relu"))
    T, ev, alpha, n = 2, 7, 0.05, 24
    eng, st = make(spec, T, ev, max_batch=32)
    loop = NativeEnvLoop(eng, batch=32, capacity=300, gamma=0.9, epsilon=0.2, alpha_w=alpha, episode_len=9, seed=4,
                         schedule=schedule, p_end=0.05)
    loop.prefill(30)
    loop.set_task(1)
    loop.record(n)
    loop.run(n)
    recs = loop.records()
    if schedule == "all":
        replay_with_oracle(st, spec, recs, alpha, ev, loop.action())
        check_state(eng, st, T, n)
    else:
        for k, rec in enumerate(recs):
            if rec["have"]:
                batch = (torch.from_numpy(rec["s"]), torch.from_numpy(rec["a"]),
                         torch.from_numpy(rec["rb"]).view(-1, 1), torch.from_numpy(rec["phi"]),
                         torch.from_numpy(rec["s1"]), torch.from_numpy(rec["gamma"]))
                R.sf_update(st, batch, 1, use_gpi=True, target_update_ev=ev)
            q, tk = R.gpi_w(R.psi_all(st.online, spec, torch.from_numpy(rec["snext"]).view(1, -1)), st.w[1])
            want = (int(tk[0]), R.select_action(q, tk[0], 1, True))
            got = (recs[k + 1]["c"], recs[k + 1]["a_greedy"]) if k + 1 < len(recs) else loop.action()
            assert got == want, f"step {k}: runner selected {got}, oracle {want}"
        params_close(torch.stack([eng.get_head(t, 0) for t in range(T)]), st.online, 1e-3 * n)
        params_close(torch.stack([eng.get_head(t, 1) for t in range(T)]), st.target, 1e-3 * n)
        rel_close(torch.stack([eng.get_w(t)[0] for t in range(T)]), st.w, rtol=1e-4, atol=1e-7)
    loop.close()
    eng.close()


def test_runner_host_rounds_with_every_queue_shared():
    """Host rounds run on the runner's side stream while the next pre-launched step spins at its
    gate on the handle's stream.  With more streams alive than hardware queues
    (GPU_MAX_HW_QUEUES) the runtime hands new streams existing queues; the runner must not pick
    a side stream on the gate's queue (the rounds would wait behind the gate until it times out,
    which cancelled bench.py's sharded run after the all-task run).  12 extra streams first, then
    the forced-host-round runner of the test above."""
    import ctypes

    from sfx.runner import NativeEnvLoop

    hip = ctypes.CDLL("libamdhip64.so")
    extra = []
    for _ in range(12):
        s = ctypes.c_void_p()
        assert hip.hipStreamCreateWithFlags(ctypes.byref(s), 1) == 0
        extra.append(s)
    try:
        spec = R.Spec(17, 32, 7, 8, ("relu", "relu"))
        T, ev, alpha, n = 4, 5, 0.05, 20
        for rep in range(3):  # a fresh runner (and side stream) each time
            eng, st = make(spec, T, ev, seed=rep)
            eng.debug_force_rerun(2)
            loop = NativeEnvLoop(eng, batch=8, capacity=100, gamma=0.9, epsilon=0.3, alpha_w=alpha, episode_len=9,
                                 seed=11 + rep)
            loop.prefill(8)
            loop.set_task(rep % T)
            loop.record(n)
            loop.run(n)
            stats = loop.stats()
            assert stats["host_round_steps"] == n and stats["retried"] == 0, stats
            replay_with_oracle(st, spec, recs := loop.records(), alpha, ev, loop.action())
            check_state(eng, st, T, len(recs))
            loop.close()
            eng.close()
            s = ctypes.c_void_p()  # and one more stream in between
            assert hip.hipStreamCreateWithFlags(ctypes.byref(s), 1) == 0
            extra.append(s)
    finally:
        torch.cuda.synchronize()
        for s in extra:
            hip.hipStreamDestroy(s)


@pytest.mark.parametrize("spec_rounds,force,T", [(2, -1, 6), (2, 1, 6), (3, -1, 6), (0, -1, 40), (0, 2, 40)],
                         ids=["r2", "r2-host-rounds", "r3", "wide-auto", "wide-auto-host-rounds"])
def test_round_skip_is_bit_exact(spec_rounds, force, T, monkeypatch):
    """Speculative rounds r >= 1 skip the backward and Adam of a policy whose next actions repeat
    round r-1's (BwdArgs::skip).  The skipped update would have repeated round r-1's bit for bit,
    so the heads, the moments and every action must be IDENTICAL with skipping off (SFX_SKIP=0)
    -- including steps finished by host rounds (force) -- and the device counters must show
    skipped policies.  T = 40 (T·A > 256): the unfused TD launch (k_tdgw) decides the skips by
    per-policy arrivals, 3 device rounds (the automatic count from 16 source tasks on)."""
    from sfx.runner import NativeEnvLoop

    spec = R.Spec(17, 64 if T < 16 else 16, 7, 8, ("relu", "relu"))
    ev, n = 9, 30
    out = {}
    for skip in ("1", "0"):
        monkeypatch.setenv("SFX_SKIP", skip)
        eng, _ = make(spec, T, ev, max_batch=32)
        eng.set_spec_rounds(spec_rounds)
        if force >= 0:
            eng.debug_force_rerun(force)
        loop = NativeEnvLoop(eng, batch=32, capacity=300, gamma=0.9, epsilon=0.2, alpha_w=0.05, episode_len=11, seed=9)
        loop.prefill(40)
        loop.set_task(2)
        loop.record(n)
        loop.run(n)
        recs = loop.records()
        heads = torch.stack([eng.get_head(t, 0) for t in range(T)])
        moms = [eng.get_adam(t) for t in range(T)]
        out[skip] = (heads, moms, [(r["c"], r["a_greedy"]) for r in recs], loop.action(), eng.skip_stats())
        loop.close()
        eng.close()
    h1, m1, a1, f1, s1 = out["1"]
    h0, m0, a0, f0, s0 = out["0"]
    assert a1 == a0 and f1 == f0
    assert torch.equal(h1, h0)
    for (ma, va, sa), (mb, vb, sb) in zip(m1, m0):
        assert torch.equal(ma, mb) and torch.equal(va, vb) and sa == sb
    assert s0["policies_checked"] == 0
    rounds = spec_rounds or (3 if T >= 16 else 2)
    assert s1["policies_checked"] >= n * (rounds - 1) * T // 2 and s1["policies_skipped"] > 0, s1


@pytest.mark.parametrize("force,ev", [(-1, 7), (1, 1000), (2, 1000)])
def test_lookahead_is_bit_exact(force, ev, monkeypatch):
    """Look-ahead: step E's final round forwards step E+1's minibatch into the other
    copy of the minibatch roles and step E+1 starts at its TD launch.  The forward is the same
    arithmetic as the step-start forward, so heads, moments and every action must be IDENTICAL to
    SFX_AHEAD=0 on the same index stream -- through dirty minibatches (a small ring: the newest
    transition is sampled often), target syncs every 7 updates, and forced host rounds (which skip
    the heads whose actions repeat)."""
    from sfx.runner import NativeEnvLoop

    spec = R.Spec(17, 64, 7, 8, ("relu", "relu"))
    T, n = 5, 60
    out = {}
    for ahead in ("1", "0"):
        monkeypatch.setenv("SFX_AHEAD", ahead)
        eng, _ = make(spec, T, ev, max_batch=16)
        if force >= 0:
            eng.debug_force_rerun(force)
        loop = NativeEnvLoop(eng, batch=16, capacity=48, gamma=0.9, epsilon=0.2, alpha_w=0.05, episode_len=13, seed=4)
        loop.prefill(20)
        loop.set_task(1)
        loop.record(n)
        loop.run(n // 2)
        loop.run(n - n // 2)  # the chain continues across runs
        recs = loop.records()
        heads = torch.stack([eng.get_head(t, 0) for t in range(T)])
        targets = torch.stack([eng.get_head(t, 1) for t in range(T)])
        moms = [eng.get_adam(t) for t in range(T)]
        ws = torch.stack([eng.get_w(t)[0] for t in range(T)])
        out[ahead] = (heads, targets, moms, ws, [(r["c"], r["a_greedy"]) for r in recs], loop.action(), loop.stats())
        loop.close()
        eng.close()
    h1, t1, m1, w1, a1, f1, s1 = out["1"]
    h0, t0, m0, w0, a0, f0, s0 = out["0"]
    assert a1 == a0 and f1 == f0
    assert torch.equal(h1, h0) and torch.equal(t1, t0) and torch.equal(w1, w0)
    for (ma, va, sa), (mb, vb, sb) in zip(m1, m0):
        assert torch.equal(ma, mb) and torch.equal(va, vb) and sa == sb
    assert s0["ahead_pre_steps"] == 0
    assert s1["ahead_pre_steps"] > n // 2, s1
    assert s1["ahead_own_forward_steps"] > 0, s1  # dirty minibatches (and syncs) ran their own forward


@pytest.mark.parametrize("between", ["load_head", "sync_target", "update_all", "gpi"])
def test_lookahead_chain_dropped_by_calls_between_runs(between, monkeypatch):
    """The look-ahead chain (the last step of a run forwarded the next step's minibatch) must not
    survive a call on the handle between two runs that writes parameters or the minibatch roles
    (sfx_handle::gen).  Each call here changes what the next step's forward would see;
    heads, moments and every action must stay IDENTICAL to SFX_AHEAD=0 with the same calls."""
    from sfx.runner import NativeEnvLoop

    spec = R.Spec(17, 64, 7, 8, ("relu", "relu"))
    T, n = 4, 24
    out = {}
    for ahead in ("1", "0"):
        monkeypatch.setenv("SFX_AHEAD", ahead)
        eng, _ = make(spec, T, 1000, max_batch=16)
        loop = NativeEnvLoop(eng, batch=16, capacity=400, gamma=0.9, epsilon=0.2, alpha_w=0.05, episode_len=50, seed=4)
        loop.prefill(200)
        loop.set_task(1)
        loop.record(2 * n)
        loop.run(n)
        gen = torch.Generator().manual_seed(11)
        if between == "load_head":
            h = eng.get_head(2, 0)
            eng.load_head(2, h + 1e-2 * torch.randn(h.shape, generator=gen), 0)
        elif between == "sync_target":
            eng.sync_target(1)
        elif between == "update_all":
            B = 16
            s, s1 = torch.randn(B, spec.n_s, generator=gen), torch.randn(B, spec.n_s, generator=gen)
            a = torch.randint(0, spec.A, (B,), generator=gen)
            phi = torch.rand(B, spec.d, generator=gen)
            eng.update_all(s.cuda(), a.cuda(), phi.cuda(), s1.cuda(), torch.full((B,), 0.9).cuda())
        else:  # a GPI over other states (forwards into the handle's activation roles)
            eng.gpi(torch.randn(16, spec.n_s, generator=gen).cuda())
        eng.synchronize()
        loop.run(n)
        recs = loop.records()
        heads = torch.stack([eng.get_head(t, 0) for t in range(T)])
        moms = [eng.get_adam(t) for t in range(T)]
        out[ahead] = (heads, moms, [(r["c"], r["a_greedy"]) for r in recs], loop.action(), loop.stats())
        loop.close()
        eng.close()
    h1, m1, a1, f1, s1 = out["1"]
    h0, m0, a0, f0, s0 = out["0"]
    assert a1 == a0 and f1 == f0
    assert torch.equal(h1, h0)
    for (ma, va, sa), (mb, vb, sb) in zip(m1, m0):
        assert torch.equal(ma, mb) and torch.equal(va, vb) and sa == sb
    assert s1["ahead_pre_steps"] > n, s1


@pytest.mark.parametrize("schedule,upd_use_gpi,ev", [("active", True, 7), ("active", False, 1000), ("tsf", True, 7),
                                                     ("tsf", False, 1000)])
def test_active_lookahead_is_bit_exact(schedule, upd_use_gpi, ev, monkeypatch):
    """Look-ahead of the active-task / TSF schedules (select_ahead_body): step E's
    select also forwards step E+1's minibatch (ψ(S1) of every head, ψ(S) and ψ⁻(S1) of the active
    head; TSF: its φ̃ and flow states) and step E+1 starts at its TD target.  Same arithmetic as the
    step-start forward, so heads, targets, moments, w (TSF: g_i, h) and every action must be
    IDENTICAL to SFX_AHEAD=0 on the same index stream -- through dirty minibatches (a small ring),
    target syncs every 7 updates and episode ends."""
    from sfx.runner import NativeEnvLoop

    spec = R.Spec(11, 48, 5, 6, ("relu", "relu"))
    T, n, task = 3, 50, 1
    out = {}
    for ahead in ("1", "0"):
        monkeypatch.setenv("SFX_AHEAD", ahead)
        eng, _ = make(spec, T, ev)
        if schedule == "tsf":
            K, G = 3, 12
            gs = R.GSpec(spec.n_s, G, K)
            gen = torch.Generator().manual_seed(4)
            g = torch.empty(T, gs.P).uniform_(-0.3, 0.3, generator=gen)
            h = torch.empty(spec.d * G + spec.d).uniform_(-0.2, 0.2, generator=gen)
            eng.tsf_setup(G, K, 1.0, 1e-3, 0.0, 1e-3, 0.0)
            for t in range(T):
                eng.tsf_load_g(t, g[t])
            eng.tsf_load_h(h)
        loop = NativeEnvLoop(eng, batch=16, capacity=40, gamma=0.9, epsilon=0.3, episode_len=11, seed=5,
                             schedule=schedule, upd_use_gpi=upd_use_gpi, p_end=0.1)
        loop.prefill(20)
        loop.set_task(task)
        loop.record(n)
        loop.run(n // 2)
        loop.run(n - n // 2)
        recs = loop.records()
        res = [torch.stack([eng.get_head(t, 0) for t in range(T)]), torch.stack([eng.get_head(t, 1) for t in range(T)]),
               torch.stack([eng.get_w(t)[0] for t in range(T)])]
        for t in range(T):
            m, v, st = eng.get_adam(t)
            res += [m, v, torch.tensor(st)]
        if schedule == "tsf":
            res += [torch.stack([eng.tsf_get_g(t)[0] for t in range(T)]), eng.tsf_get_h()]
        out[ahead] = (res, [(r["c"], r["a_greedy"]) for r in recs], loop.action(), loop.stats())
        loop.close()
        eng.close()
    (r1, a1, f1, s1), (r0, a0, f0, s0) = out["1"], out["0"]
    assert a1 == a0 and f1 == f0
    for x, y in zip(r1, r0):
        assert torch.equal(x, y)
    assert s0["ahead_pre_steps"] == 0
    assert s1["ahead_pre_steps"] > n // 2, s1
    assert s1["ahead_own_forward_steps"] > 0, s1


def test_tsf_lookahead_full_shape_is_bit_exact(monkeypatch):
    """The TSF look-ahead at the Hopper shape (T = 16, H = 256, A = 27, d = 50, G = 100, B = 32): the
    select's first forward then has 544 column tiles and the TSF forward riding along, so it runs
    with three column tiles per workgroup (one workgroup per CU there) -- heads, g_i, h, w and every
    action identical to SFX_AHEAD=0, whose step-start forward runs one tile per workgroup."""
    from sfx.runner import NativeEnvLoop

    spec = R.Spec(11, 256, 27, 50, ("relu", "relu"))
    T, n, task, K, G = 16, 8, 3, 4, 100
    out = {}
    for ahead in ("1", "0"):
        monkeypatch.setenv("SFX_AHEAD", ahead)
        eng, _ = make(spec, T, 1000, max_batch=32)
        gs = R.GSpec(spec.n_s, G, K)
        gen = torch.Generator().manual_seed(6)
        g = torch.empty(T, gs.P).uniform_(-0.1, 0.1, generator=gen)
        h = torch.empty(spec.d * G + spec.d).uniform_(-0.05, 0.05, generator=gen)
        eng.tsf_setup(G, K, 1.0, 1e-3, 0.0, 1e-3, 0.0)
        for t in range(T):
            eng.tsf_load_g(t, g[t])
        eng.tsf_load_h(h)
        loop = NativeEnvLoop(eng, batch=32, capacity=200, gamma=0.9, epsilon=0.3, episode_len=50, seed=7,
                             schedule="tsf", upd_use_gpi=True)
        loop.prefill(40)
        loop.set_task(task)
        loop.record(n)
        loop.run(n)
        recs = loop.records()
        res = [torch.stack([eng.get_head(t, 0) for t in range(T)]), torch.stack([eng.get_w(t)[0] for t in range(T)]),
               torch.stack([eng.tsf_get_g(t)[0] for t in range(T)]), eng.tsf_get_h()]
        out[ahead] = (res, [(r["c"], r["a_greedy"]) for r in recs], loop.stats())
        loop.close()
        eng.close()
    (r1, a1, s1), (r0, a0, s0) = out["1"], out["0"]
    assert a1 == a0
    for x, y in zip(r1, r0):
        assert torch.equal(x, y)
    assert s1["ahead_pre_steps"] > 0 and s0["ahead_pre_steps"] == 0


def test_lookahead_runner_matches_oracle_c2():
    """The C2 shape (T = 8, H = 256, B = 32) with look-ahead on (the bench's configuration),
    replayed through the oracle from the runner's recorded inputs."""
    from sfx.runner import NativeEnvLoop

    spec = R.Spec(17, 256, 7, 8, ("relu", "relu"))
    T, ev, alpha, n = 8, 1000, 1e-3, 24
    eng, st = make(spec, T, ev, max_batch=32)
    loop = NativeEnvLoop(eng, batch=32, capacity=400, gamma=0.9, epsilon=0.1, alpha_w=alpha, episode_len=500, seed=1)
    loop.prefill(100)
    loop.set_task(0)
    loop.record(n)
    loop.run(n)
    recs = loop.records()
    replay_with_oracle(st, spec, recs, alpha, ev, loop.action())
    check_state(eng, st, T, n)
    assert loop.stats()["ahead_pre_steps"] > n // 2
    loop.close()
    eng.close()
