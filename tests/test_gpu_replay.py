"""GPU parity of the device-resident replay (sfx_runner_device_replay).

The ring lives in HBM and each step's gate kernel appends the step's transition and draws the
uniform minibatch on the device (k_gate_replay).  The host keeps a mirror of the ring and, when
recording, draws the same rows with the same index function, so the recorded minibatch is the
one the device gathered; the oracle replays the records and must reproduce every greedy action
and the final heads / w (/ g_i, h).  A wrong gather on the device (row, field or ring slot)
changes the update and fails the comparison.  Capacities below the number of appended
transitions make the ring wrap, so overwritten slots and the step's own slot are sampled.
"""
import pytest
import torch

from oracle import ref_cpu as R
from tests.conftest import gpu_available
from tests.test_gpu_engine import params_close, rel_close
from tests.test_gpu_runner import check_state, make, replay_with_oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _need_gpu():
    if not gpu_available():
        pytest.skip("no HIP device")


@pytest.mark.parametrize("capacity", [200, 20])
def test_device_replay_all_task(capacity):
    from sfx.runner import NativeEnvLoop

    spec = R.Spec(17, 32, 7, 8, ("relu", "relu"))
    T, ev, alpha, n = 3, 4, 0.05, 30
    eng, st = make(spec, T, ev)
    loop = NativeEnvLoop(eng, batch=16, capacity=capacity, gamma=0.9, epsilon=0.3, alpha_w=alpha, episode_len=7,
                         seed=5, device_replay=True)
    loop.prefill(10)
    loop.set_task(1)
    first = loop.action()
    loop.record(n)
    loop.run(n)
    recs = loop.records()
    assert len(recs) == n and (recs[0]["c"], recs[0]["a_greedy"]) == first
    assert [r["have"] for r in recs[:6]] == [0, 0, 0, 0, 0, 1]
    replay_with_oracle(st, spec, recs, alpha, ev, loop.action())
    check_state(eng, st, T, n)
    assert loop.stats()["prelaunched"] > n // 2
    loop.close()
    eng.close()


def test_device_replay_at_the_bench_batch():
    """B = 32 at the C2 state width (the bench's device-replay leg): the staging's look-ahead block
    (2 B n_s floats, host replay only) must not count against the device-replay gate's tail."""
    from sfx.runner import NativeEnvLoop

    spec = R.Spec(17, 32, 7, 8, ("relu", "relu"))
    T, ev, alpha, n = 3, 1000, 0.05, 12
    eng, st = make(spec, T, ev, max_batch=32)
    loop = NativeEnvLoop(eng, batch=32, capacity=100, gamma=0.9, epsilon=0.3, alpha_w=alpha, episode_len=9,
                         seed=6, device_replay=True)
    loop.prefill(40)
    loop.set_task(0)
    loop.record(n)
    loop.run(n)
    replay_with_oracle(st, spec, loop.records(), alpha, ev, loop.action())
    check_state(eng, st, T, n)
    loop.close()
    eng.close()


def test_device_replay_switch_between_runs():
    """Host-replay steps, then device-replay steps on the same ring (uploaded at the switch),
    then host again: one continuous oracle replay."""
    from sfx.runner import NativeEnvLoop

    spec = R.Spec(17, 32, 7, 8, ("relu", "relu"))
    T, ev, alpha = 2, 1000, 0.05
    eng, st = make(spec, T, ev)
    loop = NativeEnvLoop(eng, batch=16, capacity=40, gamma=0.9, epsilon=0.3, alpha_w=alpha, episode_len=9, seed=2)
    loop.prefill(20)
    loop.set_task(0)
    first = loop.action()
    loop.record(36)
    loop.run(12)
    loop.set_device_replay(True)
    loop.run(12)
    loop.set_device_replay(False)
    loop.run(12)
    recs = loop.records()
    assert len(recs) == 36 and (recs[0]["c"], recs[0]["a_greedy"]) == first
    replay_with_oracle(st, spec, recs, alpha, ev, loop.action())
    check_state(eng, st, T, 36)
    loop.close()
    eng.close()


@pytest.mark.parametrize("schedule", ["active", "tsf"])
def test_device_replay_active_schedules(schedule):
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
    loop = NativeEnvLoop(eng, batch=16, capacity=24, gamma=0.9, epsilon=0.3, episode_len=11, seed=9,
                         schedule=schedule, p_end=0.1, device_replay=True)
    loop.prefill(10)
    loop.set_task(task)
    loop.record(n)
    loop.run(n)
    recs = loop.records()
    for k, rec in enumerate(recs):
        if rec["have"]:
            batch = (torch.from_numpy(rec["s"]), torch.from_numpy(rec["a"]), torch.from_numpy(rec["rb"]).view(-1, 1),
                     torch.from_numpy(rec["phi"]), torch.from_numpy(rec["s1"]), torch.from_numpy(rec["gamma"]))
            if schedule == "tsf":
                R.tsf_update(st, batch, task, use_gpi=True, target_update_ev=ev)
            else:
                R.sf_update(st, batch, task, use_gpi=True, target_update_ev=ev)
        q, tk = R.gpi_w(R.psi_all(st.online, spec, torch.from_numpy(rec["snext"]).view(1, -1)), st.w[task])
        want = (int(tk[0]), R.select_action(q, tk[0], task, True))
        got = (recs[k + 1]["c"], recs[k + 1]["a_greedy"]) if k + 1 < len(recs) else loop.action()
        assert got == want, f"step {k}: runner selected {got}, oracle {want}"
    params_close(torch.stack([eng.get_head(t, 0) for t in range(T)]), st.online, 1e-3 * n)
    rel_close(torch.stack([eng.get_w(t)[0] for t in range(T)]), st.w, rtol=1e-4, atol=1e-7)
    if schedule == "tsf":
        params_close(torch.stack([eng.tsf_get_g(t)[0] for t in range(T)]), st.g, 1e-3 * n)
        params_close(eng.tsf_get_h(), st.h, 1e-3 * n)
    loop.close()
    eng.close()
