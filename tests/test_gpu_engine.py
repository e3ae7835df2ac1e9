"""GPU parity: libsfx.so kernels vs the reference's golden vectors and the CPU oracle.

Tolerances (north_star: ψ within 1e-4 relative, GPI argmax bit-exact):
  * ψ, q, losses       : rtol 1e-4 (plus a tiny atol for values near 0)
  * task / next / action indices : exact
  * parameters after k Adam steps: rtol 1e-4 / atol 1e-5, except a vanishing fraction of
    entries whose gradient is ~0 (Adam's g/sqrt(v) can flip sign on a rounding-level
    gradient; such an entry may move by <= 2*lr per step) -- bounded by max_bad_frac.
"""
import numpy as np
import pytest
import torch

from oracle import ref_cpu as R
from tests.conftest import gpu_available

pytestmark = pytest.mark.gpu

GPI_CASES = ["reacher17", "hopper11", "cartpole", "refreacher", "tanh_odd", "tie"]


def spec_of(g):
    return R.Spec(int(g["n_s"]), int(g["H"]), int(g["A"]), int(g["d"]), tuple(str(a) for a in g["acts"]))


def engine_for(spec, T, max_batch=32):
    from sfx.engine import SFEngine

    return SFEngine(T, spec.n_s, spec.H, spec.A, spec.d, spec.acts, max_batch=max_batch)


def rel_close(a, b, rtol=1e-4, atol=1e-6):
    a = np.asarray(a.detach().cpu() if torch.is_tensor(a) else a, dtype=np.float64)
    b = np.asarray(b.detach().cpu() if torch.is_tensor(b) else b, dtype=np.float64)
    np.testing.assert_allclose(a, b, rtol=rtol, atol=atol)


def params_close(a, b, lr_steps, rtol=1e-4, atol=1e-5, max_bad_frac=2e-4):
    a = np.asarray(torch.as_tensor(a).cpu(), dtype=np.float64)
    b = np.asarray(torch.as_tensor(b).cpu(), dtype=np.float64)
    bad = np.abs(a - b) > atol + rtol * np.abs(b)
    assert bad.mean() <= max_bad_frac, f"{bad.sum()} / {bad.size} entries differ"
    if bad.any():
        assert np.abs(a - b)[bad].max() <= 2.0 * lr_steps + atol


@pytest.fixture(autouse=True)
def _need_gpu():
    if not gpu_available():
        pytest.skip("no HIP device")


@pytest.mark.parametrize("case", GPI_CASES)
def test_gpi_vs_golden(golden, case):
    g = golden("gpi_" + case)
    spec, T = spec_of(g), int(g["T"])
    eng = engine_for(spec, T)
    for t in range(T):
        eng.load_head(t, g["online"][t])
        eng.load_w(t, g["w"][t])
    for B, S in ((1, g["S1"]), (32, g["S32"])):
        S = torch.from_numpy(S).cuda()
        for i in range(T):
            psi, q, task, nxt = eng.gpi(S, w_index=i, want_psi=True)
            rel_close(psi, g[f"psi{B}"])
            rel_close(q, g[f"q{B}_{i}"], atol=1e-6)
            assert np.array_equal(task.cpu().numpy().reshape(-1), np.asarray(g[f"task{B}_{i}"]).reshape(-1))
            if B == 32:
                assert np.array_equal(nxt.cpu().numpy(), g[f"next32_{i}"])
    eng.close()


def test_gpi_full_size(golden):
    from tests.golden.recipe import full_size_heads

    g = golden("gpi_reacher17_full")
    spec, T = spec_of(g), int(g["T"])
    online, w = full_size_heads()
    eng = engine_for(spec, T)
    for t in range(T):
        eng.load_head(t, online[t])
        eng.load_w(t, w[t])
    S = torch.from_numpy(g["S32"]).cuda()
    for i in range(T):
        psi, q, task, nxt = eng.gpi(S, w_index=i, want_psi=True)
        rel_close(psi, g["psi32"], rtol=1e-4, atol=1e-5)
        rel_close(q, g[f"q32_{i}"], rtol=1e-4, atol=1e-6)
        assert np.array_equal(task.cpu().numpy(), g[f"task32_{i}"])
        assert np.array_equal(nxt.cpu().numpy(), g[f"next32_{i}"])
        _, _, t1, _ = eng.gpi(S[:1], w_index=i)
        assert int(t1) == int(g[f"task1_{i}"])
    eng.close()


@pytest.mark.parametrize("use_gpi", [True, False])
def test_select_action_vs_oracle(golden, use_gpi):
    g = golden("gpi_reacher17")
    spec, T = spec_of(g), int(g["T"])
    eng = engine_for(spec, T)
    online = torch.from_numpy(g["online"])
    for t in range(T):
        eng.load_head(t, online[t])
        eng.load_w(t, g["w"][t])
    gen = torch.Generator().manual_seed(0)
    for _ in range(20):
        s = torch.randn(1, spec.n_s, generator=gen)
        for i in range(T):
            q, task = R.gpi_w(R.psi_all(online, spec, s), torch.from_numpy(g["w"][i]))
            want = R.select_action(q, task[0], i, use_gpi)
            qd = torch.empty(T, spec.A, device="cuda")
            out = eng.select_action(s.cuda(), i, use_gpi, q_out=qd).cpu()
            assert int(out[1]) == want
            if use_gpi:
                assert int(out[0]) == int(task[0])
            rel_close(qd, q[0], atol=1e-6)
    eng.close()


def batches_of(g):
    return [tuple(torch.from_numpy(g["b_" + n][j]) for n in ("s", "a", "r", "phi", "s1", "gamma"))
            for j in range(int(g["k"]))]


@pytest.mark.parametrize("case", ["sfdqn_gpi", "sfdqn_nogpi", "sfdqn_tanh"])
def test_update_vs_golden(golden, case):
    g = golden("upd_" + case)
    spec, T = spec_of(g), int(g["T"])
    eng = engine_for(spec, T)
    eng.set_adam(1e-3, 0.0, 1e-3, 0.0)
    eng.set_target_update_ev(int(g["target_update_ev"]))
    for t in range(T):
        eng.load_head(t, g["online0"][t], 0)
        eng.load_head(t, g["target0"][t], 1)
        eng.load_w(t, g["w0"][t])
    k = int(g["k"])
    for j, (s, a, r, phi, s1, gamma) in enumerate(batches_of(g)):
        i = int(g["policies"][j])
        nxt = torch.empty(s.shape[0], dtype=torch.long, device="cuda")
        losses = eng.update(i, s, a, r, phi, s1, gamma, use_gpi=bool(g["use_gpi"]), next_actions=nxt)
        assert np.array_equal(nxt.cpu().numpy(), g["next_actions"][j]), f"step {j}"
        rel_close(losses, g["losses"][j], rtol=1e-4, atol=1e-7)
        if j == 0:
            params_close(torch.stack([eng.get_head(t) for t in range(T)]), g["online1"], 1e-3)
    online = torch.stack([eng.get_head(t, 0) for t in range(T)])
    target = torch.stack([eng.get_head(t, 1) for t in range(T)])
    params_close(online, g["online"], 1e-3 * k)
    params_close(target, g["target"], 1e-3 * k)
    w = torch.stack([eng.get_w(t)[0] for t in range(T)])
    rel_close(w, g["w"], rtol=1e-4, atol=1e-5)
    for t in range(T):
        m, v, st = eng.get_adam(t)
        assert st == int(g["steps"][t])
        params_close(m, g["m"][t], 1e-3 * k, rtol=1e-4, atol=1e-8)
        params_close(v, g["v"][t], 1e-3 * k, rtol=1e-4, atol=1e-10)
        assert eng.since_target(t) == int(g["since_target"][t])
    eng.close()


def test_update_all_vs_golden(golden):
    g = golden("upd_deep_alltask")
    spec, T = spec_of(g), int(g["T"])
    eng = engine_for(spec, T)
    eng.set_adam(1e-3, 0.0, 1e-3, 0.0)
    eng.set_target_update_ev(int(g["target_update_ev"]))
    for t in range(T):
        eng.load_head(t, g["online0"][t], 0)
        eng.load_head(t, g["online0"][t], 1)
        eng.load_w(t, g["w0"][t])
    for j, (s, a, r, phi, s1, gamma) in enumerate(batches_of(g)):
        eng.lms(int(g["lms_task"][j]), torch.from_numpy(g["lms_phi"][j]), torch.tensor([float(g["lms_r"][j])]),
                float(g["alpha_w"]))
        eng.update_all(s, a, phi, s1, gamma)
        if j == 0:
            params_close(torch.stack([eng.get_head(t) for t in range(T)]), g["online1"], 1e-3)
    k = int(g["k"])
    params_close(torch.stack([eng.get_head(t, 0) for t in range(T)]), g["online"], 1e-3 * k)
    params_close(torch.stack([eng.get_head(t, 1) for t in range(T)]), g["target"], 1e-3 * k)
    rel_close(torch.stack([eng.get_w(t)[0] for t in range(T)]), g["w"], rtol=1e-5, atol=1e-7)
    for t in range(T):
        assert eng.since_target(t) == int(g["since_target"][t])
    eng.close()


def test_update_all_host_rounds_with_temporary_inputs():
    """sfx_update_all returns with its verdict pending; the host rounds of a step whose device
    rounds are treated as failed (sfx_debug_force_rerun) run inside the NEXT call.  The caller's
    inputs are temporaries and the losses are dropped at once, as the drop-in does:
    the engine must keep them alive until that call, so every step trains on its own minibatch."""
    from sfx.init import reference_heads

    spec, T, B = R.Spec(17, 64, 7, 8), 4, 32
    online, w = reference_heads(T, spec.n_s, spec.H, spec.A, spec.d, spec.acts, seed=3)
    eng = engine_for(spec, T)
    for t in range(T):
        eng.load_head(t, online[t], 0)
        eng.load_head(t, online[t], 1)
        eng.load_w(t, w[t])
    eng.debug_force_rerun(1)
    st = R.SFState(spec, online.clone(), online.clone(), w.clone())
    gen = torch.Generator().manual_seed(11)
    batches = [(torch.randn(B, 17, generator=gen), torch.randint(0, 7, (B,), generator=gen),
                torch.rand(B, 8, generator=gen), torch.randn(B, 17, generator=gen), torch.full((B,), 0.9))
               for _ in range(4)]

    def step(b):  # every argument is a fresh host tensor that dies with this frame
        eng.update_all(*(x.clone().numpy() for x in b))

    for b in batches:
        step(b)
        R.deep_all_task_step(st, b)
    stats = eng.step_stats()
    assert stats["host_round_steps"] == len(batches)
    params_close(torch.stack([eng.get_head(t) for t in range(T)]), st.online, 4e-3)
    eng.close()


def test_gpi_right_after_update_all_sees_the_host_rounds():
    """while an update_all verdict is pending, sfx_gpi is queued speculatively on the
    update's write slots and re-run only when settle() counts a fallback.  Force the fallback
    (sfx_debug_force_rerun) and call gpi at once: q, the task and the next actions must be the
    oracle's on the post-update heads (the re-run GPI, not the speculative one), and the step must
    be counted as a host-round step."""
    from sfx.init import reference_heads

    spec, T, B = R.Spec(17, 64, 7, 8), 5, 32
    online, w = reference_heads(T, spec.n_s, spec.H, spec.A, spec.d, spec.acts, seed=8)
    eng = engine_for(spec, T)
    for t in range(T):
        eng.load_head(t, online[t], 0)
        eng.load_head(t, online[t], 1)
        eng.load_w(t, w[t])
    st = R.SFState(spec, online.clone(), online.clone(), w.clone())
    gen = torch.Generator().manual_seed(12)
    for k in range(3):
        b = (torch.randn(B, 17, generator=gen), torch.randint(0, 7, (B,), generator=gen),
             torch.rand(B, 8, generator=gen), torch.randn(B, 17, generator=gen), torch.full((B,), 0.9))
        S = torch.randn(6, 17, generator=gen)
        before = eng.step_stats()["host_round_steps"]
        eng.debug_force_rerun(1)
        eng.update_all(*(x.cuda() for x in b))
        _, q, task, nxt = eng.gpi(S.cuda(), w_index=k + 1)  # right away: the verdict is still pending
        eng.debug_force_rerun(-1)
        R.deep_all_task_step(st, b)
        q_ref, task_ref = R.gpi_w(R.psi_all(st.online, spec, S), st.w[k + 1])
        rel_close(q.cpu(), q_ref, rtol=1e-4, atol=1e-6)
        assert torch.equal(task.cpu(), task_ref)
        assert torch.equal(nxt.cpu(), R.gpi_next_actions(q_ref))
        assert eng.step_stats()["host_round_steps"] == before + 1
    eng.close()


def test_full_size_update_vs_oracle():
    """BASELINE C2 shape (H=256, T=8): one active-task and one all-task step against the oracle."""
    from tests.golden.recipe import SHAPES, full_size_heads

    n_s, H, A, d, acts = SHAPES["reacher17_full"]
    spec = R.Spec(n_s, H, A, d, acts)
    online, w = full_size_heads()
    gen = torch.Generator().manual_seed(42)
    B = 32
    s, s1 = torch.randn(B, n_s, generator=gen), torch.randn(B, n_s, generator=gen)
    a = torch.randint(0, A, (B,), generator=gen)
    phi, r = torch.rand(B, d, generator=gen), torch.rand(B, 1, generator=gen)
    gamma = torch.full((B,), 0.9)
    eng = engine_for(spec, 8)
    for t in range(8):
        eng.load_head(t, online[t], 0)
        eng.load_head(t, online[t], 1)
        eng.load_w(t, w[t])
    st = R.SFState(spec, online.clone(), online.clone(), w.clone())
    loss, l1, l2, na = R.sf_update(st, (s, a, r, phi, s1, gamma), 3, use_gpi=True)
    nxt = torch.empty(B, dtype=torch.long, device="cuda")
    lo = eng.update(3, s, a, r, phi, s1, gamma, use_gpi=True, next_actions=nxt)
    assert np.array_equal(nxt.cpu().numpy(), na.numpy())
    rel_close(lo, [float(loss), float(l1), float(l2)], rtol=1e-4, atol=1e-8)
    params_close(eng.get_head(3), st.online[3], 1e-3)
    st2 = st.clone()
    R.deep_all_task_step(st2, (s, a, phi, s1, gamma))
    eng.update_all(s, a, phi, s1, gamma)
    params_close(torch.stack([eng.get_head(t) for t in range(8)]), st2.online, 2e-3)
    eng.close()


@pytest.mark.parametrize("form", ["host", "device_phi_float_r"])
def test_lms_vs_oracle(form):
    """LMS reward fit; device_phi_float_r: the drop-in agents' call (φ on the device, r a host
    float) -- sfx_lms_value, r as a kernel argument -- bit-identical to the pointer form."""
    spec = R.Spec(17, 32, 7, 8)
    eng = engine_for(spec, 2)
    gen = torch.Generator().manual_seed(1)
    w = torch.empty(8).uniform_(-0.01, 0.01, generator=gen)
    eng.load_w(1, w)
    wr = w.reshape(-1, 1)
    for _ in range(10):
        phi = torch.rand(8, generator=gen)
        r = torch.rand((), generator=gen)
        wr = R.lms_update(wr, phi, r, 0.05)
        if form == "host":
            eng.lms(1, phi, r.reshape(1), 0.05)
        else:
            eng.lms(1, phi.cuda(), float(r), 0.05)
    rel_close(eng.get_w(1)[0], wr.reshape(-1), rtol=1e-5, atol=1e-7)
    eng.close()


RAGGED = [
    # n_s, H, A, d, acts, B
    (17, 64, 7, 8, ("relu", "relu"), 1),
    (17, 64, 7, 8, ("relu", "relu"), 64),
    (11, 48, 27, 50, ("relu", "relu"), 45),
    (6, 40, 5, 3, ("tanh",), 200),
    (33, 96, 4, 12, ("relu", "relu", "relu"), 33),
    (70, 32, 3, 17, ("relu", "relu"), 16),
]


@pytest.mark.parametrize("n_s,H,A,d,acts,B", RAGGED)
def test_ragged_shapes_update_vs_oracle(n_s, H, A, d, acts, B):
    """Edge geometries of the SF kernels: a single row, batches past one 32-row tile (up to
    200), wide ψ outputs (A·d = 1350), one and three hidden layers, tanh, odd d, fan-ins past the
    fused layer-0 limit (n_s = 70).  Active-task updates (± GPI, with l2) and all-task steps vs
    the oracle, parameters after every step."""
    from sfx.init import reference_heads

    T = 3
    spec = R.Spec(n_s, H, A, d, acts)
    online, w = reference_heads(T, n_s, H, A, d, acts, seed=4)
    eng = engine_for(spec, T, max_batch=max(B, 1))
    for t in range(T):
        eng.load_head(t, online[t], 0)
        eng.load_head(t, online[t], 1)
        eng.load_w(t, w[t])
    st = R.SFState(spec, online.clone(), online.clone(), w.clone())
    gen = torch.Generator().manual_seed(9)

    def batch():
        return (torch.randn(B, n_s, generator=gen), torch.randint(0, A, (B,), generator=gen),
                torch.rand(B, 1, generator=gen), torch.rand(B, d, generator=gen), torch.randn(B, n_s, generator=gen),
                torch.where(torch.rand(B, generator=gen) < 0.2, 0.0, 0.9))

    nxt = torch.empty(B, dtype=torch.long, device="cuda")
    for k, (i, use_gpi) in enumerate(((1, True), (2, False), (0, True))):
        s, a, r, phi, s1, gamma = batch()
        loss, l1, l2, na = R.sf_update(st, (s, a, r, phi, s1, gamma), i, use_gpi=use_gpi)
        lo = eng.update(i, s, a, r, phi, s1, gamma, use_gpi=use_gpi, next_actions=nxt)
        assert torch.equal(nxt.cpu(), na), f"update {k}: next actions differ"
        rel_close(lo, [float(loss), float(l1), float(l2)], rtol=1e-4, atol=1e-7)
    params_close(torch.stack([eng.get_head(t) for t in range(T)]), st.online, 3e-3)
    rel_close(torch.stack([eng.get_w(t)[0] for t in range(T)]), st.w, rtol=1e-4, atol=1e-7)
    for _ in range(2):
        s, a, r, phi, s1, gamma = batch()
        R.deep_all_task_step(st, (s, a, phi, s1, gamma))
        eng.update_all(s, a, phi, s1, gamma)
    params_close(torch.stack([eng.get_head(t) for t in range(T)]), st.online, 5e-3)
    eng.close()


@pytest.mark.parametrize("n_s,H,A,d,acts,B", [RAGGED[1], RAGGED[2], (17, 256, 7, 8, ("relu", "relu"), 32)])
def test_huber_update_vs_oracle(n_s, H, A, d, acts, B):
    """Opt-in HuberLoss (sfx_set_huber; not in the reference) through both TD paths --
    the fused TD launch (A·d <= 128) and k_tdg (A·d = 1350) -- against torch's huber_loss and its
    autograd gradient in the oracle: active-task updates (± GPI) and all-task steps, δ small enough
    that part of the errors fall outside it.  Tolerances as for MSE."""
    from sfx.init import reference_heads

    T, delta = 3, 0.05
    spec = R.Spec(n_s, H, A, d, acts)
    online, w = reference_heads(T, n_s, H, A, d, acts, seed=6)
    eng = engine_for(spec, T, max_batch=B)
    eng.set_huber(delta)
    assert abs(eng.huber - delta) < 1e-9
    for t in range(T):
        eng.load_head(t, online[t], 0)
        eng.load_head(t, online[t], 1)
        eng.load_w(t, w[t])
    st = R.SFState(spec, online.clone(), online.clone(), w.clone())
    gen = torch.Generator().manual_seed(12)

    def batch():
        return (torch.randn(B, n_s, generator=gen), torch.randint(0, A, (B,), generator=gen),
                torch.rand(B, 1, generator=gen), torch.rand(B, d, generator=gen), torch.randn(B, n_s, generator=gen),
                torch.full((B,), 0.9))

    nxt = torch.empty(B, dtype=torch.long, device="cuda")
    for i, use_gpi in ((1, True), (2, False)):
        s, a, r, phi, s1, gamma = batch()
        loss, l1, l2, na = R.sf_update(st, (s, a, r, phi, s1, gamma), i, use_gpi=use_gpi, huber=delta)
        lo = eng.update(i, s, a, r, phi, s1, gamma, use_gpi=use_gpi, next_actions=nxt)
        assert torch.equal(nxt.cpu(), na)
        rel_close(lo, [float(loss), float(l1), float(l2)], rtol=1e-4, atol=1e-7)
    params_close(torch.stack([eng.get_head(t) for t in range(T)]), st.online, 2e-3)
    for _ in range(2):
        s, a, r, phi, s1, gamma = batch()
        R.deep_all_task_step(st, (s, a, phi, s1, gamma), huber=delta)
        eng.update_all(s, a, phi, s1, gamma)
    params_close(torch.stack([eng.get_head(t) for t in range(T)]), st.online, 4e-3)
    eng.set_huber(0.0)  # back to the reference's MSE
    s, a, r, phi, s1, gamma = batch()
    loss, l1, l2, na = R.sf_update(st, (s, a, r, phi, s1, gamma), 0, use_gpi=True)
    lo = eng.update(0, s, a, r, phi, s1, gamma, use_gpi=True, next_actions=nxt)
    rel_close(lo, [float(loss), float(l1), float(l2)], rtol=1e-4, atol=1e-7)
    eng.close()
