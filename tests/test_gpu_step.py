"""GPU parity of the fused, speculative all-task env step (sfx_step_all / sfx_step_finish)
against the oracle's exact in-order loop (agents/sfdqn.py:57-60 over features/deep.py:93-131).

The speculation must be invisible: parameters, losses and the selected action have to match
the sequential reference whether the speculation held or the policies were re-run
(forced through sfx_debug_force_rerun).  Tolerances as in test_gpu_engine.py.
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


def setup(spec, T, seed=0, ev=3, lr=1e-3):
    from sfx.engine import SFEngine
    from sfx.init import reference_heads

    online, w = reference_heads(T, spec.n_s, spec.H, spec.A, spec.d, spec.acts, seed=seed)
    eng = SFEngine(T, spec.n_s, spec.H, spec.A, spec.d, spec.acts, max_batch=32)
    eng.set_adam(lr, 0.0, lr, 0.0)
    eng.set_target_update_ev(ev)
    for t in range(T):
        eng.load_head(t, online[t], 0)
        eng.load_head(t, online[t], 1)
        eng.load_w(t, w[t])
    st = R.SFState(spec, online.clone(), online.clone(), w.clone())
    return eng, st


def dev(x, dtype=torch.float32):
    return x.to("cuda", dtype).contiguous()


def run_steps(eng, st, spec, T, k, seed=5, lr=1e-3, ev=3, alpha=0.05):
    gen = torch.Generator().manual_seed(seed)
    B = 32
    agree = 0
    for j in range(k):
        task = j % T
        s, s1 = torch.randn(B, spec.n_s, generator=gen), torch.randn(B, spec.n_s, generator=gen)
        a = torch.randint(0, spec.A, (B,), generator=gen)
        phi = torch.rand(B, spec.d, generator=gen)
        gamma = torch.where(torch.rand(B, generator=gen) < 0.1, 0.0, 0.9)
        phi1, r1 = torch.rand(spec.d, generator=gen), torch.rand(1, generator=gen)
        s_next = torch.randn(1, spec.n_s, generator=gen)
        losses = torch.empty(T, 3, device="cuda")
        eng.step_all(dev(s), dev(a, torch.long), dev(phi), dev(s1), dev(gamma), use_gpi=True, lms_task=task,
                     lms_phi=dev(phi1), lms_r=dev(r1), lms_alpha=alpha, s_next=dev(s_next), task_index=task,
                     losses=losses)
        c, act, first = eng.step_finish()
        # oracle, in the reference's order
        st.w[task] = R.lms_update(st.w[task].view(-1, 1), phi1, r1[0], alpha).view(-1)
        res = R.deep_all_task_step(st, (s, a, phi, s1, gamma), lr=lr, target_update_ev=ev)
        q, tk = R.gpi_w(R.psi_all(st.online, spec, s_next), st.w[task])
        want_a = R.select_action(q, tk[0], task, True)
        rel_close(losses[:, 1].cpu(), [float(l1) for l1, _ in res], rtol=1e-4, atol=1e-7)
        assert c == int(tk[0]) and act == want_a, f"step {j}: got ({c},{act}) want ({int(tk[0])},{want_a})"
        agree += first == T
    online = torch.stack([eng.get_head(t, 0) for t in range(T)])
    params_close(online, st.online, 1e-3 * k)
    params_close(torch.stack([eng.get_head(t, 1) for t in range(T)]), st.target, 1e-3 * k)
    rel_close(torch.stack([eng.get_w(t)[0] for t in range(T)]), st.w, rtol=1e-5, atol=1e-7)
    for t in range(T):
        m, v, step = eng.get_adam(t)
        assert step == st.step[t]
        assert eng.since_target(t) == st.since_target[t]
    return agree


@pytest.mark.parametrize("force,rounds", [(-1, 2), (-1, 1), (0, 2), (1, 1), (3, 2)])
def test_step_all_matches_in_order_reference(force, rounds):
    spec = R.Spec(17, 32, 7, 8, ("relu", "relu"))
    T = 4
    eng, st = setup(spec, T)
    eng.set_spec_rounds(rounds)
    eng.debug_force_rerun(force)
    agree = run_steps(eng, st, spec, T, k=8)
    stats = eng.step_stats()
    assert stats["steps"] == 8
    if force >= 0:
        assert stats["host_round_steps"] == 8 and agree == 0
        assert stats["rounds"] >= 8 * (rounds + 1)
    eng.close()


def test_step_all_full_size_and_tanh():
    spec = R.Spec(17, 256, 7, 8, ("relu", "relu"))
    eng, st = setup(spec, 8)
    run_steps(eng, st, spec, 8, k=4)
    eng.close()
    spec = R.Spec(6, 48, 5, 3, ("tanh", "relu"))
    eng, st = setup(spec, 3, seed=2)
    eng.debug_force_rerun(1)
    run_steps(eng, st, spec, 3, k=5)
    eng.close()


def test_step_without_minibatch_then_active_updates():
    """B = 0 steps only select (and LMS); sfx_update after fused steps keeps the slot masks right."""
    spec = R.Spec(17, 32, 7, 8, ("relu", "relu"))
    T = 3
    eng, st = setup(spec, T, ev=1000)
    gen = torch.Generator().manual_seed(9)
    s_next = torch.randn(1, spec.n_s, generator=gen)
    phi1, r1 = torch.rand(spec.d, generator=gen), torch.rand(1, generator=gen)
    eng.step_all(lms_task=1, lms_phi=dev(phi1), lms_r=dev(r1), lms_alpha=0.05, s_next=dev(s_next), task_index=1)
    c, act, first = eng.step_finish()
    st.w[1] = R.lms_update(st.w[1].view(-1, 1), phi1, r1[0], 0.05).view(-1)
    q, tk = R.gpi_w(R.psi_all(st.online, spec, s_next), st.w[1])
    assert (c, act, first) == (int(tk[0]), R.select_action(q, tk[0], 1, True), T)
    run_steps(eng, st, spec, T, k=2, seed=11, ev=1000)
    B = 32
    s, s1 = torch.randn(B, spec.n_s, generator=gen), torch.randn(B, spec.n_s, generator=gen)
    a = torch.randint(0, spec.A, (B,), generator=gen)
    phi, r = torch.rand(B, spec.d, generator=gen), torch.rand(B, 1, generator=gen)
    gamma = torch.full((B,), 0.9)
    for i in (2, 0, 2):
        eng.update(i, s, a, r, phi, s1, gamma, use_gpi=True)
        R.sf_update(st, (s, a, r, phi, s1, gamma), i, use_gpi=True)
    params_close(torch.stack([eng.get_head(t) for t in range(T)]), st.online, 1e-2)
    eng.close()


def test_paired_forward_tiles_are_bit_exact(monkeypatch):
    """Two column tiles per forward workgroup (the layer-0+1 forward and the oversubscribed
    layer-2 forward of the first forward at the C2 shape: 384 tiles -> 192 workgroups) run each
    tile's MFMA chain in the same k order as one tile per workgroup (SFX_FWD_TPW=1): heads, Adam
    state, w and every selected action identical bit for bit after several all-task steps."""
    spec = R.Spec(17, 256, 7, 8, ("relu", "relu"))
    T, k = 8, 4
    results = []
    for tpw in ("1", "2"):
        monkeypatch.setenv("SFX_FWD_TPW", tpw)  # read when the handle is created
        eng, st = setup(spec, T)
        gen = torch.Generator().manual_seed(21)
        acts = []
        for j in range(k):
            B = 32
            s, s1 = torch.randn(B, spec.n_s, generator=gen), torch.randn(B, spec.n_s, generator=gen)
            a = torch.randint(0, spec.A, (B,), generator=gen)
            phi = torch.rand(B, spec.d, generator=gen)
            gamma = torch.full((B,), 0.9)
            phi1, r1 = torch.rand(spec.d, generator=gen), torch.rand(1, generator=gen)
            s_next = torch.randn(1, spec.n_s, generator=gen)
            eng.step_all(dev(s), dev(a, torch.long), dev(phi), dev(s1), dev(gamma), use_gpi=True, lms_task=j % T,
                         lms_phi=dev(phi1), lms_r=dev(r1), lms_alpha=0.05, s_next=dev(s_next), task_index=j % T)
            acts.append(eng.step_finish())
        heads = torch.stack([eng.get_head(t, 0) for t in range(T)])
        adam = [eng.get_adam(t) for t in range(T)]
        w = torch.stack([eng.get_w(t)[0] for t in range(T)])
        results.append((acts, heads, adam, w))
        eng.close()
    (a1, h1, m1, w1), (a2, h2, m2, w2) = results
    assert a1 == a2
    assert torch.equal(h1, h2) and torch.equal(w1, w2)
    for (p, q, s_), (p2, q2, s2) in zip(m1, m2):
        assert torch.equal(p, p2) and torch.equal(q, q2) and s_ == s2


@pytest.mark.parametrize("force", [-1, 2])
def test_step_all_many_heads(force):
    """40 heads: past the fused TD launch's bound (32·T·A <= 2048), so every round's TD target runs
    in k_tdg, and the final round's post-update ψ output layer spans more workgroups than CUs --
    the same results as the oracle's in-order loop, with and without forced host rounds."""
    spec = R.Spec(17, 32, 7, 8, ("relu", "relu"))
    T = 40
    eng, st = setup(spec, T, seed=4)
    eng.debug_force_rerun(force)
    run_steps(eng, st, spec, T, k=3, seed=8)
    assert eng.step_stats()["steps"] == 3
    eng.close()
