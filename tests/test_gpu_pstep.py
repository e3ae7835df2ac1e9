"""GPU parity of the persistent all-task step (k_pstep, csrc/sfx_pstep.h): the whole env step of
agents/sfdqn.py:57-60 over features/deep.py:93-131 -- LMS reward fit, forwards, every speculative
round until the next actions verify, Adam, action selection -- as one launch per step, checked
against the oracle's exact in-order loop (tolerances as test_gpu_step.py / test_gpu_engine.py:
losses, w within 1e-4 relative; parameters within rtol 1e-4 except at most 2e-4 of the entries by
<= 2·lr per step; selected actions, Adam step counts and target syncs exact), and against the
launch path on the same inputs.
"""
import numpy as np
import pytest
import torch

from oracle import ref_cpu as R
from tests.conftest import gpu_available
from tests.test_gpu_engine import params_close, rel_close
from tests.test_gpu_step import dev, setup

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _need_gpu():
    if not gpu_available():
        pytest.skip("no HIP device")


def run_pstep_steps(eng, st, spec, T, k, seed=5, lr=1e-3, ev=3, alpha=0.05, sel_use_gpi=True):
    gen = torch.Generator().manual_seed(seed)
    B = 32
    for j in range(k):
        task = j % T
        s, s1 = torch.randn(B, spec.n_s, generator=gen), torch.randn(B, spec.n_s, generator=gen)
        a = torch.randint(0, spec.A, (B,), generator=gen)
        phi = torch.rand(B, spec.d, generator=gen)
        gamma = torch.where(torch.rand(B, generator=gen) < 0.1, 0.0, 0.9)
        phi1, r1 = torch.rand(spec.d, generator=gen), torch.rand(1, generator=gen)
        s_next = torch.randn(1, spec.n_s, generator=gen)
        eng.step_all(dev(s), dev(a, torch.long), dev(phi), dev(s1), dev(gamma), use_gpi=True, lms_task=task,
                     lms_phi=dev(phi1), lms_r=dev(r1), lms_alpha=alpha, s_next=dev(s_next), task_index=task,
                     sel_use_gpi=sel_use_gpi)
        c, act, first = eng.step_finish()
        assert first == T, f"step {j}: the persistent step must verify on the device (flag {first})"
        st.w[task] = R.lms_update(st.w[task].view(-1, 1), phi1, r1[0], alpha).view(-1)
        R.deep_all_task_step(st, (s, a, phi, s1, gamma), lr=lr, target_update_ev=ev)
        q, tk = R.gpi_w(R.psi_all(st.online, spec, s_next), st.w[task])
        want_c = int(tk[0]) if sel_use_gpi else task
        want_a = R.select_action(q, tk[0], task, sel_use_gpi)
        assert (c, act) == (want_c, want_a), f"step {j}: got ({c},{act}) want ({want_c},{want_a})"
    online = torch.stack([eng.get_head(t, 0) for t in range(T)])
    params_close(online, st.online, lr * k)
    params_close(torch.stack([eng.get_head(t, 1) for t in range(T)]), st.target, lr * k)
    rel_close(torch.stack([eng.get_w(t)[0] for t in range(T)]), st.w, rtol=1e-5, atol=1e-7)
    for t in range(T):
        m, v, step = eng.get_adam(t)
        assert step == st.step[t]
        assert eng.since_target(t) == st.since_target[t]


@pytest.mark.parametrize("spec,T", [(R.Spec(17, 256, 7, 8, ("relu", "relu")), 8),
                                    (R.Spec(4, 256, 2, 20, ("relu", "relu")), 2),
                                    (R.Spec(6, 256, 5, 3, ("tanh", "relu", "relu")), 5)])
def test_pstep_matches_in_order_reference(spec, T):
    eng, st = setup(spec, T)
    eng.set_pstep(True)
    assert eng.pstep
    run_pstep_steps(eng, st, spec, T, k=7)
    ps = eng.pstep_stats()
    assert ps["steps"] == 7 and ps["rounds"] >= 7, ps
    eng.close()


def test_pstep_selection_without_gpi_and_many_steps():
    spec = R.Spec(17, 256, 7, 8, ("relu", "relu"))
    eng, st = setup(spec, 8, seed=3, ev=4)
    eng.set_pstep(True)
    run_pstep_steps(eng, st, spec, 8, k=12, seed=8, ev=4, sel_use_gpi=False)
    eng.close()


def _relu_ties(st, spec, s, eps=1e-6):
    """Heads whose hidden pre-activations at the minibatch states come within eps of 0 (oracle
    state): there the sign -- ReLU's gradient mask -- is a rounding tie between summation orders."""
    out = set()
    for t in range(st.T):
        x = s
        for li, (Wl, bl) in enumerate(R.unpack(st.online[t], spec)[:-1]):
            z = x @ Wl.T + bl
            if li > 0 and bool((z.abs() < eps).any()):
                out.add(t)
            x = z if li == 0 else torch.relu(z)
    return out


def test_pstep_equals_launch_path_and_reference_actions():
    """The persistent step and the launch path from the same state, beside the oracle: per step the
    selected action (identical), every policy's verified next actions (the trace of k_pstep's last
    computed round per head == the oracle's in-order GPI next actions, exactly), and parameters /
    moments within the parity tolerance -- except for a head whose hidden pre-activation came within
    1e-6 of zero at some step (a ReLU-mask rounding tie: a different fp32 summation order may take
    the other side, and Adam carries that forward; seen at seed 4, head 7, step 2, |z| = 1.7e-8)."""
    spec = R.Spec(17, 256, 7, 8, ("relu", "relu"))
    T = 8
    engs = []
    for on in (False, True):
        eng, st = setup(spec, T, seed=4, ev=1000)
        if on:
            eng.set_pstep(True)
        engs.append(eng)
    gen = torch.Generator().manual_seed(21)
    B = 32
    ties = set()
    for j in range(5):
        s, s1 = torch.randn(B, spec.n_s, generator=gen), torch.randn(B, spec.n_s, generator=gen)
        a = torch.randint(0, spec.A, (B,), generator=gen)
        phi = torch.rand(B, spec.d, generator=gen)
        gamma = torch.full((B,), 0.9)
        phi1, r1 = torch.rand(spec.d, generator=gen), torch.rand(1, generator=gen)
        s_next = torch.randn(1, spec.n_s, generator=gen)
        outs = []
        for eng in engs:
            eng.step_all(dev(s), dev(a, torch.long), dev(phi), dev(s1), dev(gamma), use_gpi=True, lms_task=j % T,
                         lms_phi=dev(phi1), lms_r=dev(r1), lms_alpha=0.05, s_next=dev(s_next), task_index=j % T)
            outs.append(eng.step_finish()[:2])
        assert outs[0] == outs[1], f"step {j}: launch path {outs[0]} vs persistent {outs[1]}"
        ties |= _relu_ties(st, spec, s)
        st.w[j % T] = R.lms_update(st.w[j % T].view(-1, 1), phi1, r1[0], 0.05).view(-1)
        res = R.deep_all_task_step(st, (s, a, phi, s1, gamma), lr=1e-3, target_update_ev=1000)
        conv, tr = engs[1].pstep_trace()
        assert 1 <= conv <= T + 1
        for t in range(T):
            last = max(r for r in range(conv) if tr[r][t][0] == 1)
            assert tr[last][t][1] == [int(x) for x in res[t][1]], f"step {j}, policy {t}: next actions"
    for t in range(T):
        if t in ties:
            continue
        params_close(engs[1].get_head(t, 0), st.online[t], 5e-3)
        params_close(engs[0].get_head(t, 0), st.online[t], 5e-3)
        m1, v1, s1_ = engs[1].get_adam(t)
        assert s1_ == engs[0].get_adam(t)[2] == st.step[t] == 5
        params_close(m1, st.m[t], 5e-3, atol=1e-7)
        rel_close(engs[1].get_w(t)[0], st.w[t], rtol=1e-5, atol=1e-7)
    assert len(ties) < T
    for eng in engs:
        eng.close()
