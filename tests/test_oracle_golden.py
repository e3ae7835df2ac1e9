"""Pin the CPU oracle (oracle/ref_cpu.py) against golden vectors from the real reference.

CPU only.  The fixtures come from tools/gen_golden.py, which runs the reference's own
sfdqn.py / features/deep.py / tsfdqn.py / tsfdqn_nf.py code in the build container.
"""
import numpy as np
import pytest
import torch

from oracle import ref_cpu as R

GPI_CASES = ["reacher17", "hopper11", "cartpole", "refreacher", "tanh_odd", "tie"]


def spec_of(g):
    return R.Spec(int(g["n_s"]), int(g["H"]), int(g["A"]), int(g["d"]), tuple(str(a) for a in g["acts"]))


def close(a, b, rtol=1e-5, atol=1e-6):
    np.testing.assert_allclose(np.asarray(a), np.asarray(b), rtol=rtol, atol=atol)


@pytest.mark.parametrize("case", GPI_CASES)
def test_gpi_matches_reference(golden, case):
    g = golden("gpi_" + case)
    spec = spec_of(g)
    online = torch.from_numpy(g["online"])
    w = torch.from_numpy(g["w"])
    assert online.shape[1] == spec.P
    for B, S in ((1, g["S1"]), (32, g["S32"])):
        S = torch.from_numpy(S)
        psi = R.psi_all(online, spec, S)
        close(psi, g[f"psi{B}"])
        for i in range(int(g["T"])):
            q, task = R.gpi_w(psi, w[i])
            close(q, g[f"q{B}_{i}"])
            assert np.array_equal(task.numpy().reshape(-1), np.asarray(g[f"task{B}_{i}"]).reshape(-1))
            if B == 32:
                assert np.array_equal(R.gpi_next_actions(q).numpy(), g[f"next32_{i}"])


def test_tie_breaks_to_first_index(golden):
    g = golden("gpi_tie")
    # head 2 is an exact copy of head 0, so task 2 can never be chosen over task 0
    for i in range(int(g["T"])):
        assert 2 not in np.asarray(g[f"task32_{i}"]).reshape(-1)


def test_full_size_recipe_and_outputs(golden):
    from tests.golden.recipe import full_size_heads

    g = golden("gpi_reacher17_full")
    online, w = full_size_heads()
    assert abs(float(online.double().sum()) - float(g["online_sum"])) < 1e-6
    spec = spec_of(g)
    psi = R.psi_all(online, spec, torch.from_numpy(g["S32"]))
    close(psi, g["psi32"], rtol=1e-4, atol=1e-6)
    for i in range(int(g["T"])):
        q, task = R.gpi_w(psi, w[i])
        close(q, g[f"q32_{i}"], rtol=1e-4, atol=1e-6)
        assert np.array_equal(task.numpy(), g[f"task32_{i}"])


def batches_of(g):
    k = int(g["k"])
    out = []
    for j in range(k):
        out.append(tuple(torch.from_numpy(g["b_" + n][j]) for n in ("s", "a", "r", "phi", "s1", "gamma")))
    return out


@pytest.mark.parametrize("case", ["sfdqn_gpi", "sfdqn_nogpi", "sfdqn_tanh"])
def test_sf_update_matches_reference(golden, case):
    g = golden("upd_" + case)
    spec = spec_of(g)
    st = R.SFState(spec, torch.from_numpy(g["online0"]).clone(), torch.from_numpy(g["target0"]).clone(),
                   torch.from_numpy(g["w0"]).clone())
    for j, b in enumerate(batches_of(g)):
        i = int(g["policies"][j])
        loss, l1, l2, na = R.sf_update(st, b, i, use_gpi=bool(g["use_gpi"]),
                                       target_update_ev=int(g["target_update_ev"]))
        assert np.array_equal(na.numpy(), g["next_actions"][j])
        close([float(loss), float(l1), float(l2)], g["losses"][j], rtol=1e-5, atol=1e-7)
        if j == 0:
            close(st.online, g["online1"])
            close(st.w, g["w1"])
    close(st.online, g["online"], rtol=1e-4, atol=1e-6)
    close(st.target, g["target"], rtol=1e-4, atol=1e-6)
    close(st.w, g["w"], rtol=1e-4, atol=1e-6)
    close(st.m, g["m"], rtol=1e-4, atol=1e-8)
    close(st.v, g["v"], rtol=1e-4, atol=1e-10)
    assert list(st.step) == list(g["steps"])
    assert list(st.since_target) == list(g["since_target"])


def test_deep_all_task_matches_reference(golden):
    g = golden("upd_deep_alltask")
    spec = spec_of(g)
    online0 = torch.from_numpy(g["online0"])
    st = R.SFState(spec, online0.clone(), online0.clone(), torch.from_numpy(g["w0"]).clone())
    for j, b in enumerate(batches_of(g)):
        t = int(g["lms_task"][j])
        st.w[t] = R.lms_update(st.w[t].reshape(-1, 1), torch.from_numpy(g["lms_phi"][j]),
                               torch.tensor(g["lms_r"][j]), float(g["alpha_w"])).reshape(-1)
        s, a, r, phi, s1, gamma = b
        R.deep_all_task_step(st, (s, a, phi, s1, gamma), target_update_ev=int(g["target_update_ev"]))
        if j == 0:
            close(st.online, g["online1"])
    close(st.w, g["w"], rtol=1e-5, atol=1e-7)
    close(st.online, g["online"], rtol=1e-4, atol=1e-6)
    close(st.target, g["target"], rtol=1e-4, atol=1e-6)
    close(st.m, g["m"], rtol=1e-4, atol=1e-8)
    close(st.v, g["v"], rtol=1e-4, atol=1e-10)
    assert list(st.since_target) == list(g["since_target"])


@pytest.mark.parametrize("case", ["tsf", "tsf_nf"])
def test_tsf_update_matches_reference(golden, case):
    g = golden("upd_" + case)
    spec = spec_of(g)
    T = int(g["T"])
    gs = R.GSpec(spec.n_s, int(g["G"]), int(g["K"]))
    online0 = torch.from_numpy(g["online0"])
    st = R.TSFState(spec, online0.clone(), online0.clone(), torch.from_numpy(g["w0"]).clone(),
                    gspec=gs, g=torch.from_numpy(g["g0"]).clone(), h=torch.from_numpy(g["h0"]).clone())
    assert st.g.shape == (T, gs.P)
    for j, b in enumerate(batches_of(g)):
        i = int(g["policies"][j])
        loss, l1, l2, _ = R.tsf_update(st, b, i, beta=float(g["beta"]),
                                       target_update_ev=int(g["target_update_ev"]))
        close([float(loss), float(l1), float(l2)], g["losses"][j], rtol=1e-5, atol=1e-7)
    close(st.online, g["online"], rtol=1e-4, atol=1e-6)
    close(st.target, g["target"], rtol=1e-4, atol=1e-6)
    close(st.w, g["w"], rtol=1e-4, atol=1e-6)
    close(st.g, g["g"], rtol=1e-4, atol=1e-6)
    close(st.h, g["h"], rtol=1e-4, atol=1e-6)


def tsf_test_problem(g):
    """The oracle state of a test_tsf* fixture (tools/gen_golden.py gen_tsf_test)."""
    spec = spec_of(g)
    gs = R.GSpec(spec.n_s, int(g["G"]), int(g["K"]))
    T = int(g["T"])
    st = R.TSFState(spec, torch.from_numpy(g["online"]).clone(), torch.from_numpy(g["target"]).clone(),
                    torch.zeros(T, spec.d), gspec=gs, g=torch.from_numpy(g["g"]).clone(),
                    h=torch.from_numpy(g["h"]).clone())
    tm = R.TestMapper(torch.from_numpy(g["w0"]).clone(), torch.from_numpy(g["omega0"]).clone())
    return st, tm


def tsf_test_hyper(g, j):
    return dict(gamma=float(g["gamma"]), beta=float(g["beta"]), lasso=float(g["lasso"]), lr_w=float(g["lr_w"]),
                wd_w=float(g["wd_w"]), lr_o=float(g["lr_o"][j]), wd_o=float(g["wd_o"]))


@pytest.mark.parametrize("case", ["tsf", "tsf_nf"])
def test_tsf_test_path_matches_reference(golden, case):
    """TSFDQN.get_test_action (greedy) and update_test_reward_mapper (tsfdqn.py:859-997) over 10
    steps with the ω learning rate decaying: actions exact, losses, w and ω per step."""
    g = golden("test_" + case)
    st, tm = tsf_test_problem(g)
    for j in range(int(g["k"])):
        s, s1 = torch.from_numpy(g["s"][j]), torch.from_numpy(g["s1"][j])
        assert R.tsf_test_action(st, s, tm.w, tm.omega) == int(g["greedy"][j])
        loss, l2, l1 = R.tsf_test_update(st, tm, s, int(g["a"][j]), float(g["r"][j]), torch.from_numpy(g["phi"][j]),
                                         s1, int(g["a1"][j]), **tsf_test_hyper(g, j))
        close([loss, l2, l1], [g["loss"][j], g["l2"][j], g["l1"][j]], rtol=1e-5, atol=1e-8)
        close(tm.w, g["w"][j], rtol=1e-5, atol=1e-8)
        close(tm.omega, g["omega"][j], rtol=1e-5, atol=1e-8)


def phi_problem(g):
    """The oracle state of an upd_phi* fixture (tools/gen_golden.py gen_phi)."""
    spec = spec_of(g)
    T = int(g["T"])
    online0 = torch.from_numpy(g["online0"])
    st = R.PhiState(spec, R.PhiSpec(spec.n_s, spec.d), online0.clone(), online0.clone(),
                    torch.from_numpy(g["w0"]).clone(), torch.from_numpy(g["wb0"]).clone(),
                    torch.from_numpy(g["phi0"]).clone(), torch.ones(T))
    return st


def phi_batches(g):
    return [tuple(torch.from_numpy(g[f"b_{n}"][j]) for n in ("s", "a", "r", "phi", "s1", "gamma"))
            for j in range(int(g["k"]))]


@pytest.mark.parametrize("case", ["phi_gpi", "phi_nogpi"])
def test_phi_update_matches_reference(golden, case):
    """features/deep_phi.py DeepSF_PHI.update_successor (learned φ): losses, the
    loss coefficient, ψ online / target, w (with bias) and the φ net after k updates."""
    g = golden("upd_" + case)
    st = phi_problem(g)
    assert st.phi.numel() == st.pspec.P
    for j, b in enumerate(phi_batches(g)):
        loss, psi_loss, phi_loss, lam, _ = R.phi_update(st, b, int(g["policies"][j]), use_gpi=bool(g["use_gpi"]),
                                                        target_update_ev=int(g["target_update_ev"]))
        close([loss, psi_loss, phi_loss, lam], g["losses"][j], rtol=1e-5, atol=1e-8)
    close(st.online, g["online"], rtol=1e-4, atol=1e-6)
    close(st.target, g["target"], rtol=1e-4, atol=1e-6)
    close(st.w, g["w"], rtol=1e-4, atol=1e-6)
    close(st.wb, g["wb"], rtol=1e-4, atol=1e-6)
    close(st.phi, g["phi"], rtol=1e-4, atol=1e-6)
    close(st.lam, g["lam"], rtol=1e-6)


def test_huber_td_grad_closed_form():
    """The oracle's opt-in Huber (td_grad(huber=δ); not in the reference, SURVEY F3 -- parity
    unpinned by the reference, pinned here to the closed form the kernels implement): gradient
    (1/N) clamp(c - t, -δ, δ) at the taken actions, 0 elsewhere; loss mean of 0.5 x² (|x| < δ) or
    δ(|x| - 0.5 δ); and for δ past every error, half the MSE gradient."""
    gen = torch.Generator().manual_seed(3)
    B, A, d, delta = 16, 5, 4, 0.3
    c = torch.randn(B, A, d, generator=gen)
    a = torch.randint(0, A, (B,), generator=gen)
    t = torch.randn(B, d, generator=gen)
    l1, g = R.td_grad(c, a, t, huber=delta)
    N = c.numel()
    x = c[torch.arange(B), a] - t
    assert (x.abs() > delta).any() and (x.abs() < delta).any()
    want = torch.zeros_like(c)
    want[torch.arange(B), a] = torch.where(x < -delta, -(1.0 / N) * delta,
                                           torch.where(x > delta, (1.0 / N) * delta, (1.0 / N) * x))
    torch.testing.assert_close(g, want, rtol=0, atol=1e-9)
    z = x.abs()
    lw = torch.where(z < delta, 0.5 * z * z, delta * (z - 0.5 * delta)).sum() / N
    torch.testing.assert_close(l1, lw, rtol=1e-6, atol=0)
    _, gm = R.td_grad(c, a, t)
    _, gh = R.td_grad(c, a, t, huber=1e3)
    torch.testing.assert_close(gh, 0.5 * gm, rtol=1e-6, atol=1e-9)
