"""CPU tests of sfx.checkpoint (SURVEY.md §5 checkpoint / resume): the exported heads load into the
reference's ψ Sequential (main_sfdqn_torch.py:44-78) and its torch.optim.Adam exactly, the optimizer
continues from the restored state bit for bit, and save -> load(weights_only=True) restores every
field.  The engine is a host stand-in with SFEngine's state-I/O methods (the GPU round trip is in
tests/test_gpu_checkpoint.py)."""
import torch

from sfx import checkpoint as ck
from sfx.init import flatten, psi_module

N_S, H, A, D, ACTS = 17, 32, 7, 8, ("relu", "relu")


class HostEngine:
    """SFEngine's state-I/O surface over host tensors."""

    def __init__(self, T):
        self.T, self.T_glob, self.n_s, self.H, self.A, self.d, self.acts = T, T, N_S, H, A, D, ACTS
        self.P = flatten(psi_module(N_S, H, A, D, ACTS)).numel()
        self.heads = torch.zeros(T, 2, self.P)
        self.m, self.v = torch.zeros(T, self.P), torch.zeros(T, self.P)
        self.step, self.since = [0] * T, [0] * T
        self.w, self.wm, self.wv = torch.zeros(T, D), torch.zeros(T, D), torch.zeros(T, D)
        self.adam_hp = dict(lr_psi=1e-3, wd_psi=0.0, lr_w=1e-3, wd_w=0.0, betas=(0.9, 0.999), eps=1e-8)

    def set_adam(self, lr_psi, wd_psi, lr_w, wd_w, betas, eps):
        self.adam_hp = dict(lr_psi=lr_psi, wd_psi=wd_psi, lr_w=lr_w, wd_w=wd_w, betas=tuple(betas), eps=eps)

    def load_head(self, t, flat, which=0):
        self.heads[t, which] = torch.as_tensor(flat).reshape(-1)

    def get_head(self, t, which=0):
        return self.heads[t, which].clone()

    def load_adam(self, t, m, v, step):
        self.m[t], self.v[t], self.step[t] = torch.as_tensor(m).reshape(-1), torch.as_tensor(v).reshape(-1), step

    def get_adam(self, t):
        return self.m[t].clone(), self.v[t].clone(), self.step[t]

    def since_target(self, t):
        return self.since[t]

    def set_since_target(self, t, c):
        self.since[t] = c

    def get_w(self, t):
        return self.w[t].clone(), self.wm[t].clone(), self.wv[t].clone()

    def load_w_state(self, t, w, wm, wv):
        self.w[t], self.wm[t], self.wv[t] = torch.as_tensor(w), torch.as_tensor(wm), torch.as_tensor(wv)


def _trained_reference(seed, steps):
    """A ψ head and its Adam after `steps` updates with seeded gradients (the reference's objects)."""
    torch.manual_seed(seed)
    model = psi_module(N_S, H, A, D, ACTS)
    opt = torch.optim.Adam(model.parameters(), lr=1e-3)
    for _ in range(steps):
        opt.zero_grad()
        model(torch.randn(16, N_S)).pow(2).mean().backward()
        opt.step()
    return model, opt


def _engine_from(models_opts):
    eng = HostEngine(len(models_opts))
    for t, (model, opt) in enumerate(models_opts):
        eng.load_head(t, flatten(model), 0)
        eng.load_head(t, flatten(model) * 0.5, 1)
        st = [opt.state[p] for p in model.parameters()]
        if st and st[0]:
            eng.load_adam(t, torch.cat([s["exp_avg"].reshape(-1) for s in st]),
                          torch.cat([s["exp_avg_sq"].reshape(-1) for s in st]), int(st[0]["step"]))
        eng.set_since_target(t, 3 * t + 1)
        eng.load_w_state(t, torch.rand(D), torch.rand(D), torch.rand(D))
    return eng


def test_heads_load_into_the_reference_module_and_adam():
    pairs = [_trained_reference(1, 5), _trained_reference(2, 0)]
    eng = _engine_from(pairs)
    sd = ck.state_dict(eng)
    for t, (model, opt) in enumerate(pairs):
        fresh = psi_module(N_S, H, A, D, ACTS)
        fresh.load_state_dict(sd["heads"][t]["model"])  # strict: the reference's key names
        for a, b in zip(fresh.parameters(), model.parameters()):
            assert torch.equal(a, b)
        fopt = torch.optim.Adam(fresh.parameters(), lr=1e-3)
        fopt.load_state_dict(sd["heads"][t]["optim"])
        # one more identical step from the restored optimizer and from the original: bit for bit
        x = torch.randn(16, N_S, generator=torch.Generator().manual_seed(9))
        for mm, oo in ((model, opt), (fresh, fopt)):
            oo.zero_grad()
            mm(x).pow(2).mean().backward()
            oo.step()
        for a, b in zip(fresh.parameters(), model.parameters()):
            assert torch.equal(a, b)
    assert sd["heads"][1]["optim"]["state"] == {}  # no Adam state before the first step, as torch


def test_save_load_round_trip(tmp_path):
    eng = _engine_from([_trained_reference(3, 4), _trained_reference(4, 2), _trained_reference(5, 1)])
    eng.set_adam(2e-3, 1e-4, 5e-3, 0.01, (0.8, 0.99), 1e-6)
    path = tmp_path / "sfx.pt"
    ck.save(eng, str(path))
    other = HostEngine(3)
    ck.load(other, str(path))  # torch.load(weights_only=True)
    assert torch.equal(other.heads, eng.heads)
    assert torch.equal(other.m, eng.m) and torch.equal(other.v, eng.v) and other.step == eng.step
    assert other.since == eng.since
    assert torch.equal(other.w, eng.w) and torch.equal(other.wm, eng.wm) and torch.equal(other.wv, eng.wv)
    assert other.adam_hp == dict(lr_psi=2e-3, wd_psi=1e-4, lr_w=5e-3, wd_w=0.01, betas=(0.8, 0.99), eps=1e-6)


def test_geometry_mismatch_is_refused():
    sd = ck.state_dict(_engine_from([_trained_reference(6, 1)]))
    other = HostEngine(1)
    other.acts = ("relu", "tanh")
    try:
        ck.load_state_dict(other, sd)
    except ValueError as e:
        assert "geometry" in str(e)
    else:
        raise AssertionError("a checkpoint of another geometry loaded")
