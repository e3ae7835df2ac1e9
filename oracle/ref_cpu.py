"""CPU restatement of the reference successor-feature hot path (fp32, PyTorch-CPU).

TEST INFRASTRUCTURE ONLY.  Nothing in the product path (the ``sfx`` package,
``libsfx.so``) imports, calls or links this module.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg use it, and
only as the checker / the timed CPU baseline.

Parity status: PINNED.  ``tests/test_oracle_golden.py`` checks every function
here against golden vectors produced by importing the real reference in the
build container (``tools/gen_golden.py`` -> ``tests/golden/*.npz``).

Each function cites the reference code (paths relative to
``/root/reference/source``) whose behaviour it restates.  The restatement uses
the same ATen primitives the reference reaches through ``nn.Linear`` / autograd /
``torch.optim.Adam`` (single-tensor CPU path), so on CPU it agrees with the
reference to the last few ulps; the HIP kernels are then checked against it.

Parameter packing (shared with the HIP library, see include/sfx.h): one ψ head
is a flat fp32 vector holding, for each Linear in ``nn.Sequential`` order,
``weight[out, in]`` (row-major) followed by ``bias[out]`` -- exactly the order
of ``model.parameters()`` for the reference's ψ lambda
(main_sfdqn_torch.py:44-78).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import List, Sequence, Tuple

import torch
import torch.nn.functional as F

ACT_NONE, ACT_RELU, ACT_TANH = 0, 1, 2
_ACT_CODES = {"none": ACT_NONE, "relu": ACT_RELU, "tanh": ACT_TANH}


# --------------------------------------------------------------------------------------
# ψ head geometry
# --------------------------------------------------------------------------------------
@dataclass
class Spec:
    """Geometry of one ψ head.

    main_sfdqn_torch.py:57-71: Linear(n_s, H) with NO activation, then one
    Linear(H, H)+act per entry of ``model_params['n_neurons']``, then
    Linear(H, A*d) and Unflatten(1, (A, d)).
    """

    n_s: int
    H: int
    A: int
    d: int
    acts: Tuple[str, ...] = ("relu", "relu")

    @property
    def n_hidden(self) -> int:
        return len(self.acts)

    @property
    def layers(self) -> List[Tuple[int, int]]:
        """(out, in) per Linear, in parameters() order."""
        return [(self.H, self.n_s)] + [(self.H, self.H)] * self.n_hidden + [(self.A * self.d, self.H)]

    @property
    def layer_acts(self) -> List[int]:
        """Activation applied to the OUTPUT of each Linear."""
        return [ACT_NONE] + [_ACT_CODES[a] for a in self.acts] + [ACT_NONE]

    @property
    def P(self) -> int:
        return sum(o * i + o for o, i in self.layers)


def unpack(flat: torch.Tensor, spec: Spec) -> List[Tuple[torch.Tensor, torch.Tensor]]:
    """Views (W[out,in], b[out]) into a packed head vector."""
    out, off = [], 0
    for o, i in spec.layers:
        W = flat[off:off + o * i].view(o, i)
        off += o * i
        b = flat[off:off + o]
        off += o
        out.append((W, b))
    assert off == spec.P
    return out


def _act(x: torch.Tensor, code: int) -> torch.Tensor:
    if code == ACT_RELU:
        return torch.relu(x)
    if code == ACT_TANH:
        return torch.tanh(x)
    return x


def _act_backward(grad: torch.Tensor, y: torch.Tensor, code: int) -> torch.Tensor:
    """Derivative expressed through the activation OUTPUT y (ReLU: y>0; tanh: 1-y^2),
    as ATen's threshold_backward / tanh_backward do."""
    if code == ACT_RELU:
        return grad * (y > 0).to(grad.dtype)
    if code == ACT_TANH:
        return grad * (1 - y * y)
    return grad


def forward(flat: torch.Tensor, spec: Spec, X: torch.Tensor):
    """ψ(X) for one head -> ([B, A, d], saved layer inputs).

    Restates ``psi(state)`` of sfdqn.py:290-293 / features/deep.py:80-83 over the
    Sequential built at main_sfdqn_torch.py:44-78."""
    xs = []
    h = X
    for (W, b), code in zip(unpack(flat, spec), spec.layer_acts):
        xs.append(h)
        h = _act(F.linear(h, W, b), code)
    xs.append(h)
    return h.view(X.shape[0], spec.A, spec.d), xs


def backward(flat: torch.Tensor, spec: Spec, xs: List[torch.Tensor], dY: torch.Tensor) -> torch.Tensor:
    """Gradient of the packed head parameters for output gradient dY [B, A, d]
    (what autograd computes through addmm / relu / tanh for the same graph)."""
    params = unpack(flat, spec)
    acts = spec.layer_acts
    grads = [None] * len(params)
    dZ = dY.reshape(dY.shape[0], -1)
    for l in range(len(params) - 1, -1, -1):
        W, _ = params[l]
        grads[l] = (dZ.t().mm(xs[l]), dZ.sum(0))
        if l > 0:
            dX = dZ.mm(W)
            dZ = _act_backward(dX, xs[l], acts[l - 1])
    return torch.cat([torch.cat([gw.reshape(-1), gb]) for gw, gb in grads])


# --------------------------------------------------------------------------------------
# Adam (torch 2.10 single-tensor CPU path, torch/optim/adam.py:_single_tensor_adam)
# --------------------------------------------------------------------------------------
def adam_(p: torch.Tensor, g: torch.Tensor, m: torch.Tensor, v: torch.Tensor, step: int,
          lr: float, betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 0.0) -> None:
    """In-place Adam step number ``step`` (1-based) on p with moments m, v.

    Restates /usr/local/lib/python3.10/dist-packages/torch/optim/adam.py:457,476,531-547
    as reached from sfdqn.py:362 / features/deep.py:123 / tsfdqn.py:700."""
    b1, b2 = betas
    if weight_decay != 0:
        g = g.add(p, alpha=weight_decay)
    m.lerp_(g, 1 - b1)
    v.mul_(b2).addcmul_(g, g, value=1 - b2)
    bc1 = 1 - b1 ** step
    bc2 = 1 - b2 ** step
    denom = (v.sqrt() / (bc2 ** 0.5)).add_(eps)
    p.addcdiv_(m, denom, value=-(lr / bc1))


# --------------------------------------------------------------------------------------
# GPI
# --------------------------------------------------------------------------------------
def psi_all(online: torch.Tensor, spec: Spec, S: torch.Tensor) -> torch.Tensor:
    """get_successors: stack of every head's ψ on axis 1 -> [B, T, A, d]
    (sfdqn.py:295-301, features/deep.py:85-91)."""
    return torch.stack([forward(online[t], spec, S)[0] for t in range(online.shape[0])], dim=1)


def gpi_w(psi: torch.Tensor, w: torch.Tensor):
    """GPI_w (features/successor.py:223-246; sfdqn.py:215-240).

    q[b,t,a] = ψ[b,t,a,:]·w ; task[b] = argmax_t max_a q[b,t,a] (first index on ties).
    Returns task with shape [B] (the reference squeezes it to 0-d at B=1)."""
    q = torch.matmul(psi, w.reshape(-1, 1))[..., 0]
    task = torch.argmax(torch.max(q, dim=2).values, dim=1)
    return q, task


def gpi_next_actions(q: torch.Tensor) -> torch.Tensor:
    """Next action in the TD target: argmax_a max_t q[b,t,a] (sfdqn.py:316; features/deep.py:103)."""
    return torch.argmax(torch.max(q, dim=1).values, dim=-1)


def select_action(q: torch.Tensor, task, task_index: int, use_gpi: bool) -> int:
    """Greedy branch of action selection (sfdqn.py:585-594; agents/sfdqn.py:39-45 + agent.py:152)."""
    c = int(task) if use_gpi else task_index
    return int(torch.argmax(q[0, c, :]))


def lms_update(w: torch.Tensor, phi: torch.Tensor, r, alpha: float) -> torch.Tensor:
    """SF.update_reward (features/successor.py:164-167): w + α (r - φ·w) φ, w shaped [d, 1]."""
    phi = phi.reshape(w.shape)
    r_fit = torch.sum(phi * w)
    return w + alpha * (r - r_fit) * phi


# --------------------------------------------------------------------------------------
# SF state and the TD update (sfdqn.py / features/deep_sequential.py semantics)
# --------------------------------------------------------------------------------------
@dataclass
class SFState:
    spec: Spec
    online: torch.Tensor          # [T, P]
    target: torch.Tensor          # [T, P]
    w: torch.Tensor               # [T, d]  (Linear(d,1,bias=False).weight rows) or LMS w
    m: torch.Tensor = None        # [T, P] Adam first moment of ψ
    v: torch.Tensor = None
    wm: torch.Tensor = None       # [T, d] Adam moments of w (sfdqn.py param group 2)
    wv: torch.Tensor = None
    step: List[int] = field(default_factory=list)
    since_target: List[int] = field(default_factory=list)

    def __post_init__(self):
        T = self.online.shape[0]
        if self.m is None:
            self.m = torch.zeros_like(self.online)
            self.v = torch.zeros_like(self.online)
        if self.wm is None:
            self.wm = torch.zeros_like(self.w)
            self.wv = torch.zeros_like(self.w)
        if not self.step:
            self.step = [0] * T
        if not self.since_target:
            self.since_target = [0] * T

    @property
    def T(self) -> int:
        return self.online.shape[0]

    def clone(self) -> "SFState":
        return SFState(self.spec, self.online.clone(), self.target.clone(), self.w.clone(),
                       self.m.clone(), self.v.clone(), self.wm.clone(), self.wv.clone(),
                       list(self.step), list(self.since_target))


def td_grad(c: torch.Tensor, actions: torch.Tensor, targets: torch.Tensor, huber: float = 0.0):
    """MSE(c, merged) with merged = clone(c); merged[b, a_b] = t_b (sfdqn.py:334-341).

    Returns (l1, dL1/dc).  Only the (b, a_b) rows differ, so the gradient is
    2 (c - t)/(B*A*d) there and 0 elsewhere.  huber > 0: the opt-in HuberLoss(delta=huber)
    instead (not in the reference) -- torch's own loss and autograd gradient."""
    B = c.shape[0]
    idx = torch.arange(B)
    merged = c.clone()
    merged[idx, actions, :] = targets
    if huber > 0:
        cc = c.detach().clone().requires_grad_(True)
        l1 = F.huber_loss(cc, merged.detach(), delta=huber)
        (g,) = torch.autograd.grad(l1, cc)
        return l1.detach(), g
    l1 = F.mse_loss(c, merged)
    g = torch.zeros_like(c)
    g[idx, actions, :] = (2.0 / c.numel()) * (c[idx, actions, :] - targets)
    return l1, g


def sf_update(st: SFState, batch, i: int, *, use_gpi: bool = True, lr_sf: float = 1e-3,
              lr_w: float = 1e-3, wd_sf: float = 0.0, wd_w: float = 0.0,
              target_update_ev: int = 1000, train_w: bool = True, huber: float = 0.0):
    """DeepSF.update_successor of sfdqn.py:303-371 (== features/deep_sequential.py:163-231).

    batch = (s [B,n_s], a [B] int64, r [B,1], phi [B,d], s1 [B,n_s], gamma [B]).
    Mutates st; returns (loss, l1, l2, next_actions)."""
    s, a, r, phi, s1, gamma = batch
    spec = st.spec
    gamma = gamma.reshape(-1, 1)
    B = s.shape[0]
    idx = torch.arange(B)
    w_i = st.w[i]
    if use_gpi:
        q1, _ = gpi_w(psi_all(st.online, spec, s1), w_i)
        next_actions = gpi_next_actions(q1)
    else:
        q1 = torch.matmul(forward(st.online[i], spec, s1)[0], w_i.reshape(-1, 1))
        next_actions = torch.argmax(q1, dim=1)[:, 0]
    c, xs = forward(st.online[i], spec, s)
    tpsi, _ = forward(st.target[i], spec, s1)
    targets = phi + gamma * tpsi[idx, next_actions, :]
    l1, gc = td_grad(c, a, targets, huber)
    r_fit = F.linear(phi, w_i.reshape(1, -1))
    l2 = F.mse_loss(r_fit, r)
    g_psi = backward(st.online[i], spec, xs, gc)
    g_w = ((2.0 / B) * (r_fit - r)).t().mm(phi).reshape(-1)
    st.step[i] += 1
    adam_(st.online[i], g_psi, st.m[i], st.v[i], st.step[i], lr_sf, weight_decay=wd_sf)
    if train_w:
        adam_(st.w[i], g_w, st.wm[i], st.wv[i], st.step[i], lr_w, weight_decay=wd_w)
    st.since_target[i] += 1
    if st.since_target[i] >= target_update_ev:
        st.target[i].copy_(st.online[i])
        st.since_target[i] = 0
    return l1 + l2, l1, l2, next_actions


def deep_update(st: SFState, batch, i: int, *, lr: float = 1e-3, target_update_ev: int = 1000, huber: float = 0.0):
    """features/deep.py:93-131 (the main_sfdqn_torch.py path): GPI next actions always,
    loss = l1 only, Adam over ψ_i only (the lambda's optimizer), w_i = LMS w [d].

    batch = (s, a, phi, s1, gamma) (agents/buffer.py:34-60 layout)."""
    s, a, phi, s1, gamma = batch
    spec = st.spec
    gamma = gamma.reshape(-1, 1)
    B = s.shape[0]
    idx = torch.arange(B)
    q1, _ = gpi_w(psi_all(st.online, spec, s1), st.w[i])
    next_actions = gpi_next_actions(q1)
    c, xs = forward(st.online[i], spec, s)
    tpsi, _ = forward(st.target[i], spec, s1)
    targets = phi + gamma * tpsi[idx, next_actions, :]
    l1, gc = td_grad(c, a, targets, huber)
    g_psi = backward(st.online[i], spec, xs, gc)
    st.step[i] += 1
    adam_(st.online[i], g_psi, st.m[i], st.v[i], st.step[i], lr)
    st.since_target[i] += 1
    if st.since_target[i] >= target_update_ev:
        st.target[i].copy_(st.online[i])
        st.since_target[i] = 0
    return l1, next_actions


def deep_all_task_step(st: SFState, batch, *, lr: float = 1e-3, target_update_ev: int = 1000, huber: float = 0.0):
    """agents/sfdqn.py:57-60: every head updated on the same minibatch, in index order
    (each GPI sees the heads already updated earlier in the same step)."""
    return [deep_update(st, batch, i, lr=lr, target_update_ev=target_update_ev, huber=huber) for i in range(st.T)]


# --------------------------------------------------------------------------------------
# TSF (tsfdqn.py:588-709; tsfdqn_nf.py with PlanarFlow g)
# --------------------------------------------------------------------------------------
@dataclass
class GSpec:
    """g_i : R^{n_s} -> R^{G}.  K planar layers (tsfdqn_nf.py:331-358) then Linear(n_s, G);
    K = 0 is the plain tsfdqn.py g (Linear(n_s, G), tsfdqn.py:537-546)."""

    n_s: int
    G: int
    K: int = 0

    @property
    def P(self) -> int:
        return self.K * (2 * self.n_s + 1) + self.G * self.n_s + self.G


def g_unpack(flat: torch.Tensor, gs: GSpec):
    """Planar layer k: weight[1,n_s], bias[1], scale[1,n_s] (registration order of
    tsfdqn_nf.py:335-337); then Linear weight[G,n_s], bias[G]."""
    off, flows = 0, []
    for _ in range(gs.K):
        wk = flat[off:off + gs.n_s].view(1, gs.n_s); off += gs.n_s
        bk = flat[off:off + 1]; off += 1
        uk = flat[off:off + gs.n_s].view(1, gs.n_s); off += gs.n_s
        flows.append((wk, bk, uk))
    W = flat[off:off + gs.G * gs.n_s].view(gs.G, gs.n_s); off += gs.G * gs.n_s
    b = flat[off:off + gs.G]; off += gs.G
    return flows, (W, b)


def g_forward(flat, gs: GSpec, X):
    flows, (W, b) = g_unpack(flat, gs)
    zs, ts = [], []
    z = X
    for wk, bk, uk in flows:
        zs.append(z)
        t = torch.tanh(F.linear(z, wk, bk))
        ts.append(t)
        z = z + uk * t
    zs.append(z)
    return F.linear(z, W, b), (zs, ts)


def g_backward(flat, gs: GSpec, saved, dY):
    flows, (W, b) = g_unpack(flat, gs)
    zs, ts = saved
    dW = dY.t().mm(zs[-1])
    db = dY.sum(0)
    dz = dY.mm(W)
    gflows = []
    for k in range(gs.K - 1, -1, -1):
        wk, bk, uk = flows[k]
        t = ts[k]
        du = (dz * t).sum(0, keepdim=True)
        da = (dz * uk).sum(1, keepdim=True) * (1 - t * t)
        dw = da.t().mm(zs[k])
        dbk = da.sum(0)
        dz = dz + da.mm(wk)
        gflows.append((dw, dbk, du))
    gflows.reverse()
    parts = []
    for dw, dbk, du in gflows:
        parts += [dw.reshape(-1), dbk.reshape(-1), du.reshape(-1)]
    parts += [dW.reshape(-1), db]
    return torch.cat(parts)


@dataclass
class TSFState(SFState):
    gspec: GSpec = None
    g: torch.Tensor = None        # [T, Pg]
    gm: torch.Tensor = None
    gv: torch.Tensor = None
    h: torch.Tensor = None        # [Ph] = Linear(G, d): weight [d, G] then bias [d]; shared
    hm: torch.Tensor = None       # [T, Ph]: each task's optimizer keeps its own h moments
    hv: torch.Tensor = None

    def __post_init__(self):
        super().__post_init__()
        T = self.online.shape[0]
        if self.gm is None:
            self.gm = torch.zeros_like(self.g)
            self.gv = torch.zeros_like(self.g)
        if self.hm is None:
            self.hm = torch.zeros(T, self.h.numel())
            self.hv = torch.zeros(T, self.h.numel())


def tsf_update(st: TSFState, batch, i: int, *, use_gpi: bool = True, beta: float = 1.0,
               lr_sf=1e-3, lr_w=1e-3, lr_g=1e-3, lr_h=1e-3, target_update_ev: int = 1000, next_actions=None):
    """TSFDQN.update_successor (tsfdqn.py:588-709; tsfdqn_nf.py identical with planar g).

    φ̃ = (h(g_i(s)) + h(g_i(s1))) ⊙ φ ; targets = φ̃ + γ ψ⁻_i(s1)[a'] carry gradient into g_i, h;
    loss = l1 + β l2 with l2 = MSE(w_i(φ̃), r); one Adam over {ψ_i, w_i, g_i, h}."""
    s, a, r, phi, s1, gamma = batch
    spec, gs = st.spec, st.gspec
    d = spec.d
    gamma = gamma.reshape(-1, 1)
    B = s.shape[0]
    idx = torch.arange(B)
    w_i = st.w[i]
    with torch.no_grad():
        if next_actions is not None:  # given (sharded heads: from the all-reduced GPI maxima)
            pass
        elif use_gpi:
            q1, _ = gpi_w(psi_all(st.online, spec, s1), w_i)
            next_actions = gpi_next_actions(q1)
        else:
            q1 = torch.matmul(forward(st.online[i], spec, s1)[0], w_i.reshape(-1, 1))
            next_actions = torch.argmax(q1, dim=1)[:, 0]
    c, xs = forward(st.online[i], spec, s)
    Wh = st.h[:d * gs.G].view(d, gs.G)
    bh = st.h[d * gs.G:]
    gs_s, sv_s = g_forward(st.g[i], gs, s)
    gs_s1, sv_s1 = g_forward(st.g[i], gs, s1)
    aff = F.linear(gs_s, Wh, bh) + F.linear(gs_s1, Wh, bh)
    tphi = aff * phi
    tpsi, _ = forward(st.target[i], spec, s1)
    targets = tphi + gamma * tpsi[idx, next_actions, :]
    l1, gc = td_grad(c, a, targets)
    r_fit = F.linear(tphi, w_i.reshape(1, -1))
    l2 = F.mse_loss(r_fit, r)
    loss = l1 + beta * l2
    # gradients
    g_psi = backward(st.online[i], spec, xs, gc)
    dr = beta * (2.0 / B) * (r_fit - r)                   # [B,1]
    g_w = dr.t().mm(tphi).reshape(-1)
    dtphi = -gc[idx, a, :] + dr.mm(w_i.reshape(1, -1))    # via targets (l1) and r_fit (l2)
    daff = dtphi * phi
    g_Wh = daff.t().mm(gs_s) + daff.t().mm(gs_s1)
    g_bh = 2 * daff.sum(0)
    dg = daff.mm(Wh)
    g_g = g_backward(st.g[i], gs, sv_s, dg) + g_backward(st.g[i], gs, sv_s1, dg)
    g_h = torch.cat([g_Wh.reshape(-1), g_bh])
    st.step[i] += 1
    k = st.step[i]
    adam_(st.online[i], g_psi, st.m[i], st.v[i], k, lr_sf)
    adam_(st.w[i], g_w, st.wm[i], st.wv[i], k, lr_w)
    adam_(st.g[i], g_g, st.gm[i], st.gv[i], k, lr_g)
    adam_(st.h, g_h, st.hm[i], st.hv[i], k, lr_h)
    st.since_target[i] += 1
    if st.since_target[i] >= target_update_ev:
        st.target[i].copy_(st.online[i])
        st.since_target[i] = 0
    return loss, l1, l2, next_actions


# --------------------------------------------------------------------------------------
# TSF test tasks: TSFDQN.get_test_action (tsfdqn.py:859-870) and
# TSFDQN.update_test_reward_mapper (tsfdqn.py:917-997; tsfdqn_nf.py identical).  A test task
# mixes the source tasks with weights ω (ω̂ = ω / Σω, ω shaped [1, T, 1, 1] in the reference)
# and fits its own reward weights w and ω by Adam on
#     l1 = MSE(Σ ω̂ ψ_t(s)[a], φ̃ + γ Σ ω̂ ψ⁻_t(s1)[a1]),  l2 = MSE(w·φ̃, r),
#     loss = l1 + β l2 + λ ||ω||_1,   φ̃ = φ ⊙ (h(Σ ω̂ g_t(s)) + h(Σ ω̂ g_t(s1)))
# with ψ, ψ⁻ and g_t under no_grad; then ω.clamp_(1e-7).
# --------------------------------------------------------------------------------------
@dataclass
class TestMapper:
    """One test task's reward mapper: w [d], ω [T] and their Adam state (one torch.optim.Adam
    with two parameter groups, tsfdqn.py:812-831)."""
    w: torch.Tensor
    omega: torch.Tensor
    wm: torch.Tensor = None
    wv: torch.Tensor = None
    om: torch.Tensor = None
    ov: torch.Tensor = None
    step: int = 0

    def __post_init__(self):
        if self.wm is None:
            self.wm, self.wv = torch.zeros_like(self.w), torch.zeros_like(self.w)
            self.om, self.ov = torch.zeros_like(self.omega), torch.zeros_like(self.omega)


def tsf_test_action(st: "TSFState", s: torch.Tensor, w: torch.Tensor, omega: torch.Tensor) -> int:
    """Greedy branch of get_test_action: argmax over the flattened q = w(Σ_t ω̂_t ψ_t(s)) [1, A, 1]."""
    on = omega.reshape(-1) / omega.reshape(-1).sum()
    psi = psi_all(st.online, st.spec, s.reshape(1, -1))[0]      # [T, A, d]
    tsf = (psi * on.view(-1, 1, 1)).sum(0)                      # [A, d]
    return int(torch.argmax(tsf @ w.reshape(-1)))


def tsf_test_update(st: "TSFState", tm: TestMapper, s, a: int, r: float, phi, s1, a1: int, *, gamma: float,
                    beta: float, lasso: float, lr_w: float, wd_w: float, lr_o: float, wd_o: float):
    """update_test_reward_mapper -> (loss, l2, l1) (the reference returns loss, phi_loss, psi_loss);
    tm is updated in place.  Gradients by autograd, as the reference's loss.backward()."""
    spec, gs, d = st.spec, st.gspec, st.spec.d
    s, s1 = s.reshape(1, -1), s1.reshape(1, -1)
    with torch.no_grad():
        gs_s = torch.cat([g_forward(st.g[t], gs, s)[0] for t in range(st.T)])     # [T, G]
        gs_s1 = torch.cat([g_forward(st.g[t], gs, s1)[0] for t in range(st.T)])
        psi = psi_all(st.online, spec, s)[0]                                     # [T, A, d]
        psi1 = psi_all(st.target, spec, s1)[0]
    w = tm.w.clone().requires_grad_(True)
    om = tm.omega.clone().requires_grad_(True)
    on = om / om.sum()
    Wh, bh = st.h[:d * gs.G].view(d, gs.G), st.h[d * gs.G:]
    ws = (gs_s * on.view(-1, 1)).sum(0)
    ws1 = (gs_s1 * on.view(-1, 1)).sum(0)
    tphi = phi.reshape(-1) * (F.linear(ws, Wh, bh) + F.linear(ws1, Wh, bh))
    nxt = tphi + gamma * (psi1 * on.view(-1, 1, 1)).sum(0)[a1]
    cur = (psi * on.view(-1, 1, 1)).sum(0)[a]
    r_fit = (tphi * w).sum()
    l1 = F.mse_loss(cur, nxt)
    l2 = (r_fit - r) ** 2
    loss = l1 + beta * l2 + lasso * om.abs().sum()
    loss.backward()
    tm.step += 1
    adam_(tm.w, w.grad, tm.wm, tm.wv, tm.step, lr_w, weight_decay=wd_w)
    adam_(tm.omega, om.grad, tm.om, tm.ov, tm.step, lr_o, weight_decay=wd_o)
    tm.omega.clamp_(1e-7)
    return float(loss.detach()), float(l2.detach()), float(l1.detach())


def sf_test_reward_update(w: torch.Tensor, phi, r) -> float:
    """SFDQN.update_test_reward_mapper (agents/sfdqn.py:168-184) on a [1, d] (or [d]) weight
    tensor, updated in place: a fresh SGD(lr=0.005, weight_decay=0.01) step of
    MSE(Linear(d, 1, bias=False)(φ), r), by autograd and torch.optim.SGD as the reference runs it.
    Returns the pre-step loss."""
    lin = torch.nn.Linear(w.numel(), 1, bias=False)
    with torch.no_grad():
        lin.weight.copy_(w.reshape(1, -1))
    optim = torch.optim.SGD(lin.parameters(), lr=0.005, weight_decay=0.01)
    r_t = torch.tensor(r).detach().float().unsqueeze(0)
    optim.zero_grad()
    loss = torch.nn.MSELoss()(lin(torch.as_tensor(phi).float()), r_t)
    loss.backward()
    optim.step()
    with torch.no_grad():
        w.copy_(lin.weight.detach().reshape(w.shape))
    return float(loss.detach())


# --------------------------------------------------------------------------------------
# Learned φ: features/deep_phi.py DeepSF_PHI.update_successor (:93-224),
# the library of main_sfdqn_phi_torch.py with agents/sfdqn_phi.py.  φ = phi_net(s ⊕ a ⊕ s1) is an
# MLP (main_sfdqn_phi_torch.py phi_model_lambda: Linear(in, 2in) + ReLU, three more
# Linear(2in, 2in) + ReLU, Linear(2in, d)); the reward model w_i is nn.Linear(d, 1) WITH bias
# (features/deep_phi.py:280); the TD targets φ + γ ψ⁻_i(s1)[a'] carry φ's gradient; loss =
# MSE(w_i(φ), r) + λ_i MSE(ψ_i(s), merged) with λ_i the agent's loss coefficient; the update
# builds a NEW torch Adam every call (so every parameter moves by Adam's first step,
# lr·g/(|g| + eps) up to rounding) over {ψ_i, φ, w_i} and λ_i with maximize=True, then clamps
# λ_i to [1e-2, 1e6].
# --------------------------------------------------------------------------------------
@dataclass
class PhiSpec:
    n_s: int
    d: int
    width_mul: int = 2   # hidden width = width_mul * in
    n_mid: int = 3       # Linear(hidden, hidden) layers between the first and the last

    @property
    def n_in(self) -> int:
        return 2 * self.n_s + 1

    @property
    def dims(self) -> List[Tuple[int, int]]:
        """(out, in) of each Linear."""
        hdim = self.width_mul * self.n_in
        return [(hdim, self.n_in)] + [(hdim, hdim)] * self.n_mid + [(self.d, hdim)]

    @property
    def P(self) -> int:
        return sum(o * i + o for o, i in self.dims)


def phi_unpack(flat: torch.Tensor, ps: PhiSpec):
    out, off = [], 0
    for o, i in ps.dims:
        W = flat[off:off + o * i].view(o, i); off += o * i
        b = flat[off:off + o]; off += o
        out.append((W, b))
    return out


def phi_forward(flat, ps: PhiSpec, X):
    layers = phi_unpack(flat, ps)
    y = X
    for l, (W, b) in enumerate(layers):
        y = F.linear(y, W, b)
        if l < len(layers) - 1:
            y = torch.relu(y)
    return y


def fresh_adam_(p: torch.Tensor, g: torch.Tensor, lr: float, maximize: bool = False) -> None:
    """One step of a freshly built torch Adam (moments zero, step 1)."""
    adam_(p, -g if maximize else g, torch.zeros_like(p), torch.zeros_like(p), 1, lr)


@dataclass
class PhiState:
    spec: Spec
    pspec: PhiSpec
    online: torch.Tensor   # [T, P]
    target: torch.Tensor   # [T, P]
    w: torch.Tensor        # [T, d]  Linear(d, 1).weight rows
    wb: torch.Tensor       # [T]     Linear(d, 1).bias
    phi: torch.Tensor      # [Pphi]  the shared φ net
    lam: torch.Tensor      # [T]     the agent's loss coefficients
    since_target: List[int] = field(default_factory=list)

    def __post_init__(self):
        if not self.since_target:
            self.since_target = [0] * self.online.shape[0]


def phi_update(st: PhiState, batch, i: int, *, use_gpi: bool = True, lr: float = 1e-3, target_update_ev: int = 1000,
               next_actions=None):
    """DeepSF_PHI.update_successor(transitions, phis_model, i, loss_coefficient, use_gpi) ->
    (loss, psi_loss, phi_loss, λ_i) and the next actions; st is updated in place.  Gradients by
    autograd, as the reference's loss.backward().  next_actions: use these instead of the argmax
    (a float64 replay following an fp32 run's actions, tests/test_gpu_phi.py error budget)."""
    s, a, r, _, s1, gamma = batch
    spec = st.spec
    B = s.shape[0]
    idx = torch.arange(B)
    gamma = gamma.reshape(-1, 1)
    with torch.no_grad():
        if use_gpi:
            q1 = torch.matmul(psi_all(st.online, spec, s1), st.w[i].reshape(-1, 1))[..., 0] + st.wb[i]
            nxt = torch.argmax(torch.max(q1, dim=1).values, dim=-1)
        else:
            q1 = torch.matmul(forward(st.online[i], spec, s1)[0], st.w[i].reshape(-1, 1))[..., 0] + st.wb[i]
            nxt = torch.argmax(q1, dim=1)
        if next_actions is not None:
            nxt = torch.as_tensor(next_actions)
        tpsi = forward(st.target[i], spec, s1)[0]
    pt = st.online[i].clone().requires_grad_(True)
    ph = st.phi.clone().requires_grad_(True)
    w = st.w[i].clone().requires_grad_(True)
    wb = st.wb[i].clone().reshape(1).requires_grad_(True)
    lam = st.lam[i].clone().reshape(1).requires_grad_(True)
    inp = torch.cat([s, a.reshape(B, 1).to(s.dtype), s1], dim=1)
    phis = phi_forward(ph, st.pspec, inp)
    cur = forward(pt, spec, s)[0]
    targets = phis + gamma * tpsi[idx, nxt, :]
    merged = cur.clone()
    merged[idx, a, :] = targets
    r_fit = F.linear(phis, w.reshape(1, -1), wb)
    phi_loss = F.mse_loss(r_fit, r.reshape(B, 1))
    psi_loss = F.mse_loss(cur, merged)
    loss = phi_loss + lam * psi_loss
    loss.backward()
    with torch.no_grad():
        fresh_adam_(st.online[i], pt.grad, lr)
        fresh_adam_(st.phi, ph.grad, lr)
        fresh_adam_(st.w[i], w.grad, lr)
        fresh_adam_(st.wb[i:i + 1], wb.grad, lr)
        fresh_adam_(st.lam[i:i + 1], lam.grad, lr, maximize=True)
        st.lam[i:i + 1].clamp_(1e-2, 1e6)
    st.since_target[i] += 1
    if st.since_target[i] >= target_update_ev:
        st.target[i].copy_(st.online[i])
        st.since_target[i] = 0
    return float(loss.detach()), float(psi_loss.detach()), float(phi_loss.detach()), float(st.lam[i]), nxt
