#!/usr/bin/env python3
"""Generate golden vectors by running the REAL reference hot path in this container.

Imports the reference read-only from /root/reference/source (with a no-op
``torch.utils.tensorboard`` stub: tensorboard is not installed and the
reference's utils/logger.py imports it at module top) and records inputs,
initial weights and outputs of:

  * GPI / get_successors              (sfdqn.py:153-240, 290-301)
  * DeepSF.update_successor           (sfdqn.py:303-371), use_gpi True / False
  * DeepSF.update_successor all-task  (features/deep.py:93-131 + agents/sfdqn.py:47-60,
                                       with SF.update_reward LMS, features/successor.py:146-167)
  * TSFDQN.update_successor           (tsfdqn.py:588-709) and the planar-flow twin (tsfdqn_nf.py)
  * TSFDQN.get_test_action / update_test_reward_mapper (tsfdqn.py:859-997), both variants

into small ``.npz`` fixtures under tests/golden/.  The fixtures are data only;
this script never travels to the GPU box (it needs /root/reference).

Usage:  python tools/gen_golden.py
"""
from __future__ import annotations

import os
import sys
import types
from collections import OrderedDict

import numpy as np
import torch

REF = "/root/reference/source"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden")
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from tests.golden.recipe import SHAPES, full_size_heads  # noqa: E402  (our own seed recipe)


def _install_reference():
    tb = types.ModuleType("torch.utils.tensorboard")

    class _NoWriter:
        def __init__(self, *a, **k):
            pass

        def add_scalar(self, *a, **k):
            pass

        add_scalars = add_histogram = flush = close = add_scalar

    tb.SummaryWriter = _NoWriter
    sys.modules["torch.utils.tensorboard"] = tb
    sys.path.insert(0, REF)
    from utils.torch import set_torch_device  # reference module
    set_torch_device(False)
    from utils.logger import set_logger_level
    set_logger_level(False)


_install_reference()
import sfdqn as ref_sfdqn          # noqa: E402
import tsfdqn as ref_tsfdqn        # noqa: E402
import tsfdqn_nf as ref_tsfdqn_nf  # noqa: E402
from features import deep as ref_deep  # noqa: E402
from features import deep_phi as ref_deep_phi  # noqa: E402

HYPER = {
    "learning_rate_sf": 1e-3, "learning_rate_w": 1e-3, "learning_rate_g": 1e-3,
    "learning_rate_h": 1e-3, "weight_decay_sf": 0, "weight_decay_w": 0,
    "weight_decay_g": 0, "weight_decay_h": 0, "g_h_function_dims": 16,
    "n_coupling_layers": 3, "beta_loss_coefficient": 0.5, "learning_rate_w_lms": 0.05,
}


def psi_lambda(H, acts, lr=1e-3):
    """The reference's ψ architecture (main_sfdqn_torch.py:44-78)."""
    act_cls = {"relu": torch.nn.ReLU, "tanh": torch.nn.Tanh}

    def build(num_inputs, output_dim, reshape_dim, reshape_axis=1):
        layers = OrderedDict()
        layers["layer_input"] = torch.nn.Linear(num_inputs, H)
        for j, a in enumerate(acts):
            layers[f"layer_{j}"] = torch.nn.Linear(H, H)
            layers[f"activation_layer_{j}"] = act_cls[a]()
        layers["layer_output"] = torch.nn.Linear(H, output_dim)
        layers["layer_unflatten"] = torch.nn.Unflatten(reshape_axis, reshape_dim)
        model = torch.nn.Sequential(layers)
        return model, torch.nn.MSELoss(), torch.optim.Adam(model.parameters(), lr=lr)

    return build


class SynthTask:
    """Minimal Task (tasks/task.py interface) for driving add_training_task."""

    def __init__(self, n_s, A, d, idx):
        self.n_s, self.A, self.d, self.idx = n_s, A, d, idx

    def action_count(self):
        return self.A

    def feature_dim(self):
        return self.d

    def encode_dim(self):
        return self.n_s

    def features(self, state, action, next_state):
        raise NotImplementedError("golden generation feeds transitions directly")

    def get_w(self):
        w = torch.zeros((self.d, 1))
        w[self.idx % self.d, 0] = 1.0
        return w

    def __repr__(self):
        return f"SynthTask({self.idx})"


def flat(module):
    return torch.cat([p.detach().reshape(-1) for p in module.parameters()]).clone()


def adam_state(optim, params):
    m, v = [], []
    for p in params:
        st = optim.state[p]
        m.append(st["exp_avg"].reshape(-1))
        v.append(st["exp_avg_sq"].reshape(-1))
    return torch.cat(m).clone(), torch.cat(v).clone()


def batch_stream(n_s, A, d, B, k, gen, terminal_p=0.1):
    out = []
    for _ in range(k):
        s = torch.randn(B, n_s, generator=gen)
        a = torch.randint(0, A, (B,), generator=gen)
        phi = torch.rand(B, d, generator=gen)
        r = torch.rand(B, 1, generator=gen)
        s1 = torch.randn(B, n_s, generator=gen)
        gamma = torch.where(torch.rand(B, generator=gen) < terminal_p, 0.0, 0.9).float()
        out.append((s, a, r, phi, s1, gamma))
    return out


def stack_batches(batches):
    names = ["s", "a", "r", "phi", "s1", "gamma"]
    return {f"b_{n}": np.stack([b[j].numpy() for b in batches]) for j, n in enumerate(names)}


def np_(t):
    return t.detach().numpy().copy()


# --------------------------------------------------------------------------------------
def build_sfdqn(shape, T, target_update_ev=1000):
    n_s, H, A, d, acts = shape
    sf = ref_sfdqn.DeepSF(pytorch_model_handle=psi_lambda(H, acts), use_true_reward=False,
                          target_update_ev=target_update_ev, hyperparameters=HYPER)
    sf.reset()
    for t in range(T):
        sf.add_training_task(SynthTask(n_s, A, d, t))
    return sf


def sfdqn_weights(sf):
    online = torch.stack([flat(sf.psi[t][0][0]) for t in range(sf.n_tasks)])
    target = torch.stack([flat(sf.psi[t][1][0]) for t in range(sf.n_tasks)])
    w = torch.stack([sf.fit_w[t].weight.detach().reshape(-1).clone() for t in range(sf.n_tasks)])
    return online, target, w


def load_sfdqn_weights(sf, online, w=None):
    with torch.no_grad():
        for t in range(sf.n_tasks):
            off = 0
            for mod in (sf.psi[t][0][0], sf.psi[t][1][0]):
                off = 0
                for p in mod.parameters():
                    n = p.numel()
                    p.copy_(online[t, off:off + n].view_as(p))
                    off += n
            if w is not None:
                sf.fit_w[t].weight.copy_(w[t].view(1, -1))


def gen_gpi(name, shape, T, tie=False):
    torch.manual_seed(100 + T)
    sf = build_sfdqn(shape, T)
    n_s, H, A, d, acts = shape
    online, _, w = sfdqn_weights(sf)
    if tie:
        # exact task tie: head 2 == head 0; exact action tie in head 1: action 3 == action 1
        online[2] = online[0]
        P_out = H * A * d + A * d
        out_off = online.shape[1] - P_out
        Wo = online[1, out_off:out_off + H * A * d].view(A * d, H)
        bo = online[1, out_off + H * A * d:].view(A * d)
        Wo[3 * d:4 * d] = Wo[1 * d:2 * d]
        bo[3 * d:4 * d] = bo[1 * d:2 * d]
        load_sfdqn_weights(sf, online)
    gen = torch.Generator().manual_seed(7)
    S1 = torch.randn(1, n_s, generator=gen)
    S32 = torch.randn(32, n_s, generator=gen)
    rec = dict(n_s=n_s, H=H, A=A, d=d, T=T, acts=np.array(acts), online=np_(online), w=np_(w),
               S1=np_(S1), S32=np_(S32))
    with torch.no_grad():
        rec["psi1"] = np_(sf.get_successors(S1))
        rec["psi32"] = np_(sf.get_successors(S32))
        for i in range(T):
            q, task = sf.GPI(S1, i)
            rec[f"q1_{i}"], rec[f"task1_{i}"] = np_(q), np.array(int(task))
            q, task = sf.GPI(S32, i)
            rec[f"q32_{i}"], rec[f"task32_{i}"] = np_(q), np_(task)
            rec[f"next32_{i}"] = np_(torch.argmax(torch.max(q, axis=1).values, axis=-1))
    np.savez_compressed(os.path.join(OUT, f"gpi_{name}.npz"), **rec)


def gen_full_size():
    """Reacher-shape C2 at H=256, T=8: weights from our seed recipe (not stored)."""
    n_s, H, A, d, acts = SHAPES["reacher17_full"]
    T = 8
    online, w = full_size_heads()
    sf = build_sfdqn(SHAPES["reacher17_full"], T)
    load_sfdqn_weights(sf, online, w)
    gen = torch.Generator().manual_seed(11)
    S32 = torch.randn(32, n_s, generator=gen)
    S1 = S32[:1].clone()
    rec = dict(n_s=n_s, H=H, A=A, d=d, T=T, acts=np.array(acts), S32=np_(S32),
               online_sum=np.float64(online.double().sum()), w=np_(w))
    with torch.no_grad():
        rec["psi32"] = np_(sf.get_successors(S32))
        for i in range(T):
            q, task = sf.GPI(S32, i)
            rec[f"q32_{i}"], rec[f"task32_{i}"] = np_(q), np_(task)
            rec[f"next32_{i}"] = np_(torch.argmax(torch.max(q, axis=1).values, axis=-1))
            q, task = sf.GPI(S1, i)
            rec[f"task1_{i}"] = np.array(int(task))
    np.savez_compressed(os.path.join(OUT, "gpi_reacher17_full.npz"), **rec)


def gen_sfdqn_updates(name, shape, T, k, use_gpi, target_update_ev):
    torch.manual_seed(200 + int(use_gpi))
    sf = build_sfdqn(shape, T, target_update_ev)
    n_s, H, A, d, acts = shape
    online0, target0, w0 = sfdqn_weights(sf)
    batches = batch_stream(n_s, A, d, 32, k, torch.Generator().manual_seed(3))
    rec = dict(n_s=n_s, H=H, A=A, d=d, T=T, acts=np.array(acts), k=k, use_gpi=int(use_gpi),
               target_update_ev=target_update_ev, online0=np_(online0), target0=np_(target0),
               w0=np_(w0), **stack_batches(batches))
    losses, nexts, policies = [], [], []
    for j, b in enumerate(batches):
        i = j % T
        policies.append(i)
        # reproduce next actions the reference uses (same code path, no state change)
        with torch.no_grad():
            if use_gpi:
                q1, _ = sf.GPI(b[4], i)
                na = torch.argmax(torch.max(q1, axis=1).values, axis=-1)
            else:
                na = torch.squeeze(torch.argmax(sf.fit_w[i](sf.get_successor(b[4], i)), axis=1), axis=1)
        nexts.append(np_(na))
        loss, l1, l2 = sf.update_successor(b, i, use_gpi)
        losses.append([float(loss), float(l1), float(l2)])
        if j == 0:
            on1, ta1, w1 = sfdqn_weights(sf)
            rec.update(online1=np_(on1), target1=np_(ta1), w1=np_(w1))
    online, target, w = sfdqn_weights(sf)
    m = torch.zeros_like(online); v = torch.zeros_like(online)
    wm = torch.zeros_like(w); wv = torch.zeros_like(w)
    steps = []
    for t in range(T):
        model = sf.psi[t][0][0]
        optim = sf.psi[t][0][2]
        if optim.state.get(next(model.parameters())) is None:
            steps.append(0)
            continue
        m[t], v[t] = adam_state(optim, list(model.parameters()))
        wm[t], wv[t] = adam_state(optim, list(sf.fit_w[t].parameters()))
        steps.append(int(optim.state[next(model.parameters())]["step"]))
    rec.update(policies=np.array(policies), losses=np.array(losses), next_actions=np.stack(nexts),
               online=np_(online), target=np_(target), w=np_(w), m=np_(m), v=np_(v), wm=np_(wm),
               wv=np_(wv), steps=np.array(steps), since_target=np.array(sf.updates_since_target_updated))
    np.savez_compressed(os.path.join(OUT, f"upd_{name}.npz"), **rec)


def gen_deep_alltask(shape, T, k, target_update_ev):
    """features/deep.py DeepSF driven like agents/sfdqn.py:47-60 (LMS w, all heads per step)."""
    torch.manual_seed(300)
    n_s, H, A, d, acts = shape
    lam = psi_lambda(H, acts, lr=1e-3)
    sf = ref_deep.DeepSF(pytorch_model_handle=lam, target_update_ev=target_update_ev,
                         hyperparameters={"learning_rate_w": HYPER["learning_rate_w_lms"]})
    sf.reset()
    for t in range(T):
        sf.add_training_task(SynthTask(n_s, A, d, t))
    online0 = torch.stack([flat(sf.psi[t][0][0]) for t in range(T)])
    w0 = torch.stack([sf.fit_w[t].reshape(-1).clone() for t in range(T)])
    gen = torch.Generator().manual_seed(5)
    batches = batch_stream(n_s, A, d, 32, k, gen)
    lms_phi = torch.rand(k, d, generator=gen)
    lms_task = torch.randint(0, T, (k,), generator=gen)
    lms_r = torch.stack([(lms_phi[j] * sf.true_w[int(lms_task[j])].reshape(-1)).sum() for j in range(k)])
    rec = dict(n_s=n_s, H=H, A=A, d=d, T=T, acts=np.array(acts), k=k, target_update_ev=target_update_ev,
               alpha_w=HYPER["learning_rate_w_lms"], online0=np_(online0), w0=np_(w0),
               lms_phi=np_(lms_phi), lms_task=np_(lms_task), lms_r=np_(lms_r), **stack_batches(batches))
    losses = []
    for j, b in enumerate(batches):
        sf.update_reward(lms_phi[j], lms_r[j], int(lms_task[j]))
        s, a, r, phi, s1, gamma = b
        step_l = []
        for i in range(T):
            sf.update_successor((s, a, phi, s1, gamma), i)
        losses.append(step_l)
        if j == 0:
            rec["online1"] = np_(torch.stack([flat(sf.psi[t][0][0]) for t in range(T)]))
    online = torch.stack([flat(sf.psi[t][0][0]) for t in range(T)])
    target = torch.stack([flat(sf.psi[t][1][0]) for t in range(T)])
    w = torch.stack([sf.fit_w[t].reshape(-1).clone() for t in range(T)])
    m, v = zip(*[adam_state(sf.psi[t][0][2], list(sf.psi[t][0][0].parameters())) for t in range(T)])
    rec.update(online=np_(online), target=np_(target), w=np_(w), m=np_(torch.stack(m)),
               v=np_(torch.stack(v)), since_target=np.array(sf.updates_since_target_updated))
    np.savez_compressed(os.path.join(OUT, "upd_deep_alltask.npz"), **rec)


def gen_tsf(name, module, shape, T, k, K):
    torch.manual_seed(400 + K)
    n_s, H, A, d, acts = shape
    hyper = dict(HYPER, n_coupling_layers=K)
    sf = module.DeepTSF(pytorch_model_handle=psi_lambda(H, acts), use_true_reward=False,
                        target_update_ev=4, hyperparameters=hyper)
    agent = module.TSFDQN(deep_sf=sf, buffer_handle=lambda: None, gamma=0.9, T=500, encoding=None,
                          use_gpi=True, hyperparameters=hyper)
    agent.reset()
    for t in range(T):
        agent.add_training_task(SynthTask(n_s, A, d, t))
    online0 = torch.stack([flat(sf.psi[t][0][0]) for t in range(T)])
    w0 = torch.stack([sf.fit_w[t].weight.detach().reshape(-1).clone() for t in range(T)])
    g0 = torch.stack([flat(agent.g_functions[t]) for t in range(T)])
    h0 = flat(agent.h_function)
    batches = batch_stream(n_s, A, d, 32, k, torch.Generator().manual_seed(9))
    rec = dict(n_s=n_s, H=H, A=A, d=d, T=T, acts=np.array(acts), k=k, K=K, G=hyper["g_h_function_dims"],
               beta=hyper["beta_loss_coefficient"], target_update_ev=4, online0=np_(online0),
               w0=np_(w0), g0=np_(g0), h0=np_(h0), **stack_batches(batches))
    losses, policies = [], []
    for j, b in enumerate(batches):
        i = j % T
        policies.append(i)
        loss, l1, l2 = agent.update_successor(b, i, True)
        losses.append([float(loss), float(l1), float(l2)])
    online = torch.stack([flat(sf.psi[t][0][0]) for t in range(T)])
    target = torch.stack([flat(sf.psi[t][1][0]) for t in range(T)])
    w = torch.stack([sf.fit_w[t].weight.detach().reshape(-1).clone() for t in range(T)])
    g = torch.stack([flat(agent.g_functions[t]) for t in range(T)])
    h = flat(agent.h_function)
    rec.update(policies=np.array(policies), losses=np.array(losses), online=np_(online),
               target=np_(target), w=np_(w), g=np_(g), h=np_(h))
    np.savez_compressed(os.path.join(OUT, f"upd_{name}.npz"), **rec)


class PhiTask(SynthTask):
    """A test task whose features() hands out the recorded φ of the current step."""

    phi = None

    def features(self, state, action, next_state):
        return self.phi


def gen_tsf_test(name, module, shape, T, k, K):
    """TSFDQN.get_test_action (greedy) and update_test_reward_mapper (tsfdqn.py:859-997): the test
    task's w and ω set up as train() does (tsfdqn.py:797-832: ω from _init_omega normalised, one
    Adam over {w, ω}, LambdaLR decaying ω's rate), then k steps of random (s, a, r, φ, s1, a1),
    with scheduler.step() after each as test_agent does."""
    torch.manual_seed(700 + K)
    n_s, H, A, d, acts = shape
    hyper = dict(HYPER, n_coupling_layers=K, omegas_l1_coefficient=0.05, learning_rate_omega=5e-3,
                 learning_rate_omega_decay=0.01, weight_decay_omega=1e-4, weight_decay_w=1e-3)
    sf = module.DeepTSF(pytorch_model_handle=psi_lambda(H, acts), use_true_reward=False,
                        target_update_ev=4, hyperparameters=hyper)
    agent = module.TSFDQN(deep_sf=sf, buffer_handle=lambda: None, gamma=0.9, T=500, encoding=None,
                          use_gpi=True, test_epsilon=-1.0, hyperparameters=hyper)
    agent.reset()
    for t in range(T):
        agent.add_training_task(SynthTask(n_s, A, d, t))
    # the target heads differ from the online ones (as after training)
    with torch.no_grad():
        for t in range(T):
            for p in sf.psi[t][1][0].parameters():
                p.add_(torch.randn_like(p) * 0.01)
        for g in agent.g_functions:  # trained-looking g / h
            for p in g.parameters():
                p.add_(torch.randn_like(p) * 0.05)
    omegas = agent._init_omega(T)
    with torch.no_grad():
        omegas = omegas / torch.sum(omegas, axis=1, keepdim=True)
    omegas = omegas.clone().detach().requires_grad_(True)
    w_approx = torch.nn.Linear(d, 1, bias=False)
    with torch.no_grad():
        w_approx.weight = torch.nn.Parameter(torch.Tensor(1, d).uniform_(-0.01, 0.01))
    optim = torch.optim.Adam([
        {"params": w_approx.parameters(), "lr": hyper["learning_rate_w"], "weight_decay": hyper["weight_decay_w"]},
        {"params": omegas, "lr": hyper["learning_rate_omega"], "weight_decay": hyper["weight_decay_omega"]}])
    decay = hyper["learning_rate_omega_decay"]
    scheduler = torch.optim.lr_scheduler.LambdaLR(optim, [lambda e: 1 ** e, lambda e: (1 - decay) ** e])
    rec = dict(n_s=n_s, H=H, A=A, d=d, T=T, acts=np.array(acts), k=k, K=K, G=hyper["g_h_function_dims"],
               beta=hyper["beta_loss_coefficient"], lasso=hyper["omegas_l1_coefficient"], gamma=0.9,
               lr_w=hyper["learning_rate_w"], wd_w=hyper["weight_decay_w"], wd_o=hyper["weight_decay_omega"],
               online=np_(torch.stack([flat(sf.psi[t][0][0]) for t in range(T)])),
               target=np_(torch.stack([flat(sf.psi[t][1][0]) for t in range(T)])),
               g=np_(torch.stack([flat(agent.g_functions[t]) for t in range(T)])), h=np_(flat(agent.h_function)),
               w0=np_(w_approx.weight.detach().reshape(-1).clone()), omega0=np_(omegas.detach().reshape(-1).clone()))
    gen = torch.Generator().manual_seed(11)
    task = PhiTask(n_s, A, d, T)
    cols = {key: [] for key in ("s", "s1", "a", "a1", "r", "phi", "lr_o", "loss", "l2", "l1", "greedy", "w", "omega")}
    for j in range(k):
        s, s1 = torch.randn(1, n_s, generator=gen), torch.randn(1, n_s, generator=gen)
        a, a1 = int(torch.randint(0, A, (1,), generator=gen)), int(torch.randint(0, A, (1,), generator=gen))
        r = float(torch.rand(1, generator=gen))
        task.phi = torch.rand(1, d, generator=gen)
        greedy = int(agent.get_test_action(s, w_approx, omegas))
        cols["lr_o"].append(optim.param_groups[1]["lr"])
        loss, l2, l1 = agent.update_test_reward_mapper(w_approx, omegas, optim, task, r, s, a, s1, a1)
        scheduler.step()
        for key, v in (("s", s), ("s1", s1), ("a", a), ("a1", a1), ("r", r), ("phi", task.phi), ("loss", float(loss)),
                       ("l2", float(l2)), ("l1", float(l1)), ("greedy", greedy),
                       ("w", w_approx.weight.detach().reshape(-1).clone()), ("omega", omegas.detach().reshape(-1).clone())):
            cols[key].append(np_(v) if torch.is_tensor(v) else v)
    rec.update({key: np.array(v) for key, v in cols.items()})
    np.savez_compressed(os.path.join(OUT, f"test_{name}.npz"), **rec)


# ---------------------------------------------------------------------------------------
# SF-boundary call logs: the reference's own agents (agents/sfdqn.py, agents/sfdqn_sequential.py,
# agents/tsfdqn_sequential.py and the single-file sfdqn.py / tsfdqn.py / tsfdqn_nf.py) run the
# seeded recipes of tests/golden/recipe.py on the CPU, and every call they make across the SF
# boundary -- GPI, get_successor(s), get_next_successors, update_reward, update_successor, and for
# TSF the agent's own update_successor (tsfdqn.py:588-709), which the drop-in binds to the library
# -- is logged in order with its inputs and outputs, together with the library state before the
# first call and after the run.  tests/test_gpu_dropin.py replays the log through sfx's drop-in
# library on the GPU.  The agents themselves never leave this container.
# ---------------------------------------------------------------------------------------
class CallLog:
    def __init__(self):
        self.calls, self.depth, self.init, self.agent = [], 0, None, None

    def call(self, sf, name, thunk, fields):
        if self.depth == 0 and self.init is None:
            self.init = lib_state(sf, self.agent)
        self.depth += 1
        try:
            out = thunk()
        finally:
            self.depth -= 1
        if self.depth == 0:  # only the agent's own calls, not the library's calls into itself
            self.calls.append((name, fields(out)))
        return out

    def save(self, path, final):
        rec = {"names": np.array([n for n, _ in self.calls])}
        for k, (_, f) in enumerate(self.calls):
            for key, v in f.items():
                rec[f"c{k}.{key}"] = _val(v)
        for key, v in self.init.items():
            rec["init." + key] = v
        for key, v in final.items():
            rec["final." + key] = v
        np.savez_compressed(path, **rec)


def _val(v):
    if isinstance(v, torch.Tensor):
        return v.detach().cpu().numpy()
    return np.asarray(v)


def _w_flat(w):
    w = w.weight if hasattr(w, "weight") else w
    return w.detach().reshape(-1).cpu().clone()


def lib_state(sf, agent=None):
    T = sf.n_tasks
    st = dict(online=np_(torch.stack([flat(sf.psi[t][0][0]) for t in range(T)])),
              target=np_(torch.stack([flat(sf.psi[t][1][0]) for t in range(T)])),
              w=np_(torch.stack([_w_flat(sf.fit_w[t]) for t in range(T)])))
    if agent is not None and getattr(agent, "g_functions", None):
        st["g"] = np_(torch.stack([flat(agent.g_functions[t]) for t in range(T)]))
        st["h"] = np_(flat(agent.h_function))
    return st


def _transitions(tr):
    return {} if tr is None else {f"t{i}": x for i, x in enumerate(tr)}


def recording_sf(cls, log):
    class Recording(cls):
        def GPI(self, state, task_index, update_counters=False):
            return log.call(self, "GPI", lambda: cls.GPI(self, state, task_index, update_counters),
                            lambda o: dict(state=state, task_index=task_index, update_counters=update_counters,
                                           q=o[0], task=o[1]))

        def get_successors(self, state):
            return log.call(self, "get_successors", lambda: cls.get_successors(self, state),
                            lambda o: dict(state=state, psi=o))

        def get_successor(self, state, policy_index):
            return log.call(self, "get_successor", lambda: cls.get_successor(self, state, policy_index),
                            lambda o: dict(state=state, policy_index=policy_index, psi=o))

        def update_reward(self, phi, r, task_index, exact=False):
            return log.call(self, "update_reward", lambda: cls.update_reward(self, phi, r, task_index, exact),
                            lambda o: dict(phi=phi, r=torch.as_tensor(r).float(), task_index=task_index,
                                           w=_w_flat(self.fit_w[task_index])))

        def update_successor(self, transitions, policy_index, *args, **kwargs):
            use_gpi = kwargs.get("use_gpi", args[0] if args else True)
            out = {}

            def fields(o):
                f = dict(_transitions(transitions), policy_index=policy_index, use_gpi=bool(use_gpi),
                         has_batch=transitions is not None)
                if isinstance(o, tuple):
                    f["losses"] = torch.stack([torch.as_tensor(x).detach().float() for x in o])
                return f

            return log.call(self, "update_successor",
                            lambda: cls.update_successor(self, transitions, policy_index, *args, **kwargs), fields)

    if hasattr(cls, "get_next_successors"):
        def get_next_successors(self, state):
            return log.call(self, "get_next_successors", lambda: cls.get_next_successors(self, state),
                            lambda o: dict(state=state, psi=o))

        Recording.get_next_successors = get_next_successors
    Recording.__name__ = cls.__name__
    return Recording


def recording_tsf_agent(cls, log):
    class Recording(cls):
        def __init__(self, *a, **k):
            super().__init__(*a, **k)
            log.agent = self

        def update_successor(self, transitions, policy_index, use_gpi=True):
            def fields(o):
                f = dict(_transitions(transitions), policy_index=policy_index, use_gpi=bool(use_gpi),
                         has_batch=transitions is not None)
                if isinstance(o, tuple):
                    f["losses"] = torch.stack([torch.as_tensor(x).detach().float() for x in o])
                return f

            return log.call(self.sf, "tsf_update",
                            lambda: cls.update_successor(self, transitions, policy_index, use_gpi), fields)

    Recording.__name__ = cls.__name__
    return Recording


def _final(agent, log):
    sf = agent.sf
    st = lib_state(sf, log.agent)
    st["gpi_counters"] = np.stack([np.asarray(c) for c in sf.gpi_counters])
    st["since_target"] = np.array(sf.updates_since_target_updated)
    return st


def gen_call_log_alltask():
    """main_sfdqn_torch.py's stack: agents/sfdqn.py SFDQN + agents/buffer.py + features/deep.py."""
    import contextlib
    import io

    from agents.buffer import ReplayBuffer
    from agents.sfdqn import SFDQN
    from tests.golden.recipe import agent_run

    log = CallLog()
    with contextlib.redirect_stdout(io.StringIO()):
        agent, *_ = agent_run(recording_sf(ref_deep.DeepSF, log), SFDQN, ReplayBuffer, torch.device("cpu"))
    log.save(os.path.join(OUT, "calls_sfdqn_alltask.npz"), _final(agent, log))


def gen_call_log_sequential(single_file=False):
    """main_sfdqn_sequential_torch.py's stack (agents/sfdqn_sequential.py + features/deep_sequential.py)
    or the single-file sfdqn.py."""
    import contextlib
    import io

    from tests.golden.recipe import agent_run_sequential

    if single_file:
        DeepSF, SFDQN, ReplayBuffer = ref_sfdqn.DeepSF, ref_sfdqn.SFDQN, ref_sfdqn.ReplayBuffer
    else:
        from agents.buffer_sequential import ReplayBuffer
        from agents.sfdqn_sequential import SFDQN
        from features.deep_sequential import DeepSF
    log = CallLog()
    with contextlib.redirect_stdout(io.StringIO()):
        agent, *_ = agent_run_sequential(recording_sf(DeepSF, log), SFDQN, ReplayBuffer, torch.device("cpu"))
    name = "calls_sfdqn_singlefile" if single_file else "calls_sfdqn_sequential"
    log.save(os.path.join(OUT, name + ".npz"), _final(agent, log))


def gen_call_log_tsf(nf=False, single_file=False):
    """main_tsfdqn_sequential_torch.py's stack (agents/tsfdqn_sequential.py +
    features/deep_sequential_tsf.py), the single-file tsfdqn.py, or tsfdqn_nf.py (planar flows)."""
    import contextlib
    import io

    from tests.golden.recipe import agent_run_tsf

    if nf:
        DeepTSF, TSFDQN, ReplayBuffer = ref_tsfdqn_nf.DeepTSF, ref_tsfdqn_nf.TSFDQN, ref_tsfdqn_nf.ReplayBuffer
    elif single_file:
        DeepTSF, TSFDQN, ReplayBuffer = ref_tsfdqn.DeepTSF, ref_tsfdqn.TSFDQN, ref_tsfdqn.ReplayBuffer
    else:
        from agents.buffer_tsf_sequential import ReplayBuffer
        from agents.tsfdqn_sequential import TSFDQN
        from features.deep_sequential_tsf import DeepTSF
    log = CallLog()
    with contextlib.redirect_stdout(io.StringIO()):
        agent, *_ = agent_run_tsf(recording_sf(DeepTSF, log), recording_tsf_agent(TSFDQN, log), ReplayBuffer,
                                  torch.device("cpu"), nf=nf)
    name = "calls_tsfdqn_nf" if nf else "calls_tsfdqn_singlefile" if single_file else "calls_tsfdqn_sequential"
    log.save(os.path.join(OUT, name + ".npz"), _final(agent, log))


def gen_call_logs():
    gen_call_log_alltask()
    gen_call_log_sequential()
    gen_call_log_sequential(single_file=True)
    gen_call_log_tsf()
    gen_call_log_tsf(single_file=True)
    gen_call_log_tsf(nf=True)


def main():
    os.makedirs(OUT, exist_ok=True)
    torch.set_num_threads(4)
    gen_gpi("reacher17", SHAPES["reacher17"], 4)
    gen_gpi("hopper11", SHAPES["hopper11"], 3)
    gen_gpi("cartpole", SHAPES["cartpole"], 2)
    gen_gpi("refreacher", SHAPES["refreacher"], 4)
    gen_gpi("tanh_odd", SHAPES["tanh_odd"], 3)
    gen_gpi("tie", SHAPES["reacher17"], 4, tie=True)
    gen_full_size()
    gen_sfdqn_updates("sfdqn_gpi", SHAPES["reacher17"], 4, 12, True, 5)
    gen_sfdqn_updates("sfdqn_nogpi", SHAPES["reacher17"], 4, 12, False, 5)
    gen_sfdqn_updates("sfdqn_tanh", SHAPES["tanh_odd"], 3, 7, True, 3)
    gen_deep_alltask(SHAPES["reacher17"], 4, 6, 3)
    gen_tsf("tsf", ref_tsfdqn, SHAPES["hopper11"], 3, 8, 0)
    gen_tsf("tsf_nf", ref_tsfdqn_nf, SHAPES["hopper11"], 3, 6, 3)
    gen_tsf_tests()
    gen_phis()
    gen_call_logs()
    print("golden vectors written to", os.path.abspath(OUT))


def gen_tsf_tests():
    gen_tsf_test("tsf", ref_tsfdqn, SHAPES["hopper11"], 3, 10, 0)
    gen_tsf_test("tsf_nf", ref_tsfdqn_nf, SHAPES["hopper11"], 3, 10, 3)


def phi_net(n_s, d):
    """main_sfdqn_phi_torch.py's phi_model_lambda (its model only): in = 2 n_s + 1 (s, a, s1)."""
    n_in = 2 * n_s + 1
    return torch.nn.Sequential(
        torch.nn.Linear(n_in, n_in * 2), torch.nn.ReLU(),
        torch.nn.Linear(n_in * 2, n_in * 2), torch.nn.ReLU(),
        torch.nn.Linear(n_in * 2, n_in * 2), torch.nn.ReLU(),
        torch.nn.Linear(n_in * 2, n_in * 2), torch.nn.ReLU(),
        torch.nn.Linear(n_in * 2, d))


def gen_phi(name, shape, T, k, use_gpi, target_update_ev):
    """features/deep_phi.py DeepSF_PHI.update_successor (:93-224): k updates of rotating policies
    with the agent's (agents/sfdqn_phi.py) φ model tuple and per-task loss coefficients."""
    torch.manual_seed(900 + int(use_gpi))
    n_s, H, A, d, acts = shape
    sf = ref_deep_phi.DeepSF_PHI(pytorch_model_handle=psi_lambda(H, acts), use_true_reward=False,
                                 target_update_ev=target_update_ev)
    sf.reset()
    for t in range(T):
        sf.add_training_task(SynthTask(n_s, A, d, t))
    pm = phi_net(n_s, d)
    phis_model = ((pm, torch.nn.MSELoss(), None), (None, None, None))
    lams = [torch.ones(1, requires_grad=True) for _ in range(T)]
    rec = dict(n_s=n_s, H=H, A=A, d=d, T=T, acts=np.array(acts), k=k, use_gpi=int(use_gpi),
               target_update_ev=target_update_ev,
               online0=np_(torch.stack([flat(sf.psi[t][0][0]) for t in range(T)])),
               w0=np_(torch.stack([sf.fit_w[t].weight.detach().reshape(-1).clone() for t in range(T)])),
               wb0=np_(torch.stack([sf.fit_w[t].bias.detach().reshape(-1).clone() for t in range(T)]).reshape(-1)),
               phi0=np_(flat(pm)))
    batches = batch_stream(n_s, A, d, 32, k, torch.Generator().manual_seed(19))
    rec.update(stack_batches(batches))
    out, policies = [], []
    for j, b in enumerate(batches):
        i = (3 * j) % T
        policies.append(i)
        loss, psi_loss, phi_loss, lam = sf.update_successor(b, phis_model, i, lams[i], use_gpi)
        out.append([float(loss), float(psi_loss), float(phi_loss), float(lam)])
    rec.update(policies=np.array(policies), losses=np.array(out),
               online=np_(torch.stack([flat(sf.psi[t][0][0]) for t in range(T)])),
               target=np_(torch.stack([flat(sf.psi[t][1][0]) for t in range(T)])),
               w=np_(torch.stack([sf.fit_w[t].weight.detach().reshape(-1).clone() for t in range(T)])),
               wb=np_(torch.stack([sf.fit_w[t].bias.detach().reshape(-1).clone() for t in range(T)]).reshape(-1)),
               phi=np_(flat(pm)), lam=np.array([float(x) for x in lams]))
    np.savez_compressed(os.path.join(OUT, f"upd_{name}.npz"), **rec)


def gen_phis():
    gen_phi("phi_gpi", SHAPES["reacher17"], 3, 8, True, 3)
    gen_phi("phi_nogpi", SHAPES["reacher17"], 3, 6, False, 1000)


if __name__ == "__main__":
    if len(sys.argv) > 1:  # only the named generators, e.g. gen_agent_run
        os.makedirs(OUT, exist_ok=True)
        for name in sys.argv[1:]:
            globals()[name]()
    else:
        main()
