"""DeepTSF on the GPU (the interface of features/deep_sequential_tsf.py:9-185, the library of
main_tsfdqn_sequential_torch.py).

The library of the transformed-successor-feature scripts: per-task ψ heads with an
Adam-trained reward model ``fit_w[i]`` (nn.Linear(d, 1, bias=False)), per-task g_i and the
shared h handed in by the agent (agents/tsfdqn_sequential.py), and one optimizer per task over
{ψ_i, w_i, g_i, h} (build_successor).  The update itself is the agent's
(TSFDQN.update_successor); here it runs as one libsfx call (sfx_tsf_update: GPI next
actions, φ̃ = (h(g_i(s)) + h(g_i(s'))) ⊙ φ, TD target on φ̃, l1 + β l2, backward through ψ_i,
w_i, g_i and h, Adam on all four, target sync).  ``get_next_successors`` (target heads) is
sfx_successors(which = 1).  g_i / h modules are refreshed from the device by
``sync_tsf_modules`` (the agent does it before its test episodes).
"""
from __future__ import annotations

import warnings

import numpy as np
import torch
from torch.utils.weak import WeakIdKeyDictionary

from sfx.dropin._host import copy_weights as update_models_weights
from . import deep_sequential as _seq


def _g_tensors(g):
    """g_i's tensors in the engine's packing (include/sfx.h sfx_tsf_load_g): per planar flow
    weight [1, n_s], bias [1], scale [1, n_s], then the Linear's weight and bias.  Flows are read by
    attribute: tsfdqn_nf.py's PlanarFlow moves its Parameters with .to(device) on a GPU, which
    leaves them unregistered -- see _flows_unregistered."""
    mods = list(g) if isinstance(g, torch.nn.Sequential) else [g]
    *flows, lin = mods
    out = []
    for f in flows:
        out += [getattr(f, "weight", None), getattr(f, "bias", None), getattr(f, "scale", None)]
    return out + [getattr(lin, "weight", None), getattr(lin, "bias", None)]


def _flows_unregistered(g) -> bool:
    """True when g_i's planar-flow tensors are not among g.parameters(): tsfdqn_nf.py's
    PlanarFlow built on a GPU (Parameter(...).to(device) is a copy the module does not register),
    so the reference's optimizer never updates them."""
    mods = list(g) if isinstance(g, torch.nn.Sequential) else [g]
    reg = {id(p) for p in g.parameters()}
    return any(id(getattr(f, k)) not in reg for f in mods[:-1] for k in ("weight", "bias", "scale"))


def _g_geometry(g, n_s):
    """(K, G) of a g_i: nn.Linear(n_s, G) (tsfdqn.py, agents/tsfdqn_sequential.py) or K planar flows
    (weight [1, n_s], bias [1], scale [1, n_s]) followed by nn.Linear(n_s, G) (tsfdqn_nf.py:331-358);
    raises for anything else."""
    mods = list(g) if isinstance(g, torch.nn.Sequential) else [g]
    *flows, lin = mods
    ok = isinstance(lin, torch.nn.Linear) and lin.bias is not None and lin.in_features == n_s
    for f in flows:
        w, b, sc = (getattr(f, k, None) for k in ("weight", "bias", "scale"))
        ok = ok and all(isinstance(x, torch.Tensor) for x in (w, b, sc))
        ok = ok and tuple(w.shape) == (1, n_s) and tuple(sc.shape) == (1, n_s) and b.numel() == 1
    if not ok:
        raise NotImplementedError("sfx DeepTSF: g_i must be nn.Linear(n_s, G) with bias, optionally after planar "
                                  f"flows (weight, bias, scale); got {g}")
    return len(flows), lin.out_features


def _params_flat(m: torch.nn.Module):
    """Parameters in registration order (h; g_i through _g_tensors)."""
    return torch.cat([p.detach().reshape(-1).float().cpu() for p in m.parameters()])


def _tensors_flat(ts):
    return torch.cat([t.detach().reshape(-1).float().cpu() for t in ts])


def _tensors_load(ts, flat):
    off = 0
    with torch.no_grad():
        for p in ts:
            p.copy_(flat[off:off + p.numel()].view_as(p).to(p.device, p.dtype))
            off += p.numel()


def _params_load(m: torch.nn.Module, flat):
    _tensors_load(list(m.parameters()), flat)


class DeepTSF(_seq.DeepSF):
    TSF_MAX_BATCH = 64  # minibatch rows of the TSF kernels (sfx_tsf.h)

    def __init__(self, pytorch_model_handle, *args, target_update_ev=1000, train_unregistered_flows=False,
                 **kwargs):
        """train_unregistered_flows: planar flows that g_i does not register (tsfdqn_nf.py on a
        GPU) stay fixed by default, as the reference's optimizer leaves them; True trains them
        anyway (the reference's CPU behaviour)."""
        super().__init__(pytorch_model_handle, *args, target_update_ev=target_update_ev, **kwargs)
        self.max_batch = min(self.max_batch, self.TSF_MAX_BATCH)
        self.train_unregistered_flows = train_unregistered_flows

    def reset(self):
        super().reset()
        self._g = []
        self._h = None
        self._tsf_stale = False
        # Adam state of each test task's {w, ω}, keyed by the ω tensor itself (weakly: it goes
        # with the agent's tensor).  Not cleared here: the reference keeps that state in the
        # agent's torch optimizers, which agent.reset() never rebuilds, so a second trial's test
        # phases continue it.
        if not isinstance(getattr(self, "_test_state", None), WeakIdKeyDictionary):
            self._test_state = WeakIdKeyDictionary()

    def add_training_task(self, task, source=None, g_function_model={}, h_function_model={}):
        """features/deep_sequential_tsf.py:40-73 (w first, then the ψ networks and the optimizer)."""
        self._flush()
        self._sync_host()
        if self._eng is not None:
            raise NotImplementedError("sfx DeepTSF: add every training task before the first update")
        true_w = task.get_w()
        n_features = task.feature_dim()
        fit_w = torch.Tensor(1, n_features).uniform_(-0.01, 0.01).to(self.device)
        # built on the CPU and moved (see features.deep_sequential.add_training_task)
        w_approx = torch.nn.Linear(n_features, 1, bias=False).to(self.device)
        with torch.no_grad():
            w_approx.weight = torch.nn.Parameter(fit_w)
        self.true_w.append(true_w)
        list.append(self.fit_w, w_approx)
        self._psi.append(self.build_successor(task, source, w_approx, g_function_model, h_function_model))
        self.n_tasks = len(self._psi)
        self.gpi_counters = [np.append(c, 0) for c in self.gpi_counters]
        self.gpi_counters.append(np.zeros((self.n_tasks,), dtype=int))
        self._g.append(g_function_model)
        self._h = h_function_model

    def build_successor(self, task, source=None, task_w={}, g_function={}, h_function={}):
        if self.n_tasks == 0:
            self.n_actions = task.action_count()
            self.n_features = task.feature_dim()
            self.inputs = task.encode_dim()
        A, d = self.n_actions, self.n_features
        model, loss, _ = self.pytorch_model_handle(self.inputs, A * d, (A, d), 1)
        if source is not None and self.n_tasks > 0:
            self._sync_host()
            update_models_weights(self._psi[source][0][0], model)
        hp = self.hyperparameters
        optim = torch.optim.Adam([
            {"params": model.parameters(), "lr": hp["learning_rate_sf"], "weight_decay": hp["weight_decay_sf"]},
            {"params": task_w.parameters(), "lr": hp["learning_rate_w"], "weight_decay": hp["weight_decay_w"]},
            {"params": g_function.parameters(), "lr": hp["learning_rate_g"], "weight_decay": hp["weight_decay_g"]},
            {"params": h_function.parameters(), "lr": hp["learning_rate_h"], "weight_decay": hp["weight_decay_h"]},
        ])
        target, _, _ = self.pytorch_model_handle(self.inputs, A * d, (A, d), 1)
        update_models_weights(model, target)
        self._since.append(0)
        target.eval()
        return (model, loss, optim), (target, None, None)

    # ------------------------------------------------------------------ engine
    def _engine(self, batch: int = 1):
        fresh = self._eng is None or self._eng_T != self.n_tasks or batch > self._eng.max_batch
        if fresh and self._eng is not None and self._eng_T > 0:
            raise NotImplementedError("sfx DeepTSF: the engine cannot be rebuilt once TSF training started")
        eng = super()._engine(batch)
        if fresh:
            h = self._h
            geos = {_g_geometry(g, self.inputs) for g in self._g}
            if len(geos) != 1:
                raise NotImplementedError("sfx DeepTSF: every g_i must have the same shape")
            (K, G), = geos
            if not isinstance(h, torch.nn.Linear) or h.bias is None or h.out_features != self.n_features or \
                    h.in_features != G:
                raise NotImplementedError("sfx DeepTSF: h must be nn.Linear(G, d) with bias")
            hp = self.hyperparameters
            eng.tsf_setup(G, K, float(hp.get("beta_loss_coefficient", 1.0)), hp["learning_rate_g"],
                          hp["weight_decay_g"], hp["learning_rate_h"], hp["weight_decay_h"])
            for t, g in enumerate(self._g):
                eng.tsf_load_g(t, _tensors_flat(_g_tensors(g)))
            eng.tsf_load_h(_params_flat(h))
            if K > 0 and any(_flows_unregistered(g) for g in self._g):
                freeze = not getattr(self, "train_unregistered_flows", False)
                warnings.warn("sfx DeepTSF: the planar flows of g_i are not registered parameters of g_i "
                              "(tsfdqn_nf.py's PlanarFlow on a GPU), so the reference's optimizer never updates "
                              "them; " + ("they are held fixed here too (train_unregistered_flows=True trains "
                                          "them)" if freeze else "train_unregistered_flows=True: they train here"),
                              RuntimeWarning, stacklevel=3)
                eng.tsf_freeze_flows(freeze)
        return eng

    def sync_tsf_modules(self):
        """Copy the device's g_i and h into the agent's modules."""
        if self._eng is None or not self._tsf_stale:
            return
        for t, g in enumerate(self._g):
            _tensors_load(_g_tensors(g), self._eng.tsf_get_g(t)[0])
        _params_load(self._h, self._eng.tsf_get_h())
        self._tsf_stale = False

    def tsf_update(self, transitions, policy_index, use_gpi=True, beta=None):
        """agents/tsfdqn_sequential.py:123-252 (TSFDQN.update_successor) -> (loss, l1, l2)."""
        states, actions, rs, phis, next_states, gammas = transitions
        eng = self._engine(len(gammas))
        if beta is not None and float(beta) != float(self.hyperparameters.get("beta_loss_coefficient", 1.0)):
            raise NotImplementedError("sfx DeepTSF: the agent's beta_loss_coefficient differs from the library's")
        self._flush()
        losses = eng.tsf_update(policy_index, states, actions, rs, phis, next_states, gammas, use_gpi=use_gpi)
        self._host_stale = True
        self._tsf_stale = True
        loss, l1, l2 = (x.to(self._out_device()) for x in losses)
        return loss, l1, l2

    # ------------------------------------------------------------------ test tasks
    # TSFDQN.get_test_action / update_test_reward_mapper (tsfdqn.py:859-997) on the device: the
    # agent's w_approx.weight [1, d] and ω [1, T, 1, 1] are updated in place when they live on the
    # engine's device (staged through it otherwise); the Adam moments of each test task's {w, ω}
    # live here, keyed by its ω tensor object (the reference keeps them in the torch optimizer).
    def _on_engine(self, t):
        dev = self._eng.device
        if t.device == dev and t.dtype == torch.float32 and t.is_contiguous():
            return t, False
        return t.detach().to(dev, torch.float32).contiguous(), True

    def tsf_test_action(self, s_enc, w_approx, omegas):
        eng = self._engine(1)
        self._flush()
        w, _ = self._on_engine(w_approx.weight.detach().reshape(-1))
        om, _ = self._on_engine(omegas.detach().reshape(-1))
        return eng.tsf_test_action(s_enc, w, om).to(self._out_device())

    def tsf_test_update(self, w_approx, omegas, phi, r, s, a, s1, a1, *, gamma, beta, lasso, lr_w, wd_w, lr_o, wd_o):
        eng = self._engine(1)
        self._flush()
        st = self._test_state.get(omegas)
        if st is None:
            st = self._test_state[omegas] = [torch.zeros(2 * (self.n_features + self.n_tasks), device=eng.device), 0]
        st[1] += 1
        w, w_staged = self._on_engine(w_approx.weight.detach().reshape(-1))
        om, om_staged = self._on_engine(omegas.detach().reshape(-1))
        losses = eng.tsf_test_update(s, s1, a, a1, float(r), phi, w, om, st[0], st[1], gamma, beta, lasso, lr_w, wd_w,
                                     lr_o, wd_o)
        with torch.no_grad():
            if w_staged:
                w_approx.weight.copy_(w.view_as(w_approx.weight))
            if om_staged:
                omegas.copy_(om.view_as(omegas))
        loss, l2, l1 = (x.to(self._out_device()) for x in losses)
        return loss, l2, l1

    # ------------------------------------------------------------------ ψ
    def get_next_successor(self, state, policy_index):
        return self.get_next_successors(state)[:, policy_index]

    def get_next_successors(self, state):
        s = self._state(state)
        eng = self._engine(s.shape[0])
        self._flush()
        return eng.successors(s, which=1).to(self._out_device())

    def update_successor(self, transitions, policy_index, use_gpi=True):
        raise Exception("This function should not be called")
