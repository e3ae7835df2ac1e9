"""DeepSF of the sequential scripts on the GPU (the interface of features/deep_sequential.py:9-231,
main_sfdqn_sequential_torch.py; the same update as sfdqn.py:303-371).

Differences from features.deep.DeepSF: the reward model of each task is an nn.Linear(d, 1)
trained by Adam together with ψ_i (loss = l1 + l2, param groups {ψ: learning_rate_sf,
weight_decay_sf}, {w: learning_rate_w, weight_decay_w}); update_successor takes
(s, a, r, φ, s', γ) plus use_gpi and returns (loss, l1, l2); GPI_w takes the Linear.
All of it runs in libsfx (sfx_update: GPI next actions, TD target, backward, Adam on ψ_i and w_i).
"""
from __future__ import annotations

import numpy as np
import torch

from sfx.dropin._host import copy_weights as update_models_weights
from . import deep as _deep


class _FitWLinear(list):
    """fit_w entries are nn.Linear(d, 1) modules, refreshed from the engine when read."""

    def __init__(self, sf):
        super().__init__()
        self._sf = sf

    def __getitem__(self, i):
        lin = super().__getitem__(i)
        sf = self._sf
        if isinstance(i, int) and sf._eng is not None and sf._eng_T == len(self):
            sf._flush()
            t = i if i >= 0 else len(self) + i
            with torch.no_grad():
                lin.weight.copy_(sf._eng.get_w(t)[0].view(1, -1).to(lin.weight.device))
        return lin

    def __setitem__(self, i, v):
        super().__setitem__(i, v)
        sf = self._sf
        if isinstance(i, int) and sf._eng is not None and sf._eng_T == len(self):
            sf._eng.load_w(i if i >= 0 else len(self) + i, v.weight.detach())


class DeepSF(_deep.DeepSF):
    def reset(self):
        super().reset()
        self.fit_w = _FitWLinear(self)

    def _w_host(self, t):
        return list.__getitem__(self.fit_w, t).weight.detach()

    def _adam_groups(self, optim):
        g0 = optim.param_groups[0]
        g1 = optim.param_groups[1] if len(optim.param_groups) > 1 else g0
        return (g0["lr"], g0.get("weight_decay", 0.0)), (g1["lr"], g1.get("weight_decay", 0.0))

    def add_training_task(self, task, source=None):
        """features/deep_sequential.py:40-73 (w first, then the ψ networks)."""
        self._flush()
        self._sync_host()
        true_w = task.get_w()
        n_features = task.feature_dim()
        fit_w = torch.Tensor(1, n_features).uniform_(-0.01, 0.01).to(self.device)
        # built on the CPU and moved: its (overwritten) init draw comes from the CPU generator, as
        # in a CPU run of the reference, so seeded runs follow the reference's trajectory
        w_approx = torch.nn.Linear(n_features, 1, bias=False).to(self.device)
        with torch.no_grad():
            w_approx.weight = torch.nn.Parameter(fit_w)
        self.true_w.append(true_w)
        list.append(self.fit_w, w_approx)
        self._psi.append(self.build_successor(task, source, w_approx))
        self.n_tasks = len(self._psi)
        self.gpi_counters = [np.append(c, 0) for c in self.gpi_counters]
        self.gpi_counters.append(np.zeros((self.n_tasks,), dtype=int))

    def build_successor(self, task, source=None, w_approx=None):
        if self.n_tasks == 0:
            self.n_actions = task.action_count()
            self.n_features = task.feature_dim()
            self.inputs = task.encode_dim()
        A, d = self.n_actions, self.n_features
        model, loss, _ = self.pytorch_model_handle(self.inputs, A * d, (A, d), 1)
        if source is not None and self.n_tasks > 0:
            self._sync_host()
            update_models_weights(self._psi[source][0][0], model)
        target, _, _ = self.pytorch_model_handle(self.inputs, A * d, (A, d), 1)
        update_models_weights(model, target)
        self._since.append(0)
        target.eval()
        hp = self.hyperparameters
        optim = torch.optim.Adam([
            {"params": model.parameters(), "lr": hp["learning_rate_sf"], "weight_decay": hp["weight_decay_sf"]},
            {"params": w_approx.parameters(), "lr": hp["learning_rate_w"], "weight_decay": hp["weight_decay_w"]},
        ])
        return (model, loss, optim), (target, None, None)

    def GPI_w(self, state, w):
        weight = w.weight if isinstance(w, torch.nn.Module) else w
        return super().GPI_w(state, torch.as_tensor(weight).reshape(-1, 1))

    def update_successor(self, transitions, policy_index, use_gpi=True):
        if transitions is None:
            return None
        states, actions, rs, phis, next_states, gammas = transitions
        eng = self._engine(len(gammas))
        self._flush()
        losses = eng.update(policy_index, states, actions, rs, phis, next_states, gammas, use_gpi=use_gpi)
        self._host_stale = True
        dev = self._out_device()
        loss, l1, l2 = (x.to(dev) for x in losses)
        return loss, l1, l2
