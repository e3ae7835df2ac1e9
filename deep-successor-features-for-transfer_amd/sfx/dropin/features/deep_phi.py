"""DeepSF_PHI on the GPU (the interface of features/deep_phi.py:11-300, the library of
main_sfdqn_phi_torch.py with agents/sfdqn_phi.py): learned φ, SURVEY §8f rank 4.

The ψ heads, their targets and each task's reward model (an nn.Linear(d, 1) WITH bias,
features/deep_phi.py:280) live in a libsfx engine; the agent's φ net (phis_model, handed to every
update_successor call) is loaded into the engine on the first update and trained there
(sfx_phi_update: φ of the minibatch, GPI / own-ψ next actions, targets φ + γ ψ⁻_i(s1)[a'] that
carry φ's gradient, loss = MSE(w_i(φ), r) + λ_i MSE(ψ_i(s), merged), one freshly built Adam step
on ψ_i, φ, w_i (lr 1e-3, as the reference hard-codes) and ascent on λ_i, clamped to [1e-2, 1e6]).
The agent's loss coefficient and each reward model's bias are updated in place when they live on
the engine's device (staged through it otherwise).
``sync_phi_module`` copies the device's φ into the agent's module (sfx.dropin.bind calls it before
the agent's test episodes, which run the φ net in torch).
"""
from __future__ import annotations

import numpy as np
import torch

from . import deep as _deep
from .deep import _flat, _unflat_into

LR = 1e-3  # features/deep_phi.py:163-175: every parameter group of the update


def _phi_geometry(model: torch.nn.Module, n_s: int, d: int):
    """(width_mul, n_mid) of main_sfdqn_phi_torch.py's phi_model_lambda net; raises otherwise."""
    mods = [m for m in model.modules() if m is not model and not isinstance(m, torch.nn.Sequential)]
    lin = [m for m in mods if isinstance(m, torch.nn.Linear)]
    n_in = 2 * n_s + 1
    ok = len(lin) >= 2 and len(mods) == 2 * len(lin) - 1 and all(l.bias is not None for l in lin)
    ok = ok and all(isinstance(mods[2 * j + 1], torch.nn.ReLU) for j in range(len(lin) - 1))
    hid = lin[0].out_features if lin else 0
    ok = ok and lin[0].in_features == n_in and hid % n_in == 0 and lin[-1].out_features == d
    ok = ok and all(l.in_features == hid and l.out_features == hid for l in lin[1:-1]) and lin[-1].in_features == hid
    if not ok:
        raise NotImplementedError("sfx DeepSF_PHI: φ net must be Linear(2 n_s + 1, k (2 n_s + 1)) + ReLU, "
                                  f"[Linear(hid, hid) + ReLU]*, Linear(hid, d); got {model}")
    return hid // n_in, len(lin) - 2


class _FitWBias(list):
    """fit_w entries: nn.Linear(d, 1) with bias.  The engine owns the weight rows once it exists
    (refreshed on read); the bias stays in the module's own tensor, which the device updates in
    place (when it lives on the engine's device) or a staging copy does."""

    def __init__(self, sf):
        super().__init__()
        self._sf = sf

    def __getitem__(self, i):
        lin = super().__getitem__(i)
        sf = self._sf
        if isinstance(i, int) and sf._phi_ready():
            t = i if i >= 0 else len(self) + i
            with torch.no_grad():
                lin.weight.copy_(sf._eng.get_w(t)[0].view(1, -1).to(lin.weight.device))
        return lin


class DeepSF_PHI(_deep.DeepSF):
    def __init__(self, pytorch_model_handle, *args, target_update_ev=1000, max_batch=64, **kwargs):
        # the φ kernels hold a minibatch of up to 64 rows (sfx_phi.h PHI_B)
        super().__init__(pytorch_model_handle, *args, target_update_ev=target_update_ev, max_batch=max_batch, **kwargs)

    def reset(self):
        super().reset()
        self.fit_w = _FitWBias(self)
        self._phi_model = self._phi_eng = None

    def add_training_task(self, task, source=None):
        """features/deep_phi.py:254-285: the ψ networks first, then a biased Linear(d, 1)."""
        self._flush()
        self._sync_host()
        if self._eng is not None:
            raise NotImplementedError("sfx DeepSF_PHI: add every training task before the first update")
        self._psi.append(self.build_successor(task, source))
        self.n_tasks = len(self._psi)
        true_w = task.get_w()
        fit_w = torch.nn.Linear(task.feature_dim(), 1).to(self.device)
        list.append(self.fit_w, fit_w)
        self.true_w.append(true_w)
        self.gpi_counters = [np.append(c, 0) for c in self.gpi_counters]
        self.gpi_counters.append(np.zeros((self.n_tasks,), dtype=int))

    def _w_host(self, t):
        return list.__getitem__(self.fit_w, t).weight.detach()

    def _phi_ready(self):
        return self._eng is not None and self._eng_T == self.n_tasks and self._phi_model is not None

    def _phi_engine(self, phi_model, batch):
        eng = self._engine(batch)
        if self._phi_model is None:
            width_mul, n_mid = _phi_geometry(phi_model, self.inputs, self.n_features)
            eng.set_adam(LR, 0.0, LR, 0.0)  # the update's own Adam (features/deep_phi.py:163-175)
            eng.phi_setup(width_mul, n_mid, LR)
            eng.phi_load(_flat(phi_model))
            self._phi_model, self._phi_eng = phi_model, eng
        elif phi_model is not self._phi_model:
            raise NotImplementedError("sfx DeepSF_PHI: one φ net per library")
        elif eng is not self._phi_eng:
            raise NotImplementedError("sfx DeepSF_PHI: the engine was rebuilt (a larger minibatch) after φ training began")
        return eng

    def _dev_scalar(self, t: torch.Tensor, eng):
        """t itself when the device can update it in place, else a staged copy (written back)."""
        if t.device == eng.device and t.dtype == torch.float32 and t.is_contiguous() and t.numel() == 1:
            return t, False
        return t.detach().reshape(1).to(eng.device, torch.float32).contiguous(), True

    def sync_phi_module(self):
        """Copy the device's φ net into the agent's module."""
        if self._phi_ready():
            _unflat_into(self._phi_model, self._eng.phi_get())

    # ------------------------------------------------------------------ GPI with the biased w
    def GPI_w(self, state, w):
        s = self._state(state)
        eng = self._engine(s.shape[0])
        self._flush()
        weight = w.weight if isinstance(w, torch.nn.Module) else torch.as_tensor(w)
        _, q, _, _ = eng.gpi(s, w=weight.detach().reshape(-1))
        if isinstance(w, torch.nn.Module) and w.bias is not None:
            q = q + w.bias.detach().to(q.device).reshape(1, 1, 1)
        task = torch.argmax(torch.max(q, dim=2).values, dim=1)
        dev = self._out_device()
        return q.to(dev), torch.squeeze(task).to(dev)

    def GPI(self, state, task_index, update_counters=False):
        q, task = self.GPI_w(state, self.fit_w[task_index])
        if update_counters:
            self._count(task_index, task)
        return q, task

    def update_reward(self, phi, r, task_index, exact=False):
        raise Exception('This function should not be used')

    # ------------------------------------------------------------------ training
    def update_successor(self, transitions, phis_model, policy_index, loss_coefficient, use_gpi):
        """features/deep_phi.py:93-224 -> (loss, psi_loss, phi_loss, loss_coefficient)."""
        if transitions is None:
            return
        states, actions, rs, _, next_states, gammas = transitions
        (phi_model, _, _), _ = phis_model
        eng = self._phi_engine(phi_model, len(gammas))
        self._flush()
        bias_mod = list.__getitem__(self.fit_w, policy_index).bias
        bias, bias_staged = self._dev_scalar(bias_mod.data, eng)
        lam, lam_staged = self._dev_scalar(loss_coefficient.data, eng)
        losses = eng.phi_update(policy_index, states, actions, rs, next_states, gammas, bias, lam, use_gpi=use_gpi)
        with torch.no_grad():
            if bias_staged:
                bias_mod.copy_(bias.view_as(bias_mod))
            if lam_staged:
                loss_coefficient.copy_(lam.view_as(loss_coefficient))
        self._host_stale = True
        dev = self._out_device()
        loss, psi_loss, phi_loss = (x.reshape(1).to(dev) for x in (losses[0], losses[1], losses[2]))
        return loss, psi_loss, phi_loss, loss_coefficient
