"""Abstract successor-feature library (the interface of features/successor.py:6-290).

Host-side bookkeeping only: the reward weights ``fit_w`` ([d, 1] tensors), the true weights,
GPI usage counters.  ``features.deep.DeepSF`` supplies the ψ evaluation and training on the
GPU and overrides the methods whose work belongs on the device.
"""
from __future__ import annotations

import numpy as np
import torch

from sfx.dropin._host import torch_device as get_torch_device


class SF:
    def __init__(self, *args, use_true_reward=False, **kwargs):
        self.use_true_reward = use_true_reward
        self.hyperparameters = kwargs.pop("hyperparameters", {})
        self.alpha_w = self.hyperparameters.get("learning_rate_w")
        if args or kwargs:
            print(f"{type(self).__name__} ignoring parameters {args} and {kwargs}")
        self.device = get_torch_device()

    # ---- library management (features/successor.py:114-144)
    def reset(self):
        self.n_tasks = 0
        self._psi = []
        self.true_w = []
        self.fit_w = []
        self.gpi_counters = []

    @property
    def psi(self):
        return self._psi

    def build_successor(self, task, source=None):
        raise NotImplementedError

    def get_successor(self, state, policy_index):
        raise NotImplementedError

    def get_successors(self, state):
        raise NotImplementedError

    def update_successor(self, transitions, policy_index):
        raise NotImplementedError

    def add_training_task(self, task, source=None):
        self._psi.append(self.build_successor(task, source))
        self.n_tasks = len(self._psi)
        true_w = task.get_w()
        self.true_w.append(true_w)
        if self.use_true_reward:
            fit_w = true_w
        else:
            fit_w = torch.Tensor(task.feature_dim(), 1).uniform_(-0.01, 0.01).to(self.device)
        self.fit_w.append(fit_w)
        self.gpi_counters = [np.append(c, 0) for c in self.gpi_counters]
        self.gpi_counters.append(np.zeros((self.n_tasks,), dtype=int))

    # ---- reward model (features/successor.py:146-173): least-mean-squares step on w
    def update_reward(self, phi, r, task_index, exact=False):
        w = self.fit_w[task_index]
        phi = phi.reshape(w.shape)
        r_fit = torch.sum(phi * w)
        self.fit_w[task_index] = w + self.alpha_w * (r - r_fit) * phi
        if exact:
            r_true = torch.sum(phi * self.true_w[task_index])
            if not torch.allclose(r, r_true):
                raise Exception(f"sampled reward {r} != linear reward {r_true} - please check task {task_index}!")

    # ---- GPE / GPI (features/successor.py:175-290)
    def GPE_w(self, state, policy_index, w):
        return self.get_successor(state, policy_index) @ w

    def GPE(self, state, policy_index, task_index):
        return self.GPE_w(state, policy_index, self.fit_w[task_index])

    def GPI_w(self, state, w):
        psi = self.get_successors(state)
        q = (psi @ w)[:, :, :, 0]
        task = torch.squeeze(torch.argmax(torch.max(q, axis=2).values, axis=1))
        return q, task

    def GPI(self, state, task_index, update_counters=False):
        q, task = self.GPI_w(state, self.fit_w[task_index])
        if update_counters:
            self._count(task_index, task)
        return q, task

    # The GPI counters (features/successor.py:266-272 increments them inside GPI).  A device task
    # tensor is not read back at every call -- that would be a device synchronisation per env step
    # beside the agent's own (its greedy action) -- but kept, and the counts are settled on the host
    # whenever ``gpi_counters`` is read (GPI_usage_percent, the agents' logs) or every _GPI_SETTLE
    # calls: one transfer for all of them.  The counts read are the reference's.
    _GPI_SETTLE = 4096

    @property
    def gpi_counters(self):
        pend = self.__dict__.get("_gpi_pending")
        if pend:
            self._gpi_pending = []
            counts = self.__dict__["_gpi_counts"]
            flat = [p[1].reshape(-1) for p in pend]
            idx = torch.cat([t.to(flat[0].device) for t in flat]).cpu().numpy()
            off = 0
            for (ti, _), t in zip(pend, flat):  # per call, as the reference's counts[ti][idx] += 1
                counts[ti][idx[off:off + t.numel()]] += 1
                off += t.numel()
        return self.__dict__.get("_gpi_counts")

    @gpi_counters.setter
    def gpi_counters(self, value):
        self.__dict__["_gpi_pending"] = []
        self.__dict__["_gpi_counts"] = value

    def _count(self, task_index, task):
        if type(task) is torch.Tensor and task.is_cuda:
            pend = self.__dict__.setdefault("_gpi_pending", [])
            pend.append((task_index, task))
            if len(pend) >= self._GPI_SETTLE:
                self.gpi_counters
            return
        idx = task.detach().numpy() if torch.is_tensor(task) else np.asarray(task)
        self.gpi_counters[task_index][idx] += 1

    def GPI_usage_percent(self, task_index):
        counts = self.gpi_counters[task_index]
        return 1.0 - float(counts[task_index]) / np.sum(counts)
