"""Synthetic Reacher-shaped task: s ~ N(0,1)^n_s, φ ~ U[0,1)^d,
r = φ·w_true with one-hot w_true, fixed episode length, own RNG (does not touch the global
torch / numpy / random streams the agent uses)."""
from __future__ import annotations

import numpy as np
import torch

from tasks.task import Task
from utils.torch import get_torch_device


class SyntheticReacher(Task):
    def __init__(self, n_s=17, n_actions=7, d=8, task_index=0, seed=0, terminal_every=0):
        self.n_s, self.A, self.d, self.task_index = n_s, n_actions, d, task_index
        self.rng = np.random.default_rng(seed)
        self.terminal_every = terminal_every
        self.t = 0
        self._phi = None

    def clone(self):
        return SyntheticReacher(self.n_s, self.A, self.d, self.task_index, int(self.rng.integers(1 << 30)),
                                self.terminal_every)

    def _dev(self):
        return get_torch_device() or torch.device("cpu")

    def initialize(self):
        return torch.from_numpy(self.rng.standard_normal(self.n_s).astype(np.float32)).to(self._dev())

    def action_count(self):
        return self.A

    def transition(self, action):
        self.t += 1
        s1 = torch.from_numpy(self.rng.standard_normal(self.n_s).astype(np.float32)).to(self._dev())
        phi = self.rng.random(self.d).astype(np.float32)
        phi += np.float32(0.01 * (int(action) % 3))
        self._phi = torch.from_numpy(phi).to(self._dev())
        r = float(phi[self.task_index % self.d])
        done = bool(self.terminal_every) and self.t % self.terminal_every == 0
        return s1, r, done

    def encode(self, state):
        return torch.as_tensor(state).detach().reshape((1, -1)).to(self._dev())

    def encode_dim(self):
        return self.n_s

    def features(self, state, action, next_state):
        return self._phi

    def feature_dim(self):
        return self.d

    def get_w(self):
        w = torch.zeros((self.d, 1)).to(self._dev())
        w[self.task_index % self.d, 0] = 1.0
        return w
