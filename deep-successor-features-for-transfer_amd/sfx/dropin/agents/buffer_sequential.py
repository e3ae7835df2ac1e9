"""Uniform experience replay of the sequential scripts (the interface of
agents/buffer_sequential.py:8-87, main_sfdqn_sequential_torch.py).

Samples are (state, action, reward, features φ, next state, γ); the reward is stored as a
float tensor.  ``replay`` draws indices with ``np.random.randint`` like the reference (seeded
runs sample the same rows) and returns tensors on the torch device, or None while fewer than
n_batch samples are stored.
"""
from __future__ import annotations

import numpy as np
import torch

from utils.torch import get_torch_device


class ReplayBuffer:
    def __init__(self, *args, n_samples=1000000, n_batch=32, **kwargs):
        self.n_samples = n_samples
        self.n_batch = n_batch
        self.device = get_torch_device()
        self.reset()

    def reset(self):
        self.buffer = np.empty(self.n_samples, dtype=object)
        self.index = 0
        self.size = 0

    def append(self, state, action, reward, phi, next_state, gamma):
        self.buffer[self.index] = (state, action, torch.as_tensor(reward).float(), phi, next_state, gamma)
        self.size = min(self.size + 1, self.n_samples)
        self.index = (self.index + 1) % self.n_samples

    def replay(self):
        if self.size < self.n_batch:
            return None
        rows = self.buffer[np.random.randint(low=0, high=self.size, size=(self.n_batch,))]
        states, actions, rewards, phis, next_states, gammas = zip(*rows)
        dev = self.device
        return (torch.vstack(states).to(dev), torch.tensor(actions).to(dev), torch.vstack(rewards).to(dev),
                torch.vstack(phis).to(dev), torch.vstack(next_states).to(dev), torch.tensor(gammas).to(dev))
