"""The single-file SF-DQN (sfdqn.py: ReplayBuffer, DeepSF, SFDQN) on libsfx.

sfdqn.py:12-994 is the sequential SF-DQN stack in one file -- the same as
agents.buffer_sequential / features.deep_sequential / agents.sfdqn_sequential here (active-task
updates with loss l1 + l2 and an Adam-trained reward model, sfdqn.py:303-371; test tasks with
Adam-trained reward models, sfdqn.py:681-738) -- except how an env action is chosen: the
ε-draw comes first and GPI (with its usage counters) runs only for greedy steps
(sfdqn.py:578-594), where agents/agent.py always runs GPI first.
"""
from __future__ import annotations

import random

import torch

from agents import sfdqn_sequential as _agent
from agents.buffer_sequential import ReplayBuffer as _ReplayBuffer
from features import deep_sequential as _lib


class ReplayBuffer(_ReplayBuffer):
    """sfdqn.py:12-92 (keyword arguments only)."""

    def __init__(self, n_samples=1000000, n_batch=32):
        super().__init__(n_samples=n_samples, n_batch=n_batch)


class DeepSF(_lib.DeepSF):
    """sfdqn.py:94-371."""

    def __init__(self, pytorch_model_handle, use_true_reward=False, target_update_ev=1000, **kwargs):
        super().__init__(pytorch_model_handle, target_update_ev=target_update_ev, use_true_reward=use_true_reward,
                         **kwargs)


class SFDQN(_agent.SFDQN):
    """sfdqn.py:374-994."""

    def _select_action(self):
        if random.random() <= self.epsilon:
            a = torch.tensor(random.randrange(self.n_actions)).to(self.device)
        else:
            with torch.no_grad():
                q, c = self.sf.GPI(self.s_enc, self.task_index, update_counters=self.use_gpi)
                if not self.use_gpi:
                    c = self.task_index
                self.c = c
                q = q[:, c, :].flatten()
                assert q.size()[0] == self.n_actions
            a = torch.argmax(q)
        self.epsilon = max(self.epsilon * self.epsilon_decay, self.epsilon_min)
        return a
