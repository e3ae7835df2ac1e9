"""The single-file TSF-DQN with planar-flow g_i (tsfdqn_nf.py, imported by
main_tsfdqn_sequential_torch_nf.py: ``from tsfdqn_nf import TSFDQN, ReplayBuffer, DeepTSF``) on libsfx.

Same agent and library as the sequential TSF stack (agents.tsfdqn_sequential,
features.deep_sequential_tsf; tsfdqn_nf.py:12-1044 repeats them in one file) except g_i: K planar
flows z <- z + u tanh(w·z + b) followed by nn.Linear(n_s, G) (PlanarFlow.build_planar_flow,
tsfdqn_nf.py:331-358), K = hyperparameters['n_coupling_layers'].  The flows, Linear, h, ψ_i and
w_i train on the device in one sfx_tsf_update call per env step.  Unlike the reference on a GPU
(its PlanarFlow parameters are moved with ``.to(device)`` after wrapping and so are not
registered), the flows here are registered and train on any device, as
they do in the reference's CPU configuration.
"""
from __future__ import annotations

import torch

from agents import tsfdqn_sequential as _agent
from agents.buffer_tsf_sequential import ReplayBuffer  # noqa: F401  (tsfdqn_nf.py:12-92)
from features import deep_sequential_tsf as _lib
from utils.torch import get_torch_device


class DeepTSF(_lib.DeepTSF):
    """tsfdqn_nf.py:95-327 (``use_true_reward`` is positional there)."""

    def __init__(self, pytorch_model_handle, use_true_reward, target_update_ev=1000, **kwargs):
        super().__init__(pytorch_model_handle, target_update_ev=target_update_ev, use_true_reward=use_true_reward,
                         **kwargs)


class PlanarFlow(torch.nn.Module):
    """z + scale * tanh(weight·z + bias) (tsfdqn_nf.py:331-358); parameters initialised on the CPU
    in the reference's order (weight, scale, bias ~ U(-0.01, 0.01)) and then moved."""

    def __init__(self, dim):
        super().__init__()
        self.weight = torch.nn.Parameter(torch.Tensor(1, dim))
        self.bias = torch.nn.Parameter(torch.Tensor(1))
        self.scale = torch.nn.Parameter(torch.Tensor(1, dim))
        self.tanh = torch.nn.Tanh()
        self.reset_parameters()

    def reset_parameters(self):
        self.weight.data.uniform_(-0.01, 0.01)
        self.scale.data.uniform_(-0.01, 0.01)
        self.bias.data.uniform_(-0.01, 0.01)

    def forward(self, z):
        return z + self.scale * self.tanh(torch.nn.functional.linear(z, self.weight, self.bias))

    @classmethod
    def build_planar_flow(cls, input_dim, output_dim, n_affine_flows):
        flows = [cls(input_dim) for _ in range(n_affine_flows)]
        flows.append(torch.nn.Linear(input_dim, output_dim, bias=True))
        return torch.nn.Sequential(*flows).to(get_torch_device())


class TSFDQN(_agent.TSFDQN):
    """tsfdqn_nf.py:361-1044: the sequential TSF agent with planar-flow g_i."""

    def _init_g_function(self, states_dim, output_dim, n_coupling_layers=1):
        return PlanarFlow.build_planar_flow(states_dim, output_dim, n_coupling_layers)

    def add_training_task(self, task):
        _agent.Agent.add_training_task(self, task)
        self.buffers.append(self.buffer_handle())
        dims = self.hyperparameters.get("g_h_function_dims")
        g_function = self._init_g_function(task.encode_dim(), dims, self.hyperparameters.get("n_coupling_layers", 1))
        self.g_functions.append(g_function)
        if self.h_function is None:
            self.h_function = self._init_h_function(dims, task.feature_dim())
        self.sf.add_training_task(task, None, g_function, self.h_function)
