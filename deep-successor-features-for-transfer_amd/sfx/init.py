"""Parameter initialisation matching the reference ψ lambda (main_sfdqn_torch.py:44-78).

Heads are built exactly as the reference builds them -- torch default nn.Linear init, in
Sequential order -- and flattened to torch packing, so a seed gives the same weights the
reference would get (the reference draws fit_w first in sfdqn.py:196-207; we follow the
features/deep.py order: ψ first, then w ~ U(-0.01, 0.01), features/successor.py:128-138).
"""
from __future__ import annotations

from collections import OrderedDict
from typing import Sequence

import torch

ACTS = {"relu": torch.nn.ReLU, "tanh": torch.nn.Tanh}


def psi_module(n_s: int, H: int, A: int, d: int, acts: Sequence[str] = ("relu", "relu")) -> torch.nn.Sequential:
    layers = OrderedDict()
    layers["layer_input"] = torch.nn.Linear(n_s, H)
    for j, a in enumerate(acts):
        layers[f"layer_{j}"] = torch.nn.Linear(H, H)
        layers[f"activation_layer_{j}"] = ACTS[a]()
    layers["layer_output"] = torch.nn.Linear(H, A * d)
    layers["layer_unflatten"] = torch.nn.Unflatten(1, (A, d))
    return torch.nn.Sequential(layers)


def flatten(module: torch.nn.Module) -> torch.Tensor:
    return torch.cat([p.detach().reshape(-1) for p in module.parameters()])


def reference_heads(T: int, n_s: int, H: int, A: int, d: int, acts=("relu", "relu"), seed: int = 0):
    """(online [T, P], w [T, d]) under torch.manual_seed(seed)."""
    torch.manual_seed(seed)
    heads, ws = [], []
    for _ in range(T):
        heads.append(flatten(psi_module(n_s, H, A, d, acts)))
        ws.append(torch.empty(d).uniform_(-0.01, 0.01))
    return torch.stack(heads), torch.stack(ws)
