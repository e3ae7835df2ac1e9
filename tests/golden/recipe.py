"""Shapes and the seed recipe behind the golden fixtures (our own code, data generation only).

Full-size (H=256) heads are too large to commit, so ``full_size_heads`` regenerates
them deterministically with torch's CPU RNG (torch 2.10.0 in this image, here and
on the GPU box); the fixture stores a checksum so a drift in the recipe is caught.
"""
from __future__ import annotations

import torch

# name: (n_s, H, A, d, hidden activations)
SHAPES = {
    "reacher17": (17, 32, 7, 8, ("relu", "relu")),        # BASELINE Reacher-shape, reduced H
    "reacher17_full": (17, 256, 7, 8, ("relu", "relu")),  # BASELINE C2 at full width
    "hopper11": (11, 24, 27, 50, ("relu", "relu")),       # BASELINE C3 shape, reduced H
    "cartpole": (4, 32, 2, 20, ("relu", "relu")),         # BASELINE C1 shape, reduced H
    "refreacher": (4, 64, 9, 12, ("relu", "relu")),       # tasks/reacher.py + reacher.cfg
    "tanh_odd": (6, 48, 5, 3, ("tanh", "relu")),          # odd sizes, tanh hidden
}


def head_modules(n_s, H, A, d, acts):
    act_cls = {"relu": torch.nn.ReLU, "tanh": torch.nn.Tanh}
    mods = [torch.nn.Linear(n_s, H)]
    for a in acts:
        mods += [torch.nn.Linear(H, H), act_cls[a]()]
    mods.append(torch.nn.Linear(H, A * d))
    return torch.nn.Sequential(*mods)


def full_size_heads(T: int = 8, seed: int = 0):
    """T heads of the Reacher-shape C2 network, torch default init under manual_seed(seed);
    w rows ~ U(-0.01, 0.01) as sfdqn.py:197."""
    n_s, H, A, d, acts = SHAPES["reacher17_full"]
    torch.manual_seed(seed)
    heads = []
    for _ in range(T):
        m = head_modules(n_s, H, A, d, acts)
        heads.append(torch.cat([p.detach().reshape(-1) for p in m.parameters()]))
    gen = torch.Generator().manual_seed(seed + 1)
    w = torch.empty(T, d).uniform_(-0.01, 0.01, generator=gen)
    return torch.stack(heads), w
