"""Process-wide torch device and model helpers (the names of the reference's utils/torch.py).

``device`` is the global the reference's modules read (agents/agent.py imports it by name at
import time, so ``set_torch_device`` must run first, as in main_sfdqn_torch.py:33).
"""
from __future__ import annotations

import os
import random

import numpy as np
import torch

device = None

_ACTIVATIONS = {"relu": torch.nn.ReLU, "tanh": torch.nn.Tanh}


def set_torch_device(use_gpu: bool = False, gpu_device_index: int = 0):
    global device
    if device is None:
        on_gpu = bool(use_gpu) and torch.cuda.is_available()
        device = torch.device(f"cuda:{gpu_device_index}" if on_gpu else "cpu")
        print(f"Using {device}")
    return device


def get_torch_device():
    return device


def get_activation(name: str):
    try:
        return _ACTIVATIONS[name]
    except KeyError:
        raise Exception("Activation name not supported") from None


def update_models_weights(model: torch.nn.Module, target_model: torch.nn.Module) -> None:
    """Copy model's parameters into target_model's, in parameters() order."""
    with torch.no_grad():
        for dst, src in zip(target_model.parameters(), model.parameters()):
            dst.data.copy_(src.data)


def set_random_seed(seed: int = 1024) -> None:
    np.random.seed(seed)
    random.seed(seed)
    torch.manual_seed(seed)
    torch.cuda.manual_seed_all(seed)
    torch.backends.cudnn.deterministic = True
    torch.backends.cudnn.benchmark = False
    os.environ["PYTHONHASHSEED"] = str(seed)
    print(f"Random seed set as {seed}")
