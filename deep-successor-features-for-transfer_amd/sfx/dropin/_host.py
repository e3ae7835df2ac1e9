"""What the drop-in library takes from the host program: the torch device the training script
chose (the reference's ``utils.torch`` global, set by ``set_torch_device`` before the library is
built) and the target-network copy of utils/torch.py:31-33.  The user's utils package is read
when it is importable; replays without it (tests/test_gpu_dropin.py) get ``None`` -- outputs then
stay on the engine's device."""
from __future__ import annotations

import sys

import torch


_absent_on = None  # sys.path for which importing utils.torch last failed (a failed import is not cached by Python)


def torch_device():
    global _absent_on
    mod = sys.modules.get("utils.torch")
    if mod is None:
        path = tuple(sys.path)
        if path == _absent_on:
            return None
        try:
            import utils.torch as mod  # the user's checkout
        except ImportError:
            _absent_on = path
            return None
    get = getattr(mod, "get_torch_device", None)
    return get() if get is not None else getattr(mod, "device", None)


def copy_weights(model: torch.nn.Module, target_model: torch.nn.Module) -> None:
    """target <- model, parameter by parameter (update_models_weights, utils/torch.py:31-33)."""
    with torch.no_grad():
        for dst, src in zip(target_model.parameters(), model.parameters()):
            dst.copy_(src)
