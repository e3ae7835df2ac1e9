"""utils/types.py: the ψ factory returns (model, loss, optim) -- any tuple."""
from typing import Any

ModelTuple = Any
