"""Drop-in module tree for the reference's training scripts.

``install()`` puts this directory first on ``sys.path`` so that the imports of
main_sfdqn_torch.py -- ``features.deep``, ``agents.sfdqn``, ``agents.buffer``,
``utils.torch``, ``utils.config``, ``utils.logger``, ``utils.types``, ``tasks.reacher``; those
of the sequential SF / TSF scripts and the single-file ``sfdqn``, ``tsfdqn``, ``tsfdqn_nf`` --
resolve to this package's modules, whose ``DeepSF`` runs every ψ / GPI / TD / Adam
computation in libsfx.so (hand-written gfx950 kernels).  The modules are written for sfx;
they reproduce the reference's public names, argument meanings, return conventions and
RNG consumption (Python ``random`` for ε-greedy, ``np.random`` for replay sampling, the
torch RNG for weight init), so a seeded run takes the same trajectory.
"""
from __future__ import annotations

import os
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))


def install() -> str:
    """Make ``import features.deep`` & co. resolve to the drop-in modules."""
    if ROOT not in sys.path:
        sys.path.insert(0, ROOT)
    for name in list(sys.modules):
        top = name.split(".")[0]
        if top in ("features", "agents", "utils", "tasks", "sfdqn", "tsfdqn", "tsfdqn_nf"):
            mod = sys.modules[name]
            if not (getattr(mod, "__file__", "") or "").startswith(ROOT):
                del sys.modules[name]
    return ROOT
