"""Drop-in binding of sfx into a checkout of the reference.

``install()`` adds an import hook so that the reference's own training scripts and agents run
unchanged on libsfx:

* ``features`` becomes sfx's package in front of the user's: ``features.deep``,
  ``features.deep_sequential``, ``features.deep_sequential_tsf``, ``features.deep_phi`` (learned φ)
  and ``features.successor`` are sfx's SF libraries (every ψ forward, GPI, TD target, backward and Adam step in the gfx950
  kernels of libsfx.so); every other ``features.*`` module stays the user's;
* the user's single-file modules ``sfdqn``, ``tsfdqn``, ``tsfdqn_nf`` and
  ``agents.tsfdqn_sequential`` load as they are and are then bound (``sfx.dropin.bind``): their
  library classes become sfx's and the TSF agents' ``update_successor`` one libsfx call;
* ``agents.buffer`` is sfx's ``ReplayBuffer`` (the reference's API over a device-resident ring,
  the same ``np.random`` index draws; ``sfx/dropin/agents/buffer.py``);
* every other ``agents`` module, ``utils``, ``tasks`` and the scripts themselves are the user's, untouched.

sfx ships no agent code: the agents are the reference's own.
"""
from __future__ import annotations

import importlib.abc
import importlib.machinery
import importlib.util
import os
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
FEATURES = os.path.join(ROOT, "features")
AGENT_ALIASES = {"agents.buffer": os.path.join(ROOT, "agents", "buffer.py")}
OURS = ("features.deep", "features.deep_sequential", "features.deep_sequential_tsf", "features.deep_phi",
        "features.successor")
BOUND = ("sfdqn", "tsfdqn", "tsfdqn_nf", "agents.tsfdqn_sequential", "agents.sfdqn_phi")


class _BindingLoader(importlib.abc.Loader):
    def __init__(self, inner, name):
        self.inner, self.name = inner, name

    def create_module(self, spec):
        return self.inner.create_module(spec)

    def exec_module(self, module):
        self.inner.exec_module(module)
        from . import bind

        bind.patch(self.name, module)


class _Finder(importlib.abc.MetaPathFinder):
    """``features`` -> sfx's package (then the user's); BOUND modules -> the user's, bound."""

    def find_spec(self, fullname, path=None, target=None):
        if fullname == "features":
            user = importlib.machinery.PathFinder.find_spec("features")
            locs = [FEATURES]
            if user is not None and user.submodule_search_locations:
                locs += [p for p in user.submodule_search_locations if os.path.abspath(p) != FEATURES]
            return importlib.util.spec_from_file_location("features", os.path.join(FEATURES, "__init__.py"),
                                                          submodule_search_locations=locs)
        if fullname in AGENT_ALIASES:  # the user's agents package, sfx's module
            return importlib.util.spec_from_file_location(fullname, AGENT_ALIASES[fullname])
        if fullname in BOUND:
            spec = importlib.machinery.PathFinder.find_spec(fullname, path)
            if spec is None or spec.loader is None:
                return None
            spec.loader = _BindingLoader(spec.loader, fullname)
            return spec
        return None


def install() -> str:
    """Install the hook (idempotent) and drop already-imported copies of the affected modules."""
    if not any(isinstance(f, _Finder) for f in sys.meta_path):
        sys.meta_path.insert(0, _Finder())
    for name in list(sys.modules):
        if name == "features" or name.startswith("features.") or name in BOUND or name in AGENT_ALIASES:
            del sys.modules[name]
    return ROOT
