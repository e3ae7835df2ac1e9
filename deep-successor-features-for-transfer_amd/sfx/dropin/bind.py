"""Binding of the reference modules that hold the SF library inside the same file as an agent.

The single-file scripts define their library next to their agent: ``sfdqn.DeepSF``
(sfdqn.py:94-371), ``tsfdqn.DeepTSF`` / ``tsfdqn_nf.DeepTSF`` (tsfdqn.py:93-326), and the TSF
agents carry the update itself (``TSFDQN.update_successor``, tsfdqn.py:588-709,
tsfdqn_nf.py:620-741, agents/tsfdqn_sequential.py:123-252).  ``sfx.dropin.install()`` lets the
user's own modules load unchanged and then applies ``patch``: the library classes become
sfx's, and the TSF agents' update_successor becomes one libsfx call (DeepTSF.tsf_update).
Nothing else of the user's agents is touched.
"""
from __future__ import annotations

import functools

from .features import deep_sequential as _seq
from .features import deep_sequential_tsf as _tsf


class SingleFileDeepSF(_seq.DeepSF):
    """sfdqn.py:94-371's constructor: (pytorch_model_handle, use_true_reward=False, target_update_ev=1000)."""

    def __init__(self, pytorch_model_handle, use_true_reward=False, target_update_ev=1000, **kwargs):
        super().__init__(pytorch_model_handle, target_update_ev=target_update_ev, use_true_reward=use_true_reward,
                         **kwargs)


class SingleFileDeepTSF(_tsf.DeepTSF):
    """tsfdqn.py:93-326 / tsfdqn_nf.py:95-327's constructor: ``use_true_reward`` is positional."""

    def __init__(self, pytorch_model_handle, use_true_reward, target_update_ev=1000, **kwargs):
        super().__init__(pytorch_model_handle, target_update_ev=target_update_ev, use_true_reward=use_true_reward,
                         **kwargs)


def tsf_update_successor(self, transitions, policy_index, use_gpi=True):
    """TSFDQN.update_successor (tsfdqn.py:588-709) as one device call: GPI (or own-ψ) next actions,
    φ̃ = (h(g_i(s)) + h(g_i(s'))) ⊙ φ, TD target, l1 + β l2, Adam over {ψ_i, w_i, g_i, h}, target
    sync -- with the agent's g_i and h, which the library received in add_training_task.
    Returns (loss, l1, l2) as the reference does."""
    if transitions is None:
        return None
    if self.h_function is None:
        raise Exception("Affine Function (h) is not initialized")
    return self.sf.tsf_update(transitions, policy_index, use_gpi,
                              beta=self.hyperparameters["beta_loss_coefficient"])


def _synced(method):
    """Run the agent's own method after the device's g_i / h are copied into its modules (the test
    tasks' reward mapper, tsfdqn.py:874-997, reads them in torch)."""
    @functools.wraps(method)
    def run(self, *args, **kwargs):
        sync = getattr(self.sf, "sync_tsf_modules", None)
        if sync is not None:
            sync()
        return method(self, *args, **kwargs)

    run.__sfx_bound__ = True
    return run


def patch_tsf_agent(cls) -> None:
    cls.update_successor = tsf_update_successor
    for name in ("test_agent", "update_test_reward_mapper"):
        m = getattr(cls, name, None)
        if m is not None and not getattr(m, "__sfx_bound__", False):
            setattr(cls, name, _synced(m))


def patch(name: str, module) -> None:
    """Bind the user's freshly loaded module ``name`` to sfx (see the module docstring)."""
    if name == "sfdqn":
        module.DeepSF = SingleFileDeepSF
    elif name in ("tsfdqn", "tsfdqn_nf"):
        module.DeepTSF = SingleFileDeepTSF
        patch_tsf_agent(module.TSFDQN)
    elif name == "agents.tsfdqn_sequential":
        patch_tsf_agent(module.TSFDQN)
