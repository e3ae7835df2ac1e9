"""Binding of the reference modules that hold the SF library inside the same file as an agent.

The single-file scripts define their library next to their agent: ``sfdqn.DeepSF``
(sfdqn.py:94-371), ``tsfdqn.DeepTSF`` / ``tsfdqn_nf.DeepTSF`` (tsfdqn.py:93-326), and the TSF
agents carry the update itself (``TSFDQN.update_successor``, tsfdqn.py:588-709,
tsfdqn_nf.py:620-741, agents/tsfdqn_sequential.py:123-252).  ``sfx.dropin.install()`` lets the
user's own modules load unchanged and then applies ``patch``: the library classes become
sfx's, the TSF agents' update_successor becomes one libsfx call (DeepTSF.tsf_update), and their
test-task methods get_test_action / update_test_reward_mapper (tsfdqn.py:859-997, SURVEY §8f
rank 1) become libsfx calls too (DeepTSF.tsf_test_action / tsf_test_update), drawing from
Python's random module exactly where the reference does.  Nothing else of the user's agents is
touched.
"""
from __future__ import annotations

import functools
import random

import torch

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


def tsf_get_test_action(self, s_enc, w, omegas):
    """TSFDQN.get_test_action (tsfdqn.py:859-870): the same ε draw from Python's random module;
    the greedy branch argmax_a w·Σ_t ω̂_t ψ_t(s)[a] is one library call (sfx_tsf_test_action)."""
    with torch.no_grad():
        if random.random() <= self.test_epsilon:
            return torch.tensor(random.randrange(self.n_actions)).to(self.device)
        return self.sf.tsf_test_action(s_enc, w, omegas)


def prints_phi_shape(agent) -> bool:
    """agents/tsfdqn_sequential.py:443 prints ``Phi values {phi.shape}`` on every call of its
    reward mapper; tsfdqn.py / tsfdqn_nf.py do not."""
    return type(agent).__module__.split(".")[-1] == "tsfdqn_sequential"


def tsf_update_test_reward_mapper(self, w_approx, omegas, optim, task, r, s, a, s1, a1):
    """TSFDQN.update_test_reward_mapper (tsfdqn.py:917-997, agents/tsfdqn_sequential.py:435-520) as
    one library call (sfx_tsf_test_update): φ from the user's task, the learning rates and weight
    decays read from the agent's optimizer groups (its LambdaLR keeps decaying ω's), the Adam step
    on the device.  Returns (loss, l2, l1) as the reference does.

    Console output: agents/tsfdqn_sequential.py's unconditional ``Phi values`` line is printed as
    the reference does; the occasional diagnostic block (every 1000th training step, when
    ``random.randint(1, 1000) < 10``) draws from the same random stream but prints ONE line (the
    task's ω and w) instead of the reference's block of intermediate tensors, and ``omegas.grad`` /
    ``w_approx.weight.grad`` are not populated (the gradients live on the device only)."""
    if self.h_function is None:
        raise Exception('Affine Function (h) is not initialized')
    phi = task.features(s, a, s1)
    if prints_phi_shape(self):
        print(f'Phi values {phi.shape}')
    gw, go = optim.param_groups[0], optim.param_groups[1]
    for grp in (gw, go):
        if tuple(grp.get("betas", (0.9, 0.999))) != (0.9, 0.999) or grp.get("eps", 1e-8) != 1e-8:
            raise NotImplementedError("sfx: the test reward mapper's Adam runs with betas (0.9, 0.999), eps 1e-8")
    hp = self.hyperparameters
    loss, l2, l1 = self.sf.tsf_test_update(w_approx, omegas, phi, r, s, a, s1, a1, gamma=self.gamma,
                                           beta=hp['beta_loss_coefficient'], lasso=hp['omegas_l1_coefficient'],
                                           lr_w=gw['lr'], wd_w=gw['weight_decay'], lr_o=go['lr'],
                                           wd_o=go['weight_decay'])
    # the reference's occasional diagnostic print draws from the same random stream
    if self.total_training_steps % 1000 == 0 and random.randint(1, 1000) < 10:
        print(f'Target Task {task} omegas {omegas.detach()} weights {w_approx.weight.detach()}')
    return loss, l2, l1


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
    if hasattr(cls, "get_test_action") and hasattr(cls, "update_test_reward_mapper"):
        cls.get_test_action = tsf_get_test_action
        cls.update_test_reward_mapper = tsf_update_test_reward_mapper
    for name in ("test_agent",):
        m = getattr(cls, name, None)
        if m is not None and not getattr(m, "__sfx_bound__", False):
            setattr(cls, name, _synced(m))


def _phi_synced(method):
    """Run the agent's own method after the device's φ net is copied into the agent's module (its
    test reward mapper, agents/sfdqn_phi.py update_test_reward_mapper, runs φ in torch)."""
    @functools.wraps(method)
    def run(self, *args, **kwargs):
        sync = getattr(self.sf, "sync_phi_module", None)
        if sync is not None:
            sync()
        return method(self, *args, **kwargs)

    run.__sfx_bound__ = True
    return run


def patch(name: str, module) -> None:
    """Bind the user's freshly loaded module ``name`` to sfx (see the module docstring)."""
    if name == "sfdqn":
        module.DeepSF = SingleFileDeepSF
    elif name in ("tsfdqn", "tsfdqn_nf"):
        module.DeepTSF = SingleFileDeepTSF
        patch_tsf_agent(module.TSFDQN)
    elif name == "agents.tsfdqn_sequential":
        patch_tsf_agent(module.TSFDQN)
    elif name == "agents.sfdqn_phi":
        m = getattr(module.SFDQN_PHI, "test_agent", None)
        if m is not None and not getattr(m, "__sfx_bound__", False):
            module.SFDQN_PHI.test_agent = _phi_synced(m)
