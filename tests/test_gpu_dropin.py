"""The main_sfdqn_torch.py stack on sfx's drop-in modules reproduces the REAL reference run.

tests/golden/run_sfdqn_agent.npz was produced by tools/gen_golden.py with the reference's own
agents/sfdqn.py SFDQN, agents/buffer.py ReplayBuffer and features/deep.py DeepSF (CPU, torch
2.10) on the synthetic tasks of tests/golden/recipe.py.  Here the same script runs with
``sfx.dropin`` installed, so ``features.deep.DeepSF`` is the libsfx-backed library.  Same
seeds => same ε-greedy draws and replay indices, so the trajectory must match exactly:
every training and test action (GPI argmax, bit-exact), GPI usage counters, target-sync
counters; heads / reward weights within the usual Adam tolerance (test_gpu_engine.py).
"""
import contextlib
import io

import numpy as np
import pytest
import torch

from tests.conftest import gpu_available
from tests.golden.recipe import agent_run
from tests.test_gpu_engine import params_close, rel_close

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _need_gpu():
    if not gpu_available():
        pytest.skip("no HIP device")


def test_dropin_reproduces_reference_agent_run(golden):
    from sfx import dropin

    dropin.install()
    import utils.torch as ut
    from utils.logger import set_logger_level

    ut.set_torch_device(True)
    set_logger_level(False, quiet=True)
    from agents.buffer import ReplayBuffer
    from agents.sfdqn import SFDQN
    from features.deep import DeepSF

    assert DeepSF.__module__ == "features.deep" and "dropin" in __import__("features.deep").__file__
    with contextlib.redirect_stdout(io.StringIO()):
        agent, tasks, test_tasks, returns = agent_run(DeepSF, SFDQN, ReplayBuffer, ut.device)
    g = golden("run_sfdqn_agent")
    sf = agent.sf
    assert sf._eng is not None, "the libsfx engine did not run"
    got = np.array([a for t in tasks for a in t.actions])
    assert np.array_equal(got, g["actions"]), f"training actions diverge at {np.argmax(got != g['actions'])}"
    assert np.array_equal(np.array(test_tasks[0].actions), g["test_actions"])
    assert np.array_equal(np.stack([np.asarray(c) for c in sf.gpi_counters]), g["gpi_counters"])
    assert list(sf.updates_since_target_updated) == list(g["since_target"])
    assert agent.total_training_steps == int(g["total_steps"])
    rel_close(torch.tensor([float(r) for r in returns]), g["returns"], rtol=1e-5, atol=1e-6)
    T = sf.n_tasks
    params_close(torch.stack([torch.cat([p.detach().reshape(-1).cpu() for p in sf.psi[t][0][0].parameters()])
                              for t in range(T)]), g["online"], 1e-3 * 60)
    params_close(torch.stack([torch.cat([p.detach().reshape(-1).cpu() for p in sf.psi[t][1][0].parameters()])
                              for t in range(T)]), g["target"], 1e-3 * 60)
    rel_close(torch.stack([sf.fit_w[t].reshape(-1).cpu() for t in range(T)]), g["w"], rtol=1e-4, atol=1e-6)
    rel_close(agent.test_tasks_weights[0].weight.detach().reshape(-1).cpu(), g["test_w"], rtol=1e-4, atol=1e-6)
