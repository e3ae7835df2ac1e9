"""The main_sfdqn_torch.py (and main_sfdqn_sequential_torch.py) stacks on sfx's drop-in modules
reproduce the REAL reference runs.

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


@pytest.mark.parametrize("single_file", [False, True])
def test_dropin_reproduces_reference_sequential_run(golden, single_file):
    """main_sfdqn_sequential_torch.py's stack (agents.sfdqn_sequential + agents.buffer_sequential +
    features.deep_sequential) on the drop-in reproduces the real reference's seeded run
    (tests/golden/run_sfdqn_sequential_agent.npz): training actions (active-task l1 + l2 updates),
    test-task actions (GPI with the test task's Adam-trained reward model), GPI counters."""
    from sfx import dropin

    dropin.install()
    import utils.torch as ut
    from utils.logger import set_logger_level

    ut.set_torch_device(True)
    set_logger_level(False, quiet=True)
    if single_file:  # sfdqn.py: the same stack in one module, ε drawn before GPI
        from sfdqn import DeepSF, ReplayBuffer, SFDQN

        assert "dropin" in __import__("sfdqn").__file__
    else:
        from agents.buffer_sequential import ReplayBuffer
        from agents.sfdqn_sequential import SFDQN
        from features.deep_sequential import DeepSF

        assert "dropin" in __import__("agents.sfdqn_sequential").sfdqn_sequential.__file__

    from tests.golden.recipe import agent_run_sequential

    with contextlib.redirect_stdout(io.StringIO()):
        agent, tasks, test_tasks, returns = agent_run_sequential(DeepSF, SFDQN, ReplayBuffer, ut.device)
    g = golden("run_sfdqn_singlefile_agent" if single_file else "run_sfdqn_sequential_agent")
    sf = agent.sf
    assert sf._eng is not None, "the libsfx engine did not run"
    got = np.array([a for t in tasks for a in t.actions])
    assert np.array_equal(got, g["actions"]), f"training actions diverge at {np.argmax(got != g['actions'])}"
    tg = np.array(test_tasks[0].actions)
    assert np.array_equal(tg, g["test_actions"]), f"test actions diverge at {np.argmax(tg != g['test_actions'])}"
    assert np.array_equal(np.stack([np.asarray(c) for c in sf.gpi_counters]), g["gpi_counters"])
    assert list(sf.updates_since_target_updated) == list(g["since_target"])
    assert agent.total_training_steps == int(g["total_steps"])
    rel_close(torch.tensor([float(r) for r in returns]), g["returns"], rtol=1e-5, atol=1e-6)
    T = sf.n_tasks
    k = int(g["total_steps"])
    params_close(torch.stack([torch.cat([p.detach().reshape(-1).cpu() for p in sf.psi[t][0][0].parameters()])
                              for t in range(T)]), g["online"], 1e-3 * k)
    rel_close(torch.stack([sf.fit_w[t].weight.detach().reshape(-1).cpu() for t in range(T)]), g["w"], rtol=1e-4,
              atol=1e-5)
    rel_close(agent.test_tasks_weights[0][0].weight.detach().reshape(-1).cpu(), g["test_w"], rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("variant", ["sequential", "nf", "singlefile"])
def test_dropin_reproduces_reference_tsf_run(golden, variant):
    """main_tsfdqn_sequential_torch.py's stack (agents.tsfdqn_sequential + agents.buffer_tsf_sequential
    + features.deep_sequential_tsf) -- nf: main_tsfdqn_sequential_torch_nf.py's single-file
    tsfdqn_nf (planar-flow g_i, 3 flows) -- on the drop-in reproduces the real reference's seeded
    run (tests/golden/run_tsfdqn_sequential_agent.npz / run_tsfdqn_nf_agent.npz): training
    actions (TSF updates of ψ_i, w_i, g_i and the shared h on the device), ω-weighted test-task
    actions, GPI counters; ψ / w / g / h within the Adam tolerance."""
    from sfx import dropin

    dropin.install()
    import utils.torch as ut
    from utils.logger import set_logger_level

    ut.set_torch_device(True)
    set_logger_level(False, quiet=True)
    nf = variant == "nf"
    if nf:
        from tsfdqn_nf import DeepTSF, ReplayBuffer, TSFDQN

        assert "dropin" in __import__("tsfdqn_nf").__file__
    elif variant == "singlefile":
        from tsfdqn import DeepTSF, ReplayBuffer, TSFDQN

        assert "dropin" in __import__("tsfdqn").__file__
    else:
        from agents.buffer_tsf_sequential import ReplayBuffer
        from agents.tsfdqn_sequential import TSFDQN
        from features.deep_sequential_tsf import DeepTSF

    from tests.golden.recipe import agent_run_tsf

    with contextlib.redirect_stdout(io.StringIO()):
        agent, tasks, test_tasks, returns = agent_run_tsf(DeepTSF, TSFDQN, ReplayBuffer, ut.device, nf=nf)
    g = golden(f"run_tsfdqn_{variant}_agent")
    sf = agent.sf
    assert sf._eng is not None, "the libsfx engine did not run"
    got = np.array([a for t in tasks for a in t.actions])
    assert np.array_equal(got, g["actions"]), f"training actions diverge at {np.argmax(got != g['actions'])}"
    tg = np.array(test_tasks[0].actions)
    assert np.array_equal(tg, g["test_actions"]), f"test actions diverge at {np.argmax(tg != g['test_actions'])}"
    assert np.array_equal(np.stack([np.asarray(c) for c in sf.gpi_counters]), g["gpi_counters"])
    assert list(sf.updates_since_target_updated) == list(g["since_target"])
    rel_close(torch.tensor([float(r) for r in returns]), g["returns"], rtol=1e-5, atol=1e-6)
    T = sf.n_tasks
    k = int(g["total_steps"])
    params_close(torch.stack([torch.cat([p.detach().reshape(-1).cpu() for p in sf.psi[t][0][0].parameters()])
                              for t in range(T)]), g["online"], 1e-3 * k)
    rel_close(torch.stack([sf.fit_w[t].weight.detach().reshape(-1).cpu() for t in range(T)]), g["w"], rtol=1e-3,
              atol=1e-5)
    sf.sync_tsf_modules()
    params_close(torch.stack([torch.cat([p.detach().reshape(-1).cpu() for p in agent.g_functions[t].parameters()])
                              for t in range(T)]), g["g"], 1e-3 * k)
    params_close(torch.cat([p.detach().reshape(-1).cpu() for p in agent.h_function.parameters()]), g["h"], 1e-3 * k)
    rel_close(agent.omegas[0].detach().reshape(-1).cpu(), g["omegas"], rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("case", ["sfdqn_gpi", "sfdqn_nogpi", "sfdqn_tanh"])
def test_dropin_sequential_deepsf_vs_reference_updates(golden, case):
    """features.deep_sequential.DeepSF (main_sfdqn_sequential_torch.py's library) driven through its
    public API reproduces the reference's update_successor sequence (tests/golden/upd_sfdqn_*)."""
    from sfx import dropin

    dropin.install()
    import utils.torch as ut

    ut.set_torch_device(True)
    from features.deep_sequential import DeepSF

    from tests.golden.recipe import AgentTask, agent_psi_lambda
    from tests.test_gpu_engine import batches_of, spec_of

    g = golden("upd_" + case)
    spec, T = spec_of(g), int(g["T"])
    hp = {"learning_rate_sf": 1e-3, "learning_rate_w": 1e-3, "weight_decay_sf": 0.0, "weight_decay_w": 0.0}
    sf = DeepSF(pytorch_model_handle=agent_psi_lambda(spec.H, spec.acts, 1e-3, ut.device),
                target_update_ev=int(g["target_update_ev"]), hyperparameters=hp)
    sf.reset()
    for t in range(T):
        sf.add_training_task(AgentTask(spec.n_s, spec.A, spec.d, t, t, ut.device))
    # the fixture's initial weights into the library's modules (before the engine exists)
    for t in range(T):
        (m, _, _), (tm, _, _) = sf.psi[t]
        for mod in (m, tm):
            off = 0
            with torch.no_grad():
                for p in mod.parameters():
                    p.copy_(torch.from_numpy(g["online0"][t][off:off + p.numel()]).view_as(p))
                    off += p.numel()
        with torch.no_grad():
            list.__getitem__(sf.fit_w, t).weight.copy_(torch.from_numpy(g["w0"][t]).view(1, -1))
    for j, (s, a, r, phi, s1, gamma) in enumerate(batches_of(g)):
        i = int(g["policies"][j])
        dev = ut.device
        loss, l1, l2 = sf.update_successor((s.to(dev), a.to(dev), r.to(dev), phi.to(dev), s1.to(dev), gamma.to(dev)),
                                           i, use_gpi=bool(g["use_gpi"]))
        rel_close(torch.stack([loss, l1, l2]).cpu(), g["losses"][j], rtol=2e-4, atol=1e-7)
    k = int(g["k"])
    online = torch.stack([torch.cat([p.detach().reshape(-1).cpu() for p in sf.psi[t][0][0].parameters()])
                          for t in range(T)])
    params_close(online, g["online"], 1e-3 * k)
    rel_close(torch.stack([sf.fit_w[t].weight.detach().reshape(-1).cpu() for t in range(T)]), g["w"], rtol=1e-4,
              atol=1e-5)
    assert list(sf.updates_since_target_updated) == [int(x) for x in g["since_target"]]
