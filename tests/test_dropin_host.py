"""CPU checks of the drop-in module tree (no GPU compute): the reference's import names
resolve to sfx's modules, the ψ architecture is recognised or rejected, the library keeps
the reference's bookkeeping, and compute fails loudly without a HIP device."""
import pytest
import torch

from tests.golden.recipe import AgentTask, agent_psi_lambda


@pytest.fixture(scope="module")
def mods():
    from sfx import dropin

    root = dropin.install()
    import agents.buffer
    import agents.sfdqn
    import features.deep
    import utils.torch as ut

    ut.set_torch_device(False)
    for m in (features.deep, agents.sfdqn, agents.buffer):
        assert m.__file__.startswith(root)
    return features.deep, agents.sfdqn, agents.buffer


def test_geometry_recognised_and_rejected(mods):
    deep, _, _ = mods
    model, _, _ = agent_psi_lambda(32, ("relu", "tanh"), 1e-3, "cpu")(17, 56, (7, 8))
    assert deep._geometry(model) == (17, 32, ("relu", "tanh"), 56)
    bad = torch.nn.Sequential(torch.nn.Linear(4, 8), torch.nn.ReLU(), torch.nn.Linear(8, 6))
    with pytest.raises(NotImplementedError):
        deep._geometry(bad)


def test_library_bookkeeping_and_loud_failure(mods):
    deep, _, _ = mods
    sf = deep.DeepSF(pytorch_model_handle=agent_psi_lambda(16, ("relu",), 1e-3, "cpu"), target_update_ev=5,
                     hyperparameters={"learning_rate_w": 0.1})
    sf.reset()
    for i in range(3):
        sf.add_training_task(AgentTask(6, 3, 4, i, i, "cpu"))
    assert sf.n_tasks == 3 and len(sf.psi) == 3 and len(sf.fit_w) == 3
    assert [c.shape for c in sf.gpi_counters] == [(3,)] * 3
    assert sf.updates_since_target_updated == [0, 0, 0]
    # target nets start as copies of the online nets (features/deep.py:69-71)
    for (m, _, _), (tm, _, _) in sf.psi:
        for a, b in zip(m.parameters(), tm.parameters()):
            assert torch.equal(a, b)
    if not torch.cuda.is_available():
        with pytest.raises(RuntimeError, match="HIP device"):
            sf.get_successors(torch.zeros(2, 6))


def test_replay_buffer_semantics(mods):
    _, _, buf = mods
    b = buf.ReplayBuffer(n_samples=4, n_batch=2)
    b.reset()
    assert b.replay() is None
    for i in range(6):
        b.append(torch.full((1, 3), float(i)), torch.tensor(i % 2), torch.ones(1, 2), torch.zeros(1, 3), 0.9)
    assert b.size == 4 and b.index == 2
    s, a, phi, s1, g = b.replay()
    assert s.shape == (2, 3) and a.shape == (2,) and phi.shape == (2, 2) and g.dtype == torch.float32


def test_sequential_modules_and_buffer(mods):
    """main_sfdqn_sequential_torch.py's imports resolve to the drop-in tree; the per-task buffer
    keeps agents/buffer_sequential.py's 6-tuples, ring order and np.random sampling."""
    import numpy as np

    from sfx import dropin

    root = dropin.install()
    import agents.buffer_sequential as bs
    import agents.buffer_tsf_sequential as bts
    import agents.sfdqn_sequential as ss
    import agents.tsfdqn_sequential as ts
    import features.deep_sequential as ds
    import features.deep_sequential_tsf as dts

    import sfdqn
    import tsfdqn
    import tsfdqn_nf

    for m in (bs, ss, ds, bts, ts, dts, sfdqn, tsfdqn, tsfdqn_nf):
        assert m.__file__.startswith(root)
    b = bs.ReplayBuffer(n_samples=4, n_batch=3)
    assert b.replay() is None
    for i in range(6):
        b.append(torch.full((1, 3), float(i)), i % 2, torch.tensor(0.5 * i), torch.ones(1, 2) * i,
                 torch.zeros(1, 3), 0.9)
    assert b.size == 4 and b.index == 2
    np.random.seed(3)
    idx = np.random.randint(low=0, high=4, size=(3,))
    np.random.seed(3)
    s, a, r, phi, s1, g = b.replay()
    # ring slots: 0 <- sample 4, 1 <- sample 5, 2 <- sample 2, 3 <- sample 3
    src = np.array([4, 5, 2, 3])[idx]
    assert torch.equal(s[:, 0], torch.tensor(src, dtype=torch.float32))
    assert torch.equal(r[:, 0], torch.tensor(0.5 * src, dtype=torch.float32))
    assert r.shape == (3, 1) and phi.shape == (3, 2) and a.tolist() == [int(x) % 2 for x in src]
    assert g.dtype == torch.float32
