"""The drop-in's agents.buffer on the device (sfx_replay_put / sfx_replay_gather: one launch per
append and per replay): the reference's collation (agents/buffer.py:52-60) of the rows numpy's
randint draws, exactly -- device-tensor inputs as main_sfdqn_torch.py's agent passes them
(states [1, n_s], φ [d], the action a 0-d int64 tensor, γ a float), through ring wrap-around,
device-tensor γ and reset()."""
import numpy as np
import pytest
import torch

from tests.conftest import gpu_available

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _need_gpu():
    if not gpu_available():
        pytest.skip("no HIP device")


def test_device_ring_matches_the_reference_collation():
    from sfx.dropin.agents.buffer import ReplayBuffer

    dev = torch.device("cuda", 0)
    n_s, d, B, cap = 17, 8, 32, 50
    buf = ReplayBuffer({}, n_samples=cap, n_batch=B)
    buf.device = dev
    gen = torch.Generator().manual_seed(2)
    rows = []
    assert buf.replay() is None
    for k in range(130):  # wraps the 50-row ring twice
        s, s1 = torch.randn(1, n_s, generator=gen), torch.randn(1, n_s, generator=gen)
        phi = torch.rand(d, generator=gen)
        a = torch.tensor(int(torch.randint(7, (1,), generator=gen)))
        g = torch.tensor(0.5) if k == 90 else (0.0 if k % 5 == 4 else 0.9)  # one device γ from k = 90 on
        buf.append(s.to(dev), a.to(dev), phi.to(dev), s1.to(dev), g.to(dev) if torch.is_tensor(g) else g)
        rows.append((s, a, phi, s1, float(g)))
        rows = rows[-cap:]
        if len(rows) >= B and k % 3 == 0:
            state = np.random.get_state()
            got = buf.replay()
            np.random.set_state(state)
            idx = np.random.randint(low=0, high=len(rows), size=(B,))
            order = rows if len(rows) < cap else rows[cap - buf.index:] + rows[:cap - buf.index]
            slot = [order[i] for i in idx]
            want = (torch.vstack([r[0] for r in slot]), torch.tensor([int(r[1]) for r in slot]),
                    torch.vstack([r[2] for r in slot]), torch.vstack([r[3] for r in slot]),
                    torch.tensor([r[4] for r in slot], dtype=torch.float32))
            for x, y in zip(got, want):
                assert x.device == dev and x.dtype == y.dtype and x.shape == y.shape and x.is_contiguous()
                assert torch.equal(x.cpu(), y)
    buf.reset()
    assert buf.replay() is None
