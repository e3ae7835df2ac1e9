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


def test_held_minibatches_survive_slot_reuse_and_ring_wrap():
    """replay() reuses a minibatch's memory only after its consumer handed it back; 300 replays queued without a synchronisation wrap the 256-slot
    index ring (its per-block events), and every held minibatch still holds its own rows."""
    from sfx.dropin.agents.buffer import ReplayBuffer

    dev = torch.device("cuda", 0)
    n_s, d, B, cap = 5, 3, 8, 40
    buf = ReplayBuffer({}, n_samples=cap, n_batch=B)
    buf.device = dev
    S = torch.arange(cap * n_s, dtype=torch.float32).reshape(cap, n_s)
    for k in range(cap):
        buf.append(S[k:k + 1].to(dev), torch.tensor(k % 7, device=dev), torch.full((d,), float(k), device=dev),
                   (S[k:k + 1] + 0.5).to(dev), 0.9)
    np.random.seed(5)
    held, want = [], []
    for _ in range(300):
        state = np.random.get_state()
        held.append(buf.replay())
        np.random.set_state(state)
        want.append(np.random.randint(low=0, high=cap, size=(B,)))
    for got, idx in zip(held, want):
        assert torch.equal(got[0].cpu(), S[idx]) and torch.equal(got[3].cpu(), S[idx] + 0.5)
        assert torch.equal(got[1].cpu(), torch.as_tensor(idx % 7)) and torch.equal(got[2][:, 0].cpu(), torch.as_tensor(idx, dtype=torch.float32))
    # reuse only after an explicit hand-back: dropping every Python reference is not enough (a fresh
    # buffer, so its first replays are its own slots, not torch allocations)
    del held
    buf = ReplayBuffer({}, n_samples=cap, n_batch=B)
    buf.device = dev
    for k in range(cap):
        buf.append(S[k:k + 1].to(dev), torch.tensor(k % 7, device=dev), torch.full((d,), float(k), device=dev),
                   (S[k:k + 1] + 0.5).to(dev), 0.9)
    a = buf.replay()
    pa = a[0].data_ptr()
    del a
    b = buf.replay()
    assert b[0].data_ptr() != pa  # the first slot was never handed back
    assert buf.release(b[0]) and not buf.release(b[0])  # a second release of one lending is a no-op
    pb = b[0].data_ptr()
    del b
    c = buf.replay()
    assert c[0].data_ptr() == pb


def test_minibatch_held_only_by_autograd_is_not_overwritten():
    """a minibatch whose only holder is C++ (autograd saved it for a backward that runs
    later) keeps its rows however many replays follow -- the buffer never infers ownership; only
    its consumer's release (sfx DeepSF, after the update that read it settled) frees a slot."""
    from sfx.dropin.agents.buffer import ReplayBuffer, release_minibatch

    dev = torch.device("cuda", 0)
    n_s, d, B, cap = 6, 4, 16, 64
    buf = ReplayBuffer({}, n_samples=cap, n_batch=B)
    buf.device = dev
    gen = torch.Generator().manual_seed(3)
    for k in range(cap):
        buf.append(torch.randn(1, n_s, generator=gen).to(dev), torch.tensor(k % 5, device=dev),
                   torch.rand(d, generator=gen).to(dev), torch.randn(1, n_s, generator=gen).to(dev), 0.9)
    lin = torch.nn.Linear(n_s, 3).to(dev)
    S = buf.replay()[0]
    ref = S.clone()
    out = (lin(S) ** 2).sum()  # autograd saves S for the weight gradient
    del S
    for _ in range(20):  # replays (some handed back) that would reuse an inferred-free slot
        t = buf.replay()
        release_minibatch(t[0])
        del t
    out.backward()
    want = torch.autograd.grad((lin(ref) ** 2).sum(), lin.weight)[0]
    torch.cuda.synchronize()
    assert torch.allclose(lin.weight.grad, want, rtol=1e-6, atol=1e-6)
