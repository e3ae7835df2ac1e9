"""The drop-in under the reference user's agent loop (tools/dropin_loop.py, the harness bench.py
times as `reacher17-all-T8-B32-dropin-*-buffer`): every env step's T update_successor calls
reach the device as ONE fused all-task step (sfx_update_all), with either replay buffer, and the
heads move.  Parity of the fused step itself: tests/test_gpu_dropin.py, test_gpu_engine.py."""
import pytest
import torch

from tests.conftest import gpu_available

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("buffer", ["reference", "objring", "host"])
def test_dropin_loop_fuses_every_env_step(buffer, monkeypatch):
    if not gpu_available():
        pytest.skip("no HIP device")
    from sfx.engine import SFEngine
    from tools import dropin_loop

    calls = {"all": 0, "one": 0}
    real_all, real_one, real_sel = SFEngine.update_all, SFEngine.update, SFEngine.update_all_select

    def count_all(self, *a, **k):
        calls["all"] += 1
        return real_all(self, *a, **k)

    def count_one(self, *a, **k):
        calls["one"] += 1
        return real_one(self, *a, **k)

    def count_sel(self, *a, **k):  # update_all with the next GPI fused in (agents.buffer alias)
        calls["all"] += 1
        return real_sel(self, *a, **k)

    monkeypatch.setattr(SFEngine, "update_all", count_all)
    monkeypatch.setattr(SFEngine, "update_all_select", count_sel)
    monkeypatch.setattr(SFEngine, "update", count_one)
    loop = dropin_loop.DropinLoop(buffer=buffer, T=4, batch=8)
    loop.run(2)
    before = torch.stack([loop.sf._eng.get_head(t, 0) for t in range(4)])
    loop.run(20)
    loop.sf._flush()
    after = torch.stack([loop.sf._eng.get_head(t, 0) for t in range(4)])
    # replay() returns None until the buffer holds a batch (8 transitions): 22 - 7 fused steps
    assert calls == {"all": 15, "one": 0}
    assert bool(torch.all((after - before).abs().amax(dim=1) > 0))
    loop.close()
