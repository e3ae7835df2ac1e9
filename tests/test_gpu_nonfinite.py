"""SURVEY §5 failure detection on the GPU: a NaN in φ makes the TD error non-finite; every TD-target
kernel (k_tdg, the fused TD of k_bwd_tdg) sets the handle's sticky flag, sfx_nonfinite
reads it, and the native runner fails the run at that step with an error instead of training on."""
import numpy as np
import pytest
import torch

from oracle import ref_cpu as R
from tests.conftest import gpu_available
from tests.test_gpu_step import dev, setup

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _need_gpu():
    if not gpu_available():
        pytest.skip("no HIP device")


@pytest.mark.parametrize("H", [32, 256])
def test_nan_phi_sets_the_flag(H):
    spec = R.Spec(17, H, 7, 8, ("relu", "relu"))
    T = 4
    eng, _ = setup(spec, T)
    gen = torch.Generator().manual_seed(3)
    B = 32
    s, s1 = torch.randn(B, spec.n_s, generator=gen), torch.randn(B, spec.n_s, generator=gen)
    a = torch.randint(0, spec.A, (B,), generator=gen)
    phi = torch.rand(B, spec.d, generator=gen)
    gamma = torch.full((B,), 0.9)
    sn = torch.randn(1, spec.n_s, generator=gen)
    eng.step_all(dev(s), dev(a, torch.long), dev(phi), dev(s1), dev(gamma), s_next=dev(sn), task_index=0)
    eng.step_finish()
    assert not eng.nonfinite()
    phi[5, 3] = float("nan")
    eng.step_all(dev(s), dev(a, torch.long), dev(phi), dev(s1), dev(gamma), s_next=dev(sn), task_index=0)
    eng.step_finish()
    assert eng.nonfinite(reset=True)
    assert not eng.nonfinite()
    # the single-head update path (k_tdg / fused TD of sfx_update) too
    r = torch.rand(B, 1, generator=gen)
    eng.update(1, s, a, r, phi, s1, gamma, use_gpi=True)
    assert eng.nonfinite(reset=True)
    eng.close()


class _NaNEnv:
    """A Reacher-shaped env whose φ turns NaN at env step `at` (the runner's env callbacks)."""

    def __init__(self, n_s, d, at):
        self.rng = np.random.default_rng(0)
        self.n_s, self.d, self.at, self.n = n_s, d, at, 0

    def reset(self, task):
        return self.rng.standard_normal(self.n_s)

    def step(self, task, a):
        self.n += 1
        phi = self.rng.random(self.d)
        if self.n >= self.at:
            phi[0] = np.nan
        return self.rng.standard_normal(self.n_s), phi, float(self.rng.random()), False


def test_runner_fails_loudly_on_a_non_finite_td_error():
    from sfx.runner import NativeEnvLoop

    spec = R.Spec(17, 256, 7, 8, ("relu", "relu"))
    eng, _ = setup(spec, 8, ev=1000)
    loop = NativeEnvLoop(eng, batch=32, seed=1, env=_NaNEnv(spec.n_s, spec.d, at=245))
    loop.prefill(200)  # the prefill steps the env too: its φ stay finite (n < 245)
    loop.set_task(0)
    loop.run(5)
    assert not eng.nonfinite()
    with pytest.raises(RuntimeError, match="non-finite"):
        loop.run(200)
    assert loop.stats()["nonfinite_steps"] == 1
    assert eng.nonfinite(reset=True)
    loop.close()
    eng.close()
