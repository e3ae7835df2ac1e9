"""GPU parity of the TSF-DQN update (sfx_tsf_*: planar-flow g_i, shared h, φ̃ in the TD target
and l2) against golden vectors from the real reference's TSFDQN.update_successor
(tsfdqn.py:588-709 and tsfdqn_nf.py with K = 3 planar layers; tests/golden/upd_tsf*.npz).
Tolerances as test_gpu_engine.py (fp32 reduction order differs from ATen's)."""
import numpy as np
import pytest
import torch

from tests.conftest import gpu_available
from tests.test_gpu_engine import batches_of, params_close, rel_close, spec_of

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _need_gpu():
    if not gpu_available():
        pytest.skip("no HIP device")


@pytest.mark.parametrize("case", ["tsf", "tsf_nf"])
def test_tsf_update_vs_golden(golden, case):
    from sfx.engine import SFEngine

    g = golden("upd_" + case)
    spec, T = spec_of(g), int(g["T"])
    eng = SFEngine(T, spec.n_s, spec.H, spec.A, spec.d, spec.acts, max_batch=32)
    eng.set_adam(1e-3, 0.0, 1e-3, 0.0)
    eng.set_target_update_ev(int(g["target_update_ev"]))
    eng.tsf_setup(int(g["G"]), int(g["K"]), float(g["beta"]), 1e-3, 0.0, 1e-3, 0.0)
    for t in range(T):
        eng.load_head(t, g["online0"][t], 0)
        eng.load_head(t, g["online0"][t], 1)
        eng.load_w(t, g["w0"][t])
        eng.tsf_load_g(t, g["g0"][t])
    eng.tsf_load_h(g["h0"])
    k = int(g["k"])
    for j, (s, a, r, phi, s1, gamma) in enumerate(batches_of(g)):
        i = int(g["policies"][j])
        losses = eng.tsf_update(i, s, a, r, phi, s1, gamma, use_gpi=True)
        rel_close(losses, g["losses"][j], rtol=2e-4, atol=1e-7)
    params_close(torch.stack([eng.get_head(t, 0) for t in range(T)]), g["online"], 1e-3 * k)
    params_close(torch.stack([eng.get_head(t, 1) for t in range(T)]), g["target"], 1e-3 * k)
    rel_close(torch.stack([eng.get_w(t)[0] for t in range(T)]), g["w"], rtol=1e-3, atol=1e-6)
    params_close(torch.stack([eng.tsf_get_g(t)[0] for t in range(T)]), g["g"], 1e-3 * k)
    params_close(eng.tsf_get_h(), g["h"], 1e-3 * k)
    eng.close()
