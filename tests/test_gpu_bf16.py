"""bf16 operand mode (sfx_set_precision, north_star "MFMA bf16 for the small dense MLP GEMMs").

Not a parity mode: the forward and dX GEMMs take bf16 operands, so ψ moves by ~2^-9 relative
per product.  Parity stays on fp32 (every other GPU test).  What is asserted here:
  * ψ within 3e-2 relative (max over entries, scaled by the row's largest |ψ|) of fp32 at the
    C2 shape, and the margin-aware GPI agreement: wherever the fp32 top-2 gap exceeds twice the
    largest |q_bf16 - q_fp32| seen, the bf16 argmax equals the fp32 one -- 100 %; the overall
    agreement rate (near-ties included) is reported;
  * training in bf16 stays finite and within Adam's 2·lr-per-step band of the fp32 run;
  * the bf16 copies the Adam epilogue writes are exactly bf16(master): a fresh bf16 engine
    loaded with the trained fp32 heads computes bit-identical ψ (online and target).
"""
import numpy as np
import pytest
import torch

from oracle import ref_cpu as R
from tests.conftest import gpu_available

pytestmark = pytest.mark.gpu

C2 = R.Spec(17, 256, 7, 8, ("relu", "relu"))


@pytest.fixture(autouse=True)
def _need_gpu():
    if not gpu_available():
        pytest.skip("no HIP device")


def engines(spec, T, seed=0, max_batch=32):
    from sfx.engine import SFEngine
    from sfx.init import reference_heads

    online, w = reference_heads(T, spec.n_s, spec.H, spec.A, spec.d, spec.acts, seed=seed)
    w = w * 50.0  # trained-scale reward weights: q spans several units, not 1e-2
    out = []
    for prec in ("fp32", "bf16"):
        eng = SFEngine(T, spec.n_s, spec.H, spec.A, spec.d, spec.acts, max_batch=max_batch)
        eng.set_adam(1e-3, 0.0, 1e-3, 0.0)
        for t in range(T):
            eng.load_head(t, online[t], 0)
            eng.load_head(t, online[t], 1)
            eng.load_w(t, w[t])
        eng.set_precision(prec)
        assert eng.precision == prec
        out.append(eng)
    return out


def top2_gap(x, dim):
    v = torch.topk(x, 2, dim=dim).values
    return (v.select(dim, 0) - v.select(dim, 1))


def test_bf16_gpi_margin_aware_agreement():
    T, n = 8, 1024
    f32, b16 = engines(C2, T)
    gen = torch.Generator().manual_seed(3)
    S = torch.randn(n, C2.n_s, generator=gen)
    agree_t = agree_a = 0
    worst_rel = 0.0
    margin_cases = margin_ok = 0
    for c in range(0, n, 32):
        s = S[c:c + 32]
        for wi in range(T):
            p0, q0, t0, n0 = f32.gpi(s, w_index=wi, want_psi=True)
            p1, q1, t1, n1 = b16.gpi(s, w_index=wi, want_psi=True)
            p0, p1, q0, q1 = p0.cpu(), p1.cpu(), q0.cpu(), q1.cpu()
            scale = p0.abs().amax(dim=(1, 2, 3), keepdim=True)
            worst_rel = max(worst_rel, float(((p1 - p0).abs() / scale).max()))
            dq = float((q1 - q0).abs().max())
            # task = argmax_t max_a q ; next action = argmax_a max_t q (torch.argmax first-index)
            m_t0, m_a0 = q0.amax(dim=2), q0.amax(dim=1)
            for got, ref, gap in ((t1.cpu(), t0.cpu(), top2_gap(m_t0, 1)), (n1.cpu(), n0.cpu(), top2_gap(m_a0, 1))):
                safe = gap > 2.0 * dq
                margin_cases += int(safe.sum())
                margin_ok += int((got[safe] == ref[safe]).sum())
            agree_t += int((t1.cpu() == t0.cpu()).sum())
            agree_a += int((n1.cpu() == n0.cpu()).sum())
    total = (n // 32) * 32 * T
    print(f"\nbf16 vs fp32 (C2, {total} GPI rows): max rel psi err {worst_rel:.2e}; task agreement "
          f"{agree_t / total:.4f}, next-action agreement {agree_a / total:.4f}; margin-aware "
          f"{margin_ok}/{margin_cases}")
    assert worst_rel < 3e-2
    assert margin_cases > total // 2  # the bound leaves most rows decidable
    assert margin_ok == margin_cases
    f32.close()
    b16.close()


def test_bf16_training_stays_in_band_and_copies_exact():
    from sfx.engine import SFEngine
    from sfx.runner import NativeEnvLoop

    T, ev, n = 8, 7, 40
    runs = {}
    for e in engines(C2, T):
        e.set_target_update_ev(ev)
        loop = NativeEnvLoop(e, batch=32, capacity=400, gamma=0.9, epsilon=0.2, alpha_w=0.05, episode_len=13, seed=4)
        loop.prefill(64)
        loop.set_task(3)
        loop.run(n)
        runs[e.precision] = e
        loop.close()
    f32, b16 = runs["fp32"], runs["bf16"]
    h0 = torch.stack([f32.get_head(t, 0) for t in range(T)])
    h1 = torch.stack([b16.get_head(t, 0) for t in range(T)])
    assert torch.isfinite(h1).all()
    lr_steps = 1e-3 * n
    assert float((h1 - h0).abs().max()) <= 2.0 * lr_steps
    # a fresh bf16 engine from b16's fp32 master weights: its copies are bf16(master) by
    # construction, so bit-equal ψ proves the epilogue's copies (and the target sync's) are too
    fresh = SFEngine(T, C2.n_s, C2.H, C2.A, C2.d, C2.acts, max_batch=32)
    for t in range(T):
        fresh.load_head(t, b16.get_head(t, 0), 0)
        fresh.load_head(t, b16.get_head(t, 1), 1)
    fresh.set_precision("bf16")
    S = torch.randn(32, C2.n_s, generator=torch.Generator().manual_seed(8))
    for which in (0, 1):
        assert torch.equal(fresh.successors(S, which).cpu(), b16.successors(S, which).cpu()), which
    fresh.close()
    f32.close()
    b16.close()


def test_bf16_switch_back_to_fp32_is_exact():
    """Switching a bf16 engine back to fp32 runs the fp32 kernels again: ψ equals an fp32 engine's
    bit for bit (the master weights were never touched by the mode)."""
    f32, b16 = engines(C2, 4)
    S = torch.randn(16, C2.n_s, generator=torch.Generator().manual_seed(2))
    b16.set_precision("fp32")
    assert torch.equal(f32.successors(S).cpu(), b16.successors(S).cpu())
    f32.close()
    b16.close()
