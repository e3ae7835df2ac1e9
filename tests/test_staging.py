"""Host logic of SFEngine's input staging (sfx/engine.py _h2d_many / _batch_in), on the CPU: the
host arguments of one call are packed 16-byte aligned into one staging slot and leave it in one
copy; each comes back with its shape, dtype and values (float64 / Python scalars converted as
torch's .to(float32) does), and a tensor already on the device is converted in place of staging.
The pinned slot and the device copy are replaced by plain CPU memory here (no HIP device)."""
import numpy as np
import torch

from sfx.engine import SFEngine


class _CpuStaging(SFEngine):
    def __init__(self, d=3):
        self.device = torch.device("cpu")
        self.d = d
        self.copies = []

    def _pin_slot(self):
        if not hasattr(self, "_pin"):
            self._pin = torch.zeros(self._PIN_SLOTS, self._PIN_BYTES, dtype=torch.uint8)
            self._pin_np = self._pin.numpy()
            self._pin_i = 0
        i = self._pin_i
        self._pin_i = (i + 1) % self._PIN_SLOTS
        return i

    def _pin_copy(self, i, nbytes, site=None):
        self.copies.append(nbytes)
        return self._pin[i, :nbytes].clone()

    def _settle_pending(self):
        self.settled = getattr(self, "settled", 0) + 1

    def __del__(self):
        pass


def test_batch_in_packs_one_copy_and_round_trips():
    st = _CpuStaging(d=3)
    g = np.random.default_rng(0)
    B = 5
    s = g.standard_normal((B, 7))  # float64: converted to float32
    s1 = torch.from_numpy(g.standard_normal((B, 7)).astype(np.float32))
    a = torch.tensor([0, 3, 1, 2, 6])
    phi = g.random((B, 3)).astype(np.float32)
    gamma = [0.9, 0.0, 0.9, 0.9, 0.9]
    r = torch.rand(B, 1)
    out = st._batch_in(s, s1, a, phi, gamma, r)
    assert st.copies == [sum((n + 15) & ~15 for n in (B * 7 * 4, B * 7 * 4, B * 8, B * 3 * 4, B * 4, B * 4))]
    want = [torch.as_tensor(s).float(), s1, a, torch.from_numpy(phi), torch.tensor(gamma).float(), r.reshape(B)]
    for got, ref, dt in zip(out, want, (torch.float32, torch.float32, torch.long, torch.float32, torch.float32,
                                        torch.float32)):
        assert got.dtype == dt and got.is_contiguous()
        assert torch.equal(got, ref.to(dt))
    assert out[3].shape == (B, 3) and out[2].shape == (B,) and out[4].shape == (B,)
    assert st.settled == 1  # a minibatch goes to the batch site only after a pending step is collected


def test_staging_slots_rotate_and_offsets_are_aligned():
    st = _CpuStaging()
    for k in range(SFEngine._PIN_SLOTS + 3):
        x, y = st._h2d_many([(np.arange(3, dtype=np.float32) + k, torch.float32), (7, torch.long)])
        assert torch.equal(x, torch.arange(3, dtype=torch.float32) + k)
        assert x.storage_offset() == 0 and y.storage_offset() * y.element_size() == 16  # packed, aligned
        assert y.dtype == torch.long and int(y) == 7
    assert st._pin_i == 3
    assert st.copies == [32] * (SFEngine._PIN_SLOTS + 3)


def test_device_and_oversized_inputs_bypass_the_slot():
    st = _CpuStaging()
    big = np.zeros(SFEngine._PIN_BYTES // 4 + 1, np.float32)
    (b,) = st._h2d_many([(big, torch.float32)])
    assert b.shape == big.shape and st.copies == []
    (e,) = st._h2d_many([(np.zeros(0, np.float32), torch.float32)])
    assert e.numel() == 0 and st.copies == []
