"""Host cost of the pieces inside the drop-in's per-step library calls (C2 shape), each timed
alone with the device idle: what the replay, the deferred update_successor calls and the GPI
wrapper spend in Python / ctypes / torch before their launches."""
import ctypes as C
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "deep-successor-features-for-transfer_amd"), os.path.join(ROOT, "tools")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from dropin_loop import DropinLoop  # noqa: E402
from sfx import _lib  # noqa: E402

loop = DropinLoop(buffer="reference")
loop.run(100)
loop.sf._flush()
torch.cuda.synchronize()
sf, buf, eng = loop.sf, loop.buffer, loop.sf._eng
dev = torch.device("cuda", 0)


def host(name, fn, n=400):
    ts = []
    for i in range(n + 20):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        t1 = time.perf_counter()
        if i >= 20:
            ts.append(t1 - t0)
    eng.step_stats()
    ts = np.array(ts) * 1e6
    print(f"{name:44s} median {np.median(ts):7.2f} us   p10 {np.percentile(ts, 10):7.2f}", flush=True)


B, n_s, d = 32, 17, 8
batch = buf.replay()
S, A, PHI, S1, G = batch
host("np.random.randint(0, size, 32)", lambda: np.random.randint(low=0, high=buf.size, size=(32,)))
idx = np.random.randint(low=0, high=buf.size, size=(32,))
hb = _lib.HostBuffer(64)
hnp = hb.np


def hw():
    hnp[:B] = idx
    hnp[B:].view(np.float32)[:B] = buf._gam[idx]


host("pinned slot writes (indices, gammas)", hw)


def alloc():
    a2, S_, PHI_, S1_, G_ = torch.empty(B * (2 * n_s + d + 3), device=dev).split((2 * B, B * n_s, B * d, B * n_s, B))
    a2.view(torch.int64), S_.view(B, n_s), PHI_.view(B, d), S1_.view(B, n_s)


host("torch.empty + split + 4 views", alloc)
host("torch.empty x1", lambda: torch.empty(4, device=dev))
ev = torch.cuda.Event()
host("Event.record (reused event)", lambda: ev.record())
host("Event.synchronize (completed)", lambda: ev.synchronize())
host("torch.cuda.Event()", lambda: torch.cuda.Event())
host("_lib.stream_ptr(0)", lambda: _lib.stream_ptr(0))
host("replay (whole)", lambda: buf.replay())
host("engine._on_dev x1", lambda: eng._on_dev(S, torch.float32))
host("engine._batch_in", lambda: eng._batch_in(S, S1, A, PHI, G))
host("5 x data_ptr()", lambda: (S.data_ptr(), A.data_ptr(), PHI.data_ptr(), S1.data_ptr(), G.data_ptr()))
lb = eng._dropin_losses
args = (eng._h, S.data_ptr(), A.data_ptr(), PHI.data_ptr(), S1.data_ptr(), G.data_ptr(), B, lb.data_ptr())
host("lib.sfx_update_all (raw ctypes)", lambda: _lib.lib.sfx_update_all(*args))
host("engine.update_all", lambda: eng.update_all(S, A, PHI, S1, G, losses=lb))


def us8():
    for i in range(8):
        sf.update_successor(batch, i)


host("DeepSF.update_successor x 8", us8)


def us7():
    for i in range(7):
        sf.update_successor(batch, i)
    sf._pending = []


host("DeepSF.update_successor x 7 (no flush)", us7)
host("lib.sfx_step_stats (ctypes, settle)", lambda: eng.step_stats())
cn = C.c_int()
host("lib.sfx_comm_state (trivial ctypes)", lambda: _lib.lib.sfx_comm_state(eng._h, C.byref(cn)))
s1 = S[:1].clone()
host("DeepSF.GPI", lambda: sf.GPI(s1, 0, update_counters=True))
host("engine.gpi", lambda: eng.gpi(s1, w_index=0))
q, c = sf.GPI(s1, 0, update_counters=True)
host("q[:, c, :].flatten() + argmax", lambda: torch.argmax(q[:, c, :].flatten()))
phi1 = PHI[0].clone()
host("DeepSF.update_reward", lambda: sf.update_reward(phi1, 0.3, 0))
host("engine.lms", lambda: eng.lms(0, phi1, 0.3, 0.05))
a1 = A[0].clone()
host("buffer.append", lambda: buf.append(s1, a1, phi1, s1, 0.9))
st = torch.from_numpy(np.zeros(17, np.float32))
host("torch.from_numpy(17).to(dev) (user env)", lambda: st.to(dev))
loop.close()
