"""Where one step of the drop-in loop (tools/dropin_loop.py, reference-buffer leg) spends its
wall time: host timestamps between the loop's calls, medians over a window.  The step's only
host/device synchronisation is ``int(a)`` inside the env transition (it waits for the previous
update and this step's GPI); everything after it runs on the host while the device is idle."""
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "deep-successor-features-for-transfer_amd"), os.path.join(ROOT, "tools")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from dropin_loop import DropinLoop  # noqa: E402

NAMES = ("GPI", "argmax", "env+sync", "update_reward", "append", "replay", "update_successor x T")


class Timed(DropinLoop):
    def step(self):
        c_ = time.perf_counter
        task = self.tasks[self.task]
        if self.s_enc is None:
            self.s_enc = task.initialize(True).reshape(1, -1)
        t0 = c_()
        q, c = self.sf.GPI(self.s_enc, self.task, update_counters=True)
        t1 = c_()
        q = q[:, c, :].flatten()
        if random.random() <= self.epsilon:
            a = torch.tensor(random.randrange(self.A)).to(self.device)
        else:
            a = torch.argmax(q)
        t2 = c_()
        s1, phi, r, term = task.transition(a, True)
        s1_enc = s1.reshape(1, -1)
        t3 = c_()
        self.sf.update_reward(phi, r, self.task)
        t4 = c_()
        g = 0.0 if term else self.gamma
        self.buffer.append(self.s_enc, a, phi, s1_enc, g)
        t5 = c_()
        batch = self.buffer.replay()
        t6 = c_()
        for i in range(self.T):
            self.sf.update_successor(batch, i)
        t7 = c_()
        self.s_enc = None if term else s1_enc
        self.rec.append((t0, t1, t2, t3, t4, t5, t6, t7))


def wrap(obj, name, acc):
    f = getattr(obj, name)

    def g(*a, **k):
        t0 = time.perf_counter()
        r = f(*a, **k)
        acc.setdefault(name, []).append(time.perf_counter() - t0)
        return r

    setattr(obj, name, g)


def main(steps=1500, warmup=200):
    loop = Timed(buffer="reference")
    loop.rec = []
    loop.run(warmup)
    acc = {}
    eng = loop.sf._eng
    for o, n in ((eng, "update_all"), (eng, "gpi"), (eng, "lms"), (loop.sf, "_flush"), (loop.buffer, "_replay_dev")):
        wrap(o, n, acc)
    loop.sf._flush()
    torch.cuda.synchronize()
    loop.rec = []
    t0 = time.perf_counter()
    loop.run(steps)
    loop.sf._flush()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    r = np.array(loop.rec)
    ph = np.diff(r, axis=1) * 1e6
    step = np.diff(r[:, 0]) * 1e6
    print(f"{steps} steps, {steps / dt:.1f} env-steps/s, step median {np.median(step):.1f} us")
    for i, n in enumerate(NAMES):
        print(f"  {n:24s} median {np.median(ph[:, i]):7.1f} us  p10 {np.percentile(ph[:, i], 10):7.1f}"
              f"  p90 {np.percentile(ph[:, i], 90):7.1f}")
    print(f"  {'after sync (host only)':24s} median {np.median((r[:, 7] - r[:, 3]) * 1e6):7.1f} us")
    for n, v in acc.items():
        v = np.array(v[-steps:]) * 1e6
        print(f"  inner {n:18s} median {np.median(v):7.1f} us  p10 {np.percentile(v, 10):7.1f}  (calls {len(v)})")
    loop.close()


if __name__ == "__main__":
    main()
