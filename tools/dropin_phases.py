"""Where the drop-in loop's step goes (tools/dropin_loop.py, `reference` buffer): host time per phase
of DropinLoop.step (no extra synchronisation -- the phase that contains `int(a)` also holds the wait
for the device), then a cProfile of the same loop.  A measurement harness, not part of the product."""
from __future__ import annotations

import cProfile
import io
import os
import pstats
import random
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "deep-successor-features-for-transfer_amd"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from dropin_loop import DropinLoop  # noqa: E402


def timed_step(loop, acc):
    t = [time.perf_counter()]

    def mark(k):
        now = time.perf_counter()
        acc[k] = acc.get(k, 0.0) + now - t[0]
        t[0] = now

    task = loop.tasks[loop.task]
    if loop.s_enc is None:
        loop.s_enc = task.initialize(True).reshape(1, -1)
    mark("top")
    q, c = loop.sf.GPI(loop.s_enc, loop.task, update_counters=True)
    mark("gpi_call")
    q = q[:, c, :].flatten()
    if random.random() <= loop.epsilon:
        a = torch.tensor(random.randrange(loop.A)).to(loop.device)
    else:
        a = torch.argmax(q)
    mark("select")
    ai = int(a)
    mark("int(a) wait")
    s1, phi, r, term = task.env.transition(ai)
    mark("env")
    s1 = torch.from_numpy(s1).to(loop.device)
    phi = torch.from_numpy(phi).to(loop.device)
    mark("to(device)")
    s1_enc = s1.reshape(1, -1)
    loop.sf.update_reward(phi, r, loop.task)
    mark("update_reward")
    g = 0.0 if term else loop.gamma
    loop.buffer.append(loop.s_enc, a, phi, s1_enc, g)
    mark("append")
    batch = loop.buffer.replay()
    mark("replay")
    for i in range(loop.T):
        loop.sf.update_successor(batch, i)
    mark("update_successor x T")
    loop.s_enc = None if term else s1_enc


def main():
    steps = int(os.environ.get("STEPS", "400"))
    buf = os.environ.get("BUFFER", "reference")
    loop = DropinLoop(buffer=buf)
    if buf != "reference":  # the loop's own step (its buffer's calls differ)
        loop.run(60)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        loop.run(steps)
        loop.sf._flush()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(f"{buf}: {1e6 * dt / steps:.1f} us/step; graph cache:", loop.sf._eng.graph_stats())
        pr = cProfile.Profile()
        pr.enable()
        loop.run(steps)
        loop.sf._flush()
        torch.cuda.synchronize()
        pr.disable()
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(25)
        print(s.getvalue())
        return
    loop.run(60)
    loop.sf._flush()
    torch.cuda.synchronize()
    acc = {}
    t0 = time.perf_counter()
    for _ in range(steps):
        timed_step(loop, acc)
    loop.sf._flush()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(f"{steps} steps, {1e6 * dt / steps:.1f} us/step ({steps / dt:.0f} env-steps/s)")
    for k, v in acc.items():
        print(f"  {k:24s} {1e6 * v / steps:8.1f} us")
    print("graph cache:", loop.sf._eng.graph_stats(), "speculation:", loop.sf._eng.step_stats())
    pr = cProfile.Profile()
    pr.enable()
    loop.run(steps)
    loop.sf._flush()
    torch.cuda.synchronize()
    pr.disable()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(35)
    print(s.getvalue())
    loop.close()


if __name__ == "__main__" and not os.environ.get("CALL_COSTS"):
    main()


def call_costs(steps=400):
    """Host time of each library call the loop makes (wrapped), per step."""
    from sfx import _lib
    from sfx.engine import SFEngine

    acc = {}

    def wrap(obj, name, label):
        real = getattr(obj, name)

        def f(*a, **k):
            t0 = time.perf_counter()
            r = real(*a, **k)
            acc[label] = acc.get(label, 0.0) + time.perf_counter() - t0
            return r
        setattr(obj, name, f)
        return real

    class L:  # ctypes entry points, timed
        pass
    names = ["sfx_update_all_select", "sfx_lms_value", "sfx_replay_put_gather", "sfx_replay_gather", "sfx_settle",
             "sfx_gpi", "sfx_replay_put"]
    saved = {n: getattr(_lib.lib, n) for n in names}
    for n in names:
        real = saved[n]

        def f(*a, _r=real, _n=n):
            t0 = time.perf_counter()
            r = _r(*a)
            acc["C " + _n] = acc.get("C " + _n, 0.0) + time.perf_counter() - t0
            return r
        setattr(_lib.lib, n, f)
    from sfx.dropin.agents.buffer import ReplayBuffer
    from sfx.dropin.features.deep import DeepSF

    wrap(SFEngine, "update_all_select", "py update_all_select")
    wrap(ReplayBuffer, "release", "py buffer.release")
    wrap(ReplayBuffer, "replay", "py buffer.replay")
    wrap(ReplayBuffer, "append", "py buffer.append")
    wrap(DeepSF, "_flush", "py DeepSF._flush")
    wrap(DeepSF, "GPI", "py DeepSF.GPI")
    wrap(DeepSF, "update_reward", "py DeepSF.update_reward")
    wrap(SFEngine, "settle_select", "py settle_select")
    loop = DropinLoop(buffer="reference")
    loop.run(60)
    loop.sf._flush()
    torch.cuda.synchronize()
    acc.clear()
    t0 = time.perf_counter()
    loop.run(steps)
    loop.sf._flush()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(f"call costs: {1e6 * dt / steps:.1f} us/step")
    for k, v in sorted(acc.items()):
        print(f"  {k:36s} {1e6 * v / steps:8.1f} us")
    loop.close()
    for n in names:
        setattr(_lib.lib, n, saved[n])


if __name__ == "__main__" and os.environ.get("CALL_COSTS"):
    call_costs()
