"""The training program a reference user runs, over the drop-in library -- for measuring the
drop-in's own env-steps/s beside the native runner's headline.

The loop is the call pattern of main_sfdqn_torch.py's agent (agents/agent.py:195-261
next_sample + agents/sfdqn.py:39-60 get_Q_values / train_agent), restated as a bench harness:

  q, c = sf.GPI(s_enc, task, update_counters=True)      # B = 1 ψ of every head, GPI
  a    = ε-greedy over q[:, c, :]                        # torch.argmax on the device
  s1, φ, r = env.transition(int(a))                     # host env (synthetic Reacher shape)
  sf.update_reward(φ, r, task)                           # LMS on fit_w[task]
  buffer.append(s_enc, a, φ, s1_enc, γ); batch = buffer.replay()
  for i in range(T): sf.update_successor(batch, i)       # fused by the drop-in into one step

over ``sfx.dropin.features.deep.DeepSF`` (the ψ library every call above lands in).  Replay
buffers:
  * ``reference``: what main_sfdqn_torch.py's ``ReplayBuffer`` is under the drop-in --
    ``agents.buffer`` resolves to ``sfx.dropin.agents.buffer`` (the reference's API and index
    draws over a device-resident ring; the agent's calls unchanged);
  * ``objring``: agents/buffer.py's own layout (without the alias) -- an object ring of
    per-transition device tensors, ``torch.vstack`` on the device and ``torch.tensor`` of the
    per-transition action tensors (one device read each) per replay;
  * ``host``: states and φ kept as numpy arrays, a numpy ring sampled on the host, one
    host->device copy per field per replay.
The env, the buffer and the agent logic are the user's program, not the library; the numbers say
what a user switching libraries gets with each.
"""
from __future__ import annotations

import random
import time

import numpy as np
import torch


def psi_model_lambda(H, acts, lr, device):
    """ψ factory shaped like main_sfdqn_torch.py's (Linear(n_s, H), [Linear(H, H) + act]*, Linear(H, A d))."""
    act_cls = {"relu": torch.nn.ReLU, "tanh": torch.nn.Tanh}

    def build(n_in, n_out, shape, axis=1):
        layers = [torch.nn.Linear(n_in, H)]
        for a in acts:
            layers += [torch.nn.Linear(H, H), act_cls[a]()]
        layers += [torch.nn.Linear(H, n_out), torch.nn.Unflatten(axis, shape)]
        model = torch.nn.Sequential(*layers).to(device)
        return model, torch.nn.MSELoss(), torch.optim.Adam(model.parameters(), lr=lr)

    return build


class _Task:
    """tasks/task.py interface over sfx.runner.SynthReacher (states as device tensors, as
    tasks/reacher.py returns them)."""

    def __init__(self, env, device):
        self.env, self.device = env, device

    def action_count(self):
        return self.env.A

    def feature_dim(self):
        return self.env.d

    def encode_dim(self):
        return self.env.n_s

    def get_w(self):
        return torch.from_numpy(self.env.w_true).reshape(-1, 1)

    def initialize(self, on_device=True):
        s = self.env.initialize()
        return torch.from_numpy(s).to(self.device) if on_device else s

    def transition(self, a, on_device=True):
        s1, phi, r, term = self.env.transition(int(a))
        if not on_device:
            return s1, phi, r, term
        return torch.from_numpy(s1).to(self.device), torch.from_numpy(phi).to(self.device), r, term


class RefReplay:
    """agents/buffer.py's layout: per-transition device tensors in an object ring."""

    def __init__(self, capacity, batch, device):
        self.buf = np.empty(capacity, dtype=object)
        self.cap, self.batch, self.device = capacity, batch, device
        self.index = self.size = 0

    def append(self, s, a, phi, s1, gamma):
        self.buf[self.index] = (s, a, phi, s1, gamma)
        self.index = (self.index + 1) % self.cap
        self.size = min(self.size + 1, self.cap)

    def replay(self):
        if self.size < self.batch:
            return None
        rows = self.buf[np.random.randint(0, self.size, size=self.batch)]
        s, a, phi, s1, g = zip(*rows)
        return (torch.vstack(s).to(self.device), torch.tensor(a).to(self.device), torch.vstack(phi).to(self.device),
                torch.vstack(s1).to(self.device), torch.tensor(g).to(self.device))


class HostReplay:
    """A numpy ring sampled on the host.  The minibatch stays on the host: DeepSF.update_successor
    hands host arrays to the engine, which stages all five fields through one pinned slot and
    one non-blocking copy (a .to(device) per field would be five synchronous pageable copies)."""

    def __init__(self, capacity, batch, device, n_s, d):
        self.s = np.zeros((capacity, n_s), np.float32)
        self.s1 = np.zeros((capacity, n_s), np.float32)
        self.phi = np.zeros((capacity, d), np.float32)
        self.a = np.zeros(capacity, np.int64)
        self.g = np.zeros(capacity, np.float32)
        self.cap, self.batch, self.device = capacity, batch, device
        self.index = self.size = 0

    def append(self, s, a, phi, s1, gamma):
        j = self.index
        self.s[j], self.a[j], self.phi[j], self.s1[j], self.g[j] = s, a, phi, s1, gamma
        self.index = (j + 1) % self.cap
        self.size = min(self.size + 1, self.cap)

    def replay(self):
        if self.size < self.batch:
            return None
        idx = np.random.randint(0, self.size, size=self.batch)
        return (torch.from_numpy(self.s[idx]), torch.from_numpy(self.a[idx]), torch.from_numpy(self.phi[idx]),
                torch.from_numpy(self.s1[idx]), torch.from_numpy(self.g[idx]))


class DropinLoop:
    """Agent.next_sample over the drop-in DeepSF (the all-task schedule of agents/sfdqn.py)."""

    def __init__(self, T=8, n_s=17, H=256, A=7, d=8, acts=("relu", "relu"), batch=32, buffer="reference",
                 gamma=0.9, epsilon=0.1, alpha_w=0.05, seed=1, device=None):
        from sfx.dropin.features.deep import DeepSF
        from sfx.runner import SynthReacher

        self.device = device or torch.device("cuda", 0)
        random.seed(seed)
        np.random.seed(seed)
        torch.manual_seed(seed)
        rng = np.random.default_rng(seed)
        self.tasks = [_Task(SynthReacher(n_s, A, d, t, rng), self.device) for t in range(T)]
        self.sf = DeepSF(pytorch_model_handle=psi_model_lambda(H, acts, 1e-3, self.device),
                         hyperparameters={"learning_rate_w": alpha_w}, target_update_ev=1000, max_batch=batch)
        self.sf.reset()
        for t in self.tasks:
            self.sf.add_training_task(t)
        if buffer == "reference":
            from sfx.dropin.agents.buffer import ReplayBuffer

            self.buffer = ReplayBuffer({}, n_batch=batch)
            self.buffer.device = self.device
        elif buffer == "objring":
            self.buffer = RefReplay(1_000_000, batch, self.device)
        else:
            self.buffer = HostReplay(1_000_000, batch, self.device, n_s, d)
        self.ref_buffer = buffer in ("reference", "objring")
        self.T, self.A, self.gamma, self.epsilon = T, A, gamma, epsilon
        self.task = 0
        self.s_enc = None

    def step(self):
        task, dev = self.tasks[self.task], self.ref_buffer  # host ring: states and φ stay numpy
        if self.s_enc is None:
            self.s_enc = task.initialize(dev).reshape(1, -1)
        q, c = self.sf.GPI(self.s_enc, self.task, update_counters=True)
        q = q[:, c, :].flatten()
        if random.random() <= self.epsilon:
            a = torch.tensor(random.randrange(self.A)).to(self.device)
        else:
            a = torch.argmax(q)
        s1, phi, r, term = task.transition(a, dev)
        s1_enc = s1.reshape(1, -1)
        self.sf.update_reward(phi, r, self.task)
        g = 0.0 if term else self.gamma
        if self.ref_buffer:
            self.buffer.append(self.s_enc, a, phi, s1_enc, g)
        else:
            self.buffer.append(self.s_enc, int(a), phi, s1, g)
        batch = self.buffer.replay()
        for i in range(self.T):
            self.sf.update_successor(batch, i)
        self.s_enc = None if term else s1_enc

    def run(self, n):
        for _ in range(n):
            self.step()

    def close(self):
        self.sf._close()


def measure(buffer="reference", steps=300, warmup=60, windows=1, **kw) -> dict:
    """env-steps/s of the loop: `warmup` untimed steps, then `windows` consecutive timed windows of
    `steps` steps each; the value is their median (every window's rate is in the record)."""
    loop = DropinLoop(buffer=buffer, **kw)
    loop.run(warmup)
    loop.sf._flush()
    torch.cuda.synchronize()
    dts = []
    for _ in range(windows):
        t0 = time.perf_counter()
        loop.run(steps)
        loop.sf._flush()
        torch.cuda.synchronize()
        dts.append(time.perf_counter() - t0)
    loop.close()
    dt = sorted(dts)[len(dts) // 2]
    out = {"value": round(steps / dt, 2), "unit": "env steps/s", "ms_per_step": round(1000.0 * dt / steps, 4),
           "steps": steps, "dtype": "fp32",
           "path": f"drop-in features.deep.DeepSF under a Python agents/sfdqn.py loop ({buffer} replay buffer)"}
    if windows > 1:
        out["windows"] = [round(steps / t, 2) for t in dts]
        out["statistic"] = f"median of {windows} consecutive {steps}-step windows after {warmup} warm-up steps"
    return out


if __name__ == "__main__":
    import json
    import os
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "deep-successor-features-for-transfer_amd"))
    for b in ("reference", "objring", "host"):
        print(json.dumps({b: measure(b)}), flush=True)
