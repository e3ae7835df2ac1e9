"""Host-side env-step loop of SF-DQN driving the libsfx engine.

Mirrors Agent.next_sample (agents/agent.py:195-261) + SFDQN.train_agent for the two
schedules the reference has:

  * "all":    agents/sfdqn.py:47-60 over features/deep.py (main_sfdqn_torch.py):
              LMS reward fit on the active task, every head updated per env step, GPI next
              actions, loss = l1.
  * "active": sfdqn.py:462-471 / agents/sfdqn_sequential.py:63-76: only the active head is
              updated (with l2 + Adam-trained w), next actions by GPI or own ψ (use_gpi).
  * "tsf":    tsfdqn.py:566-580 / tsfdqn_nf.py:598-612: only the active head is updated, by
              TSFDQN.update_successor (φ̃ from g_i and the shared h; the engine must have
              been set up with SFEngine.tsf_setup).

The environment is a synthetic Reacher-shape task: s ~ N(0,1)^n_s,
φ ~ U[0,1)^d, r = φ·w_true with one-hot w_true (tasks/reacher.py:85-88), γ constant,
episodes of T_ep steps.  Replay is a host ring (agents/buffer.py:34-82) sampled uniformly;
each step's device inputs (the minibatch, the new transition's φ/r, the next state) travel
in ONE pinned host->device copy.
"""
from __future__ import annotations

import numpy as np
import torch

from .engine import SFEngine


class SynthReacher:
    """Synthetic Reacher-shape task (never terminates, like tasks/reacher.py:112)."""

    def __init__(self, n_s: int, A: int, d: int, task_index: int, rng: np.random.Generator):
        self.n_s, self.A, self.d, self.task_index, self.rng = n_s, A, d, task_index, rng
        self.w_true = np.zeros(d, dtype=np.float32)
        self.w_true[task_index % d] = 1.0

    def initialize(self) -> np.ndarray:
        return self.rng.standard_normal(self.n_s, dtype=np.float32)

    def transition(self, a: int):
        s1 = self.rng.standard_normal(self.n_s, dtype=np.float32)
        phi = self.rng.random(self.d, dtype=np.float32)
        r = float(phi @ self.w_true)
        return s1, phi, r, False


class SynthHopper(SynthReacher):
    """Synthetic Hopper-shape task (BASELINE config C3: |s|=11, 27 actions, d=50): like
    SynthReacher, but an episode ends with probability `p_end` per step (γ = 0 then), the
    way tasks/hopper_phi.py's falls do."""

    def __init__(self, n_s: int, A: int, d: int, task_index: int, rng: np.random.Generator, p_end: float = 0.01):
        super().__init__(n_s, A, d, task_index, rng)
        self.p_end = p_end

    def transition(self, a: int):
        s1, phi, r, _ = super().transition(a)
        return s1, phi, r, bool(self.rng.random() < self.p_end)


class Staging:
    """One pinned host buffer + one device buffer with typed views at fixed offsets."""

    def __init__(self, fields, device):
        self.offsets, off = {}, 0
        for name, shape, dtype in fields:
            n = int(np.prod(shape)) * torch.empty((), dtype=dtype).element_size()
            self.offsets[name] = (off, shape, dtype)
            off += (n + 15) // 16 * 16
        self.nbytes = off
        self.host = torch.empty(off, dtype=torch.uint8, pin_memory=True)
        self.dev = torch.empty(off, dtype=torch.uint8, device=device)
        self.h = {k: self._view(self.host, k).numpy() for k in self.offsets}
        self.d = {k: self._view(self.dev, k) for k in self.offsets}

    def _view(self, buf, name):
        off, shape, dtype = self.offsets[name]
        n = int(np.prod(shape)) * torch.empty((), dtype=dtype).element_size()
        return buf[off:off + n].view(dtype).view(*shape)

    def upload(self):
        self.dev.copy_(self.host, non_blocking=True)


class Replay:
    """Uniform replay ring (agents/buffer.py:34-82) with arrays instead of object tuples."""

    def __init__(self, capacity: int, n_s: int, d: int, rng: np.random.Generator):
        self.cap, self.rng = capacity, rng
        self.s = np.zeros((capacity, n_s), np.float32)
        self.s1 = np.zeros((capacity, n_s), np.float32)
        self.phi = np.zeros((capacity, d), np.float32)
        self.r = np.zeros(capacity, np.float32)
        self.a = np.zeros(capacity, np.int64)
        self.gamma = np.zeros(capacity, np.float32)
        self.index = 0
        self.size = 0

    def append(self, s, a, r, phi, s1, gamma):
        i = self.index
        self.s[i], self.a[i], self.r[i], self.phi[i], self.s1[i], self.gamma[i] = s, a, r, phi, s1, gamma
        self.size = min(self.size + 1, self.cap)
        self.index = (i + 1) % self.cap

    def sample_into(self, st: Staging, B: int) -> bool:
        if self.size < B:
            return False
        idx = self.rng.integers(0, self.size, B)
        np.take(self.s, idx, axis=0, out=st.h["s"])
        np.take(self.s1, idx, axis=0, out=st.h["s1"])
        np.take(self.phi, idx, axis=0, out=st.h["phi"])
        if "r" in st.h:
            np.take(self.r, idx, out=st.h["r"].reshape(-1))
        np.take(self.a, idx, out=st.h["a"])
        np.take(self.gamma, idx, out=st.h["gamma"])
        return True


class EnvLoop:
    """The training env-step loop of one active task over an SFEngine of T heads."""

    def __init__(self, engine: SFEngine, schedule: str = "all", batch: int = 32, capacity: int = 1_000_000,
                 gamma: float = 0.9, epsilon: float = 0.1, alpha_w: float = 1e-3, episode_len: int = 500,
                 use_gpi: bool = True, seed: int = 1, task_cls=SynthReacher):
        assert schedule in ("all", "active", "tsf")
        self.eng, self.schedule, self.B = engine, schedule, batch
        self.gamma, self.epsilon, self.alpha_w, self.T_ep, self.use_gpi = gamma, epsilon, alpha_w, episode_len, use_gpi
        e = engine
        self.rng = np.random.default_rng(seed)
        self.tasks = [task_cls(e.n_s, e.A, e.d, t, self.rng) for t in range(e.T)]
        self.replay = Replay(capacity, e.n_s, e.d, self.rng)
        self.st = Staging([("s", (batch, e.n_s), torch.float32), ("s1", (batch, e.n_s), torch.float32),
                           ("phi", (batch, e.d), torch.float32), ("r", (batch,), torch.float32),
                           ("a", (batch,), torch.int64), ("gamma", (batch,), torch.float32),
                           ("snext", (1, e.n_s), torch.float32), ("phi1", (e.d,), torch.float32),
                           ("r1", (1,), torch.float32)], e.device)
        self.losses = torch.zeros(max(e.T, 1), 3, device=e.device)
        self.sel_host = torch.zeros(2, dtype=torch.long, pin_memory=True)
        self.gpi_counters = np.zeros((e.T, e.T), dtype=np.int64)
        self.set_task(0)

    def set_task(self, index: int):
        """Agent.set_active_training_task (agents/agent.py:121-139)."""
        self.task_index = index
        self.task = self.tasks[index]
        self.steps_in_episode = 0
        self.s = self.task.initialize()
        self.st.h["snext"][0] = self.s
        self.st.upload()
        if self.schedule == "all":
            self.eng.step_all(s_next=self.st.d["snext"], task_index=index, sel_use_gpi=self.use_gpi)
            c, a, _ = self.eng.step_finish()
            self.sel = (c, a)
        else:
            self._issue_select()

    def prefill(self, n: int):
        """Random transitions into the replay (warm-up only; not an env step)."""
        for _ in range(n):
            s = self.task.initialize()
            a = int(self.rng.integers(self.eng.A))
            s1, phi, r, _ = self.task.transition(a)
            self.replay.append(s, a, r, phi, s1, self.gamma)

    def _issue_select(self):
        e = self.eng
        sel = e.select_action(self.st.d["snext"], self.task_index, self.use_gpi)
        self.sel_host.copy_(sel, non_blocking=True)
        self.sel_event = torch.cuda.Event()
        self.sel_event.record()

    def _greedy(self):
        if self.schedule == "all":
            return self.sel
        self.sel_event.synchronize()
        return int(self.sel_host[0]), int(self.sel_host[1])

    def step(self):
        """One env step: GPI action (computed by the previous step), ε-greedy, transition, train."""
        c, a_greedy = self._greedy()
        self.gpi_counters[self.task_index, c] += 1
        if self.rng.random() <= self.epsilon:
            a = int(self.rng.integers(self.eng.A))
        else:
            a = a_greedy
        s1, phi, r, terminal = self.task.transition(a)
        g = 0.0 if terminal else self.gamma
        st = self.st
        self.replay.append(self.s, a, r, phi, s1, g)
        have = self.replay.sample_into(st, self.B)
        self.steps_in_episode += 1
        s_next = s1
        if terminal or self.steps_in_episode >= self.T_ep:  # new episode (agent.py:211-220, 248-249)
            s_next = self.task.initialize()
            self.steps_in_episode = 0
        st.h["phi1"][:] = phi
        st.h["r1"][0] = r
        st.h["snext"][0] = s_next
        st.upload()
        d, e = st.d, self.eng
        if self.schedule == "all":
            if have:
                e.step_all(d["s"], d["a"], d["phi"], d["s1"], d["gamma"], use_gpi=True, lms_task=self.task_index,
                           lms_phi=d["phi1"], lms_r=d["r1"], lms_alpha=self.alpha_w, s_next=d["snext"],
                           task_index=self.task_index, sel_use_gpi=self.use_gpi, losses=self.losses)
            else:
                e.step_all(lms_task=self.task_index, lms_phi=d["phi1"], lms_r=d["r1"], lms_alpha=self.alpha_w,
                           s_next=d["snext"], task_index=self.task_index, sel_use_gpi=self.use_gpi)
            c, a, _ = e.step_finish()
            self.sel = (c, a)
        else:
            upd = e.tsf_update if self.schedule == "tsf" else e.update
            if have:
                upd(self.task_index, d["s"], d["a"], d["r"], d["phi"], d["s1"], d["gamma"], self.use_gpi,
                    losses=self.losses[0])
            self._issue_select()
        self.s = s_next

    def run(self, n: int):
        for _ in range(n):
            self.step()


class NativeEnvLoop:
    """The env-step loop of EnvLoop run by libsfx's native runner (include/sfx.h, sfx_runner_*):
    C++ env + replay ring on the host, one pre-launched hipGraph per env step whose gate kernel
    waits for the host's inputs.  schedule: "all" (main_sfdqn_torch.py), "active" (sfdqn.py /
    agents/sfdqn_sequential.py: the active head with l2 and an Adam-trained w, no LMS), "tsf"
    (TSFDQN.update_successor; needs SFEngine.tsf_setup), "sharded" (the all-task step with the
    heads split over ranks, BASELINE config C4) or "sharded_tsf" (the TSF step with the heads split
    over ranks, config C5: tsf_setup + shard_setup + a communicator; the active task is a global
    index and its owner updates).  p_end: per-step episode-end
    probability of the built-in synthetic task (0: never terminates, like tasks/reacher.py).

    env: None for the built-in synthetic Reacher-shape task, or an object with
    ``reset(task) -> s0`` and ``step(task, a) -> (s1, phi, r, terminal)`` (numpy / floats),
    called through C callbacks (agents/agent.py's Task interface: tasks/task.py).
    """

    FIELDS = ("s", "s1", "phi", "a", "gamma", "snext", "phi1", "r1", "rb")
    SCHEDULES = {"all": 0, "active": 1, "tsf": 2, "sharded": 3, "sharded_tsf": 4}

    def __init__(self, engine: SFEngine, batch: int = 32, capacity: int = 1_000_000, gamma: float = 0.9,
                 epsilon: float = 0.1, alpha_w: float = 1e-3, episode_len: int = 500, use_gpi: bool = True,
                 seed: int = 1, env=None, schedule: str = "all", upd_use_gpi: bool = True, p_end: float = 0.0,
                 device_replay: bool = False):
        import ctypes as C

        from ._lib import ENV_RESET_FN, ENV_STEP_FN, check, lib

        self.eng, self.B, self._lib, self._check, self._C = engine, batch, lib, check, C
        self._cbs = None
        reset_fn = step_fn = None
        if env is not None:
            n_s, d = engine.n_s, engine.d

            def _reset(_ctx, task, s0):
                try:
                    v = np.asarray(env.reset(task), dtype=np.float32).reshape(n_s)
                    np.ctypeslib.as_array(s0, shape=(n_s,))[:] = v
                    return 0
                except Exception:  # reported as a failed step by libsfx
                    return 1

            def _step(_ctx, task, a, s1, phi, r, term):
                try:
                    ns, ph, rr, tt = env.step(task, a)
                    np.ctypeslib.as_array(s1, shape=(n_s,))[:] = np.asarray(ns, np.float32).reshape(n_s)
                    np.ctypeslib.as_array(phi, shape=(d,))[:] = np.asarray(ph, np.float32).reshape(d)
                    r[0] = float(rr)
                    term[0] = 1 if tt else 0
                    return 0
                except Exception:
                    return 1

            self._cbs = (ENV_RESET_FN(_reset), ENV_STEP_FN(_step))
            reset_fn, step_fn = self._cbs
        r = C.c_void_p()
        check(lib.sfx_runner_create(C.byref(r), engine._h, batch, capacity, gamma, epsilon, alpha_w, episode_len,
                                    1 if use_gpi else 0, seed, C.cast(reset_fn, C.c_void_p) if reset_fn else None,
                                    C.cast(step_fn, C.c_void_p) if step_fn else None, None), "sfx_runner_create")
        self._r = r
        off = (C.c_int64 * 10)()
        check(lib.sfx_runner_layout(r, off), "sfx_runner_layout")
        self.layout = {k: int(off[i]) for i, k in enumerate(self.FIELDS)}
        self.record_bytes = int(off[9])
        self.schedule = schedule
        check(lib.sfx_runner_config(r, self.SCHEDULES[schedule], 1 if upd_use_gpi else 0, float(p_end)),
              "sfx_runner_config")
        self.task_index = 0
        if device_replay:
            self.set_device_replay(True)

    def set_device_replay(self, on: bool):
        """SURVEY §8f rank 2 (opt-in; the north_star keeps the replay on the host): the ring in
        HBM, appended and sampled by each step's gate kernel; the host ring stays as a mirror."""
        self._check(self._lib.sfx_runner_device_replay(self._r, 1 if on else 0), "sfx_runner_device_replay")

    def close(self):
        if getattr(self, "_r", None):
            self._lib.sfx_runner_destroy(self._r)
            self._r = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_task(self, index: int):
        self._check(self._lib.sfx_runner_set_task(self._r, index), "sfx_runner_set_task")
        self.task_index = index

    def prefill(self, n: int):
        self._check(self._lib.sfx_runner_prefill(self._r, n), "sfx_runner_prefill")

    def run(self, n: int):
        self._check(self._lib.sfx_runner_run(self._r, n), "sfx_runner_run")

    def action(self):
        out = (self._C.c_int64 * 3)()
        self._check(self._lib.sfx_runner_action(self._r, out), "sfx_runner_action")
        return int(out[0]), int(out[1])

    def warm(self):
        """Instantiate this schedule's step graphs (all span lengths, both slot parities) now."""
        self._check(self._lib.sfx_runner_warm(self._r), "sfx_runner_warm")

    def set_gate_timeout(self, seconds: float):
        """Bound of each step's gate wait; a step released later is cancelled and re-issued."""
        self._check(self._lib.sfx_runner_gate_timeout(self._r, float(seconds)), "sfx_runner_gate_timeout")

    def set_wait_timeout(self, seconds: float):
        """Bound of the host's wait on a step's result (sfx_runner_wait_timeout): past it the
        queued steps are cancelled and drained; a sharded step stuck in a collective gets its
        communicators aborted and the call raises instead of hanging."""
        self._check(self._lib.sfx_runner_wait_timeout(self._r, float(seconds)), "sfx_runner_wait_timeout")

    def stats(self) -> dict:
        C = self._C
        a, b, c, w, rt = C.c_longlong(), C.c_longlong(), C.c_longlong(), C.c_double(), C.c_longlong()
        self._check(self._lib.sfx_runner_stats(self._r, C.byref(a), C.byref(b), C.byref(c), C.byref(w)),
                    "sfx_runner_stats")
        self._check(self._lib.sfx_runner_retried(self._r, C.byref(rt)), "sfx_runner_retried")
        rc, nf = C.c_longlong(), C.c_longlong()
        self._check(self._lib.sfx_runner_recomputed(self._r, C.byref(rc)), "sfx_runner_recomputed")
        self._check(self._lib.sfx_runner_nonfinite(self._r, C.byref(nf)), "sfx_runner_nonfinite")
        ps, ofs = C.c_longlong(), C.c_longlong()
        self._check(self._lib.sfx_runner_ahead_stats(self._r, C.byref(ps), C.byref(ofs)), "sfx_runner_ahead_stats")
        return {"env_steps": a.value, "prelaunched": b.value, "host_round_steps": c.value,
                "host_wait_us": round(w.value, 1), "retried": rt.value, "recomputed": rc.value,
                "nonfinite_steps": nf.value, "ahead_pre_steps": ps.value, "ahead_own_forward_steps": ofs.value}

    def gpi_counters(self) -> np.ndarray:
        T = self.eng.T_glob if self.schedule.startswith("sharded") else self.eng.T
        out = np.zeros(T * T, dtype=np.int64)
        self._check(self._lib.sfx_runner_gpi_counters(self._r, out.ctypes.data_as(self._C.POINTER(self._C.c_longlong))),
                    "sfx_runner_gpi_counters")
        return out.reshape(T, T)

    def record(self, capacity: int):
        self._check(self._lib.sfx_runner_record(self._r, capacity), "sfx_runner_record")

    def records(self) -> list:
        """Decoded input records: dict of numpy arrays + (task, have, c, a_greedy, a, terminal)."""
        C, e, B = self._C, self.eng, self.B
        shapes = {"s": ((B, e.n_s), np.float32), "s1": ((B, e.n_s), np.float32), "phi": ((B, e.d), np.float32),
                  "a": ((B,), np.int64), "gamma": ((B,), np.float32), "snext": ((e.n_s,), np.float32),
                  "phi1": ((e.d,), np.float32), "r1": ((1,), np.float32), "rb": ((B,), np.float32)}
        out = []
        for i in range(self._lib.sfx_runner_recorded(self._r)):
            buf = np.zeros(self.record_bytes, dtype=np.uint8)
            meta = (C.c_int64 * 6)()
            self._check(self._lib.sfx_runner_get_record(self._r, i, buf.ctypes.data_as(C.c_void_p), meta),
                        "sfx_runner_get_record")
            rec = {}
            for k, (shape, dt) in shapes.items():
                n = int(np.prod(shape)) * np.dtype(dt).itemsize
                rec[k] = buf[self.layout[k]:self.layout[k] + n].view(dt).reshape(shape).copy()
            rec.update(zip(("task", "have", "c", "a_greedy", "a_taken", "terminal"), (int(m) for m in meta)))
            out.append(rec)
        return out


class ShardedEnvLoop:
    """The all-task env-step loop with the heads sharded across ranks (sfx.shard): every rank
    runs the same env / replay stream (same seed), owns T_loc heads, and all-reduces the GPI
    maxima; the env action is identical on every rank."""

    def __init__(self, engine: SFEngine, T_glob: int, rank: int, all_reduce_max, batch: int = 32,
                 capacity: int = 1_000_000, gamma: float = 0.9, epsilon: float = 0.1, alpha_w: float = 1e-3,
                 episode_len: int = 500, use_gpi: bool = True, seed: int = 1, rounds: int = 2):
        from .shard import LibsfxShardBackend, ShardedAllTask

        e = engine
        self.eng, self.B, self.Tg = engine, batch, T_glob
        self.gamma, self.epsilon, self.alpha_w, self.T_ep, self.use_gpi = gamma, epsilon, alpha_w, episode_len, use_gpi
        self.backend = LibsfxShardBackend(engine, T_glob, rank * engine.T, batch)
        self.sharded = ShardedAllTask(self.backend, T_glob, e.A, all_reduce_max, rounds=rounds)
        self.rng = np.random.default_rng(seed)
        self.tasks = [SynthReacher(e.n_s, e.A, e.d, t, self.rng) for t in range(T_glob)]
        self.replay = Replay(capacity, e.n_s, e.d, self.rng)
        self.st = Staging([("s", (batch, e.n_s), torch.float32), ("s1", (batch, e.n_s), torch.float32),
                           ("phi", (batch, e.d), torch.float32), ("a", (batch,), torch.int64),
                           ("gamma", (batch,), torch.float32), ("snext", (1, e.n_s), torch.float32),
                           ("phi1", (e.d,), torch.float32), ("r1", (1,), torch.float32)], e.device)
        self.gpi_counters = np.zeros((T_glob, T_glob), dtype=np.int64)

    def set_task(self, index: int):
        self.task_index, self.task = index, self.tasks[index]
        self.steps_in_episode = 0
        self.s = self.task.initialize()
        self.st.h["snext"][0] = self.s
        self.st.upload()
        d = self.st.d
        self.sel = self.sharded.step(None, -1, None, None, 0.0, d["snext"], index, self.use_gpi)

    def prefill(self, n: int):
        for _ in range(n):
            s = self.task.initialize() if hasattr(self, "task") else self.tasks[0].initialize()
            a = int(self.rng.integers(self.eng.A))
            s1, phi, r, _ = (self.task if hasattr(self, "task") else self.tasks[0]).transition(a)
            self.replay.append(s, a, r, phi, s1, self.gamma)

    def step(self):
        c, a_greedy = self.sel
        self.gpi_counters[self.task_index, c] += 1
        a = int(self.rng.integers(self.eng.A)) if self.rng.random() <= self.epsilon else a_greedy
        s1, phi, r, terminal = self.task.transition(a)
        self.replay.append(self.s, a, r, phi, s1, 0.0 if terminal else self.gamma)
        st = self.st
        have = self.replay.sample_into(st, self.B)
        self.steps_in_episode += 1
        s_next = s1
        if terminal or self.steps_in_episode >= self.T_ep:
            s_next = self.task.initialize()
            self.steps_in_episode = 0
        st.h["phi1"][:] = phi
        st.h["r1"][0] = r
        st.h["snext"][0] = s_next
        st.upload()
        d = st.d
        batch = (d["s"], d["a"], d["phi"], d["s1"], d["gamma"]) if have else None
        self.sel = self.sharded.step(batch, self.task_index, d["phi1"], d["r1"], self.alpha_w, d["snext"],
                                     self.task_index, self.use_gpi)
        self.s = s_next

    def run(self, n: int):
        for _ in range(n):
            self.step()


class ShardedTSFEnvLoop:
    """TSF-DQN's env-step loop (tsfdqn.py next_sample + train_agent, active task) with the heads
    sharded across ranks (sfx.shard.ShardedTSF; BASELINE config C5): every rank runs the same
    env / replay stream (same seed), the GPI maxima and the action key are all-reduced, the
    active task's owner updates and broadcasts h and w_i."""

    def __init__(self, engine: SFEngine, T_glob: int, rank: int, all_reduce_max, broadcast, batch: int = 32,
                 capacity: int = 1_000_000, gamma: float = 0.9, epsilon: float = 0.1, episode_len: int = 500,
                 use_gpi: bool = True, seed: int = 1, p_end: float = 0.01):
        from .shard import LibsfxTSFShardBackend, ShardedTSF

        e = engine
        self.eng, self.B, self.Tg = engine, batch, T_glob
        self.gamma, self.epsilon, self.T_ep, self.use_gpi = gamma, epsilon, episode_len, use_gpi
        self.backend = LibsfxTSFShardBackend(engine, T_glob, rank * engine.T, batch)
        self.sharded = ShardedTSF(self.backend, T_glob, rank, e.A, all_reduce_max, broadcast)
        self.rng = np.random.default_rng(seed)
        self.tasks = [SynthHopper(e.n_s, e.A, e.d, t, self.rng, p_end) for t in range(T_glob)]
        self.replay = Replay(capacity, e.n_s, e.d, self.rng)
        self.st = Staging([("s", (batch, e.n_s), torch.float32), ("s1", (batch, e.n_s), torch.float32),
                           ("phi", (batch, e.d), torch.float32), ("r", (batch, 1), torch.float32),
                           ("a", (batch,), torch.int64), ("gamma", (batch,), torch.float32),
                           ("snext", (1, e.n_s), torch.float32)], e.device)
        self.gpi_counters = np.zeros((T_glob, T_glob), dtype=np.int64)

    def set_task(self, index: int):
        self.task_index, self.task = index, self.tasks[index]
        self.steps_in_episode = 0
        self.s = self.task.initialize()
        self.st.h["snext"][0] = self.s
        self.st.upload()
        self.sel = self.sharded.select(self.st.d["snext"], index, self.use_gpi)

    def prefill(self, n: int):
        task = getattr(self, "task", self.tasks[0])
        for _ in range(n):
            s = task.initialize()
            a = int(self.rng.integers(self.eng.A))
            s1, phi, r, _ = task.transition(a)
            self.replay.append(s, a, r, phi, s1, self.gamma)

    def step(self):
        c, a_greedy = self.sel
        self.gpi_counters[self.task_index, c] += 1
        a = int(self.rng.integers(self.eng.A)) if self.rng.random() <= self.epsilon else a_greedy
        s1, phi, r, terminal = self.task.transition(a)
        self.replay.append(self.s, a, r, phi, s1, 0.0 if terminal else self.gamma)
        st = self.st
        have = self.replay.sample_into(st, self.B)
        self.steps_in_episode += 1
        s_next = s1
        if terminal or self.steps_in_episode >= self.T_ep:
            s_next = self.task.initialize()
            self.steps_in_episode = 0
        st.h["snext"][0] = s_next
        st.upload()
        d = st.d
        if have:
            self.sharded.update(self.task_index, (d["s"], d["a"], d["r"], d["phi"], d["s1"], d["gamma"]), self.use_gpi)
        self.sel = self.sharded.select(d["snext"], self.task_index, self.use_gpi)
        self.s = s_next

    def run(self, n: int):
        for _ in range(n):
            self.step()
