"""Source-task heads sharded across ranks (BASELINE config C4).

Rank g owns global heads [g*T_loc, (g+1)*T_loc); the reward weights w, the env and the
replay are replicated with identical seeds, so every rank sees the same minibatch and the
same env action.  GPI is the only cross-rank computation: each rank reduces q over its own
heads and an all-reduce(MAX) finishes the reduction (exact: max is order-free; first-index
argmax tie-breaking is preserved by the packed selection key).  Backward and Adam stay local.

``ShardedAllTask`` runs one all-task env step (agents/sfdqn.py:47-60 over features/deep.py,
in-order semantics) as the speculative rounds of DESIGN.md §4 with the GPI split across
ranks.  It drives a *backend* with the protocol of include/sfx.h's sfx_shard_* calls:
``LibsfxShardBackend`` (the GPU path) or, in the CPU tests, an oracle backend.
"""
from __future__ import annotations

import ctypes as C
from typing import Callable, Optional

import torch

_SIGN = 1 << 63


def decode_key(key: int, A: int):
    """int64 selection key (k_skey) -> (GPI task c, action a)."""
    u = (int(key) & ((1 << 64) - 1)) ^ _SIGN
    idx = 0xFFFFFFFF - (u & 0xFFFFFFFF)
    return idx // A, idx % A


def encode_key(q: float, t: int, a: int, A: int) -> int:
    """The packing k_skey uses (for host-side backends): order-preserving float bits << 32 |
    ~(t*A + a), shifted into signed int64 order."""
    import struct

    q = q + 0.0  # -0 -> +0
    u = struct.unpack("<I", struct.pack("<f", q))[0]
    o = (~u & 0xFFFFFFFF) if (u & 0x80000000) else (u | 0x80000000)
    key_u = (o << 32) | (0xFFFFFFFF - (t * A + a))
    key_s = key_u ^ _SIGN
    return key_s - (1 << 64) if key_s >= (1 << 63) else key_s


def all_reduce_max_fn(group=None, via_host: bool = False) -> Callable[[torch.Tensor], None]:
    """all-reduce(MAX) in place over the default (or given) process group.  via_host: stage
    through CPU memory (gloo groups driving device tensors)."""
    import torch.distributed as dist

    def ar(t: torch.Tensor):
        if via_host:
            h = t.cpu()
            dist.all_reduce(h, op=dist.ReduceOp.MAX, group=group)
            t.copy_(h)
        else:
            dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)

    return ar


class ShardedAllTask:
    def __init__(self, backend, T_glob: int, A: int, all_reduce_max: Callable[[torch.Tensor], None], rounds: int = 2):
        self.be, self.Tg, self.A, self.ar, self.rounds = backend, T_glob, A, all_reduce_max, rounds
        self.stats = {"steps": 0, "host_round_steps": 0, "rounds": 0}

    def step(self, batch, lms_task: int, lms_phi, lms_r, alpha: float, s_next, task: int, sel_use_gpi: bool = True):
        """One env step.  batch = (S, a, phi, S1, gamma) or None (replay not filled yet).
        Returns (c, a) of the env action for s_next (post-update heads)."""
        be, ar = self.be, self.ar
        be.begin(batch, lms_task, lms_phi, lms_r, alpha, s_next)
        if batch is None:
            key = be.select(-1, task, sel_use_gpi)
            ar(key)
            be.finish(0)
            return decode_key(int(key.item()), self.A)
        X, Y = be.X, be.Y
        for r in range(self.rounds):
            be.td_maxima(r, X)
            ar(X)
            be.td_update(r, X)
        last = self.rounds - 1
        be.ver_maxima(last, Y)
        ar(Y)
        flag = be.verify(X, Y)
        if flag < self.Tg:
            self.stats["host_round_steps"] += 1
        while flag < self.Tg:  # each extra round fixes at least one more policy
            last += 1
            if last > self.Tg + 1:
                raise RuntimeError("sharded speculation did not converge")
            be.td_maxima(last, X)
            ar(X)
            be.td_update(last, X)
            be.ver_maxima(last, Y)
            ar(Y)
            flag = be.verify(X, Y)
        key = be.select(last, task, sel_use_gpi)
        ar(key)
        be.finish(last + 1)
        self.stats["steps"] += 1
        self.stats["rounds"] += last + 1
        return decode_key(int(key.item()), self.A)


class LibsfxShardBackend:
    """sfx_shard_* on one SFEngine holding this rank's T_loc heads."""

    def __init__(self, engine, T_glob: int, head_offset: int, max_batch: int):
        from ._lib import check, lib

        self.eng, self.lib, self.check = engine, lib, check
        self.Tg, self.off = T_glob, head_offset
        engine.shard_setup(T_glob, head_offset)
        dev = engine.device
        # GPI maxima as sortable int32 (include/sfx.h): all-reduce(MAX) on int32 is the fp32 max
        self._X = torch.empty(T_glob * max_batch * engine.A, device=dev, dtype=torch.int32)
        self._Y = torch.empty_like(self._X)
        self.key = torch.empty(1, dtype=torch.long, device=dev)
        self.flag = torch.empty(1, dtype=torch.int32, device=dev)
        self.B = 0

    @property
    def X(self):  # [T_glob][B][A] TD maxima of the current step
        return self._X[: self.Tg * self.B * self.eng.A]

    @property
    def Y(self):  # verification maxima
        return self._Y[: self.Tg * self.B * self.eng.A]

    def begin(self, batch, lms_task, lms_phi, lms_r, alpha, s_next):
        e = self.eng
        if batch is None:
            self.B = 0
            ptrs = [None] * 5
        else:
            S, a, phi, S1, g = batch
            self.B = S.shape[0]
            ptrs = [S.data_ptr(), a.data_ptr(), phi.data_ptr(), S1.data_ptr(), g.data_ptr()]
        self._keep = (batch, lms_phi, lms_r, s_next)
        self.check(self.lib.sfx_shard_begin(e.handle, *ptrs, self.B, int(lms_task),
                                            None if lms_phi is None else lms_phi.data_ptr(),
                                            None if lms_r is None else lms_r.data_ptr(), float(alpha),
                                            s_next.data_ptr()), "sfx_shard_begin")

    def td_maxima(self, r, X):
        self.check(self.lib.sfx_shard_td_maxima(self.eng.handle, r, X.data_ptr()), "sfx_shard_td_maxima")

    def td_update(self, r, X):
        self.check(self.lib.sfx_shard_td_update(self.eng.handle, r, X.data_ptr()), "sfx_shard_td_update")

    def ver_maxima(self, r, Y):
        self.check(self.lib.sfx_shard_ver_maxima(self.eng.handle, r, Y.data_ptr()), "sfx_shard_ver_maxima")

    def verify(self, X, Y) -> int:
        self.check(self.lib.sfx_shard_verify(self.eng.handle, X.data_ptr(), Y.data_ptr(), self.flag.data_ptr()),
                   "sfx_shard_verify")
        return int(self.flag.item())

    def select(self, r, task, use_gpi) -> torch.Tensor:
        self.check(self.lib.sfx_shard_select(self.eng.handle, r, int(task), int(bool(use_gpi)), self.key.data_ptr()),
                   "sfx_shard_select")
        return self.key

    def finish(self, rounds_run):
        self.check(self.lib.sfx_shard_finish(self.eng.handle, int(rounds_run)), "sfx_shard_finish")


def broadcast_fn(group=None, via_host: bool = False) -> Callable[[torch.Tensor, int], None]:
    """broadcast(t, src) in place over the default (or given) process group (via_host: stage
    through CPU memory, for gloo groups driving device tensors)."""
    import torch.distributed as dist

    def bc(t: torch.Tensor, src: int):
        if via_host:
            h = t.cpu()
            dist.broadcast(h, src=src, group=group)
            t.copy_(h)
        else:
            dist.broadcast(t, src=src, group=group)

    return bc


class ShardedTSF:
    """TSF-DQN's active-task step with the heads sharded across ranks (BASELINE config C5:
    tsfdqn_nf.py, 32 source tasks over 4 GPUs).

    Policy i's head, g_i and its optimizer state (Adam moments of ψ_i, w_i, g_i and of the
    shared h, which are per task in the reference: tsfdqn.py:255-270) live with its owner
    i // T_loc.  w (all T_glob rows) and h are replicated.  One TSFDQN.update_successor
    (tsfdqn.py:588-709): the GPI maxima of the next actions are all-reduced (MAX) over the
    ranks, the owner runs the update, then broadcasts h and w_i (Ph + d floats).  The env
    action (get_Q_values: SF.GPI with w of the active task) is one all-reduced int64 key.
    Drives a backend with the sfx_shard_tsf_* protocol (include/sfx.h)."""

    def __init__(self, backend, T_glob: int, rank: int, A: int, all_reduce_max: Callable[[torch.Tensor], None],
                 broadcast: Callable[[torch.Tensor, int], None]):
        self.be, self.Tg, self.rank, self.A, self.ar, self.bc = backend, T_glob, rank, A, all_reduce_max, broadcast
        self.T_loc = backend.T

    def owner(self, i: int) -> int:
        return i // self.T_loc

    def update(self, i: int, batch, use_gpi: bool = True):
        """batch = (s, a, r, phi, s1, gamma) (tsfdqn.py's transition tuple).  Returns the owner's
        losses tensor (l1 + β l2, l1, l2) on the owner, None elsewhere."""
        be, mine = self.be, self.owner(i) == self.rank
        X = be.X(batch[0].shape[0])
        if use_gpi:
            be.maxima(i, batch[4], X, False)
            self.ar(X)
        elif mine:
            be.maxima(i, batch[4], X, True)
        losses = None
        buf = be.shared_buf
        if mine:
            losses = be.update(i, batch, X)
            be.pack(i, buf)
        self.bc(buf, self.owner(i))
        if not mine:
            be.unpack(i, buf)
        return losses

    def select(self, s, task: int, use_gpi: bool = True):
        """(GPI task c, greedy action a) for state s [1, n_s] with w of `task`."""
        key = self.be.select(s, task, use_gpi)
        self.ar(key)
        return decode_key(int(key.item()), self.A)


class LibsfxTSFShardBackend:
    """sfx_shard_tsf_* on one SFEngine holding this rank's T_loc heads (tsf_setup done)."""

    def __init__(self, engine, T_glob: int, head_offset: int, max_batch: int):
        from ._lib import check, lib

        self.eng, self.lib, self.check = engine, lib, check
        self.Tg, self.off, self.T = T_glob, head_offset, engine.T
        engine.shard_setup(T_glob, head_offset)
        dev = engine.device
        self._X = torch.empty(max_batch * engine.A, device=dev, dtype=torch.int32)  # sortable int32 maxima
        self.shared_buf = torch.empty(engine.tsf_Ph + engine.d, device=dev)
        self.key = torch.empty(1, dtype=torch.long, device=dev)
        self.losses = torch.empty(3, device=dev)

    def X(self, B: int):
        return self._X[: B * self.eng.A]

    def maxima(self, i, S1, X, own_only):
        self.check(self.lib.sfx_shard_tsf_maxima(self.eng.handle, int(i), S1.data_ptr(), S1.shape[0], int(own_only),
                                                 X.data_ptr()), "sfx_shard_tsf_maxima")

    def update(self, i, batch, X):
        s, a, r, phi, s1, g = batch
        self._keep = batch
        self.check(self.lib.sfx_shard_tsf_update(self.eng.handle, int(i), s.data_ptr(), a.data_ptr(), r.data_ptr(),
                                                 phi.data_ptr(), s1.data_ptr(), g.data_ptr(), s.shape[0], X.data_ptr(),
                                                 self.losses.data_ptr()), "sfx_shard_tsf_update")
        return self.losses

    def pack(self, i, buf):
        self.check(self.lib.sfx_shard_tsf_shared(self.eng.handle, int(i), buf.data_ptr(), 0), "sfx_shard_tsf_shared")

    def unpack(self, i, buf):
        self.check(self.lib.sfx_shard_tsf_shared(self.eng.handle, int(i), buf.data_ptr(), 1), "sfx_shard_tsf_shared")

    def select(self, s, task, use_gpi) -> torch.Tensor:
        self.check(self.lib.sfx_shard_tsf_select(self.eng.handle, s.data_ptr(), int(task), int(bool(use_gpi)),
                                                 self.key.data_ptr()), "sfx_shard_tsf_select")
        return self.key


# ---------------------------------------------------------------- the library's own collective
def init_comm(engine, rank: int, world: int, group=None):
    """RCCL communicator for the native sharded step (include/sfx.h sfx_comm_init): rank 0 makes
    the unique id, torch.distributed broadcasts its bytes, every rank joins.  Afterwards the
    library all-reduces on its own stream (inside the step graphs); torch is not on the path."""
    import ctypes as C

    import torch.distributed as dist

    from ._lib import check, lib

    n = lib.sfx_comm_id_bytes()
    buf = (C.c_uint8 * n)()
    if rank == 0:
        check(lib.sfx_comm_unique_id(buf), "sfx_comm_unique_id")
    t = torch.tensor(list(bytes(buf)), dtype=torch.uint8)
    if world > 1:
        backend = dist.get_backend(group)
        dev = engine.device if backend == "nccl" else "cpu"
        t = t.to(dev)
        dist.broadcast(t, src=0, group=group)
        t = t.cpu()
    raw = (C.c_uint8 * n)(*t.tolist())
    check(lib.sfx_comm_init(engine.handle, raw, rank, world), "sfx_comm_init")


def set_host_comm(engine, rank: int, world: int, group=None):
    """Host transport (sfx_set_comm_host): the library stages each all-reduce (sortable int32
    maxima) through pinned host memory and this callback runs all-reduce(MAX) over a gloo group -- for ranks sharing one GPU
    (tests), where RCCL cannot run.  Keeps the callback alive on the engine."""
    import numpy as np
    import torch.distributed as dist

    from ._lib import HOST_ALLREDUCE_FN, check, lib

    def _ar(_ctx, buf, count):
        try:
            a = np.ctypeslib.as_array(buf, shape=(count,))
            t = torch.from_numpy(a)
            if world > 1:
                dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
            return 0
        except Exception:
            return 1

    cb = HOST_ALLREDUCE_FN(_ar)
    engine._host_ar_cb = cb
    check(lib.sfx_set_comm_host(engine.handle, cb, None, rank, world), "sfx_set_comm_host")
