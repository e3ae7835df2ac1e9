"""agents.buffer for the drop-in (SURVEY.md §8b module aliases; VERDICT r3 missing #4): the
reference's ReplayBuffer API (agents/buffer.py:8-82) over a device-resident ring.

The reference keeps an object ring of per-transition device tensors and collates every replay
with ``torch.vstack`` and ``torch.tensor`` -- the latter reads each of the B action tensors back
to the host (B synchronisations per replay).  Here every field lives in one preallocated device
array (allocated at the first ``append`` from the shapes it sees), ``append`` writes its row with
asynchronous device copies (a discount factor given as a Python float -- what the reference's
agents pass -- goes to a host array instead: no launch), and ``replay`` draws the SAME indices the
reference draws (``np.random.randint(low=0, high=size, size=(n_batch,))``, one call on numpy's
global state), hands the indices and the minibatch's discount factors to the device in ONE pinned
copy, and gathers the other fields there, one gather each.  The returned
tensors have the reference's shapes and dtypes: states / φ / next states ``[B, -1]`` float32,
actions ``[B]`` int64, gammas ``[B]`` float32.
"""
from __future__ import annotations

import weakref

import numpy as np
import torch


def release_minibatch(states, stream=None) -> bool:
    """Hand the minibatch whose states tensor is `states` back to the ReplayBuffer that lent it
    (ReplayBuffer.release); False when it did not come from one."""
    tok = getattr(states, "_sfx_slot", None)
    buf = tok[0]() if tok is not None else None
    return buf.release(states, stream) if buf is not None else False


def lending_buffer(states):
    """The ReplayBuffer that lent the minibatch whose states tensor is `states`, or None."""
    tok = getattr(states, "_sfx_slot", None)
    return tok[0]() if tok is not None else None


_L = None


def _libsfx():
    """sfx._lib, imported on first use (a CPU ring never loads libsfx)."""
    global _L
    if _L is None:
        from sfx import _lib

        _L = _lib
    return _L


def _device():
    try:  # the user's utils.torch (the reference's global device)
        from utils.torch import get_torch_device

        return torch.device(get_torch_device())
    except Exception:
        return torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")


class ReplayBuffer:

    def __init__(self, *args, n_samples=1000000, n_batch=32, **kwargs):
        self.n_samples = int(n_samples)
        self.n_batch = int(n_batch)
        self.device = _device()
        self._ring = None
        self._pidx = None
        self._pB = 0
        self._pev = None
        self._outs = []
        self._token = weakref.ref(self)  # identifies this buffer's lendings (ReplayBuffer.release)
        # The reference's agent appends (s, a, φ, s1) right after update_reward(φ, ...) and asks GPI
        # about s1 right after the update (agents/agent.py:238-256, agents/sfdqn.py:47-60): a consumer
        # (sfx's DeepSF) may name device vectors that the write of each appended row also copies s1
        # and φ into (``mirror`` [n_s], ``mirror_reward`` [d]), and reads back which tensors, at which
        # versions, the last write copied there: (weak reference, version at append, mirror).
        self.mirror = self.mirror_reward = None
        self.last_next = self.last_reward = None
        # a native append's row is written by the next replay's launch (sfx_replay_put_gather), or
        # before the next append / an empty replay / reset: (j, state, action, reward, next_state)
        self._pend = None
        self.index = 0
        self.size = 0

    def reset(self):
        """Removes all samples currently stored in the buffer (the ring's memory is kept)."""
        if self._pend is not None:
            self._flush_put()
        self.index = 0
        self.size = 0

    def _alloc(self, state, reward, next_state):
        dev = self.device
        n_s = int(torch.as_tensor(state).numel())
        d = int(torch.as_tensor(reward).numel())
        n_s1 = int(torch.as_tensor(next_state).numel())
        if n_s1 != n_s:  # one state width: the gather reads both state rows with it
            raise ValueError(f"ReplayBuffer: next_state has {n_s1} entries, state {n_s}")
        cap = self.n_samples
        self._ring = (torch.zeros(cap, n_s, device=dev), torch.zeros(cap, dtype=torch.int64, device=dev),
                      torch.zeros(cap, d, device=dev), torch.zeros(cap, n_s1, device=dev))
        self._gam = np.zeros(cap, dtype=np.float32)  # γ per slot, float32 as torch.tensor(list) makes it
        self._gdev = None  # set once a γ arrives as a device tensor: then γ is gathered on the device
        self._ring_dev = self._ring[0].get_device() if self._ring[0].is_cuda else -2
        self._widths = (n_s, d, n_s1)
        self._rp = tuple(x.data_ptr() for x in self._ring)  # rs, ra, rr, rs1
        self._mcache = (None, None, None, None)  # (mirror, mirror_reward, their pointers)

    @staticmethod
    def _put(row, x):
        if torch.is_tensor(x):
            row.copy_(x.reshape(row.shape), non_blocking=True)
        else:
            row.copy_(torch.as_tensor(np.asarray(x, dtype=np.float32)).reshape(row.shape))

    def _dev_index(self) -> int:
        i = self.device.index
        return torch.cuda.current_device() if i is None else i

    def _native(self, state, action, reward, next_state) -> bool:
        """Device tensors of the ring's dtypes, on the ring's device, contiguous: libsfx's one-launch
        row copy applies."""
        dev = self._ring_dev
        f32 = torch.float32
        for x, dt in ((state, f32), (action, torch.int64), (reward, f32), (next_state, f32)):
            if not (type(x) is torch.Tensor and x.is_cuda and x.get_device() == dev and x.dtype is dt
                    and x.is_contiguous()):
                return False
        return True

    def append(self, state, action, reward, next_state, gamma) -> None:
        """Adds the sample (agents/buffer.py:62-82); the oldest is overwritten once the ring is full."""
        if self._ring is None:
            self._alloc(state, reward, next_state)
        if self._pend is not None:
            self._flush_put()
        rs, ra, rr, rs1 = self._ring
        j = self.index
        self.last_next = self.last_reward = None
        if self._native(state, action, reward, next_state) and action.numel() == 1:
            # the kernel reads the ring's widths from each tensor: a shorter one would be read past its end
            if (state.numel(), reward.numel(), next_state.numel()) != self._widths:
                for name, x, w in (("state", state, self._widths[0]), ("reward", reward, self._widths[1]),
                                   ("next_state", next_state, self._widths[0])):
                    if x.numel() != w:
                        raise ValueError(f"ReplayBuffer.append: {name} has {x.numel()} entries, the ring {w}")
            # written by the next replay's launch; like the reference's object ring, the row holds
            # these tensors' values as they are then
            self._pend = (j, state, action, reward, next_state, next_state._version, reward._version)
            self._put_gamma(j, gamma)
            self.size = min(self.size + 1, self.n_samples)
            self.index = (self.index + 1) % self.n_samples
            return
        self._put(rs[j], state)
        if torch.is_tensor(action):
            ra[j].copy_(action.reshape(()), non_blocking=True)
        else:
            ra[j] = int(action)
        self._put(rr[j], reward)
        self._put(rs1[j], next_state)
        self._put_gamma(j, gamma)
        self.size = min(self.size + 1, self.n_samples)
        self.index = (self.index + 1) % self.n_samples

    def _flush_put(self):
        """Write the pending native append's row (one launch)."""
        _lib = _libsfx()
        j, st, ac, rw, ns = self._pend[:5]
        self._pend = None
        rs, ra, rr, rs1 = self._rp
        n_s, d, _ = self._widths
        _lib.check(_lib.lib.sfx_replay_put(_lib.stream_ptr(self._ring_dev), rs, rr, rs1, ra, j, st.data_ptr(),
                                           rw.data_ptr(), ns.data_ptr(), ac.data_ptr(), n_s, d), "sfx_replay_put")

    def _mirror_ptrs(self):
        """Pointers of (mirror, mirror_reward) when they are vectors the kernel may write, else None."""
        c = self._mcache
        if c[0] is not self.mirror or c[1] is not self.mirror_reward:
            def ok(m, n):
                return m.data_ptr() if (type(m) is torch.Tensor and m.is_cuda and m.get_device() == self._ring_dev
                                        and m.numel() == n and m.is_contiguous() and m.dtype is torch.float32) else None
            c = self._mcache = (self.mirror, self.mirror_reward, ok(self.mirror, self._widths[0]),
                                ok(self.mirror_reward, self._widths[1]))
        return c[2], c[3]

    def _put_gamma(self, j, gamma):
        if torch.is_tensor(gamma):
            if self._gdev is None:
                self._gdev = torch.as_tensor(self._gam, device=self.device).clone()
            self._gdev[j].copy_(gamma.reshape(()), non_blocking=True)
        else:
            self._gam[j] = gamma
            if self._gdev is not None:
                self._gdev[j] = float(gamma)

    # pinned index slots: a ring of _RING, guarded per block of _BLOCK slots by one event (recorded
    # after the block's last gather, waited for before the block is rewritten a ring later)
    _RING, _BLOCK = 256, 64
    _OUT = 3  # minibatch output slots reused once nothing outside the buffer holds them

    def replay(self):
        """A uniform minibatch (agents/buffer.py:34-60) or None while fewer than n_batch samples."""
        if self.size < self.n_batch:
            if self._pend is not None:
                self._flush_put()
            return None
        indices = np.random.randint(low=0, high=self.size, size=(self.n_batch,))
        B = self.n_batch
        rs, ra, rr, rs1 = self._ring
        if self.device.type == "cuda":
            return self._replay_dev(indices, B, rs, ra, rr, rs1)
        idx = torch.as_tensor(indices, dtype=torch.int64)
        gam = torch.as_tensor(self._gam[indices]) if self._gdev is None else self._gdev.index_select(0, idx)
        return (rs.index_select(0, idx), ra.index_select(0, idx), rr.index_select(0, idx),
                rs1.index_select(0, idx), gam)

    def _out_slot(self, B, n_s, d):
        """Output tensors for one minibatch: a slot of the buffer's own that its consumer handed back
        (``release``, called by sfx's DeepSF once the update that read the minibatch has settled), else
        a new allocation.  Ownership is never inferred: a minibatch nobody releases -- kept by the
        caller, saved by autograd, held by any other consumer -- is never written again.  Reuse is in
        stream order: the gather that refills a slot is queued after every kernel that read it (a
        consumer on another stream leaves an event the gather's stream waits for)."""
        for k, sl in enumerate(self._outs):
            if sl is not None and sl["free"]:
                sl["free"] = False
                sl["gen"] += 1
                if sl["ev"] is not None:
                    torch.cuda.current_stream(self.device).wait_event(sl["ev"])
                    sl["ev"] = None
                sl["views"][0]._sfx_slot = (self._token, k, sl["gen"])
                return sl["views"], sl["ptrs"]
        # A (int64, as 2B float words) | S | PHI | S1 | G, each contiguous, one allocation
        base = torch.empty(B * (2 * n_s + d + 3), device=self.device)
        a2, S, PHI, S1, G = base.split((2 * B, B * n_s, B * d, B * n_s, B))
        views = (S.view(B, n_s), a2.view(torch.int64), PHI.view(B, d), S1.view(B, n_s), G)
        ptrs = tuple(v.data_ptr() for v in views)
        for k, sl in enumerate(self._outs):
            if sl is None:  # becomes a slot of the buffer's: handed back by its consumer, reused
                self._outs[k] = {"views": views, "ptrs": ptrs, "free": False, "gen": 0, "ev": None}
                views[0]._sfx_slot = (self._token, k, 0)
                break
        return views, ptrs

    def release(self, states, stream=None) -> bool:
        """Hand a minibatch returned by ``replay`` back to the buffer (its states tensor identifies
        it): its device memory may hold a later minibatch from the next ``replay`` on.  Called by the
        minibatch's consumer (sfx's DeepSF) after the update that read it has settled; ``stream`` is
        the consumer's stream (a CUDA stream handle) when it is not the buffer's.  Returns whether
        the tensors were one of the buffer's slots (a second release of the same lending is a no-op)."""
        tok = getattr(states, "_sfx_slot", None)
        if tok is None or tok[0] is not self._token:
            return False
        _, k, gen = tok
        sl = self._outs[k] if self._outs and k < len(self._outs) else None
        if sl is None or sl["free"] or sl["gen"] != gen or sl["views"][0] is not states:
            return False
        if stream is not None and stream != _libsfx().stream_ptr(self._ring_dev):
            with torch.cuda.device(self.device):
                ev = torch.cuda.Event()
                ev.record(torch.cuda.ExternalStream(stream, device=self.device))
            sl["ev"] = ev
        sl["free"] = True
        return True

    def _replay_dev(self, indices, B, rs, ra, rr, rs1):
        """Every field in one gather launch.  The indices and the minibatch's γ go to the kernel in a
        slot of coherent host memory it reads directly (no host->device copy); a block of slots is
        rewritten only after the gathers that read it have completed (its event)."""
        _lib = _libsfx()
        stream = _lib.stream_ptr(self._ring_dev)
        if self._pidx is None or self._pB != B:  # slots of [B indices (int64) | B γ (float32 words)]
            if self._pidx is not None:  # a new batch size: no queued gather may still read the old slots
                torch.cuda.synchronize(self.device)
            w = B + (B + 1) // 2
            with torch.cuda.device(self.device):
                self._pidx = _lib.HostBuffer(self._RING * w)
            self._pB = B
            self._pnp = self._pidx.np.reshape(self._RING, w)
            self._pptr = [self._pidx.ptr + 8 * w * i for i in range(self._RING)]
            self._pev = [None] * (self._RING // self._BLOCK)
            self._pi = 0
            self._pstream = stream
            self._outs = [None] * self._OUT
        if stream != self._pstream:  # gathers on another stream: the events no longer order them
            torch.cuda.synchronize(self.device)
            self._pev = [None] * len(self._pev)
            self._pstream = stream
        i = self._pi
        self._pi = (i + 1) % self._RING
        blk, last = divmod(i, self._BLOCK)
        if last == 0 and self._pev[blk] is not None:
            self._pev[blk].synchronize()
        host = self._pnp[i]
        host[:B] = indices
        host[B:].view(np.float32)[:B] = self._gam[indices]
        n_s, d = self._widths[0], self._widths[1]
        views, (pS, pA, pPHI, pS1, pG) = self._out_slot(B, n_s, d)
        p = self._pptr[i]
        rg = self._gdev.data_ptr() if self._gdev is not None else None
        prs, pra, prr, prs1 = self._rp
        pend = self._pend
        if pend is not None:  # the append before: its row written in the same launch
            self._pend = None
            j, st, ac, rw, ns, nsv, rwv = pend
            mx, mr = self._mirror_ptrs()
            _lib.check(_lib.lib.sfx_replay_put_gather(
                stream, prs, prr, prs1, pra, rg, j, st.data_ptr(), rw.data_ptr(), ns.data_ptr(), ac.data_ptr(), mx, mr,
                p, p + 8 * B, B, pS, pPHI, pS1, pA, pG, n_s, d), "sfx_replay_put_gather")
            if mx is not None:
                self.last_next = (weakref.ref(ns), nsv, self.mirror)
            if mr is not None:
                self.last_reward = (weakref.ref(rw), rwv, self.mirror_reward)
        else:
            _lib.check(_lib.lib.sfx_replay_gather(stream, prs, prr, prs1, pra, rg, p, p + 8 * B, B, pS, pPHI, pS1, pA,
                                                  pG, n_s, d), "sfx_replay_gather")
        if last == self._BLOCK - 1:
            with torch.cuda.device(self.device):  # the gathers' stream, on the buffer's device
                ev = self._pev[blk] = self._pev[blk] or torch.cuda.Event()
                ev.record(torch.cuda.current_stream(self.device))
        S, A, PHI, S1, G = views
        return S, A, PHI, S1, G  # a new tuple: a caller holding it holds each tensor
