"""SFEngine: a device-resident library of T ψ heads driven through libsfx.so.

One engine = one libsfx handle = the heads, target heads, Adam state and reward weights
of T source tasks on one GPU.  Inputs are torch tensors (moved to the engine's device
when needed); outputs are torch tensors on the device.  Every compute call runs the
hand-written gfx950 kernels; there is no torch / CPU fallback.
"""
from __future__ import annotations

import ctypes as C
from typing import Optional, Sequence, Tuple

import numpy as np
import torch

from ._lib import check, dptr, fptr, lib, stream_ptr

ACT_CODES = {"none": 0, "relu": 1, "tanh": 2}


def _act_code(a) -> int:
    if isinstance(a, int):
        return a
    return ACT_CODES[str(a).lower()]


def _dev_f32(t: torch.Tensor, device) -> int:
    """Pointer of a tensor the library updates in place: float32, contiguous, on the engine's device."""
    if not (torch.is_tensor(t) and t.dtype == torch.float32 and t.is_contiguous() and t.device == torch.device(device)):
        raise ValueError("expected a contiguous float32 tensor on the engine's device")
    return t.data_ptr()


class SFEngine:
    def __init__(self, T: int, n_s: int, H: int, A: int, d: int, acts: Sequence = ("relu", "relu"),
                 max_batch: int = 32, device=None, stream: Optional[int] = None):
        if not torch.cuda.is_available():
            raise RuntimeError("SFEngine needs a HIP device (libsfx.so has no CPU path)")
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        if self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.T, self.n_s, self.H, self.A, self.d = T, n_s, H, A, d
        self.acts = tuple(acts)
        self.max_batch = max_batch
        if stream is None:
            stream = torch.cuda.current_stream(self.device).cuda_stream
        self.stream = stream
        codes = (C.c_int * max(1, len(self.acts)))(*[_act_code(a) for a in self.acts])
        h = C.c_void_p()
        check(lib.sfx_create(C.byref(h), T, n_s, H, len(self.acts), codes, A, d, max_batch,
                             self.device.index, C.c_void_p(stream)), "sfx_create")
        self._h = h
        self.P = lib.sfx_head_numel(h)
        self._sel = torch.zeros(2, dtype=torch.long, device=self.device)
        self.T_glob, self.head_offset = T, 0
        self._refresh_w_ptrs(T)
        # the library's Adam defaults (sfx_set_adam replaces them); kept for checkpoints
        self.adam_hp = dict(lr_psi=1e-3, wd_psi=0.0, lr_w=1e-3, wd_w=0.0, betas=(0.9, 0.999), eps=1e-8)

    def shard_setup(self, T_glob: int, head_offset: int):
        """This engine's T heads become the global heads [head_offset, head_offset + T) of T_glob;
        w gets T_glob rows (the rows loaded so far move to their global index)."""
        check(lib.sfx_shard_setup(self._h, int(T_glob), int(head_offset)), "sfx_shard_setup")
        self.T_glob, self.head_offset = int(T_glob), int(head_offset)
        self._refresh_w_ptrs(self.T_glob)

    def _refresh_w_ptrs(self, Tw: int):
        """Device pointers of the w rows (Tw = T, or T_glob after sfx_shard_setup)."""
        self._w_ptrs = []
        for t in range(Tw):
            p = C.c_void_p()
            check(lib.sfx_w_ptr(self._h, t, C.byref(p)), "sfx_w_ptr")
            self._w_ptrs.append(p.value)

    # ---------------------------------------------------------------- lifecycle
    def close(self):
        if getattr(self, "_h", None):
            lib.sfx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    # ---------------------------------------------------------------- helpers
    # Host inputs (numpy / CPU tensors, as the reference's agents pass them) reach the device
    # through a ring of pinned staging slots: all host arguments of one call are packed into one
    # slot (16-byte aligned) and go over in ONE non-blocking copy on torch's current stream,
    # instead of a synchronous pageable copy per argument; a slot is reused only after its copy's
    # event has completed.
    _PIN_SLOTS, _PIN_BYTES = 32, 1 << 16

    _NP = {torch.float32: np.float32, torch.long: np.int64}

    def _pin_slot(self):
        """The next staging slot (numpy view of pinned memory), once its last copy has completed."""
        if not hasattr(self, "_pin"):
            self._pin = torch.empty(self._PIN_SLOTS, self._PIN_BYTES, dtype=torch.uint8, pin_memory=True)
            self._pin_np = self._pin.numpy()
            self._pin_ev = [None] * self._PIN_SLOTS
            self._pin_i = 0
        i = self._pin_i
        self._pin_i = (i + 1) % self._PIN_SLOTS
        ev = self._pin_ev[i]
        if ev is not None:
            ev.synchronize()
        return i

    def _on_stream(self):
        """Context that makes the handle's stream torch's current one: the staging buffers are
        allocated, copied into and recorded on the stream the library's kernels read them on (the
        caching allocator then reuses a freed block only in that stream's order)."""
        import contextlib

        if self.stream == stream_ptr(self.device.index):
            return contextlib.nullcontext()
        st = getattr(self, "_xstream", None)
        if st is None:
            st = self._xstream = torch.cuda.ExternalStream(self.stream, device=self.device)
        return torch.cuda.stream(st)

    def _settle_pending(self):
        check(lib.sfx_settle(self._h, None, None), "sfx_settle")

    def _site_buf(self, site, nbytes) -> torch.Tensor:
        """The device staging buffer of one call site: the same memory every call, so the call's
        captured graph is found again instead of captured anew (a fresh buffer per call would give
        every call a new graph key).  Reuse is in stream order: the next copy into it is queued
        after every kernel that read it."""
        bufs = self.__dict__.setdefault("_sites", {})
        b = bufs.get(site)
        if b is None or b.numel() < nbytes:
            b = bufs[site] = torch.empty(max(nbytes, 256), dtype=torch.uint8, device=self.device)
        return b[:nbytes]

    def _pin_copy(self, i, nbytes, site=None) -> torch.Tensor:
        """One non-blocking copy of slot i's first nbytes into device memory -- a fresh buffer, or
        the call site's own (`site`) -- on the handle's stream."""
        with self._on_stream():
            out = torch.empty(nbytes, dtype=torch.uint8, device=self.device) if site is None else \
                self._site_buf(site, nbytes)
            out.copy_(self._pin[i, :nbytes], non_blocking=True)
            ev = self._pin_ev[i] = self._pin_ev[i] or torch.cuda.Event()
            ev.record()
        return out

    @staticmethod
    def _host_array(x, npdt):
        if torch.is_tensor(x):
            x = x.detach()
            if x.device.type != "cpu":
                return None
            x = x.numpy()
        return np.asarray(x, dtype=npdt)

    def _h2d(self, x, dtype, site=None) -> torch.Tensor:
        return self._h2d_many([(x, dtype)], site)[0]

    def _h2d_many(self, items, site=None, settle=False):
        """Host inputs [(x, dtype)] -> device tensors of their shapes, staged together through ONE
        pinned slot and ONE non-blocking copy (a step's s, a, φ, s1, γ are one copy, not five).
        Device tensors are converted in place of staging.  site: the device buffer of that call
        site (the views returned are valid until the site's next call); settle: collect a pending
        step first (its host rounds read the inputs it was given, possibly this site's)."""
        arrs = [self._host_array(x, self._NP[dt]) for x, dt in items]
        offs, tot = [], 0
        for a in arrs:
            offs.append(tot)
            if a is not None:
                tot += (a.nbytes + 15) & ~15
        if tot > self._PIN_BYTES or any(a is not None and a.nbytes == 0 for a in arrs):
            return [torch.as_tensor(x).to(device=self.device, dtype=dt) for x, dt in items]
        dev = None
        if tot:
            i = self._pin_slot()
            row = self._pin_np[i]
            for a, o in zip(arrs, offs):
                if a is not None:
                    row[o:o + a.nbytes].view(a.dtype)[:] = a.reshape(-1)
            if settle:  # a pending step's host rounds may still read the site's last inputs
                self._settle_pending()
            dev = self._pin_copy(i, tot, site)
        out = []
        for (x, dt), a, o in zip(items, arrs, offs):
            if a is None:
                out.append(torch.as_tensor(x).to(device=self.device, dtype=dt))
            else:
                out.append(dev[o:o + a.nbytes].view(dt).view(a.shape))
        return out

    def _on_dev(self, x, dt) -> bool:
        """x is already what a kernel reads: a contiguous `dt` tensor on the engine's device (the
        drop-in's agents pass device tensors: no conversion, no copy, no framework call)."""
        return (type(x) is torch.Tensor and x.is_cuda and x.dtype is dt and x.get_device() == self.device.index
                and x.is_contiguous())

    def _f(self, x, shape=None, site=None) -> torch.Tensor:
        if self._on_dev(x, torch.float32):
            return x if shape is None else x.view(shape)
        t = self._h2d(x, torch.float32, site)
        if shape is not None:
            t = t.reshape(shape)
        return t.contiguous()

    def _l(self, x) -> torch.Tensor:
        return self._h2d(x, torch.long).reshape(-1).contiguous()

    def _batch_in(self, s, s1, a, phi, gamma, r=None):
        """A minibatch's device inputs (s, s1 [B, n_s], a [B] int64, φ [B, d], γ [B], r [B] or None),
        one staged copy for all of them."""
        f32 = torch.float32
        if (self._on_dev(s, f32) and self._on_dev(s1, f32) and self._on_dev(a, torch.long)
                and self._on_dev(phi, f32) and self._on_dev(gamma, f32) and s.dim() == 2
                and (r is None or self._on_dev(r, f32))):
            B = s.shape[0]  # device tensors as the kernels read them: only their sizes are checked
            if (s.shape[1] == self.n_s and s1.shape == s.shape and a.numel() == B and phi.numel() == B * self.d
                    and gamma.numel() == B and (r is None or r.numel() == B)):
                return [s, s1, a, phi, gamma, r]
        items = [(s, torch.float32), (s1, torch.float32), (a, torch.long), (phi, torch.float32),
                 (gamma, torch.float32)] + ([] if r is None else [(r, torch.float32)])
        t = self._h2d_many(items, "batch", settle=True)
        B = t[0].shape[0]
        out = [t[0].contiguous(), t[1].contiguous(), t[2].reshape(-1).contiguous(),
               t[3].reshape(B, self.d).contiguous(), t[4].reshape(B).contiguous()]
        return out + [None if r is None else t[5].reshape(B).contiguous()]

    # ---------------------------------------------------------------- configuration
    def set_adam(self, lr_psi=1e-3, wd_psi=0.0, lr_w=1e-3, wd_w=0.0, betas=(0.9, 0.999), eps=1e-8):
        check(lib.sfx_set_adam(self._h, float(lr_psi), float(wd_psi), float(lr_w), float(wd_w),
                               float(betas[0]), float(betas[1]), float(eps)), "sfx_set_adam")
        self.adam_hp = dict(lr_psi=float(lr_psi), wd_psi=float(wd_psi), lr_w=float(lr_w), wd_w=float(wd_w),
                            betas=(float(betas[0]), float(betas[1])), eps=float(eps))

    def set_graphs(self, enable: bool):
        check(lib.sfx_set_graphs(self._h, int(bool(enable))), "sfx_set_graphs")

    def set_target_update_ev(self, ev: int):
        check(lib.sfx_set_target_update_ev(self._h, int(ev)), "sfx_set_target_update_ev")

    # ---------------------------------------------------------------- state I/O (host, synchronous)
    def load_head(self, t: int, flat, which: int = 0):
        a = np.ascontiguousarray(torch.as_tensor(flat).detach().cpu().reshape(-1).numpy(), dtype=np.float32)
        if a.size != self.P:
            raise ValueError(f"head has {a.size} parameters, engine expects {self.P}")
        check(lib.sfx_load_head(self._h, t, which, fptr(a)), "sfx_load_head")

    def get_head(self, t: int, which: int = 0) -> torch.Tensor:
        a = np.empty(self.P, dtype=np.float32)
        check(lib.sfx_get_head(self._h, t, which, fptr(a)), "sfx_get_head")
        return torch.from_numpy(a)

    def load_adam(self, t: int, m, v, step: int):
        m = np.ascontiguousarray(torch.as_tensor(m).cpu().reshape(-1).numpy(), dtype=np.float32)
        v = np.ascontiguousarray(torch.as_tensor(v).cpu().reshape(-1).numpy(), dtype=np.float32)
        check(lib.sfx_load_adam(self._h, t, fptr(m), fptr(v), int(step)), "sfx_load_adam")

    def get_adam(self, t: int) -> Tuple[torch.Tensor, torch.Tensor, int]:
        m = np.empty(self.P, dtype=np.float32)
        v = np.empty(self.P, dtype=np.float32)
        st = C.c_int()
        check(lib.sfx_get_adam(self._h, t, fptr(m), fptr(v), C.byref(st)), "sfx_get_adam")
        return torch.from_numpy(m), torch.from_numpy(v), st.value

    def load_w(self, t: int, w):
        a = np.ascontiguousarray(torch.as_tensor(w).detach().cpu().reshape(-1).numpy(), dtype=np.float32)
        if a.size != self.d:
            raise ValueError("w must have d entries")
        check(lib.sfx_load_w(self._h, t, fptr(a)), "sfx_load_w")

    def load_w_state(self, t: int, w, wm, wv):
        """w_t with its Adam moments (the sfdqn.py l2 path's w optimizer state)."""
        a = [np.ascontiguousarray(torch.as_tensor(x).detach().cpu().reshape(-1).numpy(), dtype=np.float32)
             for x in (w, wm, wv)]
        if any(x.size != self.d for x in a):
            raise ValueError("w and its moments must have d entries")
        check(lib.sfx_load_w_state(self._h, t, fptr(a[0]), fptr(a[1]), fptr(a[2])), "sfx_load_w_state")

    def get_w(self, t: int):
        w, m, v = (np.empty(self.d, dtype=np.float32) for _ in range(3))
        check(lib.sfx_get_w(self._h, t, fptr(w), fptr(m), fptr(v)), "sfx_get_w")
        return torch.from_numpy(w), torch.from_numpy(m), torch.from_numpy(v)

    def since_target(self, t: int) -> int:
        c = C.c_int()
        check(lib.sfx_get_since_target(self._h, t, C.byref(c)), "sfx_get_since_target")
        return c.value

    def set_since_target(self, t: int, count: int):
        check(lib.sfx_set_since_target(self._h, t, int(count)), "sfx_set_since_target")

    def sync_target(self, t: int):
        check(lib.sfx_sync_target(self._h, t), "sfx_sync_target")

    KINDS = {"fwd": 0, "tdg": 1, "bwd": 2, "gpi": 3, "lms": 4, "ver": 5, "tsf": 6}

    def prof_enable(self, on: bool):
        check(lib.sfx_prof_enable(self._h, int(bool(on))), "sfx_prof_enable")

    def prof_reset(self):
        check(lib.sfx_prof_reset(self._h), "sfx_prof_reset")

    def prof_collect(self):
        """{kind: (launches, total_us, algorithmic_bytes)} of the instrumented launches."""
        out = {}
        for name, k in self.KINDS.items():
            n, us, by = C.c_int(), C.c_double(), C.c_double()
            check(lib.sfx_prof_collect(self._h, k, C.byref(n), C.byref(us), C.byref(by)), "sfx_prof_collect")
            out[name] = (n.value, us.value, by.value)
        return out

    def synchronize(self):
        check(lib.sfx_synchronize(self._h), "sfx_synchronize")

    # ---------------------------------------------------------------- hot path
    def gpi(self, S, w=None, w_index: Optional[int] = None, want_psi: bool = False, want_q: bool = True,
            task_shape=None):
        """GPI over all heads.  Returns (psi [B,T,A,d] or None, q [B,T,A] or None, task [B], next [B]);
        task_shape: the task tensor's shape instead of [B] (B elements, e.g. () for one state)."""
        S = self._f(S, site="gpi_s")
        if S.dim() == 1:
            S = S.reshape(1, -1)
        B = S.shape[0]
        if w_index is not None:
            w_ptr = self._w_ptrs[w_index]
            w_keep = None
        else:
            w_keep = self._f(w, (-1,), site="gpi_w")
            w_ptr = w_keep.data_ptr()
        psi = torch.empty(B, self.T, self.A, self.d, device=self.device) if want_psi else None
        q = torch.empty(B, self.T, self.A, device=self.device) if want_q else None
        task = torch.empty(B if task_shape is None else task_shape, dtype=torch.long, device=self.device)
        if task.numel() != B:
            raise ValueError(f"task_shape {task_shape} does not hold {B} elements")
        nxt = torch.empty(B, dtype=torch.long, device=self.device)
        check(lib.sfx_gpi(self._h, S.data_ptr(), B, w_ptr, dptr(psi), dptr(q), task.data_ptr(),
                          nxt.data_ptr()), "sfx_gpi")
        return psi, q, task, nxt

    def successors(self, S, which: int = 0) -> torch.Tensor:
        """get_successors (which=0, online heads) / get_next_successors (which=1, target heads):
        [B, T, A, d]."""
        S = self._f(S, site="succ_s")
        if S.dim() == 1:
            S = S.reshape(1, -1)
        psi = torch.empty(S.shape[0], self.T, self.A, self.d, device=self.device)
        check(lib.sfx_successors(self._h, S.data_ptr(), S.shape[0], int(which), psi.data_ptr()), "sfx_successors")
        return psi

    def select_action(self, s, task_index: int, use_gpi: bool = True, q_out: Optional[torch.Tensor] = None):
        """Greedy GPI action for one state; returns the device tensor [c, a] (not synchronized)."""
        s = self._f(s, (-1,), site="sel_s")
        check(lib.sfx_select_action(self._h, s.data_ptr(), int(task_index), int(bool(use_gpi)), dptr(q_out),
                                    self._sel.data_ptr()), "sfx_select_action")
        return self._sel

    def test_actions(self, S, W, q_out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Greedy GPI actions of E test tasks in one launch set, row e under its own reward
        weights W[e] (agents/sfdqn.py:125-137 for every test task of a lockstep step).  Returns
        the device tensor [E, 2] of (c, a) (not synchronized)."""
        S = self._f(S)
        if S.dim() == 1:
            S = S.reshape(1, -1)
        E = S.shape[0]
        W = self._f(W).reshape(E, -1)
        if W.shape[1] != self.d:
            raise ValueError(f"W must be [{E}, {self.d}]")
        if q_out is not None:
            _dev_f32(q_out, self.device)
        out = torch.empty(E, 2, dtype=torch.long, device=self.device)
        check(lib.sfx_test_actions(self._h, S.data_ptr(), E, W.data_ptr(), W.stride(0), dptr(q_out),
                                   out.data_ptr()), "sfx_test_actions")
        return out

    def test_reward_updates(self, phi, r, W: torch.Tensor, lr: float = 0.005, wd: float = 0.01,
                            losses: Optional[torch.Tensor] = None) -> torch.Tensor:
        """SFDQN.update_test_reward_mapper (agents/sfdqn.py:168-184) of E test tasks in one launch:
        a fresh SGD(lr, weight_decay=wd) step on each row of W [E, d] (float32 device tensor with
        unit column stride, updated in place) against MSE(W[e]·phi[e], r[e]).  Returns the E
        pre-step losses (device tensor, not synchronized)."""
        E = W.shape[0]
        if W.dim() != 2 or W.shape[1] != self.d or W.stride(1) != 1 or W.dtype != torch.float32 \
                or W.device != self.device:
            raise ValueError(f"W must be a float32 [{E}, {self.d}] device tensor with unit column stride")
        phi, r = self._h2d_many([(phi, torch.float32), (r, torch.float32)])
        phi, r = phi.reshape(E, self.d).contiguous(), r.reshape(E).contiguous()
        losses = torch.empty(E, device=self.device) if losses is None else losses
        _dev_f32(losses, self.device)
        if losses.numel() != E:
            raise ValueError(f"losses must hold {E} floats")
        check(lib.sfx_test_reward_updates(self._h, E, phi.data_ptr(), r.data_ptr(), W.data_ptr(), W.stride(0),
                                          float(lr), float(wd), losses.data_ptr()), "sfx_test_reward_updates")
        return losses

    def update(self, policy: int, s, a, r, phi, s1, gamma, use_gpi: bool = True,
               losses: Optional[torch.Tensor] = None, next_actions: Optional[torch.Tensor] = None):
        """One TD update of head `policy` (sfdqn.py:303-371 semantics).  r=None -> no l2 / w step."""
        s, s1, a, phi, gamma, rr = self._batch_in(s, s1, a, phi, gamma, r)
        B = s.shape[0]
        if losses is None:
            losses = torch.empty(3, device=self.device)
        check(lib.sfx_update(self._h, int(policy), s.data_ptr(), a.data_ptr(), dptr(rr), phi.data_ptr(),
                             s1.data_ptr(), gamma.data_ptr(), B, int(bool(use_gpi)), losses.data_ptr(),
                             dptr(next_actions)), "sfx_update")
        return losses

    def update_all(self, s, a, phi, s1, gamma, losses: Optional[torch.Tensor] = None):
        """All-task update (agents/sfdqn.py:57-60 over features/deep.py:93-131)."""
        s, s1, a, phi, gamma, _ = self._batch_in(s, s1, a, phi, gamma)
        B = s.shape[0]
        if losses is None:
            losses = torch.empty(self.T, 3, device=self.device)
        check(lib.sfx_update_all(self._h, s.data_ptr(), a.data_ptr(), phi.data_ptr(), s1.data_ptr(),
                                 gamma.data_ptr(), B, losses.data_ptr()), "sfx_update_all")
        # sfx_update_all returns with the step's verdict pending: host rounds, if the device rounds
        # leave a policy unverified, run inside the NEXT library call (settle) and read these inputs
        # and write these losses -- keep them alive until then (replaced after the next update_all,
        # whose own call has settled this step)
        self._lazy_keep = (s, s1, a, phi, gamma, losses)
        return losses

    def _select_slots(self):
        """Persistent device inputs of the fused step (fixed pointers, so the step's graph is
        captured once per minibatch slot): ``sel_state`` [n_s], the selection's state, and
        ``lms_phi`` [d], the LMS features (filled by the caller -- the drop-in's buffer copies each
        appended next state and φ into them, sfx_replay_put_gather)."""
        if getattr(self, "sel_state", None) is None:
            TA = self.T * self.A
            self._sel_ta = TA + (TA & 1)
            self.sel_state = torch.zeros(self.n_s, device=self.device)
            self.lms_phi = torch.zeros(self.d, device=self.device)
            self._sel_ptrs = (self.sel_state.data_ptr(), self.lms_phi.data_ptr())
        return self.sel_state, self.lms_phi

    _mb_ok = None
    sel_state = None

    def update_all_select(self, s, a, phi, s1, gamma, task_index: int, s_next=None,
                          losses: Optional[torch.Tensor] = None, lms_task: int = -1, lms_r=0.0,
                          lms_alpha: float = 0.0):
        """[LMS of w[lms_task] on (``lms_phi``, lms_r: a value, or a float32 device scalar read by
        the step)], update_all, then the GPI of one next state
        with w[task_index], fused into one launch set (sfx_update_all_select).  s_next: a float32
        device tensor of n_s values, or None for ``sel_state`` (filled by the caller).  Returns
        fresh device tensors (q [1, T, A], task []) that the step's selection writes -- what
        lms + update_all + gpi(s_next, w_index=task_index) would return, bit for bit -- complete in
        stream order once the step is settled (``settle_select``, or any later call)."""
        self._select_slots()
        xp, php = self._sel_ptrs
        if s_next is not None:
            if not (self._on_dev(s_next, torch.float32) and s_next.numel() == self.n_s):
                raise ValueError("update_all_select: s_next must be a contiguous float32 device tensor of n_s values")
            xp = s_next.data_ptr()
            self._lazy_keep = s_next  # read again by host rounds
        ok = self._mb_ok  # the last minibatch checked (the drop-in's buffer lends the same few slots)
        if ok is not None and s is ok[0] and a is ok[1] and phi is ok[2] and s1 is ok[3] and gamma is ok[4] \
                and losses is ok[5]:
            ptrs = ok[6]
        else:
            s, s1, a, phi, gamma, _ = self._batch_in(s, s1, a, phi, gamma)
            if losses is None:
                losses = torch.empty(self.T, 3, device=self.device)
            ptrs = (s.data_ptr(), a.data_ptr(), phi.data_ptr(), s1.data_ptr(), gamma.data_ptr(), s.shape[0],
                    losses.data_ptr())
            self._mb_ok = (s, a, phi, s1, gamma, losses, ptrs)
        # q [T*A] then the task (int64, 8-byte aligned) in one fresh allocation; the step's graph
        # reads the two output pointers from host words each launch, so it is captured once
        out = torch.empty(self._sel_ta + 2, device=self.device)
        op = out.data_ptr()
        if type(lms_r) is torch.Tensor:
            if not (self._on_dev(lms_r, torch.float32) and lms_r.numel() == 1):
                raise ValueError("update_all_select: a tensor reward must be one float32 on the engine's device")
            self._lazy_keep_r = lms_r  # read by the step's first launch
            rv, rdev = 0.0, lms_r.data_ptr()
        else:
            rv, rdev = float(lms_r), None
        check(lib.sfx_update_all_select(self._h, *ptrs, xp, int(task_index), op, op + 4 * self._sel_ta,
                                        int(lms_task), php, rv, rdev, float(lms_alpha)), "sfx_update_all_select")
        TA = self.T * self.A
        return out[:TA].view(1, self.T, self.A), out[self._sel_ta:self._sel_ta + 2].view(torch.int64).view(())

    def settle_select(self, q, task):
        """Collect the pending step's verdict (sfx_settle); (q, task) of update_all_select hold the
        selection then (host rounds, if any, rewrote them in place).  Returns (q, task, c): c the
        task index as the host read it from the step (-1 when no step with a selection was pending)."""
        sel = (C.c_int64 * 2)()
        check(lib.sfx_settle(self._h, None, sel), "sfx_settle")
        return q, task, int(sel[0])

    def settle(self) -> int:
        """sfx_settle: collect the verdict of a pending update_all / update_all_select; returns the
        rounds that ran on the host."""
        n = C.c_int()
        check(lib.sfx_settle(self._h, C.byref(n), None), "sfx_settle")
        return n.value

    def step_all(self, s=None, a=None, phi=None, s1=None, gamma=None, *, use_gpi: bool = True, lms_task: int = -1,
                 lms_phi=None, lms_r=None, lms_alpha: float = 0.0, s_next=None, task_index: int = 0,
                 sel_use_gpi: bool = True, losses: Optional[torch.Tensor] = None):
        """Launch one fused all-task env step (see include/sfx.h: sfx_step_all).  Device tensors
        must already be float32 / int64 and contiguous (no conversion on this hot path)."""
        B = 0 if s is None else s.shape[0]
        check(lib.sfx_step_all(self._h, dptr(s), dptr(a), dptr(phi), dptr(s1), dptr(gamma), B, int(bool(use_gpi)),
                               int(lms_task), dptr(lms_phi), dptr(lms_r), float(lms_alpha), dptr(s_next),
                               int(task_index), int(bool(sel_use_gpi)), dptr(losses)), "sfx_step_all")

    def step_finish(self):
        """Complete the fused step: returns (GPI task c, greedy action, first re-run policy)."""
        out = (C.c_int64 * 3)()
        check(lib.sfx_step_finish(self._h, out), "sfx_step_finish")
        return int(out[0]), int(out[1]), int(out[2])

    def comm_state(self) -> dict:
        """sfx_comm_state: which communicators the handle holds (RCCL step / host-round split),
        whether they were aborted after a timed-out collective, or the host transport."""
        v = C.c_int()
        check(lib.sfx_comm_state(self._h, C.byref(v)), "sfx_comm_state")
        return dict(rccl=bool(v.value & 1), rounds_split=bool(v.value & 2), aborted=bool(v.value & 4),
                    host=bool(v.value & 8))

    def comm_size(self) -> dict:
        """sfx_comm_size: rank / world the handle was given and what its RCCL communicator reports
        (ncclCommUserRank / ncclCommCount; -1 / 0 without one)."""
        v = [C.c_int() for _ in range(4)]
        check(lib.sfx_comm_size(self._h, *[C.byref(x) for x in v]), "sfx_comm_size")
        return dict(rank=v[0].value, world=v[1].value, rccl_rank=v[2].value, rccl_world=v[3].value)

    def debug_stall(self, seconds: float):
        """Test hook (sfx_debug_stall): the next sharded runner step stalls on the device before it
        publishes its result."""
        check(lib.sfx_debug_stall(self._h, float(seconds)), "sfx_debug_stall")

    def debug_force_rerun(self, first_policy: int):
        check(lib.sfx_debug_force_rerun(self._h, int(first_policy)), "sfx_debug_force_rerun")

    def set_spec_rounds(self, rounds: int):
        check(lib.sfx_set_spec_rounds(self._h, int(rounds)), "sfx_set_spec_rounds")

    def step_stats(self):
        s, f, r, n = C.c_longlong(), C.c_longlong(), C.c_longlong(), C.c_longlong()
        check(lib.sfx_step_stats(self._h, C.byref(s), C.byref(f), C.byref(r), C.byref(n)), "sfx_step_stats")
        return {"steps": s.value, "host_round_steps": f.value, "unverified_policies": r.value, "rounds": n.value}

    def graph_stats(self):
        """sfx_graph_stats: graphs captured, graph launches, graphs cached on the handle."""
        v = [C.c_longlong() for _ in range(3)]
        check(lib.sfx_graph_stats(self._h, *[C.byref(x) for x in v]), "sfx_graph_stats")
        return {"captures": v[0].value, "launches": v[1].value, "cached": v[2].value}

    def nonfinite(self, reset: bool = False) -> bool:
        """SURVEY §5 failure detection: whether any TD error since the last reset was NaN / Inf."""
        v = C.c_int()
        check(lib.sfx_nonfinite(self._h, C.byref(v), int(bool(reset))), "sfx_nonfinite")
        return bool(v.value)

    PRECISIONS = {"fp32": 0, "bf16": 1}

    def set_precision(self, precision: str):
        """'fp32' (default: the reference's arithmetic, every parity test) or 'bf16' (bf16 MFMA
        operands for the forward / dX GEMMs from bf16 copies of the parameters; fp32 master
        weights, moments, gradients of W, TD targets and GPI)."""
        check(lib.sfx_set_precision(self._h, self.PRECISIONS[precision]), "sfx_set_precision")

    @property
    def precision(self) -> str:
        p = lib.sfx_get_precision(self._h)
        return {v: k for k, v in self.PRECISIONS.items()}[p]

    def set_huber(self, delta: float):
        """The ψ loss: 0 (default) = MSELoss (the reference's); delta > 0 = opt-in
        HuberLoss(delta) (sfx_set_huber)."""
        check(lib.sfx_set_huber(self._h, float(delta)), "sfx_set_huber")

    @property
    def huber(self) -> float:
        return float(lib.sfx_get_huber(self._h))

    def skip_stats(self, reset: bool = False):
        """Policies checked / skipped in speculative rounds r >= 1 (their next actions repeated
        round r-1's, so their update would have too)."""
        c, s = C.c_longlong(), C.c_longlong()
        check(lib.sfx_skip_stats(self._h, C.byref(c), C.byref(s), int(reset)), "sfx_skip_stats")
        return {"policies_checked": c.value, "policies_skipped": s.value}

    def lms(self, t: int, phi, r, alpha: float):
        if self._on_dev(phi, torch.float32) and phi.numel() == self.d and isinstance(r, (float, int)):
            # a device φ and a host reward (the reference agents' call): r as a kernel argument
            check(lib.sfx_lms_value(self._h, int(t), phi.data_ptr(), float(r), float(alpha)), "sfx_lms_value")
            return
        phi, r = self._h2d_many([(phi, torch.float32), (r, torch.float32)], "lms")  # host values: one copy
        phi, r = phi.reshape(-1).contiguous(), r.reshape(1).contiguous()
        check(lib.sfx_lms(self._h, int(t), phi.data_ptr(), r.data_ptr(), float(alpha)), "sfx_lms")

    # ---------------------------------------------------------------- TSF-DQN (tsfdqn.py / tsfdqn_nf.py)
    def tsf_freeze_flows(self, freeze: bool = True):
        """sfx_tsf_freeze_flows: hold the planar flows fixed (the Linear of g_i and h still train)."""
        check(lib.sfx_tsf_freeze_flows(self._h, int(bool(freeze))), "sfx_tsf_freeze_flows")
        self.tsf_frozen = bool(freeze)

    def tsf_setup(self, G: int, K: int = 0, beta: float = 1.0, lr_g: float = 1e-3, wd_g: float = 0.0,
                  lr_h: float = 1e-3, wd_h: float = 0.0):
        """Transformed features: g_i = K planar flows + Linear(n_s, G) per task, h = Linear(G, d) shared."""
        check(lib.sfx_tsf_setup(self._h, int(G), int(K), float(beta), float(lr_g), float(wd_g), float(lr_h),
                                float(wd_h)), "sfx_tsf_setup")
        self.tsf_G, self.tsf_K = G, K
        self.tsf_hp = dict(beta=float(beta), lr_g=float(lr_g), wd_g=float(wd_g), lr_h=float(lr_h), wd_h=float(wd_h))
        self.tsf_frozen = False
        self.tsf_Pg = K * (2 * self.n_s + 1) + G * self.n_s + G
        self.tsf_Ph = self.d * G + self.d

    def tsf_load_g(self, t: int, g):
        a = np.ascontiguousarray(torch.as_tensor(g).detach().cpu().reshape(-1).numpy(), dtype=np.float32)
        if a.size != self.tsf_Pg:
            raise ValueError(f"g has {a.size} parameters, expected {self.tsf_Pg}")
        check(lib.sfx_tsf_load_g(self._h, t, fptr(a)), "sfx_tsf_load_g")

    def tsf_get_g(self, t: int):
        g, m, v = (np.empty(self.tsf_Pg, dtype=np.float32) for _ in range(3))
        check(lib.sfx_tsf_get_g(self._h, t, fptr(g), fptr(m), fptr(v)), "sfx_tsf_get_g")
        return torch.from_numpy(g), torch.from_numpy(m), torch.from_numpy(v)

    def tsf_load_g_state(self, t: int, g, gm, gv):
        """g_t with its Adam moments (checkpoint resume)."""
        a = [np.ascontiguousarray(torch.as_tensor(x).detach().cpu().reshape(-1).numpy(), dtype=np.float32)
             for x in (g, gm, gv)]
        if any(x.size != self.tsf_Pg for x in a):
            raise ValueError(f"g and its moments must have {self.tsf_Pg} entries")
        check(lib.sfx_tsf_load_g_state(self._h, t, fptr(a[0]), fptr(a[1]), fptr(a[2])), "sfx_tsf_load_g_state")

    def tsf_get_h_state(self, t: int):
        """Task t's Adam moments of the shared h."""
        m, v = (np.empty(self.tsf_Ph, dtype=np.float32) for _ in range(2))
        check(lib.sfx_tsf_get_h_state(self._h, t, fptr(m), fptr(v)), "sfx_tsf_get_h_state")
        return torch.from_numpy(m), torch.from_numpy(v)

    def tsf_load_h_state(self, t: int, hm, hv):
        a = [np.ascontiguousarray(torch.as_tensor(x).detach().cpu().reshape(-1).numpy(), dtype=np.float32)
             for x in (hm, hv)]
        if any(x.size != self.tsf_Ph for x in a):
            raise ValueError(f"h moments must have {self.tsf_Ph} entries")
        check(lib.sfx_tsf_load_h_state(self._h, t, fptr(a[0]), fptr(a[1])), "sfx_tsf_load_h_state")

    def tsf_load_h(self, h):
        a = np.ascontiguousarray(torch.as_tensor(h).detach().cpu().reshape(-1).numpy(), dtype=np.float32)
        if a.size != self.tsf_Ph:
            raise ValueError(f"h has {a.size} parameters, expected {self.tsf_Ph}")
        check(lib.sfx_tsf_load_h(self._h, fptr(a)), "sfx_tsf_load_h")

    def tsf_get_h(self):
        a = np.empty(self.tsf_Ph, dtype=np.float32)
        check(lib.sfx_tsf_get_h(self._h, fptr(a)), "sfx_tsf_get_h")
        return torch.from_numpy(a)

    # ---------------------------------------------------------------- learned φ
    def phi_setup(self, width_mul: int = 2, n_mid: int = 3, lr: float = 1e-3):
        """features/deep_phi.py's learned φ (main_sfdqn_phi_torch.py phi_model_lambda shape)."""
        check(lib.sfx_phi_setup(self._h, int(width_mul), int(n_mid), float(lr)), "sfx_phi_setup")
        self.phi_numel = lib.sfx_phi_numel(self._h)
        self.phi_cfg = dict(width_mul=int(width_mul), n_mid=int(n_mid), lr=float(lr))

    def phi_load(self, params):
        a = np.ascontiguousarray(torch.as_tensor(params).detach().cpu().reshape(-1).numpy(), dtype=np.float32)
        if a.size != self.phi_numel:
            raise ValueError(f"φ net has {self.phi_numel} parameters, got {a.size}")
        check(lib.sfx_phi_load(self._h, fptr(a)), "sfx_phi_load")

    def phi_get(self) -> torch.Tensor:
        a = np.empty(self.phi_numel, dtype=np.float32)
        check(lib.sfx_phi_get(self._h, fptr(a)), "sfx_phi_get")
        return torch.from_numpy(a)

    def phi_update(self, policy: int, s, a, r, s1, gamma, bias: torch.Tensor, lam: torch.Tensor, use_gpi: bool = True,
                   losses: Optional[torch.Tensor] = None, next_actions: Optional[torch.Tensor] = None):
        """DeepSF_PHI.update_successor (features/deep_phi.py:93-224): losses [4] = (loss, psi_loss,
        phi_loss, λ after the step); bias / lam: one-element float32 device tensors (the policy's
        reward-model bias and loss coefficient), updated in place."""
        s, s1, a, gamma, r = self._h2d_many([(s, torch.float32), (s1, torch.float32), (a, torch.long),
                                             (gamma, torch.float32), (r, torch.float32)])
        s, s1 = s.contiguous(), s1.contiguous()
        B = s.shape[0]
        a = a.reshape(-1).contiguous()
        gamma, r = gamma.reshape(B).contiguous(), r.reshape(B).contiguous()
        if losses is None:
            losses = torch.empty(4, device=self.device)
        check(lib.sfx_phi_update(self._h, int(policy), s.data_ptr(), a.data_ptr(), r.data_ptr(), s1.data_ptr(),
                                 gamma.data_ptr(), B, int(bool(use_gpi)), _dev_f32(bias, self.device),
                                 _dev_f32(lam, self.device), losses.data_ptr(), dptr(next_actions)), "sfx_phi_update")
        return losses

    # ---------------------------------------------------------------- TSF test tasks
    def tsf_test_action(self, s, w: torch.Tensor, omega: torch.Tensor, out: Optional[torch.Tensor] = None):
        """TSFDQN.get_test_action's greedy branch (tsfdqn.py:859-870): a 0-d int64 device tensor.
        w [d] / omega [T] are float32 device tensors, read in place."""
        s = self._f(s, (-1,))
        out = torch.empty((), dtype=torch.long, device=self.device) if out is None else out
        check(lib.sfx_tsf_test_action(self._h, s.data_ptr(), _dev_f32(w, self.device), _dev_f32(omega, self.device),
                                      out.data_ptr()), "sfx_tsf_test_action")
        return out

    def tsf_test_update(self, s, s1, a, a1, r: float, phi, w: torch.Tensor, omega: torch.Tensor,
                        adam_state: torch.Tensor, step: int, gamma: float, beta: float, lasso: float,
                        lr_w: float, wd_w: float, lr_omega: float, wd_omega: float,
                        losses: Optional[torch.Tensor] = None) -> torch.Tensor:
        """TSFDQN.update_test_reward_mapper (tsfdqn.py:917-997): updates w, omega and adam_state
        ([2d + 2T], zeros initially) in place; returns losses [3] = (loss, l2, l1)."""
        s, s1, phi, a, a1 = (t.reshape(-1).contiguous() for t in self._h2d_many(
            [(s, torch.float32), (s1, torch.float32), (phi, torch.float32), (a, torch.long), (a1, torch.long)]))
        if losses is None:
            losses = torch.empty(3, device=self.device)
        check(lib.sfx_tsf_test_update(self._h, s.data_ptr(), s1.data_ptr(), a.data_ptr(), a1.data_ptr(), float(r),
                                      phi.data_ptr(), _dev_f32(w, self.device), _dev_f32(omega, self.device),
                                      _dev_f32(adam_state, self.device), int(step), float(gamma), float(beta),
                                      float(lasso), float(lr_w), float(wd_w), float(lr_omega), float(wd_omega),
                                      losses.data_ptr()), "sfx_tsf_test_update")
        return losses

    def tsf_test_actions(self, S, W: torch.Tensor, Omega: torch.Tensor, out: Optional[torch.Tensor] = None):
        """tsf_test_action for E test tasks in one launch set (lockstep test phase): S [E, n_s],
        W [E, d] / Omega [E, T] float32 device tensors with unit column stride.  Returns the
        int64 device tensor [E] (not synchronized)."""
        S = self._f(S)
        E = S.shape[0]
        _dev_f32(W, self.device)
        _dev_f32(Omega, self.device)
        if W.shape != (E, self.d) or Omega.shape != (E, self.T) or W.stride(1) != 1 or Omega.stride(1) != 1:
            raise ValueError(f"W must be [{E}, {self.d}] and Omega [{E}, {self.T}] with unit column stride")
        out = torch.empty(E, dtype=torch.long, device=self.device) if out is None else out
        check(lib.sfx_tsf_test_actions(self._h, S.data_ptr(), E, W.data_ptr(), W.stride(0), Omega.data_ptr(),
                                       Omega.stride(0), out.data_ptr()), "sfx_tsf_test_actions")
        return out

    def tsf_test_updates(self, S, S1, a, a1, phi, W: torch.Tensor, Omega: torch.Tensor, adam_state: torch.Tensor,
                         rowp: torch.Tensor, gamma: float, beta: float, lasso: float,
                         losses: Optional[torch.Tensor] = None) -> torch.Tensor:
        """tsf_test_update for E test tasks in one launch set: W [E, d], Omega [E, T],
        adam_state [E, 2d + 2T] updated in place; rowp [E, 6] device float32 (r, lr_w, wd_w,
        lr_omega, wd_omega, step per task).  Returns losses [E, 3] = (loss, l2, l1) per row."""
        S, S1, phi, a, a1 = self._h2d_many([(S, torch.float32), (S1, torch.float32), (phi, torch.float32),
                                            (a, torch.long), (a1, torch.long)])
        S, S1 = S.contiguous(), S1.contiguous()
        E = S.shape[0]
        phi = phi.reshape(E, self.d).contiguous()
        a, a1 = a.reshape(-1).contiguous(), a1.reshape(-1).contiguous()
        for t in (W, Omega, adam_state, rowp):
            _dev_f32(t, self.device)
            if t.stride(-1) != 1 or t.shape[0] != E:
                raise ValueError("sfx tsf_test_updates: row-major [E, ...] tensors expected")
        if rowp.shape != (E, 6) or not rowp.is_contiguous():
            raise ValueError(f"rowp must be a contiguous [{E}, 6] tensor")
        losses = torch.empty(E, 3, device=self.device) if losses is None else losses
        check(lib.sfx_tsf_test_updates(self._h, E, S.data_ptr(), S1.data_ptr(), a.data_ptr(), a1.data_ptr(),
                                       phi.data_ptr(), W.data_ptr(), W.stride(0), Omega.data_ptr(), Omega.stride(0),
                                       adam_state.data_ptr(), adam_state.stride(0), rowp.data_ptr(), float(gamma),
                                       float(beta), float(lasso), losses.data_ptr()), "sfx_tsf_test_updates")
        return losses

    def tsf_update(self, policy: int, s, a, r, phi, s1, gamma, use_gpi: bool = True,
                   losses: Optional[torch.Tensor] = None, next_actions: Optional[torch.Tensor] = None):
        """TSFDQN.update_successor (tsfdqn.py:588-709): returns losses [3] = (l1 + beta l2, l1, l2)."""
        s, s1, a, phi, gamma, r = self._batch_in(s, s1, a, phi, gamma, r)
        B = s.shape[0]
        if losses is None:
            losses = torch.empty(3, device=self.device)
        check(lib.sfx_tsf_update(self._h, int(policy), s.data_ptr(), a.data_ptr(), r.data_ptr(), phi.data_ptr(),
                                 s1.data_ptr(), gamma.data_ptr(), B, int(bool(use_gpi)), losses.data_ptr(),
                                 dptr(next_actions)), "sfx_tsf_update")
        return losses

