"""DeepSF on the GPU (the interface of features/deep.py:8-131, the ψ library of
main_sfdqn_torch.py).

The ψ heads, their target copies, Adam state and the reward weights live in one libsfx
engine (``sfx.engine.SFEngine``); every ψ forward, GPI reduction, TD target, backward and
Adam step runs in the hand-written gfx950 kernels.  There is no CPU path: without a HIP
device the first compute call raises.

The user's ``pytorch_model_handle`` still builds the torch modules (so weight init and the
optimizer's hyper-parameters are exactly the user's); the engine then owns the values.
``psi`` returns those modules refreshed from the device on access (read-only views:
write new weights through ``load_heads``).

``update_successor`` calls are deferred and fused: the all-task loop of
agents/sfdqn.py:57-60 (policies 0..T-1 on the same minibatch) becomes one speculative
device step with the exact sequential semantics (sfx_update_all); any other call pattern
runs head by head (sfx_update).  The deferral is invisible: features/deep.py returns
nothing from update_successor, and every method that reads state flushes first.
"""
from __future__ import annotations

import weakref

import numpy as np
import torch

from sfx import _lib
from sfx.dropin._host import copy_weights as update_models_weights
from sfx.dropin._host import torch_device as get_torch_device
from sfx.dropin.agents.buffer import lending_buffer, release_minibatch
from .successor import SF


def _geometry(model: torch.nn.Module):
    """(n_s, H, acts, out) of the reference lambda's Sequential; raises for other shapes."""
    mods = [m for m in model.modules() if m is not model and not isinstance(m, torch.nn.Sequential)]
    lin = [m for m in mods if isinstance(m, torch.nn.Linear)]
    acts = []
    seq = [m for m in mods if not isinstance(m, (torch.nn.Unflatten, torch.nn.Identity))]
    ok = len(lin) >= 2 and isinstance(seq[0], torch.nn.Linear) and isinstance(seq[-1], torch.nn.Linear)
    i = 1
    while ok and i < len(seq) - 1:
        if not isinstance(seq[i], torch.nn.Linear) or not isinstance(seq[i + 1], (torch.nn.ReLU, torch.nn.Tanh)):
            ok = False
            break
        acts.append("relu" if isinstance(seq[i + 1], torch.nn.ReLU) else "tanh")
        i += 2
    H = lin[0].out_features if lin else 0
    ok = ok and all(l.in_features == H and l.out_features == H for l in lin[1:-1]) and lin[-1].in_features == H
    ok = ok and all(l.bias is not None for l in lin)
    if not ok:
        raise NotImplementedError(
            "sfx DeepSF supports the reference ψ architecture only: Linear(n_s,H) -> [Linear(H,H) + ReLU|Tanh]* "
            f"-> Linear(H, A*d) (-> Unflatten); got {model}")
    return lin[0].in_features, H, tuple(acts), lin[-1].out_features


def _flat(model):
    return torch.cat([p.detach().reshape(-1).float().cpu() for p in model.parameters()])


def _unflat_into(model, flat):
    off = 0
    with torch.no_grad():
        for p in model.parameters():
            n = p.numel()
            p.copy_(flat[off:off + n].view_as(p).to(p.device, p.dtype))
            off += n


class _FitW(list):
    """fit_w whose entries live in the engine once it exists ([d, 1] tensors on read)."""

    def __init__(self, sf):
        super().__init__()
        self._sf = sf

    def __getitem__(self, i):
        sf = self._sf
        if isinstance(i, int) and sf._eng is not None and sf._eng_T == len(self):
            sf._flush()
            w = sf._eng.get_w(i if i >= 0 else len(self) + i)[0].view(-1, 1)
            return w.to(sf._out_device())
        return super().__getitem__(i)

    def __setitem__(self, i, v):
        super().__setitem__(i, v)
        sf = self._sf
        if isinstance(i, int) and sf._eng is not None and sf._eng_T == len(self):
            sf._flush()
            sf._pred = None  # a fused GPI computed with the old w
            sf._eng.load_w(i if i >= 0 else len(self) + i, v)



def _huber_delta(loss) -> float:
    """The ψ loss the user's model handle returns: MSELoss(mean) -- the reference's, 0 -- or the
    opt-in HuberLoss(delta, mean) / SmoothL1Loss(beta=1, mean) (the same function at δ = 1):
    δ for sfx_set_huber.  Anything else raises."""
    if getattr(loss, "reduction", None) == "mean":
        if isinstance(loss, torch.nn.MSELoss):
            return 0.0
        if isinstance(loss, torch.nn.HuberLoss) and loss.delta > 0:
            return float(loss.delta)
        if isinstance(loss, torch.nn.SmoothL1Loss) and loss.beta == 1.0:
            return 1.0
    raise NotImplementedError("sfx DeepSF trains with MSELoss, HuberLoss or SmoothL1Loss(beta=1), reduction='mean'")

class DeepSF(SF):
    _alpha_f = 0.0  # float(alpha_w) as the deferred LMS last took it
    _lms_pend = None
    _pred = None

    def __init__(self, pytorch_model_handle, *args, target_update_ev=1000, max_batch=256, **kwargs):
        super().__init__(*args, **kwargs)
        self.pytorch_model_handle = pytorch_model_handle
        self.target_update_ev = target_update_ev
        self.max_batch = max_batch
        self.device = get_torch_device()
        self._eng = None
        self._eng_T = 0
        self._pending = []
        self._host_stale = False
        # the agent loop's next GPI, fused into the last all-task update (_flush): (weak reference to
        # the state, its version, task index, q, task); _gpi_task: the task index of the last GPI
        self._pred = None
        self._gpi_task = None
        # update_reward of a device φ and a host reward, deferred to ride in the next all-task step
        # (sfx_update_all_select) or run before anything else reads w: (φ, its version, r, task)
        self._lms_pend = None

    # ------------------------------------------------------------------ library
    def reset(self):
        self._close()
        SF.reset(self)
        self.fit_w = _FitW(self)
        self._since = []

    def _close(self):
        self._pred = None
        self._lms_pend = None
        if getattr(self, "_eng", None) is not None:
            self._pending = []
            self._eng.close()
        self._eng, self._eng_T = None, 0
        self._release_held()  # the handle is gone: nothing reads the last minibatch any more

    def build_successor(self, task, source=None):
        if self.n_tasks == 0:
            self.n_actions = task.action_count()
            self.n_features = task.feature_dim()
            self.inputs = task.encode_dim()
        A, d = self.n_actions, self.n_features
        model, loss, optim = self.pytorch_model_handle(self.inputs, A * d, (A, d), 1)
        if source is not None and self.n_tasks > 0:
            self._sync_host()
            update_models_weights(self._psi[source][0][0], model)
        target, tloss, toptim = self.pytorch_model_handle(self.inputs, A * d, (A, d), 1)
        update_models_weights(model, target)
        target.eval()
        self._since.append(0)
        return (model, loss, optim), (target, tloss, toptim)

    def add_training_task(self, task, source=None):
        self._flush()
        self._pred = None
        self._sync_host()
        SF.add_training_task(self, task, source)

    @property
    def psi(self):
        self._sync_host()
        return self._psi

    @property
    def updates_since_target_updated(self):
        if self._eng is not None and self._eng_T == self.n_tasks:
            self._flush()
            return [self._eng.since_target(t) for t in range(self.n_tasks)]
        return self._since

    # ------------------------------------------------------------------ engine
    def _out_device(self):
        dev = get_torch_device() if self.device is None else self.device
        return dev if dev is not None else self._eng.device

    def _engine(self, batch: int = 1):
        """The engine holding every current head (rebuilt when tasks were added)."""
        if self._eng is not None and self._eng_T == self.n_tasks and batch <= self._eng.max_batch:
            return self._eng
        from sfx.engine import SFEngine

        if self.n_tasks == 0:
            raise RuntimeError("DeepSF has no tasks: call add_training_task first")
        self._flush()
        old, old_T = self._eng, self._eng_T
        if old is not None:  # carry the device state of the heads that already exist
            self._sync_host()
            adam = [old.get_adam(t) for t in range(old_T)]
            ws = [old.get_w(t)[0] for t in range(old_T)]
            since = [old.since_target(t) for t in range(old_T)]
        model, loss, optim = self._psi[0][0]
        n_s, H, acts, out = _geometry(model)
        if out != self.n_actions * self.n_features:
            raise ValueError("ψ output width != n_actions * n_features")
        huber = _huber_delta(loss)
        g = optim.param_groups[0] if optim is not None else {"lr": 1e-3, "betas": (0.9, 0.999), "eps": 1e-8,
                                                             "weight_decay": 0.0}
        if optim is not None and (not isinstance(optim, torch.optim.Adam) or g.get("amsgrad") or g.get("maximize")):
            raise NotImplementedError("sfx DeepSF trains ψ with torch.optim.Adam (no amsgrad / maximize) only")
        mb = max(self.max_batch, batch)
        eng = SFEngine(self.n_tasks, n_s, H, self.n_actions, self.n_features, acts, max_batch=mb)
        (lr_sf, wd_sf), (lr_w, wd_w) = self._adam_groups(optim) if optim is not None else ((1e-3, 0.0), (1e-3, 0.0))
        eng.set_adam(lr_sf, wd_sf, lr_w, wd_w, betas=tuple(g["betas"]), eps=g["eps"])
        eng.set_target_update_ev(self.target_update_ev)
        if huber:
            eng.set_huber(huber)
        for t, ((m, _, _), (tm, _, _)) in enumerate(self._psi):
            eng.load_head(t, _flat(m), 0)
            eng.load_head(t, _flat(tm), 1)
            if old is not None and t < old_T:
                eng.load_adam(t, adam[t][0], adam[t][1], adam[t][2])
                eng.load_w(t, ws[t])
                eng.set_since_target(t, since[t])
            else:
                eng.load_w(t, self._w_host(t))
                eng.set_since_target(t, self._since[t])
        if old is not None:
            old.close()
        self._eng, self._eng_T = eng, self.n_tasks
        self.max_batch = mb
        return eng

    def _w_host(self, t):
        """Host value of fit_w[t] before the engine owns it ([d, 1] tensor here)."""
        return list.__getitem__(self.fit_w, t)

    def _adam_groups(self, optim):
        """(lr, weight_decay) of the ψ group and of the w group of a task's optimizer."""
        g = optim.param_groups[0]
        return (g["lr"], g.get("weight_decay", 0.0)), (g["lr"], 0.0)

    def _sync_host(self):
        """Refresh the torch modules (online, target) from the device."""
        if self._eng is None or not self._host_stale:
            return
        self._flush()
        for t in range(self._eng_T):
            (m, _, _), (tm, _, _) = self._psi[t]
            _unflat_into(m, self._eng.get_head(t, 0))
            _unflat_into(tm, self._eng.get_head(t, 1))
        self._host_stale = False

    def load_heads(self):
        """Push the torch modules' current weights to the device (after editing ``psi``)."""
        if self._eng is not None:
            self._flush()
            self._pred = None
            for t, ((m, _, _), (tm, _, _)) in enumerate(self._psi):
                self._eng.load_head(t, _flat(m), 0)
                self._eng.load_head(t, _flat(tm), 1)
            self._host_stale = False

    def _flush(self):
        """Run deferred update_successor calls (and a deferred update_reward before them)."""
        lms = self._lms_pend
        if not self._pending or self._eng is None:
            if lms is not None:
                self._lms_now()
            return
        pend, self._pending = self._pending, []
        eng = self._eng
        T = self._eng_T
        # update_successor queues a policy after the first only when it is the next one on the same
        # minibatch, and flushes a queue that does not open with policy 0: T entries from policy 0
        # are the all-task loop of agents/sfdqn.py:57-60
        if len(pend) == T and pend[0][1] == 0:
            s, a, phi, s1, g = pend[0][2]
            lb = getattr(eng, "_dropin_losses", None)  # the losses nobody reads: one buffer per engine
            if lb is None:
                lb = eng._dropin_losses = torch.empty(T, 3, device=eng.device)
            buf = lending_buffer(s)
            nxt = self._next_state(buf)
            if nxt is not None:
                # the agent's next GPI (on the transition's next state, which the buffer copied into
                # the engine's selection input; with the task of its last GPI) rides in the update's
                # final round: GPI returns its result if that state comes.  The deferred LMS rides in
                # the step's first launch when the buffer copied its φ into the engine's LMS input.
                lt = -1
                if lms is not None:
                    lr = buf.last_reward
                    if (lr is not None and lr[2] is eng.lms_phi and lr[0]() is lms[0] and lr[1] == lms[1]
                            and lms[0]._version == lms[1]
                            and (type(lms[2]) is not torch.Tensor or lms[2]._version == lms[4])):
                        self._lms_pend, lt = None, lms[3]
                    else:
                        self._lms_now()
                q, task = eng.update_all_select(s, a, phi, s1, g, self._gpi_task, losses=lb, lms_task=lt,
                                                lms_r=lms[2] if lt >= 0 else 0.0, lms_alpha=self._alpha_f)
                self._pred = (nxt[0], nxt[1], self._gpi_task, q, task)
            else:
                if lms is not None:
                    self._lms_now()
                eng.update_all(s, a, phi, s1, g, losses=lb)
            # update_all settled the step before (host rounds included): its minibatch is read by
            # nothing queued after this point -- hand it back to the ReplayBuffer that lent it
            self._release_held()
            self._held = s
        else:
            if lms is not None:
                self._lms_now()
            for _, i, (s, a, phi, s1, g) in pend:
                eng.update(i, s, a, None, phi, s1, g, use_gpi=True)
        self._host_stale = True

    def _lms_now(self):
        """Launch the deferred update_reward.  Its φ is read now: a φ written in place since the
        update_reward call would give another reward fit than the reference's (which fits at the
        call) -- that raises instead of fitting silently on the new values."""
        phi, v, r, t, rv = self._lms_pend
        self._lms_pend = None
        if phi._version != v or (type(r) is torch.Tensor and r._version != rv):
            raise RuntimeError("DeepSF.update_reward: the φ or reward tensor was modified in place before the reward "
                               "fit ran; pass tensors that stay unchanged until the next DeepSF call (e.g. clones)")
        self._eng.lms(t, phi.reshape(-1), r, self._alpha_f)

    # ------------------------------------------------------------------ ψ / GPI
    def _state(self, state):
        s = torch.as_tensor(state)
        return s.reshape(1, -1) if s.dim() == 1 else s.reshape(s.shape[0], -1)

    def _next_state(self, buf):
        """(weak reference, version) of the state the agent's next GPI will most likely get: the
        next state the minibatch's ReplayBuffer (buf) was last given, when the buffer copied it into
        the engine's selection input (on the engine's stream) and nothing changed it since.
        Otherwise None -- and the buffer is asked to copy from its next append on (the next state
        and φ: sfx_replay_put_gather)."""
        eng = self._eng
        if self._gpi_task is None or eng is None:
            return None
        if (buf is None or getattr(buf, "_ring_dev", None) != eng.device.index
                or _lib.stream_ptr(eng.device.index) != eng.stream):
            return None
        x, _ = eng._select_slots()
        if buf.mirror is not x:
            buf.mirror, buf.mirror_reward = x, eng.lms_phi
            return None
        ln = buf.last_next
        ns = ln[0]() if ln is not None and ln[2] is x else None
        if ns is None or ns._version != ln[1]:
            return None
        return ln[0], ln[1]

    def _release_held(self):
        """The minibatch of the last fused update, once a library call has settled that update, goes
        back to the sfx ReplayBuffer that lent it (agents.buffer alias; a no-op for other tensors)."""
        held = getattr(self, "_held", None)
        if held is not None:
            self._held = None
            release_minibatch(held, self._eng.stream if self._eng is not None else None)

    def get_successor(self, state, policy_index):
        return self.get_successors(state)[:, policy_index]

    def get_successors(self, state):
        self._pred = None
        s = self._state(state)
        eng = self._engine(s.shape[0])
        self._flush()
        return eng.successors(s).to(self._out_device())

    def GPI_w(self, state, w):
        self._pred = None
        s = self._state(state)
        eng = self._engine(s.shape[0])
        self._flush()
        _, q, task, _ = eng.gpi(s, w=torch.as_tensor(w).reshape(-1))
        dev = self._out_device()
        return q.to(dev), torch.squeeze(task).to(dev)

    def GPI(self, state, task_index, update_counters=False):
        pred, self._pred = self._pred, None
        ref = pred[0]() if pred is not None else None
        if (ref is not None and state is ref and not self._pending and state._version == pred[1]
                and task_index == pred[2] and self._eng is not None and self._eng_T == self.n_tasks):
            # computed by the last update's final round, on the heads and w this call would read
            q, task, _ = self._eng.settle_select(pred[3], pred[4])
            self._release_held()
            dev = self._out_device()
            if dev != self._eng.device:
                q, task = q.to(dev), task.to(dev)
            if update_counters:
                self._count(task_index, task)
            return q, task
        s = self._state(state)
        eng = self._engine(s.shape[0])
        self._flush()
        dev = self._out_device()  # before the call: it returns once the pending update is settled
        move = dev != eng.device
        # one state: the task index is allocated 0-dim (what torch.squeeze would make of it)
        _, q, task, _ = eng.gpi(s, w_index=task_index, task_shape=() if s.shape[0] == 1 else None)
        self._gpi_task = task_index if s.shape[0] == 1 else None
        self._release_held()  # gpi settled the pending update
        if move:
            q, task = q.to(dev), task.to(dev)
        if task.dim():
            task = torch.squeeze(task)
        if update_counters:
            self._count(task_index, task)
        return q, task

    # ------------------------------------------------------------------ training
    def update_reward(self, phi, r, task_index, exact=False):
        self._pred = None
        eng = self._eng
        if eng is None or self._eng_T != self.n_tasks:
            eng = self._engine()
        if self._pending or self._lms_pend is not None:
            self._flush()
        host_r = isinstance(r, (float, int, np.floating, np.integer))
        dev_r = not host_r and eng._on_dev(r, torch.float32) and r.numel() == 1  # tasks/reacher.py's reward
        if (not exact and (host_r or dev_r) and type(phi) is torch.Tensor and eng._on_dev(phi, torch.float32)
                and phi.numel() == eng.d and 0 <= task_index < self._eng_T):
            # a device φ and a host or device reward (the reference agents' call): deferred -- it runs
            # inside the next all-task step when that step's minibatch comes from the buffer this φ was
            # appended to (one launch set), else before the next call that reads w
            self._alpha_f = float(self.alpha_w)
            self._lms_pend = (phi, phi._version, r if dev_r else float(r), task_index, r._version if dev_r else 0)
            return
        if isinstance(r, (float, int, np.floating, np.integer)) or (torch.is_tensor(r) and r.device.type == "cpu"
                                                                  and r.numel() == 1):
            rr = float(r)  # a host reward goes to the kernel as a value (rounded to float32 there)
        else:
            rr = torch.as_tensor(r, dtype=torch.float32).reshape(1)
        eng.lms(task_index, torch.as_tensor(phi).reshape(-1), rr, float(self.alpha_w))
        if exact:
            w_true = torch.as_tensor(self.true_w[task_index]).reshape(-1).cpu()
            r_true = torch.sum(torch.as_tensor(phi).reshape(-1).cpu() * w_true)
            if not torch.allclose(torch.as_tensor(r).cpu().float(), r_true.float()):
                raise Exception(f"sampled reward {r} != linear reward {r_true} - please check task {task_index}!")

    def update_successor(self, transitions, policy_index):
        self._pred = None
        if transitions is None:
            return
        pend = self._pending
        if pend and pend[0][0] is transitions and pend[-1][1] + 1 == policy_index:
            # the all-task loop's next policy on the same minibatch (checked when policy 0 came)
            pend.append((transitions, policy_index, pend[0][2]))
            if len(pend) == self._eng_T:
                self._flush()
            return
        states, actions, phis, next_states, gammas = transitions
        eng = self._engine(len(gammas))
        if self._pending and (self._pending[0][0] is not transitions or self._pending[-1][1] + 1 != policy_index):
            self._flush()
        self._pending.append((transitions, policy_index, (states, actions, phis, next_states, gammas)))
        if len(self._pending) == self._eng_T:
            self._flush()
        elif self._pending[0][1] != 0:
            self._flush()
        del eng
