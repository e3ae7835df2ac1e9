"""CPU backend of the sfx_shard_* protocol on the oracle (test infrastructure only).

It keeps one rank's heads [off, off + T_loc) in an oracle SFState plus the replicated reward
weights, and answers the same calls as sfx.shard.LibsfxShardBackend with the reference's
arithmetic (oracle/ref_cpu.py), so ShardedAllTask's orchestration (rounds, all-reduces,
verification, selection keys) can be checked against the unsharded oracle with gloo on CPU.
"""
import torch

from oracle import ref_cpu as R
from sfx.shard import encode_key


class OracleShardBackend:
    def __init__(self, spec, online, target, w_all, off, lr=1e-3, target_update_ev=1000):
        self.spec, self.off, self.lr, self.ev = spec, off, lr, target_update_ev
        self.st = R.SFState(spec, online.clone(), target.clone(), torch.zeros(online.shape[0], spec.d))
        self.w = w_all.clone()  # [T_glob, d], replicated
        self.T, self.Tg = online.shape[0], w_all.shape[0]
        self.B = 0

    @property
    def X(self):
        return self._X

    @property
    def Y(self):
        return self._Y

    def _psi(self, flat, x):
        return R.forward(flat, self.spec, x)[0]

    def begin(self, batch, lms_task, lms_phi, lms_r, alpha, s_next):
        if lms_task >= 0:
            self.w[lms_task] = R.lms_update(self.w[lms_task].view(-1, 1), lms_phi, lms_r.reshape(()), alpha).view(-1)
        self.batch, self.s_next = batch, s_next.reshape(1, -1)
        self.post = {}
        if batch is None:
            self.B = 0
            return
        S, a, phi, S1, g = batch
        self.B = S.shape[0]
        self.pre_S1 = [self._psi(self.st.online[t], S1) for t in range(self.T)]
        self._X = torch.empty(self.Tg * self.B * self.spec.A)
        self._Y = torch.empty_like(self._X)

    def _maxima(self, vals_for, out):
        A = self.spec.A
        for i in range(self.Tg):
            qs = []
            for t in range(self.T):
                vals = vals_for(t) if self.off + t < i else self.pre_S1[t]
                qs.append(torch.matmul(vals, self.w[i].view(-1, 1))[..., 0])  # [B, A]
            out.view(self.Tg, self.B, A)[i] = torch.stack(qs).max(dim=0).values

    def td_maxima(self, r, X):
        self._maxima(lambda t: self.pre_S1[t] if r == 0 else self.post[r - 1]["S1"][t], X)

    def td_update(self, r, X):
        S, a, phi, S1, g = self.batch
        A, B = self.spec.A, self.B
        Xv = X.view(self.Tg, B, A)
        post = {"p": [], "m": [], "v": [], "S1": [], "sn": []}
        for t in range(self.T):
            nxt = torch.argmax(Xv[self.off + t], dim=1)
            p, m, v = self.st.online[t].clone(), self.st.m[t].clone(), self.st.v[t].clone()
            c, xs = R.forward(p, self.spec, S)
            tpsi, _ = R.forward(self.st.target[t], self.spec, S1)
            targets = phi + g.reshape(-1, 1) * tpsi[torch.arange(B), nxt, :]
            _, gc = R.td_grad(c, a, targets)
            R.adam_(p, R.backward(p, self.spec, xs, gc), m, v, self.st.step[t] + 1, self.lr)
            for k, val in (("p", p), ("m", m), ("v", v), ("S1", self._psi(p, S1)), ("sn", self._psi(p, self.s_next))):
                post[k].append(val)
        self.post[r] = post

    def ver_maxima(self, r, Y):
        self._maxima(lambda t: self.post[r]["S1"][t], Y)

    def verify(self, X, Y):
        A = self.spec.A
        ax = X.view(self.Tg, self.B, A).argmax(dim=2)
        ay = Y.view(self.Tg, self.B, A).argmax(dim=2)
        bad = (ax != ay).any(dim=1).nonzero()
        return int(bad[0, 0]) if bad.numel() else self.Tg

    def select(self, r, task, use_gpi):
        A = self.spec.A
        best = -(1 << 63)
        for t in range(self.T):
            tg = self.off + t
            if not use_gpi and tg != task:
                continue
            vals = self._psi(self.st.online[t], self.s_next) if r < 0 else self.post[r]["sn"][t]
            q = torch.matmul(vals, self.w[task].view(-1, 1))[0, :, 0]
            for a in range(A):
                best = max(best, encode_key(float(q[a]), tg, a, A))
        self.key = torch.tensor([best], dtype=torch.long)
        return self.key

    def finish(self, rounds_run):
        if self.B == 0:
            return
        post = self.post[rounds_run - 1]
        for t in range(self.T):
            self.st.online[t] = post["p"][t]
            self.st.m[t] = post["m"][t]
            self.st.v[t] = post["v"][t]
            self.st.step[t] += 1
            self.st.since_target[t] += 1
            if self.st.since_target[t] >= self.ev:
                self.st.target[t].copy_(self.st.online[t])
                self.st.since_target[t] = 0


class OracleTSFShardBackend:
    """CPU backend of the sfx_shard_tsf_* protocol (sfx.shard.ShardedTSF): this rank's heads
    [off, off + T_loc) with their g_i and optimizer state in an oracle TSFState (local indices),
    the replicated w (T_glob rows) and h."""

    def __init__(self, spec, gspec, online, target, g, h, w_all, off, target_update_ev=1000):
        self.spec, self.off, self.ev = spec, off, target_update_ev
        self.T, self.Tg = online.shape[0], w_all.shape[0]
        self.w = w_all.clone()
        self.st = R.TSFState(spec, online.clone(), target.clone(), self.w[off:off + self.T].clone(), gspec=gspec,
                             g=g.clone(), h=h.clone())
        self.shared_buf = torch.empty(h.numel() + spec.d)
        self.losses = None

    def X(self, B):
        return torch.empty(B * self.spec.A)

    def maxima(self, i, S1, X, own_only):
        ts = [i - self.off] if own_only else range(self.T)
        qs = [torch.matmul(R.forward(self.st.online[t], self.spec, S1)[0], self.w[i].view(-1, 1))[..., 0] for t in ts]
        X.copy_(torch.stack(qs).max(dim=0).values.reshape(-1))

    def update(self, i, batch, X):
        loc = i - self.off
        nxt = torch.argmax(X.view(batch[0].shape[0], self.spec.A), dim=1)
        loss, l1, l2, _ = R.tsf_update(self.st, batch, loc, target_update_ev=self.ev, next_actions=nxt)
        self.w[i] = self.st.w[loc]
        self.losses = torch.tensor([float(loss), float(l1), float(l2)])
        return self.losses

    def pack(self, i, buf):
        buf.copy_(torch.cat([self.st.h, self.w[i]]))

    def unpack(self, i, buf):
        n = self.st.h.numel()
        self.st.h.copy_(buf[:n])
        self.w[i] = buf[n:]

    def select(self, s, task, use_gpi):
        A = self.spec.A
        best = -(1 << 63)
        for t in range(self.T):
            tg = self.off + t
            if not use_gpi and tg != task:
                continue
            q = torch.matmul(R.forward(self.st.online[t], self.spec, s.reshape(1, -1))[0], self.w[task].view(-1, 1))[0, :, 0]
            for a in range(A):
                best = max(best, encode_key(float(q[a]), tg, a, A))
        return torch.tensor([best], dtype=torch.long)
