#!/usr/bin/env python3
"""CPU simulation of the all-task step's speculation to compare guess strategies.

Not a parity tool: a batched torch restatement of features/deep.py:93-131 run for every head at
once (the heads are independent given their next actions), used to count how many speculative
rounds each env step needs before the verification passes, under different round-0 guesses:

  pre      round 0 guesses ψ_t(s') of heads t < i with the pre-step heads (the library today)
  extrap   round 0 guesses ψ_t(s') + λ (ψ_t(s') - ψ_t^{prev}(s')), ψ^{prev} = the heads before the
           previous step (Adam's momentum makes consecutive updates alike)

Round r >= 1 guesses with round r-1's post-update ψ (as on the device); a step needs rounds
until round r's next actions equal those recomputed from round r's own post-update heads.  The
trajectory follows the exact (fixpoint) result, so every strategy sees the same steps.

usage: spec_sim.py [--heads T] [--steps N] [--lams 0.5,1.0] [--threads 8]
"""
import argparse
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "deep-successor-features-for-transfer_amd")]

from sfx.init import reference_heads  # noqa: E402
from sfx.runner import Replay, SynthReacher  # noqa: E402


class Heads:
    def __init__(self, T, n_s, H, A, d, nh=2):
        self.T, self.n_s, self.H, self.A, self.d, self.O = T, n_s, H, A, d, A * d
        self.layers = [(H, n_s)] + [(H, H)] * nh + [(A * d, H)]
        self.offs = []
        off = 0
        for o, i in self.layers:
            self.offs.append((off, off + o * i, off + o * i + o))
            off += o * i + o
        self.P = off

    def views(self, flat):
        out = []
        for (o, i), (a, b, c) in zip(self.layers, self.offs):
            out.append((flat[:, a:b].view(-1, o, i), flat[:, b:c]))
        return out

    def forward(self, flat, X):
        """X [T, M, n_s] -> ([T, M, O], saved inputs per layer)."""
        xs, h = [], X
        L = self.views(flat)
        for l, (W, b) in enumerate(L):
            xs.append(h)
            h = torch.baddbmm(b.unsqueeze(1), h, W.transpose(1, 2))
            if 0 < l < len(L) - 1:
                h = torch.relu(h)
        xs.append(h)
        return h, xs

    def backward(self, flat, xs, dY):
        L = self.views(flat)
        grads = []
        dZ = dY
        for l in range(len(L) - 1, -1, -1):
            W, _ = L[l]
            grads.append((torch.bmm(dZ.transpose(1, 2), xs[l]), dZ.sum(1)))
            if l > 0:
                dX = torch.bmm(dZ, W)
                if l - 1 > 0:  # input of layer l is relu(z) for hidden layers
                    dX = dX * (xs[l] > 0)
                dZ = dX
        grads.reverse()
        return torch.cat([torch.cat([gw.reshape(self.T, -1), gb], 1) for gw, gb in grads], 1)


def adam(p, g, m, v, step, lr=1e-3, b1=0.9, b2=0.999, eps=1e-8):
    m = torch.lerp(m, g, 1 - b1)
    v = v * b2 + (1 - b2) * g * g
    bc1, bc2 = 1 - b1 ** step, 1 - b2 ** step
    return p - (lr / bc1) * m / (v.sqrt() / bc2 ** 0.5 + eps), m, v


def next_actions(guess, pre, W):
    """guess, pre [T, B, A, d]; W [T, d] -> [T_pol, B]: policy i sees heads t < i through guess."""
    T = W.shape[0]
    qg = torch.einsum("tbad,id->itba", guess, W)
    qp = torch.einsum("tbad,id->itba", pre, W)
    lower = (torch.arange(T).view(1, T) < torch.arange(T).view(T, 1)).view(T, T, 1, 1)
    q = torch.where(lower, qg, qp)
    return q.max(1).values.argmax(-1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--heads", type=int, default=64)
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--lams", default="0.5,1.0")
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--report", type=int, default=50)
    a = ap.parse_args()
    torch.set_num_threads(a.threads)
    T, n_s, H, A, d, B = a.heads, 17, 256, 7, 8, 32
    hd = Heads(T, n_s, H, A, d)
    online, w = reference_heads(T, n_s, H, A, d, seed=0)
    target = online.clone()
    m, v = torch.zeros_like(online), torch.zeros_like(online)
    prev = online.clone()  # the heads before the previous step
    step = 0
    rng = np.random.default_rng(1)
    task = SynthReacher(n_s, A, d, 0, rng)
    rep = Replay(100_000, n_s, d, rng)
    for _ in range(1000):
        s0 = task.initialize()
        a0 = int(rng.integers(A))
        s1, phi, r, _ = task.transition(a0)
        rep.append(s0, a0, r, phi, s1, 0.9)
    lams = [float(x) for x in a.lams.split(",") if x]
    strategies = ["pre"] + [f"extrap{l:g}" for l in lams]
    hist = {k: [] for k in strategies}
    wrong0 = {k: [] for k in strategies}
    s = task.initialize()
    skipc = [0, 0]
    t0 = time.time()
    for k in range(a.steps):
        with torch.no_grad():
            x = torch.from_numpy(s).view(1, 1, -1).expand(T, 1, n_s)
            psi_s = hd.forward(online, x)[0].view(T, A, d)
            q = psi_s @ w[0]
            tsk = int(q.max(1).values.argmax())
            act = int(q[tsk].argmax())
            if rng.random() <= 0.1:
                act = int(rng.integers(A))
            s1, phi, r, _ = task.transition(act)
            wl = w[0].clone()
            w[0] = wl + 1e-3 * (r - float(torch.dot(torch.from_numpy(phi), wl))) * torch.from_numpy(phi)
            rep.append(s, act, r, phi, s1, 0.9)
            idx = rng.integers(0, rep.size, B)
            S = torch.from_numpy(rep.s[idx]).expand(T, B, n_s)
            S1 = torch.from_numpy(rep.s1[idx]).expand(T, B, n_s)
            PHI = torch.from_numpy(rep.phi[idx])
            AA = torch.from_numpy(rep.a[idx])
            GAM = torch.from_numpy(rep.gamma[idx]).view(B, 1)
            c, xs = hd.forward(online, S)
            c = c.view(T, B, A, d)
            tpsi = hd.forward(target, S1)[0].view(T, B, A, d)
            pre = hd.forward(online, S1)[0].view(T, B, A, d)
            pprev = hd.forward(prev, S1)[0].view(T, B, A, d)
            step += 1
            bidx = torch.arange(B)

            def update(acts):
                tg = PHI.unsqueeze(0) + GAM.unsqueeze(0) * tpsi[torch.arange(T).view(T, 1), bidx.view(1, B), acts]
                dY = torch.zeros(T, B, A, d)
                dY[:, bidx, AA] = (2.0 / (B * A * d)) * (c[:, bidx, AA] - tg)
                g = hd.backward(online, xs, dY.view(T, B, A * d))
                p2, m2, v2 = adam(online, g, m, v, step)
                post = hd.forward(p2, S1)[0].view(T, B, A, d)
                return p2, m2, v2, post

            def run(guess0, sk=None):
                guess, rr, wrong, last = guess0, 0, None, None
                while True:
                    acts = next_actions(guess, pre, w)
                    if sk is not None and last is not None:
                        sk[0] += T
                        sk[1] += int((acts == last).all(1).sum())
                    last = acts
                    p2, m2, v2, post = update(acts)
                    ver = next_actions(post, pre, w)
                    rr += 1
                    if wrong is None:
                        wrong = -1  # filled by the caller against the exact actions
                    if torch.equal(ver, acts):
                        return rr, acts, (p2, m2, v2)
                    guess = post
                    if rr > T + 2:
                        raise RuntimeError("no convergence")

            rr, exact, newst = run(pre, skipc)
            hist["pre"].append(rr)
            wrong0["pre"].append(int((next_actions(pre, pre, w) != exact).any(1).sum()))
            for lam in lams:
                g0 = pre + lam * (pre - pprev)
                r2, acts2, _ = run(g0)
                assert torch.equal(acts2, exact)
                hist[f"extrap{lam:g}"].append(r2)
                wrong0[f"extrap{lam:g}"].append(int((next_actions(g0, pre, w) != exact).any(1).sum()))
            prev = online
            online, m, v = newst
            if step % 1000 == 0:
                target = online.clone()
            s = s1
        if (k + 1) % a.report == 0 or k + 1 == a.steps:
            line = [f"step {k + 1:5d} {time.time() - t0:6.0f}s"]
            for st in strategies:
                h = np.array(hist[st][-a.report:])
                line.append(f"{st}: rounds {h.mean():.2f} >2:{(h > 2).mean():.2f} >3:{(h > 3).mean():.2f} "
                            f"wrong0 {np.mean(wrong0[st][-a.report:]):.1f}")
            line.append(f"round>=1 skip {skipc[1] / max(skipc[0], 1):.2f}")
            skipc[:] = [0, 0]
            print(" | ".join(line), flush=True)


if __name__ == "__main__":
    main()
