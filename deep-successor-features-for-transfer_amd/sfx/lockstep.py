"""Lockstep test-task rollouts: the test phase of agents/sfdqn.py with every test task stepped
together (batched host envs).

The reference evaluates its test tasks one after the other (agents/sfdqn.py:111-115): each
``test_agent`` (:139-166) runs ``agent.T`` steps of its own env, choosing each action by GPI over
all ψ heads under that task's own reward model (``get_test_action``, :125-137) and fitting that
model after every step (``update_test_reward_mapper``, :168-184).  The ψ heads do not change during
the test phase and every test task owns its env and its ``w``, so the E episodes are independent
except for one shared thing: Python's ``random`` stream, from which each step draws
``random.random()`` (ε test) and, when exploring, ``random.randrange``.  The number of draws per
step depends only on the first draw, never on the GPU's results, so the whole schedule of draws
can be taken up front in the reference's order (task 0's steps, then task 1's, ...).  After that
the E episodes run in lockstep: one ``sfx_test_actions`` launch set per step chooses all E greedy
actions (row e under its own w), the E envs step, and the E reward models are fitted (on the device for
agents/sfdqn.py's mapper, below) -- the same arithmetic, the same draws, the same
actions, the same returns and log lines in the same order as the sequential loop, with one GPU
round trip per step instead of E.

Preconditions, checked before the first step (a phase never stops after it has moved an env or
a reward model): each test task owns its env and its random state (tasks/reacher.py: one bullet
env with its own ``np_random`` per task), since the lockstep order interleaves the tasks' env
calls; and every episode runs the full ``agent.T`` steps (``fixed_horizon``: tasks/reacher.py:112
never ends one; other tasks declare ``episodes_never_end = True``, or the caller passes
``episodes_end=False``).  An episode that ends early would shift every later task's draws, so phases
whose episodes may end run the reference's own sequential loop instead -- exact, one task after the
other.  Should a task declared endless end anyway, it stops there (as the reference's ``break``)
with a warning, and the phase goes on.

With agents/sfdqn.py's own reward mapper (``device_reward_mapper``: a fresh SGD step of
MSE(w(φ), r) per task and step) the E SGD steps of a lockstep step run as ONE device launch
(``sfx_test_reward_updates``) on a device copy of the E reward models, written back into the
users' ``w_approx`` at the end of the phase, and the E losses are read once per phase.  Other
mappers (the single-file sfdqn.py's (w, Adam) pairs, user overrides) run as written.

The TSF agents' test phase (agents/tsfdqn_sequential.py:385-420, tsfdqn.py / tsfdqn_nf.py
test_agent) runs in lockstep too (``test_tasks_lockstep_tsf``): each step draws twice (the action
at s and the next action a1 at s1, both under the pre-update w and ω) and, when
``total_training_steps % 1000 == 0``, the reward mapper's ``random.randint`` of its diagnostic
print -- all independent of the GPU, so again taken up front in the reference's order.  Per step:
one ``sfx_tsf_test_actions`` launch set for the E actions at s, the E env steps, one for the E
actions at s1, one ``sfx_tsf_test_updates`` launch set fitting the E (w, ω) pairs -- each task's
own Adam step number, LR (its LambdaLR keeps decaying ω's) and r read per row -- then each task's
scheduler steps.  The E losses of every step stay on the device until the phase ends (the
reference's ``loss.item()`` per step is one device read per task and step).  Console output of the
TSF phase: the same lines as the sequential loop over the bound reward mapper
(``sfx.dropin.bind.tsf_update_test_reward_mapper``, which shortens the reference's diagnostic
block to one line), but a step's lines are printed for all live tasks together, so across tasks
their order interleaves where the sequential loop prints task by task; the SF phase prints in the
reference's order.
"""
from __future__ import annotations

import random
import warnings
from typing import List, Sequence

import torch


def _draw_schedule(E: int, T: int, epsilon: float, n_actions: int) -> List[List[int]]:
    """The reference's random draws of E sequential test episodes of T steps (sfdqn.py:127-128):
    entry [e][j] is the explored action of task e's step j, or -1 for a greedy step."""
    sched = []
    for _ in range(E):
        row = []
        for _ in range(T):
            row.append(random.randrange(n_actions) if random.random() <= epsilon else -1)
        sched.append(row)
    return sched


def fixed_horizon(test_tasks: Sequence, episodes_end=None) -> bool:
    """Whether every episode of ``test_tasks`` is known to run the full ``agent.T`` steps -- the
    lockstep precondition, decided BEFORE the first step (a phase never stops after it has moved
    an env or a reward model).  ``episodes_end=False`` is the caller's guarantee, ``True`` its
    denial; ``None`` asks the tasks: a task attribute ``episodes_never_end = True``, or the
    reference's Reacher (tasks/reacher.py:112 returns done = False on every step)."""
    if episodes_end is not None:
        return not episodes_end
    def never(task):
        if getattr(task, "episodes_never_end", False):
            return True
        cls = type(task)
        return cls.__name__ == "Reacher" and cls.__module__ in ("tasks.reacher", "reacher")
    return len(test_tasks) > 0 and all(never(t) for t in test_tasks)


def device_reward_mapper(agent) -> bool:
    """Whether the agent's ``update_test_reward_mapper`` is agents/sfdqn.py's own (:168-184: a fresh
    SGD(lr=0.005, weight_decay=0.01) step of MSE(w(φ), r) on a bias-free Linear(d, 1)), which the
    lockstep then runs on the device for all E test tasks in one launch (sfx_test_reward_updates).
    A subclass that overrides it, or an instance attribute, keeps the user's method."""
    if "update_test_reward_mapper" in vars(agent):
        return False
    f = getattr(type(agent), "update_test_reward_mapper", None)
    if f is None:
        return False
    if getattr(f, "__sfx_mapper__", None) == "sgd":
        return True
    return f.__module__ == "agents.sfdqn" and f.__qualname__ == "SFDQN.update_test_reward_mapper"


def _warn_ended(e, j, T):
    warnings.warn(f"sfx.lockstep: test task {e} ended at step {j} of {T} although its episodes were declared "
                  "never to end; it stops there, and the random draws of the later test tasks no longer follow "
                  "the sequential loop's order", RuntimeWarning, stacklevel=3)


def test_tasks_lockstep(agent, test_tasks: Sequence, indices: Sequence[int] = None, *, episodes_end=None,
                        sequential=None) -> List:
    """``[agent.test_agent(task, i) for i, task in enumerate(test_tasks)]`` of agents/sfdqn.py
    (or of the single-file sfdqn.py, :665-721) with the episodes in lockstep.  ``agent`` is the user's SFDQN over ``sfx``'s drop-in
    ``DeepSF`` (``agent.sf``); returns the E returns R (as test_agent does).

    Lockstep runs only when ``fixed_horizon(test_tasks, episodes_end)`` holds; otherwise the
    reference's own sequential loop runs (``sequential(task, index)``, default
    ``agent.test_agent``), which is exact for episodes that end early.  With agents/sfdqn.py's
    reward mapper (``device_reward_mapper``) the E SGD steps of a lockstep step are one device
    launch and the losses one device read per phase; other mappers run as the user wrote them."""
    E = len(test_tasks)
    if E == 0:
        return []
    idx = list(range(E)) if indices is None else list(indices)
    if not fixed_horizon(test_tasks, episodes_end):
        seq = sequential or agent.test_agent
        return [seq(task, i) for i, task in zip(idx, test_tasks)]
    sf = agent.sf
    eng = sf._engine(E)
    sf._flush()
    dev, T = eng.device, int(agent.T)
    sched = _draw_schedule(E, T, float(agent.test_epsilon), int(agent.n_actions))
    # agents/sfdqn.py keeps w_approx per test task, the single-file sfdqn.py (w_approx, optim)
    # with an optimizer argument to update_test_reward_mapper (sfdqn.py:652, :723)
    entries = [agent.test_tasks_weights[i] for i in idx]
    paired = isinstance(entries[0], tuple)
    ws = [x[0] for x in entries] if paired else entries
    on_device = not paired and device_reward_mapper(agent)
    adev = getattr(agent, "device", None) or sf._out_device()
    s_enc = [agent.encoding(task.initialize()) for task in test_tasks]
    R = [0.0] * E
    acc = [0] * E
    live = list(range(E))  # tasks whose episode is still running (all of them when the declaration holds)
    W = torch.cat([w.weight.detach().to(dev, torch.float32).reshape(1, -1) for w in ws]).contiguous()
    L = torch.zeros(T, E, device=dev) if on_device else None
    for j in range(T):
        S = torch.cat([torch.as_tensor(s_enc[e]).to(dev, torch.float32).reshape(1, -1) for e in live])
        Wl = W if len(live) == E else W[live].contiguous()
        if not on_device:
            Wl = torch.cat([ws[e].weight.detach().to(dev, torch.float32).reshape(1, -1) for e in live])
        greedy = eng.test_actions(S, Wl)[:, 1].unbind()
        losses, phis, rs, ended = [], [], [], []
        for k, e in enumerate(live):
            task = test_tasks[e]
            x = sched[e][j]
            a = torch.tensor(x).to(adev) if x >= 0 else greedy[k]
            s1, r, done = task.transition(a)
            s1_enc = agent.encoding(s1)
            if on_device:
                phis.append(torch.as_tensor(task.features(s_enc[e], a, s1_enc)).to(dev, torch.float32).reshape(1, -1))
                rs.append(float(r))
            elif paired:
                losses.append(agent.update_test_reward_mapper(ws[e], entries[e][1], task, r, s_enc[e], a, s1_enc))
            else:
                losses.append(agent.update_test_reward_mapper(ws[e], task, r, s_enc[e], a, s1_enc))
            s_enc[e] = s1_enc
            R[e] += r
            if done and j + 1 < T:
                _warn_ended(idx[e], j + 1, T)
                ended.append(e)
        if on_device:
            rows = torch.tensor(live, device=dev) if len(live) < E else None
            if rows is None:
                eng.test_reward_updates(torch.cat(phis), torch.tensor(rs, dtype=torch.float32), W, losses=L[j])
            else:  # a declared-endless episode ended: the remaining rows only
                Wl = W[rows].contiguous()
                Ll = eng.test_reward_updates(torch.cat(phis), torch.tensor(rs, dtype=torch.float32), Wl)
                W[rows] = Wl
                L[j, rows] = Ll
        else:
            for e, v in zip(live, torch.stack([l.detach().reshape(()) for l in losses]).tolist()):
                acc[e] += v
        live = [e for e in live if e not in ended]
        if not live:
            break
    if on_device:
        with torch.no_grad():
            for e in range(E):
                ws[e].weight.copy_(W[e].view_as(ws[e].weight))
        Lh = L.cpu().tolist()  # one device read for the phase's losses
        for e in range(E):
            for j in range(T):
                acc[e] += Lh[j][e]
    for e in range(E):
        agent.logger.log_target_error_progress(agent.get_target_reward_mapper_error(R[e], acc[e], idx[e], T))
    return R


def _tsf_draw_schedule(E: int, T: int, epsilon: float, n_actions: int, diag: bool) -> List[List[tuple]]:
    """The random draws of E sequential TSF test episodes (agents/tsfdqn_sequential.py:377-381,
    :399-402, :502): entry [e][j] = (action at s or -1 for greedy, action at s1 or -1, whether the
    diagnostic print fires)."""
    def one():
        return random.randrange(n_actions) if random.random() <= epsilon else -1

    sched = []
    for _ in range(E):
        row = []
        for _ in range(T):
            xa = one()
            xa1 = one()
            row.append((xa, xa1, diag and random.randint(1, 1000) < 10))
        sched.append(row)
    return sched


def test_tasks_lockstep_tsf(agent, test_tasks: Sequence, indices: Sequence[int] = None, *, episodes_end=None,
                            sequential=None) -> List:
    """``[agent.test_agent(task, i) for i, task in enumerate(test_tasks)]`` of the TSF agents
    (agents/tsfdqn_sequential.py:385-420) with the episodes in lockstep.  ``agent`` is the user's
    TSFDQN over sfx's drop-in DeepTSF; ``agent.test_tasks_weights[i]`` = (w_approx, optim,
    scheduler) and ``agent.omegas[i]`` as the reference's train builds them (:320-348).  w_approx
    and ω are updated in place, the Adam moments kept where the per-call binding keeps them
    (``sf._test_state``); returns the E returns.  More test tasks than the engine's max_batch run
    as consecutive lockstep groups (the draws are taken for all of them first).  As for
    ``test_tasks_lockstep``, lockstep runs only when ``fixed_horizon(test_tasks, episodes_end)``
    holds; otherwise the sequential loop (``sequential``, default ``agent.test_agent``) runs."""
    E = len(test_tasks)
    if E == 0:
        return []
    idx = list(range(E)) if indices is None else list(indices)
    if not fixed_horizon(test_tasks, episodes_end):
        seq = sequential or agent.test_agent
        return [seq(task, i) for i, task in zip(idx, test_tasks)]
    sf = agent.sf
    eng = sf._engine(1)
    sf._flush()
    sync = getattr(sf, "sync_tsf_modules", None)  # what the bound test_agent does first
    if sync is not None:
        sync()
    if getattr(agent, "h_function", None) is None:
        raise Exception('Affine Function (h) is not initialized')
    entries = [agent.test_tasks_weights[i] for i in idx]
    omegas = [agent.omegas[i] for i in idx]
    for _, optim, _ in entries:
        for grp in optim.param_groups[:2]:
            if tuple(grp.get("betas", (0.9, 0.999))) != (0.9, 0.999) or grp.get("eps", 1e-8) != 1e-8:
                raise NotImplementedError("sfx: the test reward mapper's Adam runs with betas (0.9, 0.999), eps 1e-8")
    T = int(agent.T)
    sched = _tsf_draw_schedule(E, T, float(agent.test_epsilon), int(agent.n_actions),
                               agent.total_training_steps % 1000 == 0)
    R, Lh = [], []
    cap = int(eng.max_batch)
    for e0 in range(0, E, cap):
        sl = slice(e0, min(E, e0 + cap))
        r_, l_ = _tsf_group(agent, eng, test_tasks[sl], entries[sl], omegas[sl], sched[sl], idx[sl])
        R += r_
        Lh += l_
    hp = agent.hyperparameters
    if agent.total_training_steps % 5000 == 0:
        for e in range(E):
            acc = [0, 0, 0]  # accum_loss, total_phi_loss (l2), total_psi_loss (l1): python sums of .item()
            for row in Lh[e]:
                for k in range(3):
                    acc[k] += row[k]
            agent.logger.log_target_error_progress(agent.get_target_reward_mapper_error(
                R[e], acc[0], acc[1], acc[2], idx[e], hp['beta_loss_coefficient'], T))
            agent.logger.log_omegas_learning_rate(entries[e][1].param_groups[1]['lr'], idx[e],
                                                  agent.total_training_steps)
    return R


def _tsf_group(agent, eng, test_tasks, entries, omegas, sched, idx):
    """One lockstep group of E <= max_batch TSF test tasks: (returns, per-task [steps][3] losses)."""
    from sfx.dropin.bind import prints_phi_shape

    sf, E, T = agent.sf, len(test_tasks), int(agent.T)
    dev, d, nt = eng.device, int(sf.n_features), int(sf.n_tasks)
    phi_line = prints_phi_shape(agent)
    hp = agent.hyperparameters
    beta, lasso, gamma = hp['beta_loss_coefficient'], hp['omegas_l1_coefficient'], agent.gamma
    W = torch.stack([w.weight.detach().reshape(-1).to(dev, torch.float32) for w, _, _ in entries]).contiguous()
    Om = torch.stack([o.detach().reshape(-1).to(dev, torch.float32) for o in omegas]).contiguous()
    states = []
    for o in omegas:
        st = sf._test_state.get(o)
        if st is None:
            st = sf._test_state[o] = [torch.zeros(2 * (d + nt), device=dev), 0]
        states.append(st)
    M = torch.stack([st[0] for st in states]).contiguous()
    L = torch.zeros(T, E, 3, device=dev)
    adev = getattr(agent, "device", None) or sf._out_device()

    def write_back(rows):
        with torch.no_grad():
            for e in rows:
                w = entries[e][0].weight
                w.copy_(W[e].view_as(w))
                omegas[e].copy_(Om[e].view_as(omegas[e]))
                states[e][0].copy_(M[e])

    s_enc = [agent.encoding(task.initialize()) for task in test_tasks]
    R = [0.0] * E
    steps = [0] * E
    live = list(range(E))  # all of them unless a declared-endless episode ends
    for j in range(T):
        part = len(live) < E
        lr_ = torch.tensor(live, device=dev) if part else None
        Wl, Oml, Ml = (W[lr_].contiguous(), Om[lr_].contiguous(), M[lr_].contiguous()) if part else (W, Om, M)
        S = torch.cat([torch.as_tensor(s_enc[e]).to(dev, torch.float32).reshape(1, -1) for e in live])
        greedy = eng.tsf_test_actions(S, Wl, Oml).to(adev).unbind()
        acts, s1_enc, phis, rows, ended, shapes = [], {}, [], [], [], []
        for k, e in enumerate(live):
            task = test_tasks[e]
            xa = sched[e][j][0]
            a = torch.tensor(xa).to(adev) if xa >= 0 else greedy[k]
            s1, r, done = task.transition(a)
            s1e = agent.encoding(s1)
            phi = torch.as_tensor(task.features(s_enc[e], a, s1e))
            shapes.append(phi.shape)
            phis.append(phi.to(dev, torch.float32).reshape(1, -1))
            acts.append(a.reshape(()).to(dev, torch.long))
            s1_enc[e] = s1e
            states[e][1] += 1
            steps[e] += 1
            gw, go = entries[e][1].param_groups[0], entries[e][1].param_groups[1]
            rows.append([float(r), gw['lr'], gw['weight_decay'], go['lr'], go['weight_decay'], float(states[e][1])])
            R[e] += r
            if done and j + 1 < T:
                _warn_ended(idx[e], j + 1, T)
                ended.append(e)
        S1 = torch.cat([torch.as_tensor(s1_enc[e]).to(dev, torch.float32).reshape(1, -1) for e in live])
        A1 = eng.tsf_test_actions(S1, Wl, Oml)
        ex = [(k, sched[e][j][1]) for k, e in enumerate(live) if sched[e][j][1] >= 0]
        if ex:
            A1[[k for k, _ in ex]] = torch.tensor([x for _, x in ex], dtype=torch.long).to(dev)
        rowp = torch.tensor(rows, dtype=torch.float32).to(dev)
        Lj = eng.tsf_test_updates(S, S1, torch.stack(acts), A1, torch.cat(phis), Wl, Oml, Ml, rowp, gamma, beta,
                                  lasso, losses=None if part else L[j])
        if part:
            W[lr_], Om[lr_], M[lr_], L[j, lr_] = Wl, Oml, Ml, Lj
        if phi_line:  # agents/tsfdqn_sequential.py:443, once per task and step (bind.prints_phi_shape)
            for shp in shapes:
                print(f'Phi values {shp}')
        printed = [e for e in live if sched[e][j][2]]
        if printed:  # the binding's diagnostic print (bind.tsf_update_test_reward_mapper)
            write_back(printed)
            for e in printed:
                print(f'Target Task {test_tasks[e]} omegas {omegas[e].detach()} weights {entries[e][0].weight.detach()}')
        for e in live:
            entries[e][2].step()
        s_enc = [s1_enc.get(e, s_enc[e]) for e in range(E)]
        live = [e for e in live if e not in ended]
        if not live:
            break
    write_back(range(E))
    Lh = L.cpu().tolist()  # one device read for the group's losses
    return R, [[Lh[j][e] for j in range(steps[e])] for e in range(E)]


def enable(agent, episodes_end=None) -> None:
    """Bind lockstep test rollouts into an SFDQN or TSFDQN instance without touching its code: ``train``
    records its ``test_tasks``; the first ``test_agent`` call of a test phase (test_index 0) runs
    all of them in lockstep and the later calls of that phase return the stored returns, so the
    reference's loop (agents/sfdqn.py:111-120) sees the same values in the same order.  A
    ``test_agent`` call outside that pattern runs its one task alone (E = 1, sequential
    semantics).  ``episodes_end`` is passed to ``fixed_horizon``: phases whose episodes may end
    early run the agent's own sequential ``test_agent``."""
    train, state = agent.train, {"tasks": None, "R": None}
    own = agent.test_agent  # the user's sequential loop: the fallback
    # the TSF agents (test_tasks_weights of (w_approx, optim, scheduler) and per-task ω) or SFDQN
    rollout = test_tasks_lockstep_tsf if hasattr(agent, "omegas") else test_tasks_lockstep

    def train_recording(*args, **kwargs):
        tasks = kwargs.get("test_tasks", args[4] if len(args) > 4 else [])
        state["tasks"], state["R"] = list(tasks), None
        return train(*args, **kwargs)

    def test_agent(task, test_index):
        tasks = state["tasks"]
        if tasks and test_index < len(tasks) and tasks[test_index] is task:
            if test_index == 0 or state["R"] is None:
                state["R"] = rollout(agent, tasks, episodes_end=episodes_end, sequential=own)
            return state["R"][test_index]
        return rollout(agent, [task], [test_index], episodes_end=episodes_end, sequential=own)[0]

    agent.train = train_recording
    agent.test_agent = test_agent
