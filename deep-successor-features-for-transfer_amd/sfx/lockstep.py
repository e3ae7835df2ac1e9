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
actions (row e under its own w), the E envs step, and the E reward models are fitted by the
user's own ``update_test_reward_mapper`` -- the same arithmetic, the same draws, the same
actions, the same returns and log lines in the same order as the sequential loop, with one GPU
round trip per step instead of E.

Preconditions: each test task owns its env and its random state (tasks/reacher.py: one bullet
env with its own ``np_random`` per task), since the lockstep order interleaves the tasks' env calls;
and episodes run the full ``agent.T`` steps (tasks/reacher.py:112 never ends one) -- an episode that
ended early would have shifted every later task's draws, so the rollout raises.

The TSF agents' test phase (agents/tsfdqn_sequential.py:385-420, tsfdqn.py / tsfdqn_nf.py
test_agent) runs in lockstep too (``test_tasks_lockstep_tsf``): each step draws twice (the action
at s and the next action a1 at s1, both under the pre-update w and ω) and, when
``total_training_steps % 1000 == 0``, the reward mapper's ``random.randint`` of its diagnostic
print -- all independent of the GPU, so again taken up front in the reference's order.  Per step:
one ``sfx_tsf_test_actions`` launch set for the E actions at s, the E env steps, one for the E
actions at s1, one ``sfx_tsf_test_updates`` launch set fitting the E (w, ω) pairs -- each task's
own Adam step number, LR (its LambdaLR keeps decaying ω's) and r read per row -- then each task's
scheduler steps.  The E losses of every step stay on the device until the phase ends (the
reference's ``loss.item()`` per step is one device read per task and step).
"""
from __future__ import annotations

import random
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


def test_tasks_lockstep(agent, test_tasks: Sequence, indices: Sequence[int] = None) -> List:
    """``[agent.test_agent(task, i) for i, task in enumerate(test_tasks)]`` of agents/sfdqn.py
    (or of the single-file sfdqn.py, :665-721) with the episodes in lockstep.  ``agent`` is the user's SFDQN over ``sfx``'s drop-in
    ``DeepSF`` (``agent.sf``); returns the E returns R (as test_agent does)."""
    E = len(test_tasks)
    if E == 0:
        return []
    idx = list(range(E)) if indices is None else list(indices)
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
    adev = getattr(agent, "device", None) or sf._out_device()
    s_enc = [agent.encoding(task.initialize()) for task in test_tasks]
    R = [0.0] * E
    acc = [0] * E
    for j in range(T):
        S = torch.cat([torch.as_tensor(s).to(dev, torch.float32).reshape(1, -1) for s in s_enc])
        W = torch.cat([w.weight.detach().to(dev, torch.float32).reshape(1, -1) for w in ws])
        greedy = eng.test_actions(S, W)[:, 1].unbind()
        losses = []
        for e, task in enumerate(test_tasks):
            x = sched[e][j]
            a = torch.tensor(x).to(adev) if x >= 0 else greedy[e]
            s1, r, done = task.transition(a)
            s1_enc = agent.encoding(s1)
            if paired:
                loss = agent.update_test_reward_mapper(ws[e], entries[e][1], task, r, s_enc[e], a, s1_enc)
            else:
                loss = agent.update_test_reward_mapper(ws[e], task, r, s_enc[e], a, s1_enc)
            losses.append(loss)
            s_enc[e] = s1_enc
            R[e] += r
            if done and j + 1 < T:
                raise RuntimeError("lockstep test rollouts need full-length episodes: test task "
                                   f"{idx[e]} ended at step {j + 1} of {T}")
        for e, v in enumerate(torch.stack([l.detach().reshape(()) for l in losses]).tolist()):
            acc[e] += v
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


def test_tasks_lockstep_tsf(agent, test_tasks: Sequence, indices: Sequence[int] = None) -> List:
    """``[agent.test_agent(task, i) for i, task in enumerate(test_tasks)]`` of the TSF agents
    (agents/tsfdqn_sequential.py:385-420) with the episodes in lockstep.  ``agent`` is the user's
    TSFDQN over sfx's drop-in DeepTSF; ``agent.test_tasks_weights[i]`` = (w_approx, optim,
    scheduler) and ``agent.omegas[i]`` as the reference's train builds them (:320-348).  w_approx
    and ω are updated in place, the Adam moments kept where the per-call binding keeps them
    (``sf._test_state``); returns the E returns.  More test tasks than the engine's max_batch run
    as consecutive lockstep groups (the draws are taken for all of them first)."""
    E = len(test_tasks)
    if E == 0:
        return []
    idx = list(range(E)) if indices is None else list(indices)
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
        r_, l_ = _tsf_group(agent, eng, test_tasks[sl], entries[sl], omegas[sl], sched[sl])
        R += r_
        Lh += l_
    hp = agent.hyperparameters
    if agent.total_training_steps % 5000 == 0:
        for e in range(E):
            acc = [0, 0, 0]  # accum_loss, total_phi_loss (l2), total_psi_loss (l1): python sums of .item()
            for j in range(T):
                for k in range(3):
                    acc[k] += Lh[e][j][k]
            agent.logger.log_target_error_progress(agent.get_target_reward_mapper_error(
                R[e], acc[0], acc[1], acc[2], idx[e], hp['beta_loss_coefficient'], T))
            agent.logger.log_omegas_learning_rate(entries[e][1].param_groups[1]['lr'], idx[e],
                                                  agent.total_training_steps)
    return R


def _tsf_group(agent, eng, test_tasks, entries, omegas, sched):
    """One lockstep group of E <= max_batch TSF test tasks: (returns, per-task [T][3] losses)."""
    sf, E, T = agent.sf, len(test_tasks), int(agent.T)
    dev, d, nt = eng.device, int(sf.n_features), int(sf.n_tasks)
    hp = agent.hyperparameters
    beta, lasso, gamma = hp['beta_loss_coefficient'], hp['omegas_l1_coefficient'], agent.gamma
    W = torch.stack([w.weight.detach().reshape(-1).to(dev, torch.float32) for w, _, _ in entries]).contiguous()
    Om = torch.stack([o.detach().reshape(-1).to(dev, torch.float32) for o in omegas]).contiguous()
    states = []
    for o in omegas:
        st = sf._test_state.get(id(o))
        if st is None:
            st = sf._test_state[id(o)] = [torch.zeros(2 * (d + nt), device=dev), 0]
        states.append(st)
    M = torch.stack([st[0] for st in states]).contiguous()
    L = torch.empty(T, E, 3, device=dev)
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
    for j in range(T):
        S = torch.cat([torch.as_tensor(s).to(dev, torch.float32).reshape(1, -1) for s in s_enc])
        greedy = eng.tsf_test_actions(S, W, Om).to(adev).unbind()
        acts, s1_enc, phis, rows = [], [], [], []
        for e, task in enumerate(test_tasks):
            xa = sched[e][j][0]
            a = torch.tensor(xa).to(adev) if xa >= 0 else greedy[e]
            s1, r, done = task.transition(a)
            s1e = agent.encoding(s1)
            phis.append(torch.as_tensor(task.features(s_enc[e], a, s1e)).to(dev, torch.float32).reshape(1, -1))
            acts.append(a.reshape(()).to(dev, torch.long))
            s1_enc.append(s1e)
            states[e][1] += 1
            gw, go = entries[e][1].param_groups[0], entries[e][1].param_groups[1]
            rows.append([float(r), gw['lr'], gw['weight_decay'], go['lr'], go['weight_decay'], float(states[e][1])])
            R[e] += r
            if done and j + 1 < T:
                raise RuntimeError("lockstep test rollouts need full-length episodes: a test task ended at "
                                   f"step {j + 1} of {T}")
        S1 = torch.cat([torch.as_tensor(s).to(dev, torch.float32).reshape(1, -1) for s in s1_enc])
        A1 = eng.tsf_test_actions(S1, W, Om)
        ex = [(e, sched[e][j][1]) for e in range(E) if sched[e][j][1] >= 0]
        if ex:
            A1[[e for e, _ in ex]] = torch.tensor([x for _, x in ex], dtype=torch.long).to(dev)
        rowp = torch.tensor(rows, dtype=torch.float32).to(dev)
        eng.tsf_test_updates(S, S1, torch.stack(acts), A1, torch.cat(phis), W, Om, M, rowp, gamma, beta, lasso,
                             losses=L[j])
        printed = [e for e in range(E) if sched[e][j][2]]
        if printed:  # the binding's diagnostic print (bind.tsf_update_test_reward_mapper)
            write_back(printed)
            for e in printed:
                print(f'Target Task {test_tasks[e]} omegas {omegas[e].detach()} weights {entries[e][0].weight.detach()}')
        for _, _, scheduler in entries:
            scheduler.step()
        s_enc = s1_enc
    write_back(range(E))
    Lh = L.cpu().tolist()  # one device read for the group's losses
    return R, [[Lh[j][e] for j in range(T)] for e in range(E)]


def enable(agent) -> None:
    """Bind lockstep test rollouts into an SFDQN or TSFDQN instance without touching its code: ``train``
    records its ``test_tasks``; the first ``test_agent`` call of a test phase (test_index 0) runs
    all of them in lockstep and the later calls of that phase return the stored returns, so the
    reference's loop (agents/sfdqn.py:111-120) sees the same values in the same order.  A
    ``test_agent`` call outside that pattern runs its one task alone (E = 1, sequential
    semantics)."""
    train, state = agent.train, {"tasks": None, "R": None}
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
                state["R"] = rollout(agent, tasks)
            return state["R"][test_index]
        return rollout(agent, [task], [test_index])[0]

    agent.train = train_recording
    agent.test_agent = test_agent
