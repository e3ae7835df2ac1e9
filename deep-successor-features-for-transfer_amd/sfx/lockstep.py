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
ended early would have shifted every later task's draws, so the rollout raises.  The TSF agents'
test phase (two actions per step, an LR schedule, conditional logs) keeps the sequential loop over
the HIP test-task calls of ``sfx.dropin.bind``.
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


def enable(agent) -> None:
    """Bind lockstep test rollouts into an SFDQN instance without touching its code: ``train``
    records its ``test_tasks``; the first ``test_agent`` call of a test phase (test_index 0) runs
    all of them in lockstep and the later calls of that phase return the stored returns, so the
    reference's loop (agents/sfdqn.py:111-120) sees the same values in the same order.  A
    ``test_agent`` call outside that pattern runs its one task alone (E = 1, sequential
    semantics)."""
    train, state = agent.train, {"tasks": None, "R": None}

    def train_recording(*args, **kwargs):
        tasks = kwargs.get("test_tasks", args[4] if len(args) > 4 else [])
        state["tasks"], state["R"] = list(tasks), None
        return train(*args, **kwargs)

    def test_agent(task, test_index):
        tasks = state["tasks"]
        if tasks and test_index < len(tasks) and tasks[test_index] is task:
            if test_index == 0 or state["R"] is None:
                state["R"] = test_tasks_lockstep(agent, tasks)
            return state["R"][test_index]
        return test_tasks_lockstep(agent, [task], [test_index])[0]

    agent.train = train_recording
    agent.test_agent = test_agent
