"""Episodic RL agent skeleton (the interface and loop of agents/agent.py:8-307).

``next_sample`` is one env step: Q-values of the current state, ε-greedy action (Python
``random``, as the reference), env transition, ``train_agent``, episode bookkeeping.
"""
from __future__ import annotations

import random

import torch

import utils.torch as _ut


class Agent:
    def __init__(self, gamma, T, encoding, *args, epsilon=0.1, epsilon_decay=1.0, epsilon_min=0.0,
                 print_ev=1000, save_ev=100, **kwargs):
        self.gamma = gamma
        self.T = T
        self.encoding = (lambda s: s) if encoding is None else encoding
        self.epsilon_init = epsilon
        self.epsilon_decay = epsilon_decay
        self.epsilon_min = epsilon_min
        self.print_ev = print_ev
        self.save_ev = save_ev
        self.total_training_steps = 0
        self.sf = None
        if args or kwargs:
            print(f"{type(self).__name__} ignoring parameters {args} and {kwargs}")

    def get_Q_values(self, s, s_enc):
        raise NotImplementedError

    def train_agent(self, s, s_enc, a, r, s1, s1_enc, gamma):
        raise NotImplementedError

    # ---- tasks (agents/agent.py:96-139)
    def reset(self):
        self.tasks = []
        self.phis = []
        self.cum_reward = 0.0
        self.reward_hist = []
        self.cum_reward_hist = []

    def add_training_task(self, task):
        self.tasks.append(task)
        self.n_tasks = len(self.tasks)
        self.phis.append(task.features)
        if self.n_tasks == 1:
            self.n_actions = task.action_count()
            self.n_features = task.feature_dim()
            if self.encoding == "task":
                self.encoding = task.encode

    def set_active_training_task(self, index):
        self.task_index = index
        self.active_task = self.tasks[index]
        self.phi = self.phis[index]
        self.s = self.s_enc = None
        self.new_episode = True
        self.episode, self.episode_reward = 0, 0.0
        self.steps_since_last_episode, self.reward_since_last_episode = 0, 0.0
        self.steps, self.reward = 0, 0.0
        self.epsilon = self.epsilon_init
        self.episode_reward_hist = []

    # ---- acting (agents/agent.py:144-157)
    def _epsilon_greedy(self, q):
        q = q.flatten()
        assert q.size()[0] == self.n_actions
        if random.random() <= self.epsilon:
            a = torch.tensor(random.randrange(self.n_actions)).to(_ut.device)
        else:
            a = torch.argmax(q)
        self.epsilon = max(self.epsilon * self.epsilon_decay, self.epsilon_min)
        return a

    def get_progress_strings(self):
        sample = "task \t {} \t steps \t {} \t episodes \t {} \t eps \t {:.4f}".format(
            self.task_index, self.steps, self.episode, self.epsilon)
        reward = "ep_reward \t {:.4f} \t reward \t {:.4f}".format(self.episode_reward, self.reward)
        return sample, reward

    def get_progress_dict(self):
        gpi = w_err = None
        if self.sf is not None:
            gpi = self.sf.GPI_usage_percent(self.task_index)
            w_err = torch.linalg.norm(self.sf.fit_w[self.task_index] - self.sf.true_w[self.task_index])
        return {"task": self.task_index, "steps": self.total_training_steps, "episodes": self.episode,
                "eps": self.epsilon, "ep_reward": self.episode_reward, "reward": self.reward,
                "reward_hist": self.reward_hist, "cum_reward": self.cum_reward,
                "cum_reward_hist": self.cum_reward_hist, "GPI%": gpi, "w_err": w_err}

    # ---- one env step (agents/agent.py:195-261)
    def _select_action(self):
        """Q-values of the current state (GPI), then ε-greedy (agents/agent.py:221-225)."""
        return self._epsilon_greedy(self.get_Q_values(self.s, self.s_enc))

    def next_sample(self, viewer=None, n_view_ev=None):
        if self.new_episode:
            self.s = self.active_task.initialize()
            self.s_enc = self.encoding(self.s)
            self.new_episode = False
            self.episode += 1
            self.steps_since_last_episode = 0
            self.episode_reward = self.reward_since_last_episode
            self.reward_since_last_episode = 0.0
            if self.episode > 1:
                self.episode_reward_hist.append(self.episode_reward)
        a = self._select_action()
        s1, r, terminal = self.active_task.transition(a)
        s1_enc = self.encoding(s1)
        gamma = 0.0 if terminal else self.gamma
        if terminal:
            self.new_episode = True
        self.train_agent(self.s, self.s_enc, a, r, s1, s1_enc, gamma)
        self.s, self.s_enc = s1, s1_enc
        self.steps += 1
        self.reward += r
        self.steps_since_last_episode += 1
        self.reward_since_last_episode += r
        self.cum_reward += r
        if self.steps_since_last_episode >= self.T:
            self.new_episode = True
        if self.steps % self.save_ev == 0:
            self.reward_hist.append(self.reward)
            self.cum_reward_hist.append(self.cum_reward)
        if viewer is not None and self.episode % n_view_ev == 0:
            viewer.update()

    def train_on_task(self, train_task, n_samples, viewer=None, n_view_ev=None):
        self.add_training_task(train_task)
        self.set_active_training_task(self.n_tasks - 1)
        for _ in range(n_samples):
            self.next_sample(viewer, n_view_ev)

    def train(self, train_tasks, n_samples, viewers=None, n_view_ev=None):
        viewers = [None] * len(train_tasks) if viewers is None else viewers
        self.reset()
        for task, viewer in zip(train_tasks, viewers):
            self.train_on_task(task, n_samples, viewer, n_view_ev)
