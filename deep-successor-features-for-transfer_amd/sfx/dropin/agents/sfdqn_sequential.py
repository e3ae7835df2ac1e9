"""Sequential SFDQN agent over a DeepSF library (the interface of agents/sfdqn_sequential.py:11-245,
main_sfdqn_sequential_torch.py).

One replay buffer per training task (``buffer_handle()``); each env step appends
(s, a, r, φ, s', γ) to the active task's buffer and runs ONE ``update_successor`` on the active
task (l1 + l2 with the Adam-trained reward model, features.deep_sequential -> libsfx).  Test
tasks (agents/sfdqn_sequential.py:177-234, the same as sfdqn.py:681-738): actions by GPI over the
source heads with the test task's own reward model ``w`` (one B=1 GPI launch in libsfx), and
``w`` trained by Adam on the observed rewards (d parameters, torch on the configured device).
"""
from __future__ import annotations

import random

import torch

from agents.agent import Agent
from utils.logger import get_logger_level, set_logger_level
from utils.torch import get_torch_device


class SFDQN(Agent):
    def __init__(self, deep_sf, buffer_handle, *args, use_gpi=True, test_epsilon=0.03, **kwargs):
        super().__init__(*args, **kwargs)
        self.sf = deep_sf
        self.buffer_handle = buffer_handle
        self.use_gpi = use_gpi
        self.test_epsilon = test_epsilon
        self.logger = get_logger_level() or set_logger_level(False, quiet=True)
        self.device = get_torch_device()
        self.test_tasks_weights = []
        self.hyperparameters = kwargs.get("hyperparameters", {})
        self.buffers = []

    def set_active_training_task(self, index):
        super().set_active_training_task(index)
        self.buffer = self.buffers[index]

    def get_Q_values(self, s, s_enc):
        with torch.no_grad():
            q, c = self.sf.GPI(s_enc, self.task_index, update_counters=self.use_gpi)
            if not self.use_gpi:
                c = self.task_index
            self.c = c
            return q[:, c, :]

    def train_agent(self, s, s_enc, a, r, s1, s1_enc, gamma):
        phi = self.phi(s, a, s1)
        self.buffer.append(s_enc, a, r, phi, s1_enc, gamma)
        transitions = self.buffer.replay()
        losses = self.sf.update_successor(transitions, self.task_index, self.use_gpi)
        if isinstance(losses, tuple):
            total_loss, psi_loss, phi_loss = losses
            self.logger.log_losses(total_loss.item(), psi_loss.item(), phi_loss.item(), [1], self.total_training_steps)
        if self.total_training_steps % 1000 == 0:
            print(f"Current task {self.task_index} Reward Mapper {self.sf.fit_w[self.task_index].weight}")

    def reset(self):
        super().reset()
        self.sf.reset()
        for buffer in self.buffers:
            buffer.reset()

    def add_training_task(self, task):
        super().add_training_task(task)
        self.sf.add_training_task(task, source=None)
        self.buffers.append(self.buffer_handle())

    def get_progress_dict(self):
        gpi = self.sf.GPI_usage_percent(self.task_index)
        w_err = torch.linalg.norm(self.sf.fit_w[self.task_index].weight.T - self.sf.true_w[self.task_index])
        return {"task": self.task_index, "steps": self.total_training_steps, "episodes": self.episode,
                "eps": self.epsilon, "ep_reward": self.episode_reward, "reward": self.reward,
                "reward_hist": self.reward_hist, "cum_reward": self.cum_reward,
                "cum_reward_hist": self.cum_reward_hist, "GPI%": gpi, "w_err": w_err}

    def get_progress_strings(self):
        sample, reward = super().get_progress_strings()
        gpi = self.sf.GPI_usage_percent(self.task_index)
        w_err = torch.linalg.norm(self.sf.fit_w[self.task_index].weight.T - self.sf.true_w[self.task_index])
        return sample, reward, "GPI% \t {:.4f} \t w_err \t {:.4f}".format(gpi, w_err)

    def train(self, train_tasks, n_samples, viewers=None, n_view_ev=None, test_tasks=[], n_test_ev=1000,
              cycles_per_task=1):
        viewers = [None] * len(train_tasks) if viewers is None else viewers
        self.reset()
        for task in train_tasks:
            self.add_training_task(task)
        hp = self.hyperparameters
        for test_task in test_tasks:
            fit_w = torch.Tensor(1, test_task.feature_dim()).uniform_(-0.01, 0.01).to(self.device)
            # CPU init draw (see features.deep_sequential.add_training_task)
            w_approx = torch.nn.Linear(test_task.feature_dim(), 1, bias=False).to(self.device)
            with torch.no_grad():
                w_approx.weight = torch.nn.Parameter(fit_w)
            optim = torch.optim.Adam([{"params": w_approx.parameters(), "lr": hp["learning_rate_w"],
                                       "weight_decay": hp["weight_decay_w"]}])
            self.test_tasks_weights.append((w_approx, optim))
        returns = []
        for _ in range(cycles_per_task):
            for index, (task, viewer) in enumerate(zip(train_tasks, viewers)):
                self.set_active_training_task(index)
                for t in range(n_samples):
                    self.next_sample(viewer, n_view_ev)
                    if t % n_test_ev == 0:
                        Rs = [self.test_agent(tt, ti) for ti, tt in enumerate(test_tasks)]
                        avg = torch.mean(torch.Tensor(Rs).to(self.device))
                        returns.append(avg)
                        self.logger.log_progress(self.get_progress_dict())
                        self.logger.log_average_reward(avg, self.total_training_steps)
                        self.logger.log_accumulative_reward(torch.sum(torch.Tensor(returns).to(self.device)),
                                                            self.total_training_steps)
                    self.total_training_steps += 1
        return returns

    # ---- test tasks (agents/sfdqn_sequential.py:177-245)
    def get_test_action(self, s_enc, w):
        with torch.no_grad():
            if random.random() <= self.test_epsilon:
                return torch.tensor(random.randrange(self.n_actions)).to(self.device)
            q, c = self.sf.GPI_w(s_enc, w)
            return torch.argmax(q[:, c, :])

    def test_agent(self, task, test_index):
        R = 0.0
        w, optim = self.test_tasks_weights[test_index]
        s = task.initialize()
        s_enc = self.encoding(s)
        accum_loss = 0
        for _ in range(self.T):
            a = self.get_test_action(s_enc, w)
            s1, r, done = task.transition(a)
            s1_enc = self.encoding(s1)
            accum_loss += self.update_test_reward_mapper(w, optim, task, r, s_enc, a, s1_enc).item()
            s, s_enc = s1, s1_enc
            R += r
            if done:
                break
        self.logger.log_target_error_progress(self.get_target_reward_mapper_error(R, accum_loss, test_index, self.T))
        return R

    def update_test_reward_mapper(self, w_approx, optim, task, r, s, a, s1):
        phi = task.features(s, a, s1)
        r_t = torch.as_tensor(r).detach().float().reshape(1).to(self.device)
        optim.zero_grad()
        loss = torch.nn.MSELoss()(w_approx(phi), r_t)
        loss.backward()
        optim.step()
        return loss

    def get_target_reward_mapper_error(self, r, loss, task_index, ts):
        return {"task": task_index, "reward": r, "steps": 500 * (self.total_training_steps // 1000) + ts,
                "w_error": loss}
