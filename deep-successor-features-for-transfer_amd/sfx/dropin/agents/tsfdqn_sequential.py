"""Transformed-SF agent over a DeepTSF library (the interface of agents/tsfdqn_sequential.py:12-531,
main_tsfdqn_sequential_torch.py).

One replay buffer per training task; per task a g_i = nn.Linear(n_s, G) and one shared
h = nn.Linear(G, d) (handed to the library, which trains them on the device); each env step
runs ONE ``update_successor`` on the active task -- GPI next actions, φ̃ = (h(g_i(s)) +
h(g_i(s'))) ⊙ φ, TD target on φ̃, loss l1 + β l2 and the Adam step over {ψ_i, w_i, g_i, h}, all
in one libsfx call (features.deep_sequential_tsf.DeepTSF.tsf_update).

Test tasks keep the reference's ω-weighted transfer (agents/tsfdqn_sequential.py:369-508): the
action is argmax_a w(Σ_t ω̂_t ψ_t(s)) with ψ from the device (one B=1 launch), and {w, ω} are
trained by Adam (with the ω learning-rate schedule) in torch on the configured device -- a
handful of parameters, using the g_i / h the device trained (synced before each test episode).
"""
from __future__ import annotations

import random

import torch

from agents.agent import Agent
from utils.logger import get_logger_level, set_logger_level
from utils.torch import get_torch_device


class TSFDQN(Agent):
    def __init__(self, deep_sf, buffer_handle, *args, use_gpi=True, test_epsilon=0.03, **kwargs):
        super().__init__(*args, **kwargs)
        self.sf = deep_sf
        self.buffer_handle = buffer_handle
        self.use_gpi = use_gpi
        self.test_epsilon = test_epsilon
        self.hyperparameters = kwargs.get("hyperparameters", {})
        self.logger = get_logger_level() or set_logger_level(False, quiet=True)
        self.device = get_torch_device()
        self.test_tasks_weights = []
        self.buffers = []
        self.omegas_per_source_task = []
        self.omegas = []
        self.g_functions = []
        self.h_function = None

    def set_active_training_task(self, index):
        super().set_active_training_task(index)
        self.buffer = self.buffers[index]
        self.active_g_function = self.g_functions[index]

    def get_Q_values(self, s, s_enc):
        with torch.no_grad():
            q, c = self.sf.GPI(s_enc, self.task_index, update_counters=self.use_gpi)
            if not self.use_gpi:
                c = self.task_index
            self.c = c
            return q[:, c, :]

    # built on the CPU and moved: their init draws come from the CPU generator, as in a CPU run
    def _init_g_function(self, states_dim, output_dim):
        return torch.nn.Linear(states_dim, output_dim, bias=True).to(self.device)

    def _init_h_function(self, input_dim, features_dim):
        return torch.nn.Linear(input_dim, features_dim, bias=True).to(self.device)

    def _init_omega(self, num_source_tasks):
        return torch.Tensor(1, num_source_tasks, 1, 1).uniform_(0, 1).to(self.device).requires_grad_(True)

    def train_agent(self, s, s_enc, a, r, s1, s1_enc, gamma):
        phi = self.phi(s, a, s1)
        self.buffer.append(s_enc, a, r, phi, s1_enc, gamma)
        transitions = self.buffer.replay()
        losses = self.update_successor(transitions, self.task_index, self.use_gpi)
        if isinstance(losses, tuple):
            total_loss, psi_loss, phi_loss = losses
            self.logger.log_losses(total_loss.item(), psi_loss.item(), phi_loss.item(),
                                   [self.hyperparameters["beta_loss_coefficient"]], self.total_training_steps)
        if self.total_training_steps % 1000 == 0:
            print(f"Current task {self.task_index} Reward Mapper {self.sf.fit_w[self.task_index].weight}")
            print(f"Current omegas {self.task_index} OMEGAS Weights {self.omegas}")

    def update_successor(self, transitions, policy_index, use_gpi=True):
        if transitions is None:
            return
        if self.h_function is None:
            raise Exception("Affine Function (h) is not initialized")
        return self.sf.tsf_update(transitions, policy_index, use_gpi,
                                  beta=self.hyperparameters["beta_loss_coefficient"])

    def reset(self):
        super().reset()
        self.sf.reset()
        for buffer in self.buffers:
            buffer.reset()

    def add_training_task(self, task):
        super().add_training_task(task)
        self.buffers.append(self.buffer_handle())
        dims = self.hyperparameters.get("g_h_function_dims")
        g_function = self._init_g_function(task.encode_dim(), dims)
        self.g_functions.append(g_function)
        if self.h_function is None:
            self.h_function = self._init_h_function(dims, task.feature_dim())
        self.sf.add_training_task(task, None, g_function, self.h_function)

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
        omegas0 = self._init_omega(len(train_tasks))
        with torch.no_grad():
            omegas0 = omegas0 / torch.sum(omegas0, axis=1, keepdim=True)
        omegas0 = omegas0.clone().detach().requires_grad_(True)
        for test_task in test_tasks:
            omegas_target_task = omegas0.clone().detach().requires_grad_(True)
            fit_w = torch.Tensor(1, test_task.feature_dim()).uniform_(-0.01, 0.01).to(self.device)
            w_approx = torch.nn.Linear(test_task.feature_dim(), 1, bias=False).to(self.device)  # CPU init draw
            with torch.no_grad():
                w_approx.weight = torch.nn.Parameter(fit_w)
            optim = torch.optim.Adam([
                {"params": w_approx.parameters(), "lr": hp["learning_rate_w"], "weight_decay": hp["weight_decay_w"]},
                {"params": omegas_target_task, "lr": hp["learning_rate_omega"],
                 "weight_decay": hp["weight_decay_omega"]},
            ])
            decay = hp["learning_rate_omega_decay"]
            scheduler = torch.optim.lr_scheduler.LambdaLR(optim, [lambda epoch: 1 ** epoch,
                                                                  lambda epoch: (1 - decay) ** epoch])
            self.test_tasks_weights.append((w_approx, optim, scheduler))
            self.omegas.append(omegas_target_task)
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

    # ---- test tasks (agents/tsfdqn_sequential.py:369-508)
    def get_test_action(self, s_enc, w, omegas):
        with torch.no_grad():
            if random.random() <= self.test_epsilon:
                return torch.tensor(random.randrange(self.n_actions)).to(self.device)
            normalized = omegas / torch.sum(omegas, axis=1, keepdim=True)
            tsf = torch.sum(self.sf.get_successors(s_enc) * normalized, axis=1)
            return torch.argmax(w(tsf))

    def test_agent(self, task, test_index):
        self.sf.sync_tsf_modules()
        R = 0.0
        w, optim, scheduler = self.test_tasks_weights[test_index]
        omegas = self.omegas[test_index]
        s = task.initialize()
        s_enc = self.encoding(s)
        accum_loss = total_phi_loss = total_psi_loss = 0
        for _ in range(self.T):
            a = self.get_test_action(s_enc, w, omegas)
            s1, r, done = task.transition(a)
            s1_enc = self.encoding(s1)
            a1 = self.get_test_action(s1_enc, w, omegas)
            loss_t, phi_loss, psi_loss = self.update_test_reward_mapper(w, omegas, optim, task, r, s_enc, a, s1_enc, a1)
            accum_loss += loss_t.item()
            total_phi_loss += phi_loss.item()
            total_psi_loss += psi_loss.item()
            scheduler.step()
            s, s_enc = s1, s1_enc
            R += r
            if done:
                break
        if self.total_training_steps % 5000 == 0:
            beta = self.hyperparameters["beta_loss_coefficient"]
            self.logger.log_target_error_progress(self.get_target_reward_mapper_error(
                R, accum_loss, total_phi_loss, total_psi_loss, test_index, beta, self.T))
            self.logger.log_omegas_learning_rate(optim.param_groups[1]["lr"], test_index, self.total_training_steps)
        self.omegas[test_index] = omegas
        return R

    def update_test_reward_mapper(self, w_approx, omegas, optim, task, r, s, a, s1, a1):
        if self.h_function is None:
            raise Exception("Affine Function (h) is not initialized")
        phi = task.features(s, a, s1)
        self.h_function.eval()
        normalized = omegas / torch.sum(omegas, axis=1, keepdim=True)
        with torch.no_grad():
            t_states = torch.vstack([g(s) for g in self.g_functions]).unsqueeze(1)
            t_next_states = torch.vstack([g(s1) for g in self.g_functions]).unsqueeze(1)
        weighted_states = torch.sum(t_states * normalized, axis=1)
        weighted_next_states = torch.sum(t_next_states * normalized, axis=1)
        affine_states = self.h_function(weighted_states) + self.h_function(weighted_next_states)
        transformed_phi = phi * affine_states.squeeze(0)
        with torch.no_grad():
            successor_features = self.sf.get_successors(s)
            next_successor_features = self.sf.get_next_successors(s1)
            r_tensor = torch.as_tensor(r).detach().float().reshape(1).to(self.device)
        next_tsf = transformed_phi + self.gamma * torch.sum(next_successor_features * normalized, axis=1)[:, a1, :]
        tsf = torch.sum(successor_features * normalized, axis=1)[:, a, :]
        loss_task = torch.nn.MSELoss()
        r_fit = w_approx(transformed_phi)
        beta = torch.tensor(self.hyperparameters["beta_loss_coefficient"])
        lasso = torch.tensor(self.hyperparameters["omegas_l1_coefficient"])
        l1 = loss_task(tsf, next_tsf)
        l2 = loss_task(r_fit, r_tensor)
        loss = l1 + beta * l2 + lasso * torch.norm(omegas, 1)
        optim.zero_grad()
        loss.backward()
        optim.step()
        with torch.no_grad():
            omegas.clamp_(1e-7)
        # the reference's occasional diagnostics draw from Python's RNG: same draw, same stream
        if self.total_training_steps % 1000 == 0 and random.randint(1, 1000) < 10:
            print(f"Target Task {task} Omegas Gradients {omegas.grad}")
            print(f"Target Task {task} Weights {w_approx.weight}")
        self.h_function.train()
        return loss, l2, l1

    def get_target_reward_mapper_error(self, r, loss, phi_loss, psi_loss, task_index, target_loss_coefficient, ts):
        return {"task": task_index, "reward": r, "steps": 500 * (self.total_training_steps // 1000) + ts,
                "w_error": loss, "psi_loss": psi_loss, "phi_loss": phi_loss,
                "target_loss_coefficient": target_loss_coefficient}
