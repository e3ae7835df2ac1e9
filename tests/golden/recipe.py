"""Shapes and the seed recipe behind the golden fixtures (our own code, data generation only).

Full-size (H=256) heads are too large to commit, so ``full_size_heads`` regenerates
them deterministically with torch's CPU RNG (torch 2.10.0 in this image, here and
on the GPU box); the fixture stores a checksum so a drift in the recipe is caught.
"""
from __future__ import annotations

import torch

# name: (n_s, H, A, d, hidden activations)
SHAPES = {
    "reacher17": (17, 32, 7, 8, ("relu", "relu")),        # BASELINE Reacher-shape, reduced H
    "reacher17_full": (17, 256, 7, 8, ("relu", "relu")),  # BASELINE C2 at full width
    "hopper11": (11, 24, 27, 50, ("relu", "relu")),       # BASELINE C3 shape, reduced H
    "cartpole": (4, 32, 2, 20, ("relu", "relu")),         # BASELINE C1 shape, reduced H
    "refreacher": (4, 64, 9, 12, ("relu", "relu")),       # tasks/reacher.py + reacher.cfg
    "tanh_odd": (6, 48, 5, 3, ("tanh", "relu")),          # odd sizes, tanh hidden
}


def head_modules(n_s, H, A, d, acts):
    act_cls = {"relu": torch.nn.ReLU, "tanh": torch.nn.Tanh}
    mods = [torch.nn.Linear(n_s, H)]
    for a in acts:
        mods += [torch.nn.Linear(H, H), act_cls[a]()]
    mods.append(torch.nn.Linear(H, A * d))
    return torch.nn.Sequential(*mods)


def full_size_heads(T: int = 8, seed: int = 0):
    """T heads of the Reacher-shape C2 network, torch default init under manual_seed(seed);
    w rows ~ U(-0.01, 0.01) as sfdqn.py:197."""
    n_s, H, A, d, acts = SHAPES["reacher17_full"]
    torch.manual_seed(seed)
    heads = []
    for _ in range(T):
        m = head_modules(n_s, H, A, d, acts)
        heads.append(torch.cat([p.detach().reshape(-1) for p in m.parameters()]))
    gen = torch.Generator().manual_seed(seed + 1)
    w = torch.empty(T, d).uniform_(-0.01, 0.01, generator=gen)
    return torch.stack(heads), w


# ---------------------------------------------------------------------------------------
# End-to-end agent run (agents/sfdqn.py SFDQN over features/deep.py DeepSF, the
# main_sfdqn_torch.py stack) -- generated with the real reference by tools/gen_golden.py,
# replayed on the GPU through sfx's drop-in modules by tests/test_gpu_dropin.py.
# ---------------------------------------------------------------------------------------
AGENT_RUN = dict(seed=7, n_s=17, H=32, A=7, d=8, acts=("relu", "relu"), T_tasks=3, lr=1e-3, alpha_w=0.05,
                 target_update_ev=6, n_samples=20, n_test_ev=10, episode_T=9, epsilon=0.2, gamma=0.9,
                 buffer=dict(n_samples=500, n_batch=8), task_terminal_every=7)


class AgentTask:
    """Reacher-shaped Task (tasks/task.py interface) with its own RNG; records its actions."""

    def __init__(self, n_s, A, d, index, seed, device, terminal_every=0, tensor_reward=False):
        import numpy as np

        self.n_s, self.A, self.d, self.index, self.device = n_s, A, d, index, device
        self.tensor_reward = tensor_reward  # tasks/reacher.py returns r as a 0-d tensor
        self.rng = np.random.default_rng(seed)
        self.terminal_every, self.t = terminal_every, 0
        self.actions, self._phi = [], None

    def initialize(self):
        import numpy as np

        return torch.from_numpy(self.rng.standard_normal(self.n_s).astype(np.float32)).to(self.device)

    def action_count(self):
        return self.A

    def transition(self, action):
        import numpy as np

        a = int(action)
        self.actions.append(a)
        self.t += 1
        s1 = torch.from_numpy(self.rng.standard_normal(self.n_s).astype(np.float32)).to(self.device)
        phi = (self.rng.random(self.d).astype(np.float32) + np.float32(0.05 * (a % 3))).astype(np.float32)
        self._phi = torch.from_numpy(phi).to(self.device)
        r = float(phi[self.index % self.d])
        done = bool(self.terminal_every) and self.t % self.terminal_every == 0
        if self.tensor_reward:
            r = torch.tensor(r).to(self.device)
        return s1, r, done

    def encode(self, state):
        return torch.as_tensor(state).detach().reshape((1, -1)).to(self.device)

    def encode_dim(self):
        return self.n_s

    def features(self, state, action, next_state):
        return self._phi

    def feature_dim(self):
        return self.d

    def get_w(self):
        w = torch.zeros((self.d, 1)).to(self.device)
        w[self.index % self.d, 0] = 1.0
        return w


def agent_psi_lambda(H, acts, lr, device):
    """ψ factory with the structure of main_sfdqn_torch.py:44-78 (our code)."""
    from collections import OrderedDict

    act_cls = {"relu": torch.nn.ReLU, "tanh": torch.nn.Tanh}

    def build(num_inputs, output_dim, reshape_dim, reshape_axis=1):
        layers = OrderedDict(layer_input=torch.nn.Linear(num_inputs, H))
        for j, a in enumerate(acts):
            layers[f"layer_{j}"] = torch.nn.Linear(H, H)
            layers[f"activation_layer_{j}"] = act_cls[a]()
        layers["layer_output"] = torch.nn.Linear(H, output_dim)
        layers["layer_unflatten"] = torch.nn.Unflatten(reshape_axis, reshape_dim)
        model = torch.nn.Sequential(layers).to(device)
        return model, torch.nn.MSELoss().to(device), torch.optim.Adam(model.parameters(), lr=lr)

    return build


def agent_run(DeepSF, SFDQN, ReplayBuffer, device):
    """Build and train the agent of AGENT_RUN with the given classes; returns (agent, tasks)."""
    import random

    import numpy as np

    c = AGENT_RUN
    random.seed(c["seed"])
    np.random.seed(c["seed"])
    torch.manual_seed(c["seed"])
    tasks = [AgentTask(c["n_s"], c["A"], c["d"], i, 100 + i, device, c["task_terminal_every"])
             for i in range(c["T_tasks"])]
    test_tasks = [AgentTask(c["n_s"], c["A"], c["d"], c["T_tasks"], 200, device)]
    sf = DeepSF(pytorch_model_handle=agent_psi_lambda(c["H"], c["acts"], c["lr"], device),
                target_update_ev=c["target_update_ev"], hyperparameters={"learning_rate_w": c["alpha_w"]})
    agent = SFDQN(deep_sf=sf, buffer=ReplayBuffer(**c["buffer"]), gamma=c["gamma"], T=c["episode_T"],
                  encoding="task", epsilon=c["epsilon"], use_gpi=True, test_epsilon=0.03)
    returns = agent.train(tasks, c["n_samples"], test_tasks=test_tasks, n_test_ev=c["n_test_ev"])
    return agent, tasks, test_tasks, returns


# The main_sfdqn_sequential_torch.py stack: agents/sfdqn_sequential.py SFDQN (one buffer per
# task, active-task updates, l1 + l2 with Adam-trained reward models, Adam-trained test-task
# reward models) + agents/buffer_sequential.py + features/deep_sequential.py.
AGENT_RUN_SEQ = dict(seed=11, n_s=17, H=32, A=7, d=8, acts=("relu", "relu"), T_tasks=3, lr=1e-3,
                     hp=dict(learning_rate_sf=1e-3, weight_decay_sf=0.0, learning_rate_w=5e-3, weight_decay_w=1e-2),
                     target_update_ev=5, n_samples=24, n_test_ev=8, episode_T=9, epsilon=0.2, gamma=0.9,
                     buffer=dict(n_samples=500, n_batch=8), task_terminal_every=7)


def agent_run_sequential(DeepSF, SFDQN, ReplayBuffer, device):
    """Build and train the sequential agent of AGENT_RUN_SEQ; returns (agent, tasks, test_tasks, returns)."""
    import random

    import numpy as np

    c = AGENT_RUN_SEQ
    random.seed(c["seed"])
    np.random.seed(c["seed"])
    torch.manual_seed(c["seed"])
    tasks = [AgentTask(c["n_s"], c["A"], c["d"], i, 300 + i, device, c["task_terminal_every"], tensor_reward=True)
             for i in range(c["T_tasks"])]
    test_tasks = [AgentTask(c["n_s"], c["A"], c["d"], c["T_tasks"], 400, device, tensor_reward=True)]
    sf = DeepSF(pytorch_model_handle=agent_psi_lambda(c["H"], c["acts"], c["lr"], device),
                target_update_ev=c["target_update_ev"], hyperparameters=c["hp"])
    agent = SFDQN(deep_sf=sf, buffer_handle=lambda: ReplayBuffer(**c["buffer"]), gamma=c["gamma"], T=c["episode_T"],
                  encoding="task", epsilon=c["epsilon"], use_gpi=True, test_epsilon=0.03, hyperparameters=c["hp"])
    returns = agent.train(tasks, c["n_samples"], test_tasks=test_tasks, n_test_ev=c["n_test_ev"])
    return agent, tasks, test_tasks, returns


# The main_tsfdqn_sequential_torch.py stack: agents/tsfdqn_sequential.py TSFDQN (per-task g_i =
# Linear(n_s, G), shared h = Linear(G, d), loss l1 + beta l2, ω-weighted test tasks) +
# agents/buffer_tsf_sequential.py + features/deep_sequential_tsf.py DeepTSF.
AGENT_RUN_TSF = dict(seed=13, n_s=17, H=32, A=7, d=8, acts=("relu", "relu"), T_tasks=3, lr=1e-3,
                     hp=dict(learning_rate_sf=1e-3, learning_rate_w=1e-3, learning_rate_g=1e-3, learning_rate_h=1e-3,
                             learning_rate_omega=1e-3, learning_rate_omega_decay=0.0, weight_decay_sf=0.0,
                             weight_decay_w=0.0, weight_decay_g=0.0, weight_decay_h=0.0, weight_decay_omega=0.0,
                             g_h_function_dims=16, beta_loss_coefficient=1.0, omegas_l1_coefficient=0.0),
                     target_update_ev=5, n_samples=24, n_test_ev=8, episode_T=9, epsilon=0.2, gamma=0.9,
                     buffer=dict(n_samples=500, n_batch=8), task_terminal_every=7)


def agent_run_tsf(DeepTSF, TSFDQN, ReplayBuffer, device, nf=False):
    """Build and train the TSF agent of AGENT_RUN_TSF (nf: tsfdqn_nf.py's planar-flow g_i with
    n_coupling_layers = 3); returns (agent, tasks, test_tasks, returns)."""
    import random

    import numpy as np

    c = dict(AGENT_RUN_TSF)
    if nf:
        c["hp"] = dict(c["hp"], n_coupling_layers=3)
        c["seed"] = 17
    random.seed(c["seed"])
    np.random.seed(c["seed"])
    torch.manual_seed(c["seed"])
    tasks = [AgentTask(c["n_s"], c["A"], c["d"], i, 500 + i, device, c["task_terminal_every"], tensor_reward=True)
             for i in range(c["T_tasks"])]
    test_tasks = [AgentTask(c["n_s"], c["A"], c["d"], c["T_tasks"], 600, device, tensor_reward=True)]
    sf = DeepTSF(pytorch_model_handle=agent_psi_lambda(c["H"], c["acts"], c["lr"], device), use_true_reward=False,
                 target_update_ev=c["target_update_ev"], hyperparameters=c["hp"])
    agent = TSFDQN(deep_sf=sf, buffer_handle=lambda: ReplayBuffer(**c["buffer"]), gamma=c["gamma"], T=c["episode_T"],
                   encoding="task", epsilon=c["epsilon"], use_gpi=True, test_epsilon=0.03, hyperparameters=c["hp"])
    returns = agent.train(tasks, c["n_samples"], test_tasks=test_tasks, n_test_ev=c["n_test_ev"])
    return agent, tasks, test_tasks, returns
