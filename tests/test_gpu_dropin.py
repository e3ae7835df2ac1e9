"""The reference's own agents on sfx's SF library: replay of SF-boundary call logs.

tools/gen_golden.py ran each training stack of the reference -- its own agents, buffers and SF
libraries, on the CPU, with the seeded recipes of tests/golden/recipe.py -- and logged, in order,
every call its agents made across the SF boundary with inputs and outputs (GPI,
get_successor(s), get_next_successors, update_reward, update_successor; for TSF the agent's own
update_successor, tsfdqn.py:588-709, which sfx.dropin.bind routes to DeepTSF.tsf_update), plus the
library state before the first call and after the last (tests/golden/calls_*.npz).

Here the same calls, with the same inputs, go to sfx's drop-in libraries (sfx.dropin.features.*,
sfx.dropin.bind) on the GPU, starting from the same state.  Every GPI task index must match
bit-exactly; q, ψ and the losses within 1e-4 relative; the final ψ / target / w (and g, h) within
the Adam tolerance of test_gpu_engine.py; GPI counters and target-sync counters exactly.  The
agents never run here: the log is their trace.
"""
import numpy as np
import pytest
import torch

from tests.conftest import gpu_available
from tests.golden.recipe import AGENT_RUN, AGENT_RUN_SEQ, AGENT_RUN_TSF, AgentTask, agent_psi_lambda
from tests.test_gpu_engine import params_close, rel_close

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


@pytest.fixture(autouse=True)
def _need_gpu():
    if not gpu_available():
        pytest.skip("no HIP device")


class _Flow(torch.nn.Module):
    """A planar flow's tensors in tsfdqn_nf.py's order (weight [1, n_s], bias [1], scale [1, n_s])."""

    def __init__(self, n_s):
        super().__init__()
        self.weight = torch.nn.Parameter(torch.zeros(1, n_s))
        self.bias = torch.nn.Parameter(torch.zeros(1))
        self.scale = torch.nn.Parameter(torch.zeros(1, n_s))

    def forward(self, z):
        return z + self.scale * torch.tanh(torch.nn.functional.linear(z, self.weight, self.bias))


def _load(module, flat):
    off = 0
    with torch.no_grad():
        for p in module.parameters():
            p.copy_(torch.from_numpy(flat[off:off + p.numel()]).view_as(p))
            off += p.numel()


def _build(stack, g):
    """sfx's library for `stack`, with the recipe's hyper-parameters and the logged initial state."""
    from sfx.dropin import bind
    from sfx.dropin.features import deep, deep_sequential, deep_sequential_tsf

    tsf = stack.startswith("tsfdqn")
    c = AGENT_RUN if stack == "sfdqn_alltask" else AGENT_RUN_SEQ if stack.startswith("sfdqn") else dict(AGENT_RUN_TSF)
    if stack == "tsfdqn_nf":
        c["hp"] = dict(c["hp"], n_coupling_layers=3)
    handle = agent_psi_lambda(c["H"], c["acts"], c["lr"], DEV)
    if stack == "sfdqn_alltask":
        sf = deep.DeepSF(pytorch_model_handle=handle, target_update_ev=c["target_update_ev"],
                         hyperparameters={"learning_rate_w": c["alpha_w"]})
    elif stack == "sfdqn_sequential":
        sf = deep_sequential.DeepSF(pytorch_model_handle=handle, target_update_ev=c["target_update_ev"],
                                    hyperparameters=c["hp"])
    elif stack == "sfdqn_singlefile":
        sf = bind.SingleFileDeepSF(pytorch_model_handle=handle, target_update_ev=c["target_update_ev"],
                                   hyperparameters=c["hp"])
    elif stack == "tsfdqn_sequential":
        sf = deep_sequential_tsf.DeepTSF(pytorch_model_handle=handle, use_true_reward=False,
                                         target_update_ev=c["target_update_ev"], hyperparameters=c["hp"])
    else:
        sf = bind.SingleFileDeepTSF(handle, False, target_update_ev=c["target_update_ev"], hyperparameters=c["hp"])
    sf.reset()
    T, n_s, d = c["T_tasks"], c["n_s"], c["d"]
    gfun, h = [], None
    if tsf:
        G, K = c["hp"]["g_h_function_dims"], c["hp"].get("n_coupling_layers", 0) if stack == "tsfdqn_nf" else 0
        h = torch.nn.Linear(G, d).to(DEV)
        _load(h, g["init.h"])
    for t in range(T):
        task = AgentTask(n_s, c["A"], d, t, t, DEV)
        if tsf:
            gt = torch.nn.Sequential(*[_Flow(n_s) for _ in range(K)], torch.nn.Linear(n_s, G)) if K else \
                torch.nn.Linear(n_s, G)
            gt = gt.to(DEV)
            _load(gt, g["init.g"][t])
            gfun.append(gt)
            sf.add_training_task(task, None, gt, h)
        else:
            sf.add_training_task(task)
    for t in range(T):  # the logged initial state, before the engine exists
        (m, _, _), (tm, _, _) = sf.psi[t]
        _load(m, g["init.online"][t])
        _load(tm, g["init.target"][t])
        w = list.__getitem__(sf.fit_w, t)
        with torch.no_grad():
            if isinstance(w, torch.nn.Linear):
                w.weight.copy_(torch.from_numpy(g["init.w"][t]).view(1, -1))
            else:
                list.__setitem__(sf.fit_w, t, torch.from_numpy(g["init.w"][t]).view(-1, 1).to(DEV))
    return sf, c, gfun, h


def _w(x):
    return (x.weight if hasattr(x, "weight") else x).detach().reshape(-1).cpu()


STACKS = ["sfdqn_alltask", "sfdqn_sequential", "sfdqn_singlefile", "tsfdqn_sequential", "tsfdqn_singlefile",
          "tsfdqn_nf"]


@pytest.mark.parametrize("stack", STACKS)
def test_dropin_replays_reference_call_log(golden, stack):
    g = golden("calls_" + stack)
    sf, c, gfun, h = _build(stack, g)
    names = [str(n) for n in g["names"]]
    seq = stack != "sfdqn_alltask"
    counts = {}

    def arr(k, key, dtype=None):
        t = torch.from_numpy(np.asarray(g[f"c{k}.{key}"]))
        return t.to(DEV) if dtype is None else t.to(DEV, dtype)

    for k, name in enumerate(names):
        counts[name] = counts.get(name, 0) + 1
        if name == "GPI":
            q, task = sf.GPI(arr(k, "state"), int(g[f"c{k}.task_index"]), bool(g[f"c{k}.update_counters"]))
            assert int(task) == int(g[f"c{k}.task"]), f"call {k} (GPI): task {int(task)} vs {int(g[f'c{k}.task'])}"
            rel_close(q, g[f"c{k}.q"], rtol=1e-4, atol=1e-6)
        elif name in ("get_successors", "get_next_successors"):
            rel_close(getattr(sf, name)(arr(k, "state")), g[f"c{k}.psi"], rtol=1e-4, atol=1e-6)
        elif name == "get_successor":
            rel_close(sf.get_successor(arr(k, "state"), int(g[f"c{k}.policy_index"])), g[f"c{k}.psi"], rtol=1e-4,
                      atol=1e-6)
        elif name == "update_reward":
            ti = int(g[f"c{k}.task_index"])
            sf.update_reward(arr(k, "phi"), arr(k, "r"), ti)
            rel_close(_w(sf.fit_w[ti]), g[f"c{k}.w"], rtol=1e-5, atol=1e-7)
        elif name in ("update_successor", "tsf_update"):
            pi, use_gpi = int(g[f"c{k}.policy_index"]), bool(g[f"c{k}.use_gpi"])
            tr = None
            if bool(g[f"c{k}.has_batch"]):
                n = len([f for f in g if f.startswith(f"c{k}.t")])
                tr = tuple(arr(k, f"t{i}") for i in range(n))
            if name == "tsf_update":
                out = None if tr is None else sf.tsf_update(tr, pi, use_gpi, beta=c["hp"]["beta_loss_coefficient"])
            else:
                out = sf.update_successor(tr, pi, use_gpi) if seq else sf.update_successor(tr, pi)
            if f"c{k}.losses" in g:
                rel_close(torch.stack([torch.as_tensor(x).float().cpu() for x in out]), g[f"c{k}.losses"], rtol=1e-4,
                          atol=1e-7)
            else:
                assert out is None
        else:
            raise AssertionError(f"unknown call {name}")
    assert counts.get("GPI", 0) > 0 and (counts.get("update_successor", 0) + counts.get("tsf_update", 0)) > 0
    T = sf.n_tasks
    steps = counts.get("update_successor", 0) + counts.get("tsf_update", 0)
    online = torch.stack([torch.cat([p.detach().reshape(-1).cpu() for p in sf.psi[t][0][0].parameters()])
                          for t in range(T)])
    target = torch.stack([torch.cat([p.detach().reshape(-1).cpu() for p in sf.psi[t][1][0].parameters()])
                          for t in range(T)])
    params_close(online, g["final.online"], 1e-3 * steps)
    params_close(target, g["final.target"], 1e-3 * steps)
    rel_close(torch.stack([_w(sf.fit_w[t]) for t in range(T)]), g["final.w"], rtol=1e-4, atol=1e-7)
    assert np.array_equal(np.stack([np.asarray(x) for x in sf.gpi_counters]), g["final.gpi_counters"])
    assert list(sf.updates_since_target_updated) == [int(x) for x in g["final.since_target"]]
    if gfun:
        sf.sync_tsf_modules()
        params_close(torch.stack([torch.cat([p.detach().reshape(-1).cpu() for p in m.parameters()]) for m in gfun]),
                     g["final.g"], 1e-3 * steps)
        params_close(torch.cat([p.detach().reshape(-1).cpu() for p in h.parameters()]), g["final.h"], 1e-3 * steps)


@pytest.mark.parametrize("case", ["sfdqn_gpi", "sfdqn_nogpi", "sfdqn_tanh"])
def test_dropin_sequential_deepsf_vs_reference_updates(golden, case):
    """features.deep_sequential.DeepSF (main_sfdqn_sequential_torch.py's library) driven through its
    public API reproduces the reference's update_successor sequence (tests/golden/upd_sfdqn_*)."""
    from sfx.dropin.features.deep_sequential import DeepSF

    from tests.golden.recipe import AgentTask, agent_psi_lambda
    from tests.test_gpu_engine import batches_of, spec_of

    g = golden("upd_" + case)
    spec, T = spec_of(g), int(g["T"])
    hp = {"learning_rate_sf": 1e-3, "learning_rate_w": 1e-3, "weight_decay_sf": 0.0, "weight_decay_w": 0.0}
    sf = DeepSF(pytorch_model_handle=agent_psi_lambda(spec.H, spec.acts, 1e-3, DEV),
                target_update_ev=int(g["target_update_ev"]), hyperparameters=hp)
    sf.reset()
    for t in range(T):
        sf.add_training_task(AgentTask(spec.n_s, spec.A, spec.d, t, t, DEV))
    # the fixture's initial weights into the library's modules (before the engine exists)
    for t in range(T):
        (m, _, _), (tm, _, _) = sf.psi[t]
        for mod in (m, tm):
            off = 0
            with torch.no_grad():
                for p in mod.parameters():
                    p.copy_(torch.from_numpy(g["online0"][t][off:off + p.numel()]).view_as(p))
                    off += p.numel()
        with torch.no_grad():
            list.__getitem__(sf.fit_w, t).weight.copy_(torch.from_numpy(g["w0"][t]).view(1, -1))
    for j, (s, a, r, phi, s1, gamma) in enumerate(batches_of(g)):
        i = int(g["policies"][j])
        dev = DEV
        loss, l1, l2 = sf.update_successor((s.to(dev), a.to(dev), r.to(dev), phi.to(dev), s1.to(dev), gamma.to(dev)),
                                           i, use_gpi=bool(g["use_gpi"]))
        rel_close(torch.stack([loss, l1, l2]).cpu(), g["losses"][j], rtol=1e-4, atol=1e-7)
    k = int(g["k"])
    online = torch.stack([torch.cat([p.detach().reshape(-1).cpu() for p in sf.psi[t][0][0].parameters()])
                          for t in range(T)])
    params_close(online, g["online"], 1e-3 * k)
    rel_close(torch.stack([sf.fit_w[t].weight.detach().reshape(-1).cpu() for t in range(T)]), g["w"], rtol=1e-4,
              atol=1e-5)
    assert list(sf.updates_since_target_updated) == [int(x) for x in g["since_target"]]
