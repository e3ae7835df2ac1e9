"""Checkpoint / resume of an SFEngine's training state (the reference has none --
no torch.save / state_dict anywhere -- and the survey's option is an export "with the same per-task
nn.Sequential key names, so the reference can load them").

The checkpoint is a plain dict of tensors, ints and strings (loadable with
``torch.load(path, weights_only=True)``):

* ``heads[t]["model"]`` / ``["target_model"]`` -- the state_dict of the reference's ψ Sequential
  (main_sfdqn_torch.py:44-78 sf_model_lambda: ``layer_input``, ``layer_{j}``, ``layer_output``;
  the activation and Unflatten layers hold no parameters);
* ``heads[t]["optim"]`` -- the state_dict of the ``torch.optim.Adam(model.parameters(), ...)``
  that lambda builds: per parameter ``step`` / ``exp_avg`` / ``exp_avg_sq`` (no entries before the
  first step, as torch keeps them), one param group with the engine's hyper-parameters;
* ``heads[t]["since_target"]`` -- updates since the last target sync (utils/torch.py:31-33 bookkeeping);
* ``w`` / ``w_exp_avg`` / ``w_exp_avg_sq`` -- the reward weights of every task (the LMS fit of
  features/successor.py, or sfdqn.py's Adam-trained w with its moments);
* ``geometry``, ``adam`` -- what the engine was built with.

So a reference user resumes with ``model.load_state_dict(ck["heads"][t]["model"])`` and
``optim.load_state_dict(ck["heads"][t]["optim"])``, and an engine with ``load(eng, path)``.
TSF (g_i, h, ω) and learned-φ state are not part of it.
"""
from __future__ import annotations

from collections import OrderedDict
from typing import Dict, List, Tuple

import torch

FORMAT = "sfx-checkpoint-1"


def param_shapes(n_s: int, H: int, A: int, d: int, acts) -> List[Tuple[str, Tuple[int, ...]]]:
    """Names and shapes of the ψ head's parameters in torch packing order (module.parameters())."""
    out = [("layer_input.weight", (H, n_s)), ("layer_input.bias", (H,))]
    for j in range(len(acts)):
        out += [(f"layer_{j}.weight", (H, H)), (f"layer_{j}.bias", (H,))]
    out += [("layer_output.weight", (A * d, H)), ("layer_output.bias", (A * d,))]
    return out


def unpack(flat: torch.Tensor, shapes) -> "OrderedDict[str, torch.Tensor]":
    flat = flat.detach().reshape(-1).to(torch.float32).cpu()
    out, o = OrderedDict(), 0
    for name, shp in shapes:
        n = 1
        for s in shp:
            n *= s
        out[name] = flat[o:o + n].reshape(shp).clone()
        o += n
    if o != flat.numel():
        raise ValueError(f"packed head has {flat.numel()} floats, the geometry {o}")
    return out


def pack(named: Dict[str, torch.Tensor], shapes) -> torch.Tensor:
    parts = []
    for name, shp in shapes:
        x = torch.as_tensor(named[name], dtype=torch.float32).cpu()
        if tuple(x.shape) != tuple(shp):
            raise ValueError(f"{name}: shape {tuple(x.shape)}, expected {tuple(shp)}")
        parts.append(x.reshape(-1))
    return torch.cat(parts)


def _adam_group(hp: dict, n_params: int) -> dict:
    """torch.optim.Adam's own param-group record for these hyper-parameters (every key its
    load_state_dict expects in this torch version)."""
    dummy = [torch.zeros(1) for _ in range(n_params)]
    g = torch.optim.Adam(dummy, lr=hp["lr_psi"], betas=tuple(hp["betas"]), eps=hp["eps"],
                         weight_decay=hp["wd_psi"]).state_dict()["param_groups"][0]
    g["params"] = list(range(n_params))
    return g


def state_dict(eng) -> dict:
    """The engine's training state (host copies; synchronous)."""
    shapes = param_shapes(eng.n_s, eng.H, eng.A, eng.d, eng.acts)
    group = _adam_group(eng.adam_hp, len(shapes))
    heads = []
    for t in range(eng.T):
        m, v, step = eng.get_adam(t)
        ms, vs = unpack(m, shapes), unpack(v, shapes)
        state = {}
        if step > 0:  # torch keeps no per-parameter state before the first step
            for i, (name, _) in enumerate(shapes):
                state[i] = {"step": torch.tensor(float(step), dtype=torch.float32), "exp_avg": ms[name],
                            "exp_avg_sq": vs[name]}
        heads.append({"model": unpack(eng.get_head(t, 0), shapes),
                      "target_model": unpack(eng.get_head(t, 1), shapes),
                      "optim": {"state": state, "param_groups": [dict(group)]},
                      "since_target": int(eng.since_target(t))})
    Tw = getattr(eng, "T_glob", eng.T)
    ws = [eng.get_w(t) for t in range(Tw)]
    return {"format": FORMAT,
            "geometry": {"T": eng.T, "n_s": eng.n_s, "H": eng.H, "A": eng.A, "d": eng.d, "acts": list(eng.acts),
                         "T_w": Tw},
            "adam": {k: (list(v) if isinstance(v, tuple) else v) for k, v in eng.adam_hp.items()},
            "heads": heads,
            "w": torch.stack([w for w, _, _ in ws]),
            "w_exp_avg": torch.stack([m for _, m, _ in ws]),
            "w_exp_avg_sq": torch.stack([v for _, _, v in ws])}


def load_state_dict(eng, ck: dict) -> None:
    """Restore an engine of the same geometry from `ck` (heads, targets, Adam moments and step
    counts, target-sync counters, w and its moments, Adam hyper-parameters)."""
    if ck.get("format") != FORMAT:
        raise ValueError(f"not an sfx checkpoint (format {ck.get('format')!r})")
    g = ck["geometry"]
    mine = {"T": eng.T, "n_s": eng.n_s, "H": eng.H, "A": eng.A, "d": eng.d, "acts": list(eng.acts),
            "T_w": getattr(eng, "T_glob", eng.T)}
    if {k: g[k] for k in mine} != mine:
        raise ValueError(f"checkpoint geometry {g} does not match the engine's {mine}")
    hp = ck["adam"]
    eng.set_adam(hp["lr_psi"], hp["wd_psi"], hp["lr_w"], hp["wd_w"], tuple(hp["betas"]), hp["eps"])
    shapes = param_shapes(eng.n_s, eng.H, eng.A, eng.d, eng.acts)
    for t, hd in enumerate(ck["heads"]):
        eng.load_head(t, pack(hd["model"], shapes), 0)
        eng.load_head(t, pack(hd["target_model"], shapes), 1)
        st = hd["optim"]["state"]
        if st:
            steps = {int(round(float(st[i]["step"]))) for i in range(len(shapes))}
            if len(steps) != 1:
                raise ValueError(f"head {t}: per-parameter Adam steps differ ({sorted(steps)})")
            step = steps.pop()
            m = pack({name: st[i]["exp_avg"] for i, (name, _) in enumerate(shapes)}, shapes)
            v = pack({name: st[i]["exp_avg_sq"] for i, (name, _) in enumerate(shapes)}, shapes)
        else:
            step, m, v = 0, torch.zeros(eng.P), torch.zeros(eng.P)
        eng.load_adam(t, m, v, step)
        eng.set_since_target(t, int(hd["since_target"]))
    for t in range(mine["T_w"]):
        eng.load_w_state(t, ck["w"][t], ck["w_exp_avg"][t], ck["w_exp_avg_sq"][t])


def save(eng, path: str) -> None:
    torch.save(state_dict(eng), path)


def load(eng, path: str) -> None:
    load_state_dict(eng, torch.load(path, weights_only=True))
