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
* ``geometry``, ``adam`` -- what the engine was built with (with ``head_offset`` / ``T_w`` of a
  sharded rank: a rank's checkpoint loads only into the same rank's engine).

TSF-DQN engines (tsfdqn.py / tsfdqn_nf.py; ``eng.tsf_setup``) add, per task, the reference's task
modules and ONE 4-group ``torch.optim.Adam`` (tsfdqn.py:255-270: {ψ_i}, {w_i}, {g_i}, {h}):

* ``heads[t]["w_model"]`` -- ``Linear(d, 1, bias=False)`` (tsfdqn.py:154-161): ``weight`` [1, d];
* ``heads[t]["g_model"]`` -- g_i: ``Linear(n_s, G)`` (``weight``, ``bias``; tsfdqn.py:537-546) or, with K
  planar layers, the ``Sequential`` of K ``PlanarFlow`` (``{k}.weight`` [1, n_s], ``{k}.bias`` [1],
  ``{k}.scale`` [1, n_s]) and the ``Linear`` (``{K}.weight``, ``{K}.bias``; tsfdqn_nf.py:331-358, flows
  registered as on the reference's CPU configuration);
* ``heads[t]["optim"]`` -- that Adam's state_dict: parameters in the order ψ, w, g, h, each with the
  step / exp_avg / exp_avg_sq of task t (its own moments of the shared h), groups with the engine's
  hyper-parameters (lr_sf / wd_sf, lr_w / wd_w, lr_g / wd_g, lr_h / wd_h);
* ``h_model`` -- the shared ``Linear(G, d)``; ``tsf`` -- G, K, β, the g / h hyper-parameters, frozen flows.

Learned-φ engines (features/deep_phi.py; ``eng.phi_setup``) add ``phi``: the φ network's packed
parameters and its configuration (the reference rebuilds its Adam at every update, so there is
no optimizer state to keep).

So a reference user resumes with ``model.load_state_dict(ck["heads"][t]["model"])`` and
``optim.load_state_dict(ck["heads"][t]["optim"])``, and an engine with ``load(eng, path)``.
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


def _adam_group(hp: dict, n_params: int, lr=None, wd=None, first: int = 0) -> dict:
    """torch.optim.Adam's own param-group record for these hyper-parameters (every key its
    load_state_dict expects in this torch version), parameters first .. first + n_params - 1."""
    dummy = [torch.zeros(1) for _ in range(n_params)]
    g = torch.optim.Adam(dummy, lr=hp["lr_psi"] if lr is None else lr, betas=tuple(hp["betas"]), eps=hp["eps"],
                         weight_decay=hp["wd_psi"] if wd is None else wd).state_dict()["param_groups"][0]
    g["params"] = list(range(first, first + n_params))
    return g


def g_shapes(n_s: int, G: int, K: int) -> List[Tuple[str, Tuple[int, ...]]]:
    """g_i's parameters in the engine's packing (flow k: weight, bias, scale; then the Linear), with
    the reference module's state_dict names."""
    if K == 0:
        return [("weight", (G, n_s)), ("bias", (G,))]
    out = []
    for k in range(K):
        out += [(f"{k}.weight", (1, n_s)), (f"{k}.bias", (1,)), (f"{k}.scale", (1, n_s))]
    return out + [(f"{K}.weight", (G, n_s)), (f"{K}.bias", (G,))]


def h_shapes(G: int, d: int):
    return [("weight", (d, G)), ("bias", (d,))]


def _state_entries(step: int, named_m, named_v, names, first: int) -> dict:
    return {first + i: {"step": torch.tensor(float(step), dtype=torch.float32), "exp_avg": named_m[n],
                        "exp_avg_sq": named_v[n]} for i, n in enumerate(names)}


def _geometry(eng) -> dict:
    return {"T": eng.T, "n_s": eng.n_s, "H": eng.H, "A": eng.A, "d": eng.d, "acts": list(eng.acts),
            "T_w": getattr(eng, "T_glob", eng.T), "head_offset": getattr(eng, "head_offset", 0)}


def state_dict(eng) -> dict:
    """The engine's training state (host copies; synchronous)."""
    shapes = param_shapes(eng.n_s, eng.H, eng.A, eng.d, eng.acts)
    tsf = getattr(eng, "tsf_G", None) is not None
    Tw = getattr(eng, "T_glob", eng.T)
    ws = [eng.get_w(t) for t in range(Tw)]
    hp = eng.adam_hp
    if tsf:
        gsh, hsh = g_shapes(eng.n_s, eng.tsf_G, eng.tsf_K), h_shapes(eng.tsf_G, eng.d)
        th = eng.tsf_hp
        nps, ng = len(shapes), len(gsh)
        groups = [_adam_group(hp, nps), _adam_group(hp, 1, hp["lr_w"], hp["wd_w"], nps),
                  _adam_group(hp, ng, th["lr_g"], th["wd_g"], nps + 1),
                  _adam_group(hp, 2, th["lr_h"], th["wd_h"], nps + 1 + ng)]
    else:
        groups = [_adam_group(hp, len(shapes))]
    heads = []
    for t in range(eng.T):
        m, v, step = eng.get_adam(t)
        ms, vs = unpack(m, shapes), unpack(v, shapes)
        state = {}
        if step > 0:  # torch keeps no per-parameter state before the first step
            state.update(_state_entries(step, ms, vs, [n for n, _ in shapes], 0))
        head = {"model": unpack(eng.get_head(t, 0), shapes),
                "target_model": unpack(eng.get_head(t, 1), shapes),
                "optim": {"state": state, "param_groups": [dict(g) for g in groups]},
                "since_target": int(eng.since_target(t))}
        if tsf:
            w, wm, wv = ws[getattr(eng, "head_offset", 0) + t]
            g, gm, gv = eng.tsf_get_g(t)
            hm, hv = eng.tsf_get_h_state(t)
            head["w_model"] = OrderedDict(weight=w.reshape(1, -1).clone())
            head["g_model"] = unpack(g, gsh)
            if step > 0:
                state.update(_state_entries(step, {"w": wm.reshape(1, -1)}, {"w": wv.reshape(1, -1)}, ["w"], nps))
                state.update(_state_entries(step, unpack(gm, gsh), unpack(gv, gsh), [n for n, _ in gsh], nps + 1))
                state.update(_state_entries(step, unpack(hm, hsh), unpack(hv, hsh), [n for n, _ in hsh], nps + 1 + ng))
        heads.append(head)
    out = {"format": FORMAT,
           "geometry": _geometry(eng),
           "adam": {k: (list(v) if isinstance(v, tuple) else v) for k, v in hp.items()},
           "heads": heads,
           "w": torch.stack([w for w, _, _ in ws]),
           "w_exp_avg": torch.stack([m for _, m, _ in ws]),
           "w_exp_avg_sq": torch.stack([v for _, _, v in ws])}
    if tsf:
        out["h_model"] = unpack(eng.tsf_get_h(), h_shapes(eng.tsf_G, eng.d))
        out["tsf"] = dict(G=eng.tsf_G, K=eng.tsf_K, frozen_flows=bool(getattr(eng, "tsf_frozen", False)),
                          **eng.tsf_hp)
    if getattr(eng, "phi_numel", None):
        out["phi"] = {"params": eng.phi_get().clone(), "cfg": dict(eng.phi_cfg)}
    return out


def load_state_dict(eng, ck: dict) -> None:
    """Restore an engine of the same geometry from `ck` (heads, targets, Adam moments and step
    counts, target-sync counters, w and its moments, Adam hyper-parameters)."""
    if ck.get("format") != FORMAT:
        raise ValueError(f"not an sfx checkpoint (format {ck.get('format')!r})")
    g = dict(ck["geometry"])
    g.setdefault("head_offset", 0)
    mine = _geometry(eng)
    if {k: g.get(k) for k in mine} != mine:
        raise ValueError(f"checkpoint geometry {g} does not match the engine's {mine}")
    tsf = getattr(eng, "tsf_G", None) is not None
    if tsf != ("tsf" in ck):
        raise ValueError("checkpoint and engine disagree on TSF state (eng.tsf_setup before loading a TSF checkpoint)")
    if tsf:
        want = {k: ck["tsf"][k] for k in ("G", "K")}
        if want != {"G": eng.tsf_G, "K": eng.tsf_K}:
            raise ValueError(f"checkpoint TSF geometry {want} does not match the engine's (G={eng.tsf_G}, K={eng.tsf_K})")
    phi = bool(getattr(eng, "phi_numel", None))
    if phi != ("phi" in ck):
        raise ValueError("checkpoint and engine disagree on learned-φ state (eng.phi_setup before loading)")
    if phi and dict(ck["phi"]["cfg"]) != dict(eng.phi_cfg):
        raise ValueError(f"checkpoint φ configuration {ck['phi']['cfg']} does not match the engine's {eng.phi_cfg}")
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
        if tsf:
            gsh, hsh = g_shapes(eng.n_s, eng.tsf_G, eng.tsf_K), h_shapes(eng.tsf_G, eng.d)
            nps, ng = len(shapes), len(gsh)
            if st:
                gm = pack({n: st[nps + 1 + i]["exp_avg"] for i, (n, _) in enumerate(gsh)}, gsh)
                gv = pack({n: st[nps + 1 + i]["exp_avg_sq"] for i, (n, _) in enumerate(gsh)}, gsh)
                hm = pack({n: st[nps + 1 + ng + i]["exp_avg"] for i, (n, _) in enumerate(hsh)}, hsh)
                hv = pack({n: st[nps + 1 + ng + i]["exp_avg_sq"] for i, (n, _) in enumerate(hsh)}, hsh)
            else:
                gm = gv = torch.zeros(eng.tsf_Pg)
                hm = hv = torch.zeros(eng.tsf_Ph)
            eng.tsf_load_g_state(t, pack(hd["g_model"], gsh), gm, gv)
            eng.tsf_load_h_state(t, hm, hv)
    for t in range(mine["T_w"]):
        eng.load_w_state(t, ck["w"][t], ck["w_exp_avg"][t], ck["w_exp_avg_sq"][t])
    if tsf:
        eng.tsf_load_h(pack(ck["h_model"], h_shapes(eng.tsf_G, eng.d)))
        if bool(ck["tsf"].get("frozen_flows", False)) != bool(getattr(eng, "tsf_frozen", False)):
            eng.tsf_freeze_flows(bool(ck["tsf"].get("frozen_flows", False)))
    if phi:
        eng.phi_load(ck["phi"]["params"])


def save(eng, path: str) -> None:
    torch.save(state_dict(eng), path)


def load(eng, path: str) -> None:
    load_state_dict(eng, torch.load(path, weights_only=True))
