"""GPU check of the sharded all-task step (sfx_shard_* kernels + sfx.shard.ShardedAllTask):
two ranks share this box's GPU, each owning half of the heads; the all-reduces run over gloo
through host memory (RCCL needs one GPU per rank; the data path of the kernels is the same).
Against the unsharded oracle: identical env actions (GPI argmax, bit-exact), heads within the
Adam tolerance of test_gpu_engine.py."""
import os
import socket

import numpy as np
import pytest
import torch

from oracle import ref_cpu as R
from tests.conftest import gpu_available

pytestmark = pytest.mark.gpu

SPEC = dict(n_s=17, H=32, A=7, d=8, acts=("relu", "relu"))
TG, STEPS, EV, B = 4, 8, 3, 16


@pytest.fixture(autouse=True)
def _need_gpu():
    if not gpu_available():
        pytest.skip("no HIP device")


# BASELINE config C4's per-rank shape (Reacher, 256-wide heads), two ranks of 8 heads each
FULL = dict(spec=dict(n_s=17, H=256, A=7, d=8, acts=("relu", "relu")), tg=16, b=32, steps=5)
SMALL = dict(spec=SPEC, tg=TG, b=B, steps=STEPS)


def _stream(seed, cfg=SMALL):
    spec, tg, b = cfg["spec"], cfg["tg"], cfg["b"]
    g = torch.Generator().manual_seed(seed)
    out = []
    for j in range(cfg["steps"]):
        batch = None
        if j > 0:
            batch = (torch.randn(b, spec["n_s"], generator=g), torch.randint(0, spec["A"], (b,), generator=g),
                     torch.rand(b, spec["d"], generator=g), torch.randn(b, spec["n_s"], generator=g),
                     torch.where(torch.rand(b, generator=g) < 0.2, 0.0, 0.9))
        out.append((batch, j % tg, torch.rand(spec["d"], generator=g), torch.rand(1, generator=g),
                    torch.randn(spec["n_s"], generator=g)))
    return out


def _run_rank(rank, world, rounds, ar, cfg=SMALL):
    from sfx.engine import SFEngine
    from sfx.init import reference_heads
    from sfx.shard import LibsfxShardBackend, ShardedAllTask

    sp, tg, b = cfg["spec"], cfg["tg"], cfg["b"]
    online, w = reference_heads(tg, sp["n_s"], sp["H"], sp["A"], sp["d"], sp["acts"], seed=3)
    T_loc = tg // world
    eng = SFEngine(T_loc, sp["n_s"], sp["H"], sp["A"], sp["d"], sp["acts"], max_batch=b)
    eng.set_adam(1e-3, 0.0, 1e-3, 0.0)
    eng.set_target_update_ev(EV)
    be = LibsfxShardBackend(eng, tg, rank * T_loc, b)
    for t in range(T_loc):
        eng.load_head(t, online[rank * T_loc + t], 0)
        eng.load_head(t, online[rank * T_loc + t], 1)
    for t in range(tg):
        eng.load_w(t, w[t])
    step = ShardedAllTask(be, tg, sp["A"], ar, rounds=rounds)
    actions = []
    dev = eng.device
    for batch, task, phi1, r1, s_next in _stream(11, cfg):
        db = None if batch is None else tuple(x.to(dev).contiguous() for x in batch)
        actions.append(step.step(db, task, phi1.to(dev), r1.to(dev), 0.05, s_next.to(dev), task))
    heads = torch.stack([eng.get_head(t) for t in range(T_loc)])
    targets = torch.stack([eng.get_head(t, 1) for t in range(T_loc)])
    ws = torch.stack([eng.get_w(t)[0] for t in range(tg)])
    eng.close()
    return actions, heads, targets, ws, step.stats


def _oracle(cfg=SMALL):
    sp, tg = cfg["spec"], cfg["tg"]
    spec = R.Spec(**sp)
    from sfx.init import reference_heads

    online, w0 = reference_heads(tg, sp["n_s"], sp["H"], sp["A"], sp["d"], sp["acts"], seed=3)
    st = R.SFState(spec, online.clone(), online.clone(), w0.clone())
    want = []
    for batch, task, phi1, r1, s_next in _stream(11, cfg):
        st.w[task] = R.lms_update(st.w[task].view(-1, 1), phi1, r1[0], 0.05).view(-1)
        if batch is not None:
            R.deep_all_task_step(st, batch, lr=1e-3, target_update_ev=EV)
        qv, tk = R.gpi_w(R.psi_all(st.online, spec, s_next.view(1, -1)), st.w[task])
        want.append((int(tk[0]), R.select_action(qv, tk[0], task, True)))
    return want, st


def _check(actions, heads, targets, ws, want, st, steps=STEPS):
    from tests.test_gpu_engine import params_close, rel_close

    assert actions == want
    params_close(heads, st.online, 1e-3 * steps)
    params_close(targets, st.target, 1e-3 * steps)
    rel_close(ws, st.w, rtol=1e-5, atol=1e-7)


@pytest.mark.parametrize("rounds", [1, 2])
def test_single_rank_shard_protocol(rounds):
    actions, heads, targets, ws, stats = _run_rank(0, 1, rounds, lambda t: None)
    want, st = _oracle()
    _check(actions, heads, targets, ws, want, st)
    assert stats["steps"] == STEPS - 1


def _worker(rank, port, q, cfg=SMALL):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=2)
    from sfx.shard import all_reduce_max_fn

    try:
        actions, heads, targets, ws, stats = _run_rank(rank, 2, 2, all_reduce_max_fn(via_host=True), cfg)
        parts = [None, None]
        dist.all_gather_object(parts, (heads, targets))
        if rank == 0:
            q.put((actions, torch.cat([p[0] for p in parts]).numpy(), torch.cat([p[1] for p in parts]).numpy(),
                   ws.numpy(), stats))
            q.close()
            q.join_thread()  # flushed into the pipe before the teardown
    finally:
        dist.destroy_process_group()


def _two_ranks(worker, cfg):
    import torch.multiprocessing as mp

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=worker, args=(r, port, q, cfg)) for r in range(cfg.get("world", 2))]
    for p in procs:
        p.start()
    # tensors travel as numpy arrays (pickled by value): torch's fd-shared storages need the
    # sending rank alive until the parent has unpickled them, and rank 0 exits right after
    out = tuple(torch.from_numpy(x) if isinstance(x, np.ndarray) else x for x in q.get(timeout=300))
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    return out


@pytest.mark.parametrize("cfg", [SMALL, FULL], ids=["small", "c4-shape"])
def test_two_ranks_on_one_gpu(cfg):
    actions, heads, targets, ws, stats = _two_ranks(_worker, cfg)
    want, st = _oracle(cfg)
    _check(actions, heads, targets, ws, want, st, cfg["steps"])


# ---- sharded TSF-DQN (sfx_shard_tsf_*, BASELINE config C5) ---------------------------------
TSF_SMALL = dict(spec=dict(n_s=11, H=32, A=9, d=6, acts=("relu", "relu")), tg=TG, b=B, G=10, K=3, steps=8,
                 init=0.3)
# C5's shape (Hopper, tsfdqn_nf.py): 256-wide heads, 27 actions, d=50, g_i width 100 with 100 planar
# layers; two ranks of 8 heads, flows at a small init (PlanarFlow's U(-0.01, 0.01) scale, widened)
TSF_FULL = dict(spec=dict(n_s=11, H=256, A=27, d=50, acts=("relu", "relu")), tg=16, b=32, G=100, K=100, steps=4,
                init=0.05)
# BASELINE config C5 at its stated size: 32 TSF-NF tasks over 4 ranks (8 heads each), K = 100
TSF_C5 = dict(TSF_FULL, tg=32, world=4)


def _tsf_problem(cfg):
    from sfx.init import reference_heads

    sp, tg = cfg["spec"], cfg["tg"]
    online, w = reference_heads(tg, sp["n_s"], sp["H"], sp["A"], sp["d"], sp["acts"], seed=5)
    gs = R.GSpec(sp["n_s"], cfg["G"], cfg["K"])
    gen = torch.Generator().manual_seed(6)
    g = torch.empty(tg, gs.P).uniform_(-cfg["init"], cfg["init"], generator=gen)
    h = torch.empty(sp["d"] * cfg["G"] + sp["d"]).uniform_(-cfg["init"], cfg["init"], generator=gen)
    return online, w, gs, g, h


def _tsf_stream(seed, cfg):
    sp, tg, b = cfg["spec"], cfg["tg"], cfg["b"]
    g = torch.Generator().manual_seed(seed)
    out = []
    for j in range(cfg["steps"]):
        batch = (torch.randn(b, sp["n_s"], generator=g), torch.randint(0, sp["A"], (b,), generator=g),
                 torch.rand(b, 1, generator=g), torch.rand(b, sp["d"], generator=g),
                 torch.randn(b, sp["n_s"], generator=g), torch.where(torch.rand(b, generator=g) < 0.2, 0.0, 0.9))
        out.append((batch, (3 * j + 1) % tg, torch.randn(sp["n_s"], generator=g)))
    return out


def _tsf_run_rank(rank, world, use_gpi, ar, bc, cfg=TSF_SMALL):
    from sfx.engine import SFEngine
    from sfx.shard import LibsfxTSFShardBackend, ShardedTSF

    sp, TGc, Bc = cfg["spec"], cfg["tg"], cfg["b"]
    online, w, gs, g, h = _tsf_problem(cfg)
    T_loc = TGc // world
    eng = SFEngine(T_loc, sp["n_s"], sp["H"], sp["A"], sp["d"], sp["acts"], max_batch=Bc)
    eng.set_adam(1e-3, 0.0, 1e-3, 0.0)
    eng.set_target_update_ev(EV)
    eng.tsf_setup(cfg["G"], cfg["K"], 1.0, 1e-3, 0.0, 1e-3, 0.0)
    be = LibsfxTSFShardBackend(eng, TGc, rank * T_loc, Bc)
    for t in range(T_loc):
        eng.load_head(t, online[rank * T_loc + t], 0)
        eng.load_head(t, online[rank * T_loc + t], 1)
        eng.tsf_load_g(t, g[rank * T_loc + t])
    for t in range(TGc):
        eng.load_w(t, w[t])
    eng.tsf_load_h(h)
    step = ShardedTSF(be, TGc, rank, sp["A"], ar, bc)
    dev = eng.device
    actions = []
    for batch, i, s in _tsf_stream(13, cfg):
        step.update(i, tuple(x.to(dev).contiguous() for x in batch), use_gpi=use_gpi)
        actions.append(step.select(s.to(dev).view(1, -1), i))
    out = (actions, torch.stack([eng.get_head(t) for t in range(T_loc)]),
           torch.stack([eng.tsf_get_g(t)[0] for t in range(T_loc)]), eng.tsf_get_h(),
           torch.stack([eng.get_w(t)[0] for t in range(TGc)]))
    eng.close()
    return out


def _tsf_oracle(use_gpi, cfg):
    spec = R.Spec(**cfg["spec"])
    online, w0, gs, g0, h0 = _tsf_problem(cfg)
    st = R.TSFState(spec, online.clone(), online.clone(), w0.clone(), gspec=gs, g=g0.clone(), h=h0.clone())
    want = []
    for batch, i, s in _tsf_stream(13, cfg):
        R.tsf_update(st, batch, i, use_gpi=use_gpi, target_update_ev=EV)
        qv, tk = R.gpi_w(R.psi_all(st.online, spec, s.view(1, -1)), st.w[i])
        want.append((int(tk[0]), R.select_action(qv, tk[0], i, True)))
    return want, st


def _tsf_check(res, use_gpi, cfg=TSF_SMALL):
    from tests.test_gpu_engine import params_close, rel_close

    actions, heads, gg, h, w = res
    want, st = _tsf_oracle(use_gpi, cfg)
    assert actions == want
    n = cfg["steps"]
    params_close(heads, st.online, 1e-3 * n)
    params_close(gg, st.g, 1e-3 * n)
    params_close(h, st.h, 1e-3 * n)
    rel_close(w, st.w, rtol=1e-4, atol=1e-7)


@pytest.mark.parametrize("use_gpi", [True, False])
def test_tsf_single_rank_shard_protocol(use_gpi):
    _tsf_check(_tsf_run_rank(0, 1, use_gpi, lambda t: None, lambda t, src: None), use_gpi)


def _tsf_worker(rank, port, q, cfg=TSF_SMALL):
    import torch.distributed as dist

    world = cfg.get("world", 2)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from sfx.shard import all_reduce_max_fn, broadcast_fn

    try:
        actions, heads, gg, h, w = _tsf_run_rank(rank, world, True, all_reduce_max_fn(via_host=True),
                                                 broadcast_fn(via_host=True), cfg)
        parts = [None] * world
        dist.all_gather_object(parts, (heads, gg))
        if rank == 0:
            q.put((actions, torch.cat([p[0] for p in parts]).numpy(), torch.cat([p[1] for p in parts]).numpy(),
                   h.numpy(), w.numpy()))
            q.close()
            q.join_thread()  # flushed into the pipe before the teardown
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("cfg", [TSF_SMALL, TSF_FULL, TSF_C5], ids=["small", "c5-shape", "c5-4x8-k100"])
def test_tsf_two_ranks_on_one_gpu(cfg):
    _tsf_check(_two_ranks(_tsf_worker, cfg), True, cfg)


# ---- the NATIVE sharded TSF loop (sfx_runner schedule "sharded_tsf") --------
def _native_tsf_rank(rank, world, cfg, comm, use_gpi=True, steps=10, task=None):
    """One rank of the native runner's sharded TSF step: T_glob / world heads, the env and replay
    replicated (same seed), every collective issued by libsfx (RCCL inside the step graphs, or the
    host transport for ranks sharing the GPU)."""
    from sfx.engine import SFEngine
    from sfx.runner import NativeEnvLoop
    from sfx.shard import init_comm, set_host_comm

    sp, TGc, Bc = cfg["spec"], cfg["tg"], cfg["b"]
    online, w, gs, g, h = _tsf_problem(cfg)
    T_loc = TGc // world
    eng = SFEngine(T_loc, sp["n_s"], sp["H"], sp["A"], sp["d"], sp["acts"], max_batch=Bc)
    eng.set_adam(1e-3, 0.0, 1e-3, 0.0)
    eng.set_target_update_ev(EV)
    eng.tsf_setup(cfg["G"], cfg["K"], 1.0, 1e-3, 0.0, 1e-3, 0.0)
    eng.shard_setup(TGc, rank * T_loc)
    for t in range(T_loc):
        eng.load_head(t, online[rank * T_loc + t], 0)
        eng.load_head(t, online[rank * T_loc + t], 1)
        eng.tsf_load_g(t, g[rank * T_loc + t])
    for t in range(TGc):
        eng.load_w(t, w[t])
    eng.tsf_load_h(h)
    if comm == "rccl":
        init_comm(eng, rank, world)
    else:
        set_host_comm(eng, rank, world)
    loop = NativeEnvLoop(eng, batch=Bc, capacity=300, gamma=0.9, epsilon=0.3, episode_len=9, seed=21,
                         schedule="sharded_tsf", upd_use_gpi=use_gpi, p_end=0.1)
    loop.prefill(Bc - 3)  # the first 2 steps run without a minibatch
    loop.set_task(TGc - 2 if task is None else task)  # owned by the last rank
    loop.record(steps)
    loop.run(steps)
    recs = loop.records()
    final = loop.action()
    stats = loop.stats()
    out = (recs, final, torch.stack([eng.get_head(t) for t in range(T_loc)]),
           torch.stack([eng.tsf_get_g(t)[0] for t in range(T_loc)]), eng.tsf_get_h(),
           torch.stack([eng.get_w(t)[0] for t in range(TGc)]), stats, loop.gpi_counters())
    loop.close()
    eng.close()
    return out


def _native_tsf_check(cfg, recs, final, heads, gg, h, w, use_gpi=True):
    from tests.test_gpu_engine import params_close, rel_close

    spec = R.Spec(**cfg["spec"])
    online, w0, gs, g0, h0 = _tsf_problem(cfg)
    st = R.TSFState(spec, online.clone(), online.clone(), w0.clone(), gspec=gs, g=g0.clone(), h=h0.clone())
    assert [r["have"] for r in recs[:4]] == [0, 0, 1, 1]
    for k, rec in enumerate(recs):
        task = rec["task"]
        if rec["have"]:
            batch = (torch.from_numpy(rec["s"]), torch.from_numpy(rec["a"]), torch.from_numpy(rec["rb"]).view(-1, 1),
                     torch.from_numpy(rec["phi"]), torch.from_numpy(rec["s1"]), torch.from_numpy(rec["gamma"]))
            R.tsf_update(st, batch, task, use_gpi=use_gpi, target_update_ev=EV)
        q, tk = R.gpi_w(R.psi_all(st.online, spec, torch.from_numpy(rec["snext"]).view(1, -1)), st.w[task])
        want = (int(tk[0]), R.select_action(q, tk[0], task, True))
        got = (recs[k + 1]["c"], recs[k + 1]["a_greedy"]) if k + 1 < len(recs) else final
        assert got == want, f"step {k}: runner selected {got}, oracle {want}"
    n = len(recs)
    params_close(heads, st.online, 1e-3 * n)
    params_close(gg, st.g, 1e-3 * n)
    params_close(h, st.h, 1e-3 * n)
    rel_close(w, st.w, rtol=1e-4, atol=1e-7)


@pytest.mark.parametrize("use_gpi,ahead", [(True, "1"), (False, "1"), (True, "0")],
                         ids=["gpi", "own-psi", "gpi-no-lookahead"])
def test_native_tsf_single_rank_rccl(use_gpi, ahead, monkeypatch):
    """World 1 with the library's own RCCL communicator, the collectives forced (SFX_RCCL_WORLD1=1):
    the GPI maxima all-reduce and the h / w_task ++ selection-table all-reduce are ncclAllReduce
    calls inside the pre-launched step graphs; with the look-ahead (default) each step's selection
    also forwards the next minibatch (select_ahead_body; the owner's TSF forward riding along).
    Every recorded env action bit-exact to the oracle's TSFDQN.update_successor replay
    (tsfdqn.py:588-709), parameters within tolerance."""
    monkeypatch.setenv("SFX_RCCL_WORLD1", "1")
    monkeypatch.setenv("SFX_AHEAD", ahead)
    recs, final, heads, gg, h, w, stats, counters = _native_tsf_rank(0, 1, TSF_SMALL, "rccl", use_gpi, steps=16)
    assert stats["prelaunched"] >= 8, stats
    assert counters.sum() == 16
    _native_tsf_check(TSF_SMALL, recs, final, heads, gg, h, w, use_gpi)


def _native_tsf_worker(rank, port, q, cfg):
    import torch.distributed as dist

    world = cfg.get("world", 2)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        recs, final, heads, gg, h, w, stats, _ = _native_tsf_rank(rank, world, cfg, "host", steps=10)
        parts = [None] * world
        dist.all_gather_object(parts, (heads, gg, [(r["c"], r["a_greedy"], r["a_taken"]) for r in recs]))
        if rank == 0:
            q.put((recs, final, torch.cat([p[0] for p in parts]).numpy(), torch.cat([p[1] for p in parts]).numpy(),
                   h.numpy(), w.numpy(), [p[2] for p in parts]))
            q.close()
            q.join_thread()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("cfg", [TSF_SMALL, TSF_C5], ids=["2x2-small", "c5-4x8-k100"])
def test_native_tsf_ranks_on_one_gpu(cfg):
    """The native sharded TSF loop at several ranks sharing this GPU (host transport over gloo),
    including BASELINE config C5 at its stated size (4 ranks x 8 Hopper TSF-NF heads, K = 100): the
    ranks record the same stream, and the oracle's in-order replay reproduces every env action."""
    recs, final, heads, gg, h, w, streams = _two_ranks(_native_tsf_worker, cfg)
    assert all(s == streams[0] for s in streams), "ranks diverged"
    _native_tsf_check(cfg, recs, final, heads, gg, h, w)
