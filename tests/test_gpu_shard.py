"""GPU check of the sharded all-task step (sfx_shard_* kernels + sfx.shard.ShardedAllTask):
two ranks share this box's GPU, each owning half of the heads; the all-reduces run over gloo
through host memory (RCCL needs one GPU per rank; the data path of the kernels is the same).
Against the unsharded oracle: identical env actions (GPI argmax, bit-exact), heads within the
Adam tolerance of test_gpu_engine.py."""
import os
import socket

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


def _stream(seed):
    g = torch.Generator().manual_seed(seed)
    out = []
    for j in range(STEPS):
        batch = None
        if j > 0:
            batch = (torch.randn(B, SPEC["n_s"], generator=g), torch.randint(0, SPEC["A"], (B,), generator=g),
                     torch.rand(B, SPEC["d"], generator=g), torch.randn(B, SPEC["n_s"], generator=g),
                     torch.where(torch.rand(B, generator=g) < 0.2, 0.0, 0.9))
        out.append((batch, j % TG, torch.rand(SPEC["d"], generator=g), torch.rand(1, generator=g),
                    torch.randn(SPEC["n_s"], generator=g)))
    return out


def _run_rank(rank, world, rounds, ar):
    from sfx.engine import SFEngine
    from sfx.init import reference_heads
    from sfx.shard import LibsfxShardBackend, ShardedAllTask

    online, w = reference_heads(TG, SPEC["n_s"], SPEC["H"], SPEC["A"], SPEC["d"], SPEC["acts"], seed=3)
    T_loc = TG // world
    eng = SFEngine(T_loc, SPEC["n_s"], SPEC["H"], SPEC["A"], SPEC["d"], SPEC["acts"], max_batch=B)
    eng.set_adam(1e-3, 0.0, 1e-3, 0.0)
    eng.set_target_update_ev(EV)
    be = LibsfxShardBackend(eng, TG, rank * T_loc, B)
    for t in range(T_loc):
        eng.load_head(t, online[rank * T_loc + t], 0)
        eng.load_head(t, online[rank * T_loc + t], 1)
    for t in range(TG):
        eng.load_w(t, w[t])
    step = ShardedAllTask(be, TG, SPEC["A"], ar, rounds=rounds)
    actions = []
    dev = eng.device
    for batch, task, phi1, r1, s_next in _stream(11):
        db = None if batch is None else tuple(x.to(dev).contiguous() for x in batch)
        actions.append(step.step(db, task, phi1.to(dev), r1.to(dev), 0.05, s_next.to(dev), task))
    heads = torch.stack([eng.get_head(t) for t in range(T_loc)])
    targets = torch.stack([eng.get_head(t, 1) for t in range(T_loc)])
    ws = torch.stack([eng.get_w(t)[0] for t in range(TG)])
    eng.close()
    return actions, heads, targets, ws, step.stats


def _oracle():
    spec = R.Spec(**SPEC)
    from sfx.init import reference_heads

    online, w0 = reference_heads(TG, SPEC["n_s"], SPEC["H"], SPEC["A"], SPEC["d"], SPEC["acts"], seed=3)
    st = R.SFState(spec, online.clone(), online.clone(), w0.clone())
    want = []
    for batch, task, phi1, r1, s_next in _stream(11):
        st.w[task] = R.lms_update(st.w[task].view(-1, 1), phi1, r1[0], 0.05).view(-1)
        if batch is not None:
            R.deep_all_task_step(st, batch, lr=1e-3, target_update_ev=EV)
        qv, tk = R.gpi_w(R.psi_all(st.online, spec, s_next.view(1, -1)), st.w[task])
        want.append((int(tk[0]), R.select_action(qv, tk[0], task, True)))
    return want, st


def _check(actions, heads, targets, ws, want, st):
    from tests.test_gpu_engine import params_close, rel_close

    assert actions == want
    params_close(heads, st.online, 1e-3 * STEPS)
    params_close(targets, st.target, 1e-3 * STEPS)
    rel_close(ws, st.w, rtol=1e-5, atol=1e-7)


@pytest.mark.parametrize("rounds", [1, 2])
def test_single_rank_shard_protocol(rounds):
    actions, heads, targets, ws, stats = _run_rank(0, 1, rounds, lambda t: None)
    want, st = _oracle()
    _check(actions, heads, targets, ws, want, st)
    assert stats["steps"] == STEPS - 1


def _worker(rank, port, q):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=2)
    from sfx.shard import all_reduce_max_fn

    try:
        actions, heads, targets, ws, stats = _run_rank(rank, 2, 2, all_reduce_max_fn(via_host=True))
        parts = [None, None]
        dist.all_gather_object(parts, (heads, targets))
        if rank == 0:
            q.put((actions, torch.cat([p[0] for p in parts]), torch.cat([p[1] for p in parts]), ws, stats))
    finally:
        dist.destroy_process_group()


def test_two_ranks_on_one_gpu():
    import torch.multiprocessing as mp

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    actions, heads, targets, ws, stats = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    want, st = _oracle()
    _check(actions, heads, targets, ws, want, st)


# ---- sharded TSF-DQN (sfx_shard_tsf_*, BASELINE config C5) ---------------------------------
TSF_SPEC = dict(n_s=11, H=32, A=9, d=6, acts=("relu", "relu"))
TSF_G, TSF_K, TSF_STEPS = 10, 3, 8


def _tsf_problem():
    from sfx.init import reference_heads

    online, w = reference_heads(TG, TSF_SPEC["n_s"], TSF_SPEC["H"], TSF_SPEC["A"], TSF_SPEC["d"], TSF_SPEC["acts"],
                                seed=5)
    gs = R.GSpec(TSF_SPEC["n_s"], TSF_G, TSF_K)
    gen = torch.Generator().manual_seed(6)
    g = torch.empty(TG, gs.P).uniform_(-0.3, 0.3, generator=gen)
    h = torch.empty(TSF_SPEC["d"] * TSF_G + TSF_SPEC["d"]).uniform_(-0.3, 0.3, generator=gen)
    return online, w, gs, g, h


def _tsf_stream(seed):
    g = torch.Generator().manual_seed(seed)
    out = []
    for j in range(TSF_STEPS):
        batch = (torch.randn(B, TSF_SPEC["n_s"], generator=g), torch.randint(0, TSF_SPEC["A"], (B,), generator=g),
                 torch.rand(B, 1, generator=g), torch.rand(B, TSF_SPEC["d"], generator=g),
                 torch.randn(B, TSF_SPEC["n_s"], generator=g), torch.where(torch.rand(B, generator=g) < 0.2, 0.0, 0.9))
        out.append((batch, (3 * j + 1) % TG, torch.randn(TSF_SPEC["n_s"], generator=g)))
    return out


def _tsf_run_rank(rank, world, use_gpi, ar, bc):
    from sfx.engine import SFEngine
    from sfx.shard import LibsfxTSFShardBackend, ShardedTSF

    online, w, gs, g, h = _tsf_problem()
    T_loc = TG // world
    eng = SFEngine(T_loc, TSF_SPEC["n_s"], TSF_SPEC["H"], TSF_SPEC["A"], TSF_SPEC["d"], TSF_SPEC["acts"], max_batch=B)
    eng.set_adam(1e-3, 0.0, 1e-3, 0.0)
    eng.set_target_update_ev(EV)
    eng.tsf_setup(TSF_G, TSF_K, 1.0, 1e-3, 0.0, 1e-3, 0.0)
    be = LibsfxTSFShardBackend(eng, TG, rank * T_loc, B)
    for t in range(T_loc):
        eng.load_head(t, online[rank * T_loc + t], 0)
        eng.load_head(t, online[rank * T_loc + t], 1)
        eng.tsf_load_g(t, g[rank * T_loc + t])
    for t in range(TG):
        eng.load_w(t, w[t])
    eng.tsf_load_h(h)
    step = ShardedTSF(be, TG, rank, TSF_SPEC["A"], ar, bc)
    dev = eng.device
    actions = []
    for batch, i, s in _tsf_stream(13):
        step.update(i, tuple(x.to(dev).contiguous() for x in batch), use_gpi=use_gpi)
        actions.append(step.select(s.to(dev).view(1, -1), i))
    out = (actions, torch.stack([eng.get_head(t) for t in range(T_loc)]),
           torch.stack([eng.tsf_get_g(t)[0] for t in range(T_loc)]), eng.tsf_get_h(),
           torch.stack([eng.get_w(t)[0] for t in range(TG)]))
    eng.close()
    return out


def _tsf_oracle(use_gpi):
    spec = R.Spec(**TSF_SPEC)
    online, w0, gs, g0, h0 = _tsf_problem()
    st = R.TSFState(spec, online.clone(), online.clone(), w0.clone(), gspec=gs, g=g0.clone(), h=h0.clone())
    want = []
    for batch, i, s in _tsf_stream(13):
        R.tsf_update(st, batch, i, use_gpi=use_gpi, target_update_ev=EV)
        qv, tk = R.gpi_w(R.psi_all(st.online, spec, s.view(1, -1)), st.w[i])
        want.append((int(tk[0]), R.select_action(qv, tk[0], i, True)))
    return want, st


def _tsf_check(res, use_gpi):
    from tests.test_gpu_engine import params_close, rel_close

    actions, heads, gg, h, w = res
    want, st = _tsf_oracle(use_gpi)
    assert actions == want
    params_close(heads, st.online, 1e-3 * TSF_STEPS)
    params_close(gg, st.g, 1e-3 * TSF_STEPS)
    params_close(h, st.h, 1e-3 * TSF_STEPS)
    rel_close(w, st.w, rtol=1e-3, atol=1e-6)


@pytest.mark.parametrize("use_gpi", [True, False])
def test_tsf_single_rank_shard_protocol(use_gpi):
    _tsf_check(_tsf_run_rank(0, 1, use_gpi, lambda t: None, lambda t, src: None), use_gpi)


def _tsf_worker(rank, port, q):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=2)
    from sfx.shard import all_reduce_max_fn, broadcast_fn

    try:
        actions, heads, gg, h, w = _tsf_run_rank(rank, 2, True, all_reduce_max_fn(via_host=True),
                                                 broadcast_fn(via_host=True))
        parts = [None, None]
        dist.all_gather_object(parts, (heads, gg))
        if rank == 0:
            q.put((actions, torch.cat([p[0] for p in parts]), torch.cat([p[1] for p in parts]), h, w))
    finally:
        dist.destroy_process_group()


def test_tsf_two_ranks_on_one_gpu():
    import torch.multiprocessing as mp

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_tsf_worker, args=(r, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    _tsf_check(res, True)
