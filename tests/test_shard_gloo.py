"""Multi-rank (gloo, world size 2, CPU) check of the sharded all-task step: heads split over
ranks, GPI maxima and the selection key all-reduced (MAX).  Against the unsharded oracle
(agents/sfdqn.py:47-60 over features/deep.py in index order): same env actions, same heads."""
import os
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import ref_cpu as R

SPEC = dict(n_s=6, H=16, A=5, d=4, acts=("relu", "relu"))
TG, WORLD, STEPS, EV = 4, 2, 6, 3


def _stream(seed):
    g = torch.Generator().manual_seed(seed)
    out = []
    for j in range(STEPS):
        B = 0 if j == 0 else 8
        batch = None
        if B:
            batch = (torch.randn(B, SPEC["n_s"], generator=g), torch.randint(0, SPEC["A"], (B,), generator=g),
                     torch.rand(B, SPEC["d"], generator=g), torch.randn(B, SPEC["n_s"], generator=g),
                     torch.where(torch.rand(B, generator=g) < 0.2, 0.0, 0.9))
        out.append((batch, j % TG, torch.rand(SPEC["d"], generator=g), torch.rand(1, generator=g),
                    torch.randn(SPEC["n_s"], generator=g)))
    return out


def _heads():
    from sfx.init import reference_heads

    return reference_heads(TG, SPEC["n_s"], SPEC["H"], SPEC["A"], SPEC["d"], SPEC["acts"], seed=3)


def _worker(rank, port, q, rounds):
    # a file rendezvous: no TCP port to race other processes for
    dist.init_process_group("gloo", init_method="file://" + port, rank=rank, world_size=WORLD)
    from sfx.shard import ShardedAllTask, all_reduce_max_fn
    from tests.shard_oracle import OracleShardBackend

    spec = R.Spec(**SPEC)
    online, w = _heads()
    T_loc = TG // WORLD
    sl = slice(rank * T_loc, (rank + 1) * T_loc)
    be = OracleShardBackend(spec, online[sl], online[sl], w, rank * T_loc, target_update_ev=EV)
    step = ShardedAllTask(be, TG, SPEC["A"], all_reduce_max_fn(), rounds=rounds)
    actions = []
    for batch, task, phi1, r1, s_next in _stream(11):
        actions.append(step.step(batch, task, phi1, r1, 0.05, s_next, task))
    heads = [None] * WORLD
    dist.all_gather_object(heads, be.st.online)
    if rank == 0:
        # numpy, pickled by value: a torch tensor goes through a shared-memory fd that the parent
        # fetches from this process while unpickling -- refused once this process has exited
        q.put((actions, torch.cat(heads).numpy(), np.asarray(be.w), step.stats))
        q.close()
        q.join_thread()  # the result is in the pipe before the teardown (a crash there reset the pipe once)
    dist.destroy_process_group()


def _free_port():
    """A fresh rendezvous file for the ranks' FileStore (the name kept from the TCP version)."""
    fd, path = tempfile.mkstemp(prefix="sfx_gloo_")
    os.close(fd)
    os.unlink(path)  # the store creates it; a leftover file would carry an old run's keys
    return path


@pytest.mark.parametrize("rounds", [1, 2])
def test_sharded_step_matches_unsharded_oracle(rounds):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, port, q, rounds)) for r in range(WORLD)]
    for p in procs:
        p.start()
    actions, heads, w, stats = q.get(timeout=300)
    heads, w = torch.from_numpy(heads), torch.from_numpy(w)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # unsharded reference order
    spec = R.Spec(**SPEC)
    online, w0 = _heads()
    st = R.SFState(spec, online.clone(), online.clone(), w0.clone())
    want = []
    for batch, task, phi1, r1, s_next in _stream(11):
        st.w[task] = R.lms_update(st.w[task].view(-1, 1), phi1, r1[0], 0.05).view(-1)
        if batch is not None:
            R.deep_all_task_step(st, batch, lr=1e-3, target_update_ev=EV)
        qv, tk = R.gpi_w(R.psi_all(st.online, spec, s_next.view(1, -1)), st.w[task])
        want.append((int(tk[0]), R.select_action(qv, tk[0], task, True)))
    assert actions == want
    assert torch.allclose(heads, st.online, rtol=1e-5, atol=1e-6)
    assert torch.allclose(w, st.w)
    assert stats["steps"] == STEPS - 1
    if rounds == 1:  # one device round rarely verifies: the extra-round path must have run
        assert stats["host_round_steps"] > 0


# ---- sharded TSF-DQN (BASELINE config C5; sfx.shard.ShardedTSF) -----------------------------
TSF_SPEC = dict(n_s=5, H=16, A=4, d=3, acts=("relu", "relu"))
TSF_G, TSF_K, TSF_STEPS = 6, 2, 7


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
    B, out = 8, []
    for j in range(TSF_STEPS):
        batch = (torch.randn(B, TSF_SPEC["n_s"], generator=g), torch.randint(0, TSF_SPEC["A"], (B,), generator=g),
                 torch.rand(B, 1, generator=g), torch.rand(B, TSF_SPEC["d"], generator=g),
                 torch.randn(B, TSF_SPEC["n_s"], generator=g), torch.where(torch.rand(B, generator=g) < 0.2, 0.0, 0.9))
        out.append((batch, (3 * j + 1) % TG, torch.randn(TSF_SPEC["n_s"], generator=g)))
    return out


def _tsf_worker(rank, port, q, use_gpi):
    # a file rendezvous: no TCP port to race other processes for
    dist.init_process_group("gloo", init_method="file://" + port, rank=rank, world_size=WORLD)
    from sfx.shard import ShardedTSF, all_reduce_max_fn, broadcast_fn
    from tests.shard_oracle import OracleTSFShardBackend

    spec = R.Spec(**TSF_SPEC)
    online, w, gs, g, h = _tsf_problem()
    T_loc = TG // WORLD
    sl = slice(rank * T_loc, (rank + 1) * T_loc)
    be = OracleTSFShardBackend(spec, gs, online[sl], online[sl], g[sl], h, w, rank * T_loc, target_update_ev=EV)
    step = ShardedTSF(be, TG, rank, TSF_SPEC["A"], all_reduce_max_fn(), broadcast_fn())
    actions = []
    for batch, i, s in _tsf_stream(13):
        step.update(i, batch, use_gpi=use_gpi)
        actions.append(step.select(s, i))
    parts = [None] * WORLD
    dist.all_gather_object(parts, (be.st.online, be.st.g))
    if rank == 0:
        q.put((actions, torch.cat([p[0] for p in parts]).numpy(), torch.cat([p[1] for p in parts]).numpy(),
               np.asarray(be.st.h), np.asarray(be.w)))  # by value (see _worker)
        q.close()
        q.join_thread()
    dist.destroy_process_group()


@pytest.mark.parametrize("use_gpi", [True, False])
def test_sharded_tsf_matches_unsharded_oracle(use_gpi):
    """tsfdqn.py's update_successor over a stream of active tasks owned by both ranks: GPI
    maxima all-reduced, the owner's update, h and w_i broadcast from the owner; env actions
    by the all-reduced key.  Same actions, heads, g_i, h and w as the unsharded oracle."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_tsf_worker, args=(r, port, q, use_gpi)) for r in range(WORLD)]
    for p in procs:
        p.start()
    actions, heads, gg, h, w = q.get(timeout=300)
    heads, gg, h, w = (torch.from_numpy(x) for x in (heads, gg, h, w))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    spec = R.Spec(**TSF_SPEC)
    online, w0, gs, g0, h0 = _tsf_problem()
    st = R.TSFState(spec, online.clone(), online.clone(), w0.clone(), gspec=gs, g=g0.clone(), h=h0.clone())
    want = []
    for batch, i, s in _tsf_stream(13):
        R.tsf_update(st, batch, i, use_gpi=use_gpi, target_update_ev=EV)
        qv, tk = R.gpi_w(R.psi_all(st.online, spec, s.view(1, -1)), st.w[i])
        want.append((int(tk[0]), R.select_action(qv, tk[0], i, True)))
    assert actions == want
    assert torch.allclose(heads, st.online, rtol=1e-5, atol=1e-6)
    assert torch.allclose(gg, st.g, rtol=1e-5, atol=1e-6)
    assert torch.allclose(h, st.h, rtol=1e-5, atol=1e-6)
    assert torch.allclose(w, st.w, rtol=1e-5, atol=1e-6)
