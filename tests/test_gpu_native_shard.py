"""GPU parity of the NATIVE sharded all-task runner (sfx_runner schedule "sharded"; SURVEY §8e,
BASELINE config C4): each rank owns T_loc heads, every rank runs the same env / replay stream
(same seed), and the GPI maxima -- plus the selection table of the env action -- are all-reduced
(MAX) by the library itself, inside the step.

* one rank with an RCCL communicator the library creates (sfx_comm_init): the all-reduces are
  ncclAllReduce calls captured into the pre-launched step graphs;
* several ranks sharing this box's one GPU through the host transport (sfx_set_comm_host over
  gloo; RCCL refuses two ranks on one device), including C4 at its stated size: 8 ranks x 8
  Reacher heads = 64 source tasks, 256-wide heads, minibatch 32.

The oracle replays rank 0's recorded inputs with ALL heads in the reference's order
(agents/sfdqn.py:47-60 over features/deep.py) and must reproduce every recorded env action
(bit-exact GPI argmax); the gathered heads, target heads and w must match it within the Adam
tolerance of test_gpu_engine.py; every rank must have recorded the same stream."""
import os
import socket

import numpy as np
import pytest
import torch

from oracle import ref_cpu as R
from tests.conftest import gpu_available

pytestmark = pytest.mark.gpu

SMALL = dict(spec=dict(n_s=17, H=32, A=7, d=8, acts=("relu", "relu")), world=2, t_loc=2, b=16, steps=16, ev=5,
             eps=0.3, ep=7, prefill=8)
C4 = dict(spec=dict(n_s=17, H=256, A=7, d=8, acts=("relu", "relu")), world=8, t_loc=8, b=32, steps=6, ev=1000,
          eps=0.1, ep=500, prefill=30)
ALPHA = 0.05


@pytest.fixture(autouse=True)
def _need_gpu():
    if not gpu_available():
        pytest.skip("no HIP device")


def _run_rank(rank, cfg, comm, force_rerun=None, gate_timeout=None):
    from sfx.engine import SFEngine
    from sfx.init import reference_heads
    from sfx.runner import NativeEnvLoop
    from sfx.shard import init_comm, set_host_comm

    sp, world, T_loc, b = cfg["spec"], cfg["world"], cfg["t_loc"], cfg["b"]
    Tg = world * T_loc
    online, w = reference_heads(Tg, sp["n_s"], sp["H"], sp["A"], sp["d"], sp["acts"], seed=3)
    eng = SFEngine(T_loc, sp["n_s"], sp["H"], sp["A"], sp["d"], sp["acts"], max_batch=b)
    eng.set_adam(1e-3, 0.0, 1e-3, 0.0)
    eng.set_target_update_ev(cfg["ev"])
    eng.shard_setup(Tg, rank * T_loc)
    for t in range(T_loc):
        eng.load_head(t, online[rank * T_loc + t], 0)
        eng.load_head(t, online[rank * T_loc + t], 1)
    for t in range(Tg):
        eng.load_w(t, w[t])
    if comm == "rccl":
        init_comm(eng, rank, world)
    else:
        set_host_comm(eng, rank, world)
    loop = NativeEnvLoop(eng, batch=b, capacity=500, gamma=0.9, epsilon=cfg["eps"], alpha_w=ALPHA,
                         episode_len=cfg["ep"], seed=17, schedule="sharded")
    if force_rerun is not None:
        eng.debug_force_rerun(force_rerun)  # every step's device rounds count as failed: host rounds
    loop.prefill(cfg["prefill"])  # the first steps run without a minibatch
    loop.set_task(Tg - 1)
    if gate_timeout is not None:
        loop.set_gate_timeout(gate_timeout)
    loop.record(cfg["steps"])
    loop.run(cfg["steps"])
    recs = loop.records()
    final = loop.action()
    stats = loop.stats()
    heads = torch.stack([eng.get_head(t) for t in range(T_loc)])
    targets = torch.stack([eng.get_head(t, 1) for t in range(T_loc)])
    ws = torch.stack([eng.get_w(t)[0] for t in range(Tg)])
    counters = loop.gpi_counters()
    loop.close()
    eng.close()
    return recs, final, heads, targets, ws, stats, counters


def _oracle_check(cfg, recs, final, heads, targets, ws):
    from tests.test_gpu_engine import params_close, rel_close
    from tests.test_gpu_runner import replay_with_oracle

    sp, Tg = cfg["spec"], cfg["world"] * cfg["t_loc"]
    spec = R.Spec(**sp)
    from sfx.init import reference_heads

    online, w = reference_heads(Tg, sp["n_s"], sp["H"], sp["A"], sp["d"], sp["acts"], seed=3)
    st = R.SFState(spec, online.clone(), online.clone(), w.clone())
    replay_with_oracle(st, spec, recs, ALPHA, cfg["ev"], final)
    n = len(recs)
    params_close(heads, st.online, 1e-3 * n)
    params_close(targets, st.target, 1e-3 * n)
    rel_close(ws, st.w, rtol=1e-5, atol=1e-7)


@pytest.mark.parametrize("fused,force", [(True, True), (False, True), (True, False)],
                         ids=["fused-maxima", "qmax-launches", "no-collective-8-step-graphs"])
def test_native_sharded_single_rank_rccl(fused, force, monkeypatch):
    """World 1 with the library's own RCCL communicator; SFX_RCCL_WORLD1=1 makes the one-rank
    all-reduces real ncclAllReduce calls inside the step graphs, pre-launched behind the step in
    flight as at N > 1 (host rounds all-reduce on the split-off communicator); without it there is
    nothing to reduce.  fused: the maxima come out of the ψ output layer's
    forward tiles (d | 16); else from separate k_qmax launches."""
    if force:
        monkeypatch.setenv("SFX_RCCL_WORLD1", "1")
    if not fused:
        monkeypatch.setenv("SFX_SHARD_QA", "0")
    cfg = dict(SMALL, world=1, t_loc=4)
    recs, final, heads, targets, ws, stats, counters = _run_rank(0, cfg, "rccl")
    # pre-launched behind the step in flight (the host rounds have their own communicator), none
    # across a target sync (every 5 updates here)
    assert stats["prelaunched"] >= cfg["steps"] // 2, stats
    assert counters.sum() == cfg["steps"]
    _oracle_check(cfg, recs, final, heads, targets, ws)


@pytest.mark.parametrize("t_loc,force", [(40, None), (64, 1)], ids=["40-heads", "64-heads-host-rounds"])
def test_native_sharded_single_rank_many_heads(t_loc, force, monkeypatch):
    """BASELINE config C4's 64 source tasks on ONE GPU: the sharded schedule at
    world 1 with T_loc * A > 256 takes its GPI maxima from the wide kernels (k_qmaxw: one workgroup
    per (row, 8 policies), lane = head), three device rounds by
    default (T_glob >= 16) with round skipping in the unfused TD launch (tdg_skip_report) -- through
    real RCCL all-reduces and, forced, host rounds.  Every env action bit-exact to the in-order
    oracle."""
    monkeypatch.setenv("SFX_RCCL_WORLD1", "1")
    cfg = dict(SMALL, spec=dict(n_s=17, H=16, A=7, d=8, acts=("relu", "relu")), world=1, t_loc=t_loc, steps=14)
    recs, final, heads, targets, ws, stats, counters = _run_rank(0, cfg, "rccl", force_rerun=force)
    assert counters.sum() == cfg["steps"]
    if force is not None:
        assert stats["host_round_steps"] >= 4, stats
    _oracle_check(cfg, recs, final, heads, targets, ws)


def test_native_sharded_rccl_host_rounds_pipelined(monkeypatch):
    """Host rounds on the split communicator while the next step is pre-launched: RCCL forced at
    world 1, every step's device rounds treated as failed (sfx_debug_force_rerun), so each step's
    host rounds all-reduce on the host-round communicator (side stream) while the next step's
    graph -- with its own all-reduces on the step communicator -- already waits at its gate.
    The oracle replay must still reproduce every env action and the parameters."""
    monkeypatch.setenv("SFX_RCCL_WORLD1", "1")
    cfg = dict(SMALL, world=1, t_loc=4)
    recs, final, heads, targets, ws, stats, counters = _run_rank(0, cfg, "rccl", force_rerun=1)
    assert stats["host_round_steps"] >= 4, stats
    assert stats["prelaunched"] >= cfg["steps"] // 2, stats
    _oracle_check(cfg, recs, final, heads, targets, ws)


def test_native_sharded_one_rank_gate_timeouts_recompute():
    """one rank, no collective, a 10 ns gate bound and every step's device rounds
    treated as failed: each step's host rounds find the next pre-launched steps cancelled at their
    gates (their launches ran over the step's transient buffers), so the runner recomputes the
    step's forward and device rounds from the pre-step slot before its host rounds -- as the
    all-task schedule does -- instead of failing the run.  The oracle replay must still reproduce
    every env action and the parameters."""
    cfg = dict(SMALL, world=1, t_loc=4)
    recs, final, heads, targets, ws, stats, counters = _run_rank(0, cfg, "rccl", force_rerun=1, gate_timeout=1e-8)
    assert stats["retried"] > 0 and stats["recomputed"] > 0, stats
    assert counters.sum() == cfg["steps"]
    _oracle_check(cfg, recs, final, heads, targets, ws)


def test_native_sharded_wait_bound_aborts_communicators(monkeypatch):
    """a sharded step whose result never arrives (here: a one-shot 4 s stall
    of the finish kernel, after the step's all-reduces) is bounded by sfx_runner_wait_timeout --
    the runner cancels and drains what it can, reads RCCL's async error, aborts both
    communicators and raises; later collectives fail fast instead of hanging, and the handle
    still closes."""
    import time

    from sfx._lib import SFXError
    from sfx.engine import SFEngine
    from sfx.init import reference_heads
    from sfx.runner import NativeEnvLoop
    from sfx.shard import init_comm

    monkeypatch.setenv("SFX_RCCL_WORLD1", "1")
    monkeypatch.setenv("SFX_RUNNER_PIPELINE", "0")  # nothing queued behind the stalled step
    sp = SMALL["spec"]
    T = 2
    online, w = reference_heads(T, sp["n_s"], sp["H"], sp["A"], sp["d"], sp["acts"], seed=3)
    eng = SFEngine(T, sp["n_s"], sp["H"], sp["A"], sp["d"], sp["acts"], max_batch=16)
    eng.set_adam(1e-3, 0.0, 1e-3, 0.0)
    eng.shard_setup(T, 0)
    for t in range(T):
        eng.load_head(t, online[t], 0)
        eng.load_head(t, online[t], 1)
        eng.load_w(t, w[t])
    init_comm(eng, 0, 1)
    assert eng.comm_state() == dict(rccl=True, rounds_split=True, aborted=False, host=False)
    loop = NativeEnvLoop(eng, batch=16, capacity=200, gamma=0.9, epsilon=0.2, alpha_w=ALPHA, episode_len=50,
                         seed=5, schedule="sharded")
    loop.prefill(20)
    loop.set_task(0)
    loop.run(3)
    loop.set_wait_timeout(1.0)
    eng.debug_stall(4.0)
    t0 = time.time()
    with pytest.raises(SFXError, match="did not complete within 1 s.*communicators aborted"):
        loop.run(3)
    assert time.time() - t0 < 20.0
    assert eng.comm_state()["aborted"]
    t0 = time.time()
    with pytest.raises(SFXError, match="aborted after a collective timed out"):
        loop.run(1)
    assert time.time() - t0 < 5.0
    loop.close()
    eng.close()


def _worker(rank, port, q, cfg):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), **cfg.get("env", {}))
    dist.init_process_group("gloo", rank=rank, world_size=cfg["world"])
    try:
        recs, final, heads, targets, ws, stats, _ = _run_rank(rank, cfg, "host")
        parts = [None] * cfg["world"]
        dist.all_gather_object(parts, (heads.numpy(), targets.numpy(), [(r["c"], r["a_greedy"], r["a_taken"])
                                                                        for r in recs]))
        if rank == 0:
            q.put((recs, final, np.concatenate([p[0] for p in parts]), np.concatenate([p[1] for p in parts]),
                   ws.numpy(), stats, [p[2] for p in parts]))
            q.close()
            q.join_thread()  # flushed into the pipe before the teardown
    finally:
        dist.destroy_process_group()


def _ranks(cfg):
    import torch.multiprocessing as mp

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, port, q, cfg)) for r in range(cfg["world"])]
    for p in procs:
        p.start()
    out = q.get(timeout=600)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    return out


# d = 6 does not divide 16: the maxima of every round come from k_qmax launches
ODD_D = dict(SMALL, spec=dict(n_s=9, H=32, A=5, d=6, acts=("relu", "relu")), world=3, t_loc=2)


@pytest.mark.parametrize("cfg", [SMALL, dict(SMALL, env={"SFX_SHARD_QA": "0"}), ODD_D, C4],
                         ids=["2x2-small", "2x2-qmax-launches", "3x2-d6", "c4-8x8-h256"])
def test_native_sharded_ranks_on_one_gpu(cfg):
    recs, final, heads, targets, ws, stats, streams = _ranks(cfg)
    assert all(s == streams[0] for s in streams), "ranks diverged"
    assert len(recs) == cfg["steps"]
    _oracle_check(cfg, recs, final, torch.from_numpy(heads), torch.from_numpy(targets), torch.from_numpy(ws))
