#!/usr/bin/env python3
"""bench.py -- env steps/sec of SF-DQN on synthetic Reacher-shape tasks, MI355X.

Metric (BASELINE.json): "env steps/sec (whole node), Reacher 8-task SF-DQN at 1/2/4/8 MI355X".
One step = one Agent.next_sample iteration (agents/agent.py:195-261): GPI action selection
for the current state (B=1), ε-greedy, a synthetic Reacher-shape transition (|s|=17,
|a|=7, d=8), the LMS reward fit, replay append + uniform B=32 sample, and the SF update.
Default schedule "all" is the main_sfdqn_torch.py path (agents/sfdqn.py:47-60 over
features/deep.py): every one of the 8 heads is updated per env step.

Multi-GPU: one process per GPU.  `python bench.py --gpus N` (N > 1, no WORLD_SIZE in the env) is
its own launcher: the parent starts N rank processes (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR
127.0.0.1 / MASTER_PORT) before anything touches the GPU, waits for them and exits with their
status; rank 0 prints the line.  Under `torch.distributed.run` (WORLD_SIZE set) it runs as that
rank.  The N > 1 headline is BASELINE config C4's layout: 8 heads per GPU, 8N source
tasks, ONE env stream replicated on every rank, GPI maxima all-reduced (MAX) over RCCL inside the
step graphs -- weak scaling in source tasks; N independent 8-head replicas are timed beside it
(`replicas`).  See DESIGN.md §7.

`other_workloads` (N=1 only; --no-other skips it) times the other one-GPU BASELINE configs through
the same native runner: the active-task schedule of sfdqn.py (C2 shape), Hopper TSF-DQN (C3) and
TSF-DQN with 100 planar layers (C5's per-GPU work); `--workload hopper-tsf[-nf]` makes one of
them the measured line instead.

Prints ONE JSON line on rank 0.  `roofline` is for the dominant kernel kind, measured live
in this process with HIP events (libsfx instrumentation, eager launches) right after the
timed region; `cpu_baseline` times the CPU oracle (oracle/ref_cpu.py) on a bounded sample
of the same workload on this box's host cores.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [ROOT, os.path.join(ROOT, "deep-successor-features-for-transfer_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

METRIC = "env steps/sec (whole node), Reacher 8-task SF-DQN at 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
MFMA_PEAK = {"fp32": 157.3e12, "bf16": 2.5e15}  # dense matrix peaks, MI355X_MICROARCH.md:42-43
CLK_HZ, SIMDS = 2.4e9, 256 * 4  # max clock, CUs x SIMDs (MI355X_MICROARCH.md:30-34)
SHAPE = dict(n_s=17, H=256, A=7, d=8, acts=("relu", "relu"))
# BASELINE.json configs C3 / C5 (one GPU): Hopper-shape TSF-DQN, |s|=11, 27 actions, d=50, 16 source
# tasks, g_i / h width 100; K planar layers in g_i for tsfdqn_nf.py (reacher.cfg n_coupling_layers=100)
TSF_SHAPE = dict(n_s=11, H=256, A=27, d=50, acts=("relu", "relu"), G=100)
C1_SHAPE = dict(n_s=4, H=256, A=2, d=20, acts=("relu", "relu"))  # BASELINE C1 (CartPole-v2)
WORKLOADS = {"reacher-sf": None, "hopper-tsf": 0, "hopper-tsf-nf": 100}
KIND_NAMES = {"fwd": "k_fwd", "tdg": "k_tdg", "bwd": "k_bwd", "gpi": "k_gpi", "lms": "k_lms", "ver": "k_ver",
              "tsf": "k_tsf"}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=None,
                   help="ranks (one per GPU); N > 1 without WORLD_SIZE: this process launches the N ranks")
    p.add_argument("--steps", type=int, default=2000)
    p.add_argument("--warmup", type=int, default=200)
    p.add_argument("--schedule", choices=["all", "active"], default="all")
    p.add_argument("--loop", choices=["native", "python"], default="native",
                   help="native: libsfx's C++ env-step runner (pipelined graphs); python: sfx.runner.EnvLoop")
    p.add_argument("--workload", choices=list(WORKLOADS), default="reacher-sf",
                   help="reacher-sf: the metric's workload (C2, default); hopper-tsf / hopper-tsf-nf: BASELINE "
                        "configs C3 / C5 on one GPU (TSF-DQN, active-task schedule, python host loop)")
    p.add_argument("--heads", type=int, default=None, help="source tasks (ψ heads) per GPU (8; 16 for hopper-tsf*)")
    p.add_argument("--batch", type=int, default=32)
    p.add_argument("--precision", choices=["fp32", "bf16"], default="fp32",
                   help="operands of the ψ forward / dX GEMMs (fp32: the reference's arithmetic, parity-tested)")
    p.add_argument("--replay", choices=["host", "device"], default="host",
                   help="replay ring on the host (north_star; the headline) or in HBM with on-device sampling "
                        "(SURVEY §8f rank 2; native loop only)")
    p.add_argument("--spec-rounds", type=int, default=0,
                   help="speculative rounds of the all-task step launched on the device (more run from the host); "
                        "0: libsfx's choice from the source-task count (2 below 16 tasks, 3 from 16)")
    p.add_argument("--prof-steps", type=int, default=50)
    p.add_argument("--repeats", type=int, default=3,
                   help="time the same K-step window this many more times after the measured one (spread only)")
    p.add_argument("--cpu-seconds", type=float, default=15.0)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-other", dest="other", action="store_false",
                   help="skip the other one-GPU configs (active-task C2, TSF C3, TSF-NF) reported beside the headline")
    p.add_argument("--layout", choices=["sharded", "replicas"], default="sharded",
                   help="N > 1 headline: the north-star sharded layout (C4: 8 heads per GPU, one env stream, "
                        "libsfx RCCL all-reduces; default) or N independent single-GPU replicas (side key otherwise)")
    p.add_argument("--shard-steps", type=int, default=400,
                   help="also time the north-star sharded mode (heads split over ranks, RCCL all-reduce-max "
                        "GPI) for this many env steps; 0 skips it")
    args = p.parse_args()
    args.tsf_K = WORKLOADS[args.workload]
    if args.heads is None:
        args.heads = 8 if args.tsf_K is None else 16
    if args.tsf_K is not None:
        args.schedule = "tsf"
    return args


def shape_of(args):
    if getattr(args, "c1", False):
        return C1_SHAPE
    return SHAPE if args.tsf_K is None else TSF_SHAPE


def tsf_problem(T: int, K: int, seed: int):
    """ψ heads as the reference lambda builds them; g_i = K planar layers (PlanarFlow.reset_parameters,
    tsfdqn_nf.py:341-345: weight, bias, scale ~ U(-0.01, 0.01)) + nn.Linear(n_s, G); h = nn.Linear(G, d)."""
    from sfx.init import reference_heads

    sh = TSF_SHAPE
    online, w = reference_heads(T, sh["n_s"], sh["H"], sh["A"], sh["d"], sh["acts"], seed=seed)
    gs = []
    for _ in range(T):
        parts = []
        for _k in range(K):
            parts += [torch.empty(sh["n_s"] + 1 + sh["n_s"]).uniform_(-0.01, 0.01)]
        lin = torch.nn.Linear(sh["n_s"], sh["G"])
        parts += [lin.weight.detach().reshape(-1), lin.bias.detach()]
        gs.append(torch.cat(parts))
    hl = torch.nn.Linear(sh["G"], sh["d"])
    return online, w, torch.stack(gs), torch.cat([hl.weight.detach().reshape(-1), hl.bias.detach()])


def head_params(sh) -> int:
    """P of SURVEY §8: parameters of one ψ head, (n_s·H + H) + n_hidden·(H² + H) + (H·A·d + A·d)."""
    n_s, H, A, d, nh = sh["n_s"], sh["H"], sh["A"], sh["d"], len(sh["acts"])
    return (n_s * H + H) + nh * (H * H + H) + (H * A * d + A * d)


def algorithmic_step_bytes(T: int, U: int, P: int, weight_bytes: int) -> float:
    """bytes one env step must move at minimum -- the action-select GPI reads all T
    heads, the update-path GPI over s' reads them once more, and each of the U updated heads is
    read by the target and online forwards and the backward, plus Adam's fp32 read of p, g, m, v
    (16 B) and write of p, m, v (12 B).  weight_bytes = 2 is §8(d)'s bf16-weights figure
    (U·P·34); 4 is the same count for fp32 weights, the arithmetic this build runs (U·P·40)."""
    wb = weight_bytes
    return 2.0 * wb * T * P + U * P * (3 * wb + 28)


def head_flops(sh) -> float:
    """f of SURVEY 8(d): forward FLOPs of one ψ head for one row, 2(n_s·H + n_hidden·H² + H·A·d)."""
    n_s, H, A, d, nh = sh["n_s"], sh["H"], sh["A"], sh["d"], len(sh["acts"])
    return 2.0 * (n_s * H + nh * H * H + H * A * d)


def mfma_from_profiles(kind: str, workload: str, precision: str):
    """MFMA counters per launch of `kind` from the committed rocprofv3 --pmc pass
    (profiles/pmc_mfma.json, tools/pmc_mfma.py), or None."""
    try:
        rec = json.load(open(os.path.join(ROOT, "profiles", "pmc_mfma.json")))
        return rec.get(workload + ("@bf16" if precision == "bf16" else ""), {}).get(KIND_NAMES[kind])
    except Exception:
        return None


def skippable_head_bytes(sh, M: int) -> float:
    """Algorithmic bytes (fp32, the formulas of sfx.hip run_bwd / run_fwd) of one head's work in one
    speculative round that a skipped policy does not move: dX of layers NL-1 .. 1, dW + Adam of
    every layer, the post-update forward of every layer."""
    n_s, H, A, d, nh = sh["n_s"], sh["H"], sh["A"], sh["d"], len(sh["acts"])
    layers = [(H, n_s)] + [(H, H)] * nh + [(A * d, H)]  # (N, K) per Linear
    dx = sum(4.0 * (N * K + M * N + 2.0 * M * K) for N, K in layers[1:])
    dw = sum(24.0 * (N * K + N) + 4.0 * (M * N + M * K) for N, K in layers)
    # and its post-update forward over the S1 rows ++ s_next (the head keeps last round's values)
    fw = sum(4.0 * (N * K + N + (M + 1) * K + (M + 1) * N) for N, K in layers)
    return dx + dw, fw  # (k_bwd launches, k_fwd launches)


def cpu_info() -> dict:
    """Host CPU model and physical core count (unique (package, core) pairs of /proc/cpuinfo)."""
    model, cores = None, set()
    try:
        phys = core = None
        for line in open("/proc/cpuinfo"):
            k, _, v = line.partition(":")
            k, v = k.strip(), v.strip()
            if k == "model name" and model is None:
                model = v
            elif k == "physical id":
                phys = v
            elif k == "core id":
                core = v
            elif not k and phys is not None:
                cores.add((phys, core))
                phys = core = None
        if phys is not None:
            cores.add((phys, core))
    except OSError:
        pass
    return {"cpu_model": model, "physical_cores_on_host": len(cores) or None, "logical_cpus_on_host": os.cpu_count()}


def cpu_share() -> int:
    """Host threads this job may use: the box allots a one-GPU job its CPU share through
    OMP_NUM_THREADS (16 on the MI355X pool, whose hosts have 128 physical cores shared by 8 GPUs);
    os.cpu_count() otherwise."""
    return min(int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or os.cpu_count(), os.cpu_count())


def cpu_baseline(args, seconds: float, threads: int = None):
    """The CPU oracle (a from-scratch PyTorch-CPU restatement of the reference path,
    oracle/ref_cpu.py) running the same env-step loop on the host cores."""
    from oracle import ref_cpu as R
    from sfx.init import reference_heads
    from sfx.runner import Replay, SynthHopper, SynthReacher

    cores = threads or cpu_share()
    torch.set_num_threads(cores)
    T, B = args.heads, args.batch
    sh = shape_of(args)
    spec = R.Spec(sh["n_s"], sh["H"], sh["A"], sh["d"], sh["acts"])
    if args.tsf_K is None:
        online, w = reference_heads(T, spec.n_s, spec.H, spec.A, spec.d, spec.acts, seed=0)
        st = R.SFState(spec, online.clone(), online.clone(), w.clone())
        task = SynthReacher(spec.n_s, spec.A, spec.d, 0, np.random.default_rng(1))
    else:
        online, w, g, h = tsf_problem(T, args.tsf_K, seed=0)
        st = R.TSFState(spec, online.clone(), online.clone(), w.clone(), gspec=R.GSpec(spec.n_s, sh["G"], args.tsf_K),
                        g=g.clone(), h=h.clone())
        task = SynthHopper(spec.n_s, spec.A, spec.d, 0, np.random.default_rng(1))
    rng = task.rng
    rep = Replay(100_000, spec.n_s, spec.d, rng)
    for _ in range(1000):
        s0 = task.initialize()
        a0 = int(rng.integers(spec.A))  # random actions, as the runners' prefill draws them
        s1, phi, r, _ = task.transition(a0)
        rep.append(s0, a0, r, phi, s1, 0.9)
    s = task.initialize()
    steps = 0
    t0 = time.perf_counter()
    with torch.no_grad():
        while True:
            q, c = R.gpi_w(R.psi_all(st.online, spec, torch.from_numpy(s).view(1, -1)), st.w[0])
            a = R.select_action(q, c[0], 0, True)
            if rng.random() <= 0.1:
                a = int(rng.integers(spec.A))
            s1, phi, r, term = task.transition(a)
            if args.schedule == "all":
                st.w[0] = R.lms_update(st.w[0].view(-1, 1), torch.from_numpy(phi), torch.tensor(r), 1e-3).view(-1)
            rep.append(s, a, r, phi, s1, 0.0 if term else 0.9)
            idx = rng.integers(0, rep.size, B)
            batch = (torch.from_numpy(rep.s[idx]), torch.from_numpy(rep.a[idx]), torch.from_numpy(rep.phi[idx]),
                     torch.from_numpy(rep.s1[idx]), torch.from_numpy(rep.gamma[idx]))
            if args.schedule == "all":
                R.deep_all_task_step(st, batch)
            else:
                b6 = (batch[0], batch[1], torch.from_numpy(rep.r[idx]).view(-1, 1), batch[2], batch[3], batch[4])
                if args.schedule == "tsf":
                    R.tsf_update(st, b6, 0, use_gpi=True)
                else:
                    R.sf_update(st, b6, 0, use_gpi=True)
            s = task.initialize() if term else s1
            steps += 1
            el = time.perf_counter() - t0
            if el >= seconds:
                break
    out = {"value": steps / el, "unit": "env steps/s", "cores": cores, "kind": "port",
           "sample": f"{steps} env steps ({el:.1f} s) of the same {args.schedule}-task loop, T={T}, B={B}, "
                     f"oracle/ref_cpu.py on torch CPU with {cores} threads (cores = torch intra-op threads used)"}
    out.update(cpu_info())
    return out


def bench_sharded(args, world, rank, device, barrier, dist, steps=None, warmup=None):
    """North-star multi-GPU layout (BASELINE config C4): T_loc = --heads heads per rank,
    T_glob = T_loc * world source tasks, ONE env / replay stream replicated on every rank with the
    same seed, every head updated per env step (agents/sfdqn.py:47-60), GPI maxima and the env
    action's q table all-reduced (MAX) by libsfx itself -- RCCL calls captured in the step graphs
    of the native runner (sfx_runner schedule "sharded").  Returns env-steps/s of that stream
    (max-over-ranks time)."""
    from sfx.engine import SFEngine
    from sfx.init import reference_heads
    from sfx.runner import NativeEnvLoop
    from sfx.shard import init_comm, set_host_comm

    steps = args.shard_steps if steps is None else steps
    warmup = max(20, steps // 10) if warmup is None else warmup
    T_loc, B = args.heads, args.batch
    Tg = T_loc * world
    eng = SFEngine(T_loc, SHAPE["n_s"], SHAPE["H"], SHAPE["A"], SHAPE["d"], SHAPE["acts"], max_batch=B, device=device)
    online, w = reference_heads(Tg, SHAPE["n_s"], SHAPE["H"], SHAPE["A"], SHAPE["d"], SHAPE["acts"], seed=0)
    eng.set_adam(1e-3, 0.0, 1e-3, 0.0)
    eng.set_target_update_ev(1000)
    eng.set_spec_rounds(args.spec_rounds)
    eng.set_precision(args.precision)
    eng.shard_setup(Tg, rank * T_loc)
    for t in range(T_loc):
        eng.load_head(t, online[rank * T_loc + t], 0)
        eng.load_head(t, online[rank * T_loc + t], 1)
    for t in range(Tg):
        eng.load_w(t, w[t])
    if args.via_host:
        set_host_comm(eng, rank, world)
    else:
        init_comm(eng, rank, world)
    loop = NativeEnvLoop(eng, batch=B, seed=1, schedule="sharded")
    loop.set_wait_timeout(30.0)  # a collective that never completes: abort + error, not a hang
    loop.prefill(1000)
    loop.set_task(0)
    loop.warm()
    loop.run(warmup)
    barrier()
    t0 = time.perf_counter()
    loop.run(steps)
    barrier()
    dt = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([dt], device="cpu" if args.via_host else device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    st = loop.stats()
    st.update(eng.step_stats())
    eng_comm = eng.comm_state()
    eng_comm.update(eng.comm_size())
    if world > 1 and not args.via_host and eng_comm["rccl_world"] != world:
        raise RuntimeError(f"RCCL communicator reports world {eng_comm['rccl_world']}, expected {world}")
    eng_comm["rccl_forced_world1"] = os.environ.get("SFX_RCCL_WORLD1") == "1"
    loop.close()
    eng.close()
    v = steps / dt
    return {"value": round(v, 2), "unit": "env steps/s", "ms_per_step": round(1000.0 * dt / steps, 4),
            "steps": steps, "warmup": warmup, "heads_total": Tg, "heads_per_gpu": T_loc,
            "head_updates_per_s": round(v * Tg, 1), "parallelism": f"heads sharded over {world} GPU(s)",
            "loop": "native C++ runner (sfx_runner schedule sharded): one pre-launched graph per env step",
            "comm": eng_comm,
            "collective": ("gloo via host (rehearsal)" if args.via_host else "RCCL (library-owned communicator)") +
                          " all-reduce(MAX): GPI maxima [T_glob,B,A] per speculative round, then verification "
                          "maxima ++ the env action's q table [T_glob,A] in one call",
            "rounds": st}


def bench_sharded_tsf(args, world, rank, device, barrier, dist, steps=None, warmup=None, heads=None):
    """BASELINE config C5 (tsfdqn_nf.py, 32 source tasks over 4 GPUs): T_loc = --heads per rank,
    T_glob = T_loc * world, one env / replay stream replicated on every rank (same seed), the native
    runner's "sharded_tsf" schedule: the active policy's GPI maxima and (one call) the owner's h and
    w_task ++ the env action's q table all-reduced (MAX) by libsfx inside the pre-launched step
    graphs (RCCL; the host transport for gloo rehearsals)."""
    from sfx.engine import SFEngine
    from sfx.runner import NativeEnvLoop
    from sfx.shard import init_comm, set_host_comm

    sh, B = TSF_SHAPE, args.batch
    T_loc = heads or args.heads
    Tg = T_loc * world
    steps = args.shard_steps if steps is None else steps
    warmup = max(20, steps // 10) if warmup is None else warmup
    eng = SFEngine(T_loc, sh["n_s"], sh["H"], sh["A"], sh["d"], sh["acts"], max_batch=B, device=device)
    eng.set_adam(1e-3, 0.0, 1e-3, 0.0)
    eng.set_target_update_ev(1000)
    eng.tsf_setup(sh["G"], args.tsf_K, 1.0, 1e-3, 0.0, 1e-3, 0.0)
    eng.shard_setup(Tg, rank * T_loc)
    online, w, g, h = tsf_problem(Tg, args.tsf_K, seed=0)
    for t in range(T_loc):
        eng.load_head(t, online[rank * T_loc + t], 0)
        eng.load_head(t, online[rank * T_loc + t], 1)
        eng.tsf_load_g(t, g[rank * T_loc + t])
    for t in range(Tg):
        eng.load_w(t, w[t])
    eng.tsf_load_h(h)
    if args.via_host:
        set_host_comm(eng, rank, world)
    else:
        init_comm(eng, rank, world)
    loop = NativeEnvLoop(eng, batch=B, seed=1, schedule="sharded_tsf", p_end=0.01)
    loop.set_wait_timeout(30.0)
    loop.prefill(1000)
    loop.set_task(0)
    loop.warm()
    loop.run(warmup)
    barrier()
    t0 = time.perf_counter()
    loop.run(steps)
    barrier()
    dt = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([dt], device="cpu" if args.via_host else device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    st = loop.stats()
    comm = eng.comm_state()
    comm.update(eng.comm_size())
    comm["rccl_forced_world1"] = os.environ.get("SFX_RCCL_WORLD1") == "1"
    loop.close()
    eng.close()
    v = steps / dt
    return {"value": round(v, 2), "unit": "env steps/s", "ms_per_step": round(1000.0 * dt / steps, 4),
            "steps": steps, "warmup": warmup, "heads_total": Tg, "heads_per_gpu": T_loc,
            "parallelism": f"TSF heads sharded over {world} GPU(s)",
            "loop": "native C++ runner (sfx_runner schedule sharded_tsf): one pre-launched graph per env step",
            "comm": comm, "prelaunched": st["prelaunched"],
            "collective": ("gloo via host (rehearsal)" if args.via_host else "RCCL (library-owned communicator)") +
                          " all-reduce(MAX): the active policy's GPI maxima [B,A], then the owner's h ++ w_task "
                          "(raw bits, a broadcast) ++ the env action's q table [T_glob,A] in one call"}


def bench_other_workloads(args, device, steps: int = 1000, warmup: int = 200) -> dict:
    """The other BASELINE configs that fit one GPU, each through the native runner on its own
    engine (reported beside the headline, never as `value`): the active-task schedule of
    sfdqn.py on the C2 shape, Hopper TSF-DQN (C3) and TSF-DQN with 100 planar layers (C5's
    per-GPU work).  env-steps/s of the same timed loop as the headline."""
    from sfx.engine import SFEngine
    from sfx.init import reference_heads
    from sfx.runner import NativeEnvLoop

    out = {}
    # the -fp32 / -bf16 pair: the headline workload in the same 1000-step window, operands in fp32
    # (the reference's arithmetic) and in bf16 (sfx_set_precision; not a parity mode)
    for name, sched, K, dev, prec in (("reacher17-active-T8-B32", "active", None, False, "fp32"),
                                      ("reacher17-all-T8-B32-device-replay", "all", None, True, "fp32"),
                                      ("reacher17-all-T8-B32-fp32", "all", None, False, "fp32"),
                                      ("reacher17-all-T8-B32-bf16", "all", None, False, "bf16"),
                                      ("hopper11-tsf-T16-B32", "tsf", 0, False, "fp32"),
                                      ("hopper11-tsf-T16-B32-bf16", "tsf", 0, False, "bf16"),
                                      ("hopper11-tsf-nf100-T16-B32", "tsf", 100, False, "fp32"),
                                      ("cartpole4-all-T2-B32", "all", None, False, "fp32")):
        # C1: CartPole-v2 SF-DQN (n_s 4, A 2, d 20: configs/cartpole_phi.cfg:52), 2 source tasks
        c1 = name.startswith("cartpole")
        sh = C1_SHAPE if c1 else SHAPE if K is None else TSF_SHAPE
        T = 2 if c1 else 8 if K is None else 16
        eng = SFEngine(T, sh["n_s"], sh["H"], sh["A"], sh["d"], sh["acts"], max_batch=args.batch, device=device)
        if K is None:
            online, w = reference_heads(T, sh["n_s"], sh["H"], sh["A"], sh["d"], sh["acts"], seed=0)
        else:
            online, w, g, h = tsf_problem(T, K, seed=0)
            eng.tsf_setup(sh["G"], K, 1.0, 1e-3, 0.0, 1e-3, 0.0)
            for t in range(T):
                eng.tsf_load_g(t, g[t])
            eng.tsf_load_h(h)
        for t in range(T):
            eng.load_head(t, online[t], 0)
            eng.load_head(t, online[t], 1)
            eng.load_w(t, w[t])
        eng.set_adam(1e-3, 0.0, 1e-3, 0.0)
        eng.set_target_update_ev(1000)
        eng.set_spec_rounds(args.spec_rounds)
        eng.set_precision(prec)
        loop = NativeEnvLoop(eng, batch=args.batch, seed=1, schedule=sched, p_end=0.0 if K is None else 0.01,
                             device_replay=dev)
        loop.prefill(1000)
        loop.set_task(0)
        loop.run(warmup)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        loop.run(steps)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        out[name] = {"value": round(steps / dt, 2), "unit": "env steps/s", "ms_per_step": round(1000.0 * dt / steps, 4),
                     "steps": steps, "dtype": prec}
        loop.close()
        eng.close()
    # BASELINE configs C4 / C5 in their sharded layouts on ONE GPU, every collective a real RCCL call
    # at world 1 (SFX_RCCL_WORLD1=1): C4's 64 Reacher tasks (the sharded all-task step, 3 device
    # rounds from 16 tasks on), and C5's per-rank share, 8 Hopper TSF-NF heads (schedule sharded_tsf)
    os.environ["SFX_RCCL_WORLD1"] = "1"
    try:
        c4 = argparse.Namespace(**vars(args))
        c4.heads, c4.spec_rounds, c4.via_host = 64, 0, False
        r = bench_sharded(c4, 1, 0, device, torch.cuda.synchronize, None, steps=2000, warmup=200)
        out["reacher17-sharded-T64-B32-rccl-world1"] = {k: r[k] for k in ("value", "unit", "ms_per_step", "steps",
                                                                          "heads_total")} | {
            "speculation": {k: r["rounds"][k] for k in ("steps", "host_round_steps", "rounds", "unverified_policies")},
            "layout": "BASELINE C4's 64 source tasks on one GPU: sharded schedule at world 1, RCCL forced"}
        c5 = argparse.Namespace(**vars(args))
        c5.heads, c5.tsf_K, c5.via_host, c5.shard_steps = 8, 100, False, 1000
        r = bench_sharded_tsf(c5, 1, 0, device, torch.cuda.synchronize, None, steps=1000, warmup=100)
        out["hopper11-sharded-tsf-nf100-T8-B32-rccl-world1"] = {k: r[k] for k in ("value", "unit", "ms_per_step", "steps",
                                                                                 "heads_total")} | {
            "layout": "BASELINE C5's per-GPU share (8 of 32 TSF-NF heads) through the sharded_tsf schedule, RCCL forced"}
    except Exception as e:  # an error return (a bounded collective), not a hang
        out["sharded-one-gpu-error"] = repr(e)[:400]
    finally:
        os.environ.pop("SFX_RCCL_WORLD1", None)
    # the drop-in: features.deep.DeepSF under the reference user's Python agent loop (tools/dropin_loop.py)
    from tools import dropin_loop

    # the median of three consecutive 1,000-step windows (≈0.25 s each with the alias buffer): one
    # 300-step window moved ±5 % run to run
    for buf in ("reference", "objring", "host"):
        out[f"reacher17-all-T8-B32-dropin-{buf}-buffer"] = dropin_loop.measure(
            buf, steps=1000, warmup=60, windows=3 if buf != "objring" else 1, batch=args.batch, device=device)
    # the test phase (agents/sfdqn.py:111-115): 8 test tasks one after the other as the reference
    # runs them, and in lockstep (sfx/lockstep.py, one sfx_test_actions launch set per step)
    from tools import test_phase

    for ls in (False, True):
        out[f"reacher-test-phase-E8-{'lockstep' if ls else 'sequential'}"] = test_phase.measure(ls, device=device)
    # the TSF agents' test phase (agents/tsfdqn_sequential.py:385-420) at the Hopper TSF shape:
    # the per-call drop-in binding vs sfx.lockstep.test_tasks_lockstep_tsf
    from tools import tsf_test_phase

    for ls in (False, True):
        out[f"hopper-tsf-test-phase-E8-{'lockstep' if ls else 'sequential'}"] = tsf_test_phase.measure(
            ls, device=device)
    return out


def traffic_from_profiles(kind: str, workload: str):
    """HBM bytes per launch of `kind` from a committed rocprofv3 --pmc pass (profiles/), or None."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(path):
        return None
    try:
        rec = json.load(open(path))
        ent = rec.get(workload, {}).get(KIND_NAMES[kind])
        return None if ent is None else float(ent["hbm_bytes_per_launch"])
    except Exception:
        return None


def rocprof_avg_from_profiles(kind: str):
    """Average duration (µs) of `kind`'s launches in the committed rocprofv3 --kernel-trace --stats
    summary of the headline workload (profiles/headline_kernel_stats.csv, copied from the latest
    round-end profile run), or None."""
    path = os.path.join(ROOT, "profiles", "headline_kernel_stats.csv")
    if not os.path.exists(path):
        return None
    try:
        import csv
        base = KIND_NAMES[kind]
        n = ns = 0.0
        for r in csv.DictReader(open(path)):
            name = r["Name"].split("(")[0].split("<")[0].split("::")[-1].strip()
            if name == base or name.startswith(base + "_"):
                n += float(r["Calls"])
                ns += float(r["TotalDurationNs"])
        return ns / n / 1000.0 if n else None
    except Exception:
        return None


def rocprof_window_from_profiles(kernel: str):
    """tools/rocprof_window.py's summary of the committed kernel trace of the default command: the
    average duration of `kernel`'s launches inside the bench's own prof window, or None."""
    path = os.path.join(ROOT, "profiles", "rocprof_window.json")
    try:
        d = json.load(open(path))
        return d if d.get("kernel") == kernel and d.get("window_launches") else None
    except Exception:
        return None


def unskipped_window(args, device, prof_steps: int, warmup: int = 200) -> dict:
    """The dominant kernel kind's live average over launches in which NO head skips: a fresh engine
    of the headline workload with round skipping off (SFX_SKIP=0 at its creation), the same warmup
    and an eagerly launched prof window like the headline's.  Every launch then moves its whole
    algorithmic bytes, so achieved / peak is the kernel's efficiency independent of how many
    policies the training phase lets skip."""
    from sfx.engine import SFEngine
    from sfx.init import reference_heads
    from sfx.runner import NativeEnvLoop

    sh, T, B = SHAPE, args.heads, args.batch
    old = os.environ.get("SFX_SKIP")
    os.environ["SFX_SKIP"] = "0"
    try:
        eng = SFEngine(T, sh["n_s"], sh["H"], sh["A"], sh["d"], sh["acts"], max_batch=B, device=device)
    finally:
        if old is None:
            os.environ.pop("SFX_SKIP", None)
        else:
            os.environ["SFX_SKIP"] = old
    online, w = reference_heads(T, sh["n_s"], sh["H"], sh["A"], sh["d"], sh["acts"], seed=0)
    for t in range(T):
        eng.load_head(t, online[t], 0)
        eng.load_head(t, online[t], 1)
        eng.load_w(t, w[t])
    eng.set_adam(1e-3, 0.0, 1e-3, 0.0)
    eng.set_target_update_ev(1000)
    eng.set_spec_rounds(args.spec_rounds)
    eng.set_precision(args.precision)
    loop = NativeEnvLoop(eng, batch=B, seed=1, schedule="all")
    loop.prefill(1000)
    loop.set_task(0)
    loop.warm()
    loop.run(warmup)
    eng.prof_reset()
    sk0 = eng.skip_stats()
    eng.prof_enable(True)
    loop.run(prof_steps)
    stats = eng.prof_collect()
    eng.prof_enable(False)
    skipped = eng.skip_stats()["policies_skipped"] - sk0["policies_skipped"]
    loop.close()
    eng.close()
    return {"stats": stats, "skipped": skipped, "steps": prof_steps}


def launch_ranks(n: int, argv=None, dry_run: bool = False) -> int:
    """`bench.py --gpus N` as its own launcher (N > 1 and no WORLD_SIZE in the environment): start
    N rank processes of this script, one per GPU, with the torch.distributed env contract
    (RANK, LOCAL_RANK, WORLD_SIZE, LOCAL_WORLD_SIZE, MASTER_ADDR=127.0.0.1, a free MASTER_PORT),
    wait for all of them and return the first nonzero exit status (0 if all succeed).  The parent
    never initialises the GPU (no torch.cuda call happens before this point), so the ranks own
    their devices; a rank that fails ends the others (their exact PIDs).  dry_run: the children
    print their rank env as one JSON line and exit (tests/test_bench_launch.py)."""
    import socket
    import subprocess

    argv = sys.argv[1:] if argv is None else list(argv)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        if dry_run:
            env["SFX_BENCH_DRYRUN"] = "1"
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env))
    rc = 0
    pending = list(procs)
    try:
        while pending:
            for p in list(pending):
                code = p.poll()
                if code is None:
                    continue
                pending.remove(p)
                if code != 0 and rc == 0:
                    rc = code
                    print(f"bench launcher: rank {procs.index(p)} exited with {code}; stopping the others",
                          file=sys.stderr, flush=True)
                    for q in pending:
                        q.terminate()
            if pending:
                time.sleep(0.05)
    finally:  # an interrupted launcher (KeyboardInterrupt, SIGTERM) leaves no rank behind
        for q in pending:
            if q.poll() is None:
                q.terminate()
        for q in pending:
            try:
                q.wait(timeout=10)
            except subprocess.TimeoutExpired:
                q.kill()
                q.wait()
    return rc


def main():
    args = parse()
    if args.gpus is not None and args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus is None:
        args.gpus = world
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    if os.environ.get("SFX_BENCH_DRYRUN") == "1":  # launcher test: report the rank env, touch no GPU
        print(json.dumps({k: os.environ.get(k) for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR",
                                                         "MASTER_PORT")} | {"gpus": args.gpus}), flush=True)
        return
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # SFX_BENCH_BACKEND=gloo rehearses the multi-rank path on a box with fewer GPUs than ranks
    # (ranks share GPUs, collectives through host memory); the real run is RCCL ("nccl").
    backend = os.environ.get("SFX_BENCH_BACKEND", "nccl")
    ndev = torch.cuda.device_count()
    local = local % max(ndev, 1) if backend == "gloo" else local
    if world > 1:
        import torch.distributed as dist

        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")
    else:
        dist = None
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)
    args.via_host = backend != "nccl"

    from sfx.engine import SFEngine
    from sfx.init import reference_heads
    from sfx.runner import EnvLoop, NativeEnvLoop, SynthHopper, SynthReacher

    T, B = args.heads, args.batch
    sh = shape_of(args)
    eng = SFEngine(T, sh["n_s"], sh["H"], sh["A"], sh["d"], sh["acts"], max_batch=B, device=device)
    if args.tsf_K is None:
        online, w = reference_heads(T, sh["n_s"], sh["H"], sh["A"], sh["d"], sh["acts"], seed=rank)
    else:
        online, w, g, h = tsf_problem(T, args.tsf_K, seed=rank)
        eng.tsf_setup(sh["G"], args.tsf_K, 1.0, 1e-3, 0.0, 1e-3, 0.0)
        for t in range(T):
            eng.tsf_load_g(t, g[t])
        eng.tsf_load_h(h)
    for t in range(T):
        eng.load_head(t, online[t], 0)
        eng.load_head(t, online[t], 1)
        eng.load_w(t, w[t])
    eng.set_adam(1e-3, 0.0, 1e-3, 0.0)
    eng.set_target_update_ev(1000)
    eng.set_spec_rounds(args.spec_rounds)
    eng.set_precision(args.precision)
    native = args.loop == "native"
    if native:
        loop = NativeEnvLoop(eng, batch=B, seed=1 + rank, schedule=args.schedule,
                             p_end=0.0 if args.tsf_K is None else 0.01, device_replay=args.replay == "device")
        loop.prefill(1000)
        loop.set_task(0)
        loop.warm()  # instantiate every step graph now: the timed steps replay graphs, never capture
    else:
        task_cls = SynthReacher if args.tsf_K is None else SynthHopper
        loop = EnvLoop(eng, schedule=args.schedule, batch=B, seed=1 + rank, task_cls=task_cls)
        loop.prefill(1000)

    def barrier():
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    loop.run(args.warmup)
    barrier()
    t0 = time.perf_counter()
    loop.run(args.steps)
    barrier()
    dt = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([dt], device="cpu" if args.via_host else device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    value = world * args.steps / dt
    # spread: the same K-step window timed again (not part of `value`)
    repeats = []
    if args.repeats > 0:
        for _ in range(args.repeats):
            barrier()
            t1 = time.perf_counter()
            loop.run(args.steps)
            barrier()
            repeats.append(round(world * args.steps / (time.perf_counter() - t1), 2))

    # live per-kernel durations (HIP events around each launch) for the roofline figure
    eng.prof_reset()
    skip0 = eng.skip_stats()
    eng.prof_enable(True)
    # the window on CLOCK_MONOTONIC, rocprofv3's timestamp domain: tools/rocprof_window.py averages
    # the same launches in a kernel trace of this command (profiles/rocprof_window.json)
    torch.cuda.synchronize(device)
    t_prof0 = time.monotonic_ns()
    loop.run(args.prof_steps)
    stats = eng.prof_collect()
    t_prof1 = time.monotonic_ns()
    eng.prof_enable(False)
    eng.prof_reset()
    prof_skip = {k: v - skip0[k] for k, v in eng.skip_stats().items()}
    # the launches' algorithmic bytes (host-side, per launch) count every head of every round; a
    # skipped policy's tiles return at once, so its bytes are not moved: take them off the kinds
    # they belong to (device counters over the same steps), so achieved GB/s stays honest
    launched = sum(v[2] for v in stats.values()) / max(args.prof_steps, 1)
    skb, skf = skippable_head_bytes(sh, B)
    nsk = prof_skip["policies_skipped"]
    for kd, per in (("bwd", skb), ("fwd", skf)):
        if kd in stats:
            n_, us_, by_ = stats[kd]
            stats[kd] = (n_, us_, max(0.0, by_ - nsk * per))

    unsk = None
    if world == 1 and args.schedule == "all" and args.tsf_K is None and rank == 0 and args.prof_steps > 0:
        unsk = unskipped_window(args, device, args.prof_steps)
    sharded = replicas = sharded_rccl1 = None
    layout = "single" if world == 1 else f"replica{world}"
    if world > 1 and args.schedule == "all" and args.tsf_K is None and args.layout == "sharded":
        # the headline at N > 1 is config C4's layout, timed with the same W / K; the replicas just
        # measured stay beside it
        replicas = {"value": round(value, 2), "unit": "env steps/s", "ms_per_step": round(1000.0 * dt / args.steps, 4),
                    "parallelism": f"replica{world}", "note": f"{world} independent 8-head learners, no collective"}
        try:
            sharded = bench_sharded(args, world, rank, device, barrier, dist, steps=args.steps, warmup=args.warmup)
        except Exception as e:  # an error return (not a hang): keep the replicas' line, say why
            print(f"rank {rank}: sharded C4 layout failed: {e!r}", file=sys.stderr, flush=True)
            sharded = {"error": repr(e)[:400]}
        if "error" not in sharded:
            value = sharded["value"]
            dt = sharded["ms_per_step"] * args.steps / 1000.0
            layout = f"shard{world}"
    elif args.shard_steps > 0 and args.schedule == "all":
        # the same window of training as the headline (its warmup, then its step count), so the two
        # rates compare like for like (the all-task rate rises as more speculative rounds skip)
        sharded = bench_sharded(args, world, rank, device, barrier, dist, steps=max(args.steps, args.shard_steps),
                                warmup=args.warmup)
        if world == 1 and not args.via_host:
            # the per-step cost the N > 1 headline pays: the same stream with real (captured)
            # ncclAllReduce calls at one rank, pipelined through the host rounds' split communicator
            os.environ["SFX_RCCL_WORLD1"] = "1"
            try:
                sharded_rccl1 = bench_sharded(args, world, rank, device, barrier, dist,
                                              steps=max(args.steps, args.shard_steps), warmup=args.warmup)
            except Exception as e:  # an error return (a bounded collective), not a hang
                sharded_rccl1 = {"error": repr(e)[:400]}
            finally:
                os.environ.pop("SFX_RCCL_WORLD1", None)
    elif args.shard_steps > 0 and args.schedule == "tsf":
        sharded = bench_sharded_tsf(args, world, rank, device, barrier, dist)
        if world == 1 and not args.via_host:
            os.environ["SFX_RCCL_WORLD1"] = "1"  # the collectives really issued, at one rank
            try:
                sharded_rccl1 = bench_sharded_tsf(args, world, rank, device, barrier, dist)
            except Exception as e:
                sharded_rccl1 = {"error": repr(e)[:400]}
            finally:
                os.environ.pop("SFX_RCCL_WORLD1", None)

    workload = (f"reacher17-{args.schedule}-T{T}-B{B}" if args.tsf_K is None else
                f"hopper11-tsf{'-nf' + str(args.tsf_K) if args.tsf_K else ''}-T{T}-B{B}")
    if rank == 0:
        kind = max(stats, key=lambda k: stats[k][1])
        n, us, by = stats[kind]
        avg_us = us / max(n, 1)
        bpl = by / max(n, 1)
        achieved = bpl / (avg_us * 1e-6) / 1e9 if n else 0.0
        traffic = traffic_from_profiles(kind, workload)
        roofline = {"bound": "hbm", "kernel": KIND_NAMES[kind], "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                    "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
                    "bytes_per_launch": round(bpl), "avg_launch_us": round(avg_us, 3),
                    "share_of_gpu_time": round(us / max(sum(v[1] for v in stats.values()), 1e-9), 3),
                    "per_kind_avg_us": {KIND_NAMES[k]: round(v[1] / max(v[0], 1), 3) for k, v in stats.items() if v[0]},
                    "prof_window": {"steps": args.prof_steps, "launches": n, "t0_ns": t_prof0, "t1_ns": t_prof1,
                                    "clock": "CLOCK_MONOTONIC", "where": "after the timed window and its repeats"}}
        if args.tsf_K is None and args.schedule == "all" and world == 1:
            # the same kind's average in the committed rocprofv3 kernel trace of this command: over the
            # same window of launches (profiles/rocprof_window.json), and over the whole profiled run
            # (one-GPU traces only: at N > 1 they would be another workload's numbers)
            rw = rocprof_window_from_profiles(KIND_NAMES[kind])
            rp = rocprof_avg_from_profiles(kind)
            if rw:
                roofline["rocprof_avg_us"] = round(rw["window_avg_us"], 3)
                roofline["rocprof_frac"] = round(bpl / (rw["window_avg_us"] * 1e-6) / 1e9 / HBM_PEAK_GBS, 5)
                roofline["rocprof_window_launches"] = rw["window_launches"]
                roofline["rocprof_source"] = "profiles/rocprof_window.json (same prof window of the same command)"
            if rp:
                roofline["rocprof_run_avg_us"] = round(rp, 3)
                roofline["rocprof_run_source"] = "profiles/headline_kernel_stats.csv (the whole profiled run)"
                if not rw:
                    roofline["rocprof_avg_us"] = round(rp, 3)
                    roofline["rocprof_frac"] = round(bpl / (rp * 1e-6) / 1e9 / HBM_PEAK_GBS, 5)
                    roofline["rocprof_source"] = "profiles/headline_kernel_stats.csv"
        if unsk is not None and kind in unsk["stats"]:
            un, uus, uby = unsk["stats"][kind]
            if un:
                ua = uby / un / (uus / un * 1e-6) / 1e9
                roofline["frac_unskipped"] = round(ua / HBM_PEAK_GBS, 5)
                roofline["unskipped"] = {"achieved": round(ua, 2), "avg_launch_us": round(uus / un, 3),
                                         "bytes_per_launch": round(uby / un), "launches": un,
                                         "steps": unsk["steps"], "policies_skipped": unsk["skipped"],
                                         "how": "fresh engine, SFX_SKIP=0, 200 warmup steps, eager prof window"}
        # SURVEY §8(d)'s whole-step figure: the ALGORITHMIC bytes of one env step x env-steps/s / peak,
        # per GPU.  Launched bytes (each launch's own minimum, summed -- speculative re-work included)
        # are reported beside it as a ratio, never as achieved bandwidth.
        P = head_params(sh)
        U = T if args.schedule == "all" else 1
        alg = algorithmic_step_bytes(T, U, P, 2)
        alg32 = algorithmic_step_bytes(T, U, P, 4)
        launched_moved = sum(v[2] for v in stats.values()) / max(args.prof_steps, 1)  # net of skipped work
        # each GPU runs every env step of the sharded stream (its T heads); replicas split the total
        per_gpu_rate = value if layout.startswith("shard") else value / world
        roofline["per_step"] = {
            "formula": "SURVEY 8(d): 2*wb*T*P + U*P*(3*wb + 28), P = params per head",
            "T": T, "U": U, "P": P,
            "algorithmic_bytes_per_env_step": round(alg), "achieved": round(alg * per_gpu_rate / 1e9, 2),
            "frac": round(alg * per_gpu_rate / 1e9 / HBM_PEAK_GBS, 5),
            "fp32_algorithmic_bytes_per_env_step": round(alg32),
            "fp32_achieved": round(alg32 * per_gpu_rate / 1e9, 2),
            "fp32_frac": round(alg32 * per_gpu_rate / 1e9 / HBM_PEAK_GBS, 5),
            "launched_bytes_per_env_step": round(launched),
            "skipped_policy_rounds_per_env_step": round(prof_skip["policies_skipped"] / max(args.prof_steps, 1), 3),
            "moved_bytes_per_env_step": round(launched_moved),
            "moved_over_fp32_algorithmic": round(launched_moved / alg32, 3), "unit": "GB/s"}
        # compute side (north_star: "MFMA utilisation against gfx950 peak"): the dominant kind's
        # algorithmic FLOPs per env step -- the backward half of 8(d)'s U*4*B*f, dX + dW = 2 forwards
        # -- over its GPU time per env step, and the MFMA busy cycles of the committed --pmc pass over
        # the live launch time (profiles/pmc_mfma.json)
        f = head_flops(sh)
        peak_c = MFMA_PEAK[args.precision]
        kind_flops = {"bwd": U * 2.0 * B * f}.get(kind)
        if kind_flops and us > 0:
            roofline["compute_frac"] = round(kind_flops * args.prof_steps / (us * 1e-6) / peak_c, 5)
            roofline["compute_peak_tflops"] = peak_c / 1e12
        mf = mfma_from_profiles(kind, workload, args.precision)
        if mf and avg_us > 0:
            roofline["mfma_util"] = round(mf["mfma_busy_cycles_per_launch"] / (avg_us * 1e-6 * CLK_HZ * SIMDS), 5)
            ex = mf["mfma_flops_f32_per_launch"] / MFMA_PEAK["fp32"] + mf["mfma_flops_bf16_per_launch"] / MFMA_PEAK["bf16"]
            roofline["mfma_executed_frac"] = round(ex / (avg_us * 1e-6), 5)
            roofline["mfma_source"] = ("profiles/pmc_mfma.json: SQ_VALU_MFMA_BUSY_CYCLES / (live avg launch x 2.4 GHz x "
                                       "1024 SIMDs); executed = MOPS_F32/BF16 x 512 FLOPs / live launch / peak")
        roofline["per_step"]["flops_per_env_step"] = round(T * f + T * B * f + U * 4 * B * f)
        roofline["per_step"]["compute_frac"] = round((T * f + T * B * f + U * 4 * B * f) * per_gpu_rate / peak_c, 5)
        spec_stats = eng.step_stats()
        spec_stats.update(eng.skip_stats())
        if native:
            spec_stats.update(loop.stats())
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            # the reference's CPU path on the box's cores.  The value is the best of
            # the thread counts this job may use (its CPU share: 8 and 16 threads timed), for both
            # schedules; the share is the ceiling -- more threads would take other jobs' cores
            share = cpu_share()
            tried = {}
            for th in sorted({max(1, share // 2), share}):
                tried[th] = cpu_baseline(args, args.cpu_seconds / 2, threads=th)
            best = max(tried.values(), key=lambda x: x["value"])
            cpu = dict(best)
            cpu["threads_tried"] = {str(k): round(v["value"], 2) for k, v in tried.items()}
            cpu["note"] = (f"cores = the best of {sorted(tried)} torch threads; this job's CPU share is {share} "
                           f"(OMP_NUM_THREADS) of the host's {cpu.get('physical_cores_on_host')} physical cores")
            if args.tsf_K is None and args.schedule == "all":
                act = argparse.Namespace(**vars(args))
                act.schedule = "active"
                cpu["active_task_schedule"] = {k: v for k, v in cpu_baseline(act, args.cpu_seconds / 2, threads=best["cores"]).items()
                                               if k in ("value", "unit", "cores", "kind", "sample")}
            if args.tsf_K is None and args.schedule == "all" and args.other:
                # C1 (CartPole shape, 2 source tasks) on the same host cores, beside the headline's
                c1 = argparse.Namespace(**vars(args))
                c1.c1, c1.heads = True, 2
                cpu["c1_cartpole4_all_T2_B32"] = {k: v for k, v in cpu_baseline(c1, 5.0).items()
                                                  if k in ("value", "unit", "cores", "kind", "sample")}
        other = None
        if world == 1 and args.other and args.tsf_K is None and args.schedule == "all":
            other = bench_other_workloads(args, device)
        out = {
            "metric": METRIC if args.tsf_K is None else
                      f"env steps/sec, Hopper 16-task TSF-DQN{' + planar-flow g' if args.tsf_K else ''} (BASELINE config "
                      f"{'C5' if args.tsf_K else 'C3'}, one GPU)", "value": round(value, 2), "unit": "env steps/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(1000.0 * dt / args.steps, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": args.precision, "data": "synthetic",
            "config": {"workload": (f"C4 layout: {T * world} Reacher tasks, {T} heads per GPU, one env stream; " if
                                    layout.startswith("shard") else "") + workload + (f" (Reacher-shape |s|=17 |a|=7 d=8, psi MLP 256x2, "
                                               f"{'all heads updated per env step: main_sfdqn_torch.py path' if args.schedule == 'all' else 'active head only: sfdqn.py path'})"
                                               if args.tsf_K is None else
                                               f" (Hopper-shape |s|=11 |a|=27 d=50, psi MLP 256x2, g/h width 100, "
                                               f"{args.tsf_K} planar layers, active head only: "
                                               f"{'tsfdqn_nf.py' if args.tsf_K else 'tsfdqn.py'} path)"),
                       "heads_per_gpu": T, "heads_total": T * world if layout.startswith("shard") else T,
                       "global_batch": B if layout.startswith("shard") else B * world,
                       "replay": args.replay if native else "host", "parallelism": layout,
                       "loop": (f"native C++ runner (sfx_runner_run, {args.schedule} schedule): host env + replay, one "
                                "pre-launched gated hipGraph per env step" if native else "python host loop over libsfx graphs")},
            "roofline": roofline,
            "repeats": {"values": repeats, "steps_each": args.steps} if repeats else None,
            "speculation": spec_stats,
            "sharded": sharded,
            "comm": (sharded or {}).get("comm") if world > 1 else None,
            "sharded_rccl_world1": sharded_rccl1,
            "replicas": replicas,
            "other_workloads": other,
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()
    if native:
        loop.close()
    eng.close()


if __name__ == "__main__":
    main()
