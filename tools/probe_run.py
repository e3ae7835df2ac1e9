"""In-kernel timing breakdown of the native env step (debug build with -DSFX_PROBE).

Build:  hipcc ... -DSFX_PROBE -o deep-successor-features-for-transfer_amd/sfx/libsfx_probe.so sfx.hip
Run:    SFX_LIB=.../libsfx_probe.so python tools/probe_run.py [steps]

Every probed workgroup logs (kernel id, block, t_entry, t_mark, t_end) on the 100 MHz wall
clock (t_end after its stores completed).  Launches are recovered by time clustering (a
stream's launches do not overlap); per launch we print the workgroup start spread, the
median / max body time, the median time to the mark (operands landed / MFMA done) and the
gap since the previous launch's last store.
"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "deep-successor-features-for-transfer_amd")]
import numpy as np
import torch

KIDS = {1: "fwd", 2: "fwdL0", 3: "bwd_tdg", 4: "dx", 5: "dw", 6: "dw_v0", 7: "round", 8: "ver", 9: "gate",
        10: "tsf_fwd", 11: "tsf_flows", 12: "tsf_h", 13: "tsf_glin", 14: "tsf_w", 15: "tsf_flow", 16: "gpi", 17: "tdg",
        18: "publish", 19: "fwd_gemv"}


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    # workload: all (default, the headline), active, tsf, tsf-nf
    work = sys.argv[2] if len(sys.argv) > 2 else "all"
    from bench import SHAPE, TSF_SHAPE, tsf_problem
    from sfx import _lib
    from sfx.engine import SFEngine
    from sfx.init import reference_heads
    from sfx.runner import NativeEnvLoop

    lib = _lib.lib
    lib.sfx_probe_dump.argtypes = [C.c_void_p, C.c_int]
    B = 32
    K = {"tsf": 0, "tsf-nf": 100}.get(work)
    sh = SHAPE if K is None else TSF_SHAPE
    T = 8 if K is None else 16
    eng = SFEngine(T, sh["n_s"], sh["H"], sh["A"], sh["d"], sh["acts"], max_batch=B)
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
    eng.set_precision(os.environ.get("SFX_PROBE_PREC", "fp32"))  # bf16: the operand mode's timeline
    loop = NativeEnvLoop(eng, batch=B, seed=1, schedule="all" if work == "all" else ("active" if work == "active" else "tsf"),
                         p_end=0.0 if K is None else 0.01)
    loop.prefill(1000)
    loop.set_task(0)
    dt = np.dtype([("kid", "<u4"), ("blk", "<u4"), ("t", "<u8", (10,))])
    buf = np.zeros(1 << 16, dtype=dt)
    loop.run(60)
    torch.cuda.synchronize()
    lib.sfx_probe_dump(buf.ctypes.data, len(buf))
    loop.run(steps)
    torch.cuda.synchronize()
    n = lib.sfx_probe_dump(buf.ctypes.data, len(buf))
    rec = buf[:n][np.argsort(buf[:n]["t"][:, 0], kind="stable")]
    if os.environ.get("SFX_PROBE_RAW"):
        np.save(os.environ["SFX_PROBE_RAW"], rec)
    # cluster into launches (a stream's launches do not overlap)
    launches, start, cur_end = [], 0, 0
    for i in range(len(rec)):
        t = rec[i]["t"]
        if i > start and t[0] > cur_end:
            launches.append(rec[start:i])
            start, cur_end = i, 0
        cur_end = max(cur_end, int(t[9]))
    launches.append(rec[start:])

    def marks(L):
        t = L["t"].astype(np.int64)
        rel = (t - t[:, :1]) * 10e-3
        out = [np.median(rel[:, 9]), rel[:, 9].max()]
        for j in (1, 2, 3, 4, 5, 6, 7, 8):
            ok = t[:, j] > 0
            out.append(np.median(rel[ok, j]) if ok.any() else np.nan)
        return out

    agg, sub, order = {}, {}, []
    prev_end, pos = None, 0
    for L in launches:
        kinds = tuple(sorted(set(int(k) for k in L["kid"])))
        if 9 in kinds:
            pos = 0
        key = (pos, kinds)
        pos += 1
        t = L["t"].astype(np.int64)
        gap = (t[:, 0].min() - prev_end) * 10e-3 if prev_end is not None else np.nan
        prev_end = t[:, 9].max()
        row = [(t[:, 0].max() - t[:, 0].min()) * 10e-3, (t[:, 9].max() - t[:, 0].min()) * 10e-3, gap] + marks(L) + [len(L)]
        if key not in agg:
            agg[key], sub[key] = [], {k: [] for k in kinds}
            order.append(key)
        agg[key].append(row)
        if len(kinds) > 1:
            for k in kinds:
                sub[key][k].append([int((L["kid"] == k).sum())] + marks(L[L["kid"] == k]))
    print(f"{n} records, {len(launches)} launches over {steps} steps (us; marks relative to workgroup entry:"
          " m1 = kernel arguments landed, m2 = operands landed / MFMA done, m3 / m4 kernel specific; k_round: m1..m6 after each phase)")
    print(f"{'pos':>3} {'kernel':16s} {'WGs':>5} {'spread':>6} {'span':>6} {'gap':>5} | {'body50':>6} {'bodymx':>6}"
          f" {'m1':>5} {'m2':>5} {'m3':>5} {'m4':>5} {'m5':>5} {'m6':>5} {'m7':>5} {'m8':>5}")
    tot_span = tot_gap = 0.0
    f = lambda x: "    -" if np.isnan(x) else f"{x:5.2f}"
    for key in order:
        pos, kinds = key
        a = np.array(agg[key], dtype=float)
        if len(a) < steps // 3:
            continue
        m = np.nanmedian(a, axis=0)
        nwg = int(m[-1])
        tot_span += m[1]
        tot_gap += 0 if np.isnan(m[2]) else m[2]
        name = "+".join(KIDS.get(k, str(k)) for k in kinds)
        print(f"{pos:3d} {name:16s} {nwg:5d} {m[0]:6.2f} {m[1]:6.2f} {f(m[2])} | {m[3]:6.2f} {m[4]:6.2f} "
              + " ".join(f(x) for x in m[5:13]))
        for k, v in sub[key].items():
            if v:
                u = np.nanmedian(np.array(v, dtype=float), axis=0)
                print(f"    {'- ' + KIDS.get(k, str(k)):16s} {int(u[0]):5d} {'':6s} {'':6s} {'':5s} | {u[1]:6.2f} {u[2]:6.2f} "
                      + " ".join(f(x) for x in u[3:11]))
    print(f"sum span {tot_span:.1f} us, sum gap {tot_gap:.1f} us")


if __name__ == "__main__":
    main()
