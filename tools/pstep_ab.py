"""A/B of the persistent all-task step (k_pstep) against the launch path on the headline C2
workload (Reacher shape, T=8, B=32, native runner), alternating the two in one process so both see
the same box; with SFX_PSTEP_PROBE=1 also prints the last launch's per-head phase marks
(csrc/sfx_pstep.h PS_MARK ids, µs since the earliest mark)."""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "deep-successor-features-for-transfer_amd")]
import torch  # noqa: E402

from sfx._lib import lib  # noqa: E402
from sfx.engine import SFEngine  # noqa: E402
from sfx.init import reference_heads  # noqa: E402
from sfx.runner import NativeEnvLoop  # noqa: E402

SH = dict(n_s=17, H=256, A=7, d=8, acts=("relu", "relu"))


def run(pstep: bool, steps: int, warmup: int, T: int = 8, B: int = 32):
    eng = SFEngine(T, SH["n_s"], SH["H"], SH["A"], SH["d"], SH["acts"], max_batch=B, device="cuda")
    online, w = reference_heads(T, SH["n_s"], SH["H"], SH["A"], SH["d"], SH["acts"], seed=0)
    for t in range(T):
        eng.load_head(t, online[t], 0)
        eng.load_head(t, online[t], 1)
        eng.load_w(t, w[t])
    eng.set_adam(1e-3, 0.0, 1e-3, 0.0)
    eng.set_target_update_ev(1000)
    if pstep:
        eng.set_pstep(True)
    loop = NativeEnvLoop(eng, batch=B, seed=1, schedule="all", p_end=0.0)
    loop.prefill(1000)
    loop.set_task(0)
    loop.run(warmup)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    loop.run(steps)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    out = {"pstep": pstep, "env_steps_per_s": round(steps / dt, 1), "us_per_step": round(1e6 * dt / steps, 2)}
    if pstep:
        st = eng.pstep_stats()
        out["rounds_per_step"] = round(st["rounds"] / max(1, st["steps"]), 3)
        if os.environ.get("SFX_PSTEP_PROBE") == "1":
            buf = (ctypes.c_longlong * (8 * 64))()
            if lib.sfx_pstep_timeline(eng._h, buf) == 0:
                marks = [[buf[h * 64 + i] for i in range(64)] for h in range(8)]
                t_min = min(m for row in marks for m in row if m > 0)
                out["timeline_us"] = {i: [round((marks[h][i] - t_min) / 100.0, 2) if marks[h][i] > 0 else None
                                          for h in range(T)] for i in range(64)
                                      if any(marks[h][i] > 0 for h in range(T))}
    loop.close()
    eng.close()
    return out


if __name__ == "__main__":
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    for rep in range(reps):
        for ps in (False, True):
            r = run(ps, steps, 200)
            tl = r.pop("timeline_us", None)
            print(json.dumps(r), flush=True)
            if tl and rep == reps - 1:
                for i, row in tl.items():
                    print(f"  mark {i:2d} " + " ".join(f"{x:8.2f}" if x is not None else "       -" for x in row))
