"""In-kernel timing of the TSF kernels (debug build with -DSFX_PROBE), per kernel / role.

Build:  cd deep-successor-features-for-transfer_amd/csrc && hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC
        -shared -ffp-contract=off -DSFX_PROBE -o ../sfx/libsfx_probe.so sfx.hip
Run:    SFX_LIB=.../libsfx_probe.so python tools/probe_tsf.py [K] [updates]

Prints, per TSF kernel role, the median time (us, from workgroup entry) to each mark and to
the end of its stores: k_tsf_fwd m1 staged / m2 flows done; flow role m1 staged+daff / m2 dg /
m3 dz; other roles m1 staged+daff.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "deep-successor-features-for-transfer_amd")]
import ctypes as C

import numpy as np
import torch

NAMES = {10: "tsf_fwd", 11: "bwd:flows", 12: "bwd:h", 13: "bwd:g-lin", 14: "bwd:w", 15: "tsf_flow"}


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 100
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    import bench
    from sfx import _lib
    from sfx.engine import SFEngine

    lib = _lib.lib
    lib.sfx_probe_dump.argtypes = [C.c_void_p, C.c_int]
    sh = bench.TSF_SHAPE
    T, B = 16, 32
    online, w, g, h = bench.tsf_problem(T, K, seed=0)
    eng = SFEngine(T, sh["n_s"], sh["H"], sh["A"], sh["d"], sh["acts"], max_batch=B)
    eng.tsf_setup(sh["G"], K, 1.0, 1e-3, 0.0, 1e-3, 0.0)
    for t in range(T):
        eng.load_head(t, online[t], 0)
        eng.load_head(t, online[t], 1)
        eng.load_w(t, w[t])
        eng.tsf_load_g(t, g[t])
    eng.tsf_load_h(h)
    gen = torch.Generator().manual_seed(1)
    dev = eng.device
    batch = [torch.randn(B, sh["n_s"], generator=gen).to(dev), torch.randint(0, sh["A"], (B,), generator=gen).to(dev),
             torch.rand(B, generator=gen).to(dev), torch.rand(B, sh["d"], generator=gen).to(dev),
             torch.randn(B, sh["n_s"], generator=gen).to(dev), torch.full((B,), 0.9, device=dev)]
    dt = np.dtype([("kid", "<u4"), ("blk", "<u4"), ("t", "<u8", (10,))])
    buf = np.zeros(1 << 16, dtype=dt)
    for _ in range(10):
        eng.tsf_update(0, *batch)
    torch.cuda.synchronize()
    lib.sfx_probe_dump(buf.ctypes.data, len(buf))
    for _ in range(n):
        eng.tsf_update(0, *batch)
    torch.cuda.synchronize()
    cnt = lib.sfx_probe_dump(buf.ctypes.data, len(buf))
    rec = buf[:cnt]
    print(f"K={K}: {cnt} records over {n} updates (us from workgroup entry, medians; end = stores done)")
    print(f"{'role':12s} {'WGs/upd':>7} {'m1':>7} {'m2':>7} {'m3':>7} {'end':>7} {'end max':>8}")
    for kid, name in NAMES.items():
        r = rec[rec["kid"] == kid]
        if not len(r):
            continue
        t = r["t"].astype(np.int64)
        rel = (t - t[:, :1]) * 10e-3
        cols = []
        for j in (1, 2, 3):
            ok = t[:, j] > 0
            cols.append(f"{np.median(rel[ok, j]):7.2f}" if ok.any() else "      -")
        print(f"{name:12s} {len(r) / n:7.1f} " + " ".join(cols) + f" {np.median(rel[:, 9]):7.2f} {rel[:, 9].max():8.2f}")
    eng.close()


if __name__ == "__main__":
    main()
