"""Build libsfx.so for gfx950 in-tree (the .so travels to the GPU box with the snapshot)."""
from __future__ import annotations

import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(os.path.dirname(HERE), "csrc")
LIB = os.path.join(HERE, "libsfx.so")


def build(force: bool = False, verbose: bool = False) -> str:
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    cmd = ["make", "-C", CSRC, f"HIPCC={hipcc}", f"OUT={LIB}"]
    if force:
        cmd.insert(1, "-B")
    res = subprocess.run(cmd, capture_output=True, text=True)
    if verbose or res.returncode != 0:
        print(res.stdout)
        print(res.stderr)
    if res.returncode != 0:
        raise RuntimeError("building libsfx.so failed")
    return LIB


if __name__ == "__main__":
    print(build(force=True, verbose=True))
