#!/usr/bin/env python3
"""One sharded leg of bench.py on its own (for rocprofv3 traces and quick A/Bs): the C4 layout
(all-task, --heads per rank) or the C5 layout (--workload hopper-tsf-nf) at world 1, RCCL forced
(SFX_RCCL_WORLD1=1) unless --no-rccl.  Prints one JSON line."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "deep-successor-features-for-transfer_amd")]

import bench  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--workload", default="reacher-sf", choices=list(bench.WORKLOADS))
    p.add_argument("--heads", type=int, default=64)
    p.add_argument("--steps", type=int, default=2000)
    p.add_argument("--warmup", type=int, default=200)
    p.add_argument("--no-rccl", action="store_true")
    a = p.parse_args()
    import torch

    if not a.no_rccl:
        os.environ["SFX_RCCL_WORLD1"] = "1"
    args = argparse.Namespace(heads=a.heads, batch=32, spec_rounds=0, precision="fp32", via_host=False,
                              shard_steps=a.steps, tsf_K=bench.WORKLOADS[a.workload])
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    barrier = torch.cuda.synchronize
    if args.tsf_K is None:
        out = bench.bench_sharded(args, 1, 0, dev, barrier, None, steps=a.steps, warmup=a.warmup)
    else:
        out = bench.bench_sharded_tsf(args, 1, 0, dev, barrier, None, steps=a.steps, warmup=a.warmup)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
