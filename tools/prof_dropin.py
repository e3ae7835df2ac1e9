"""cProfile of the drop-in host loop (tools/dropin_loop.py) -- where a drop-in env step's host time goes."""
import cProfile
import os
import pstats
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "deep-successor-features-for-transfer_amd")]
import torch  # noqa: E402

from tools import dropin_loop  # noqa: E402

buf = sys.argv[1] if len(sys.argv) > 1 else "host"
loop = dropin_loop.DropinLoop(buffer=buf)
loop.run(60)
torch.cuda.synchronize()
pr = cProfile.Profile()
pr.enable()
loop.run(300)
loop.sf._flush()
torch.cuda.synchronize()
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(35)
loop.close()
