"""Forward-only (eval, no_grad) passes of the config-3 model over one 32-story batch in two
16-story micro-batches: the north-star forward leg of bench.py, as a small rocprofv3 target.
usage: python tools/fwd_only.py [iters]"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import synthetic_batch  # noqa: E402
from multimodal_sequencing_amd import model_zoo  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 3
m = model_zoo.build_preset("config3", device="cuda", dtype=torch.bfloat16)
m.eval()
data = synthetic_batch(32, 5, 60, 50265, 224, "cuda", seed=1000)
mbs = [{k: v[o:o + 16] for k, v in data.items()} for o in (0, 16)]
with torch.no_grad():
    for b in mbs:
        m(b)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        for b in mbs:
            m(b)
    torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / iters
print(f"forward 32 stories: {dt * 1e3:.1f} ms = {32 / dt:.1f} stories/s = "
      f"{32 / dt * 3.411:.0f} TFLOP/s ({32 / dt * 3.411 / 2500:.3f} of 2.5 PF)", flush=True)
